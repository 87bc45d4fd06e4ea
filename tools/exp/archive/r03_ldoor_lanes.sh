# ldoor stand-in: lane streams forced (both directions) vs the default layouts; tile counts
mkdir -p gpurun_out; export TMPDIR=/tmp
V="VBC_X=0;VBC_PLANAR_LANES=1;VBC_PLANAR_LANES=1,VBC_TARGET_RANGES_L=2048;VBC_PLANAR_LANES=1,VBC_TARGET_RANGES_L=1024"
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --workload ldoor --trans 0 --variants "$V" > gpurun_out/r03_ldoor_lanes_fwd.log 2>&1 && tail -4 gpurun_out/r03_ldoor_lanes_fwd.log &&
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --workload ldoor --variants "$V" > gpurun_out/r03_ldoor_lanes_t.log 2>&1 && tail -4 gpurun_out/r03_ldoor_lanes_t.log
