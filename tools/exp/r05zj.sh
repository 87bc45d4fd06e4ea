# range-count knobs at HEAD on the other bench workloads (fewer, longer ranges, as for the FE-3D lane tiles)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab.py --workload c5 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "@multi;@multi,VBC_TARGET_RANGES_M=2048;@multi,VBC_TARGET_RANGES_M=8192" > gpurun_out/r05zj_c5.log 2>&1 || { tail -20 gpurun_out/r05zj_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zj_c5.log | tail -3
timeout -k 10 600 python -u tools/ab.py --workload ns --graph --reps 20 --rounds 3 --variants "VBC_NONE=0;VBC_TARGET_RANGES_S=2048;VBC_TARGET_RANGES_S=8192" > gpurun_out/r05zj_ns.log 2>&1 || { tail -20 gpurun_out/r05zj_ns.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zj_ns.log | tail -3
timeout -k 10 600 python -u tools/ab.py --workload ldoor --graph --reps 50 --rounds 3 --variants "VBC_NONE=0;VBC_PLANAR_WPS_PAIR=2;VBC_TARGET_RANGES_P=2048" > gpurun_out/r05zj_ldoor.log 2>&1 || { tail -20 gpurun_out/r05zj_ldoor.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zj_ldoor.log | tail -3
