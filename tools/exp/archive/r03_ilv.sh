# Interleaved lane streams (every 64th stripe per lane) vs contiguous sub-blocks: parity (lanes tests with the
# mode forced on) and FE-3D / ldoor A/B
mkdir -p gpurun_out; export TMPDIR=/tmp
VBC_LANES_INTERLEAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_ilv_tests.log 2>&1; tail -2 gpurun_out/r03_ilv_tests.log
run() { timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 "$@"; }
V="VBC_LANES_INTERLEAVE=0;VBC_LANES_INTERLEAVE=1"
run --workload fe3d --variants "$V" > gpurun_out/r03_ilv_fe3d.log 2>&1 && tail -2 gpurun_out/r03_ilv_fe3d.log &&
run --workload fe3d --trans 0 --variants "$V" > gpurun_out/r03_ilv_fe3dfwd.log 2>&1 && tail -2 gpurun_out/r03_ilv_fe3dfwd.log &&
run --workload fe3d --dtype f32 --variants "$V" > gpurun_out/r03_ilv_fe3df32.log 2>&1 && tail -2 gpurun_out/r03_ilv_fe3df32.log
