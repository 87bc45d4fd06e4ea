set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sweep_tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SWEEP=0;VBC_SWEEP=1,VBC_SWEEP_TILE=8;VBC_SWEEP=1,VBC_SWEEP_TILE=16;VBC_SWEEP=1,VBC_SWEEP_TILE=32;VBC_SWEEP=1,VBC_SWEEP_TILE=16,VBC_SWEEP_DIAG=1;VBC_SWEEP=1,VBC_SWEEP_TILE=16,VBC_SWEEP_DIAG=2"
timeout -k 10 400 python tools/ab.py --workload ns --dtype f64 --variants "$V" > gpurun_out/sw3_ns.log 2>&1 || exit $?
V="VBC_SWEEP=0;VBC_SWEEP=1,VBC_SWEEP_TILE=8;VBC_SWEEP=1,VBC_SWEEP_TILE=16;VBC_SWEEP=1,VBC_SWEEP_TILE=32"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f32 --variants "$V" > gpurun_out/sw3_ns32.log 2>&1 || exit $?
cat gpurun_out/sw3_ns.log gpurun_out/sw3_ns32.log | grep -v amdgpu.ids
