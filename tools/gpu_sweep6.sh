set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1; rc=$?; tail -15 gpurun_out/sweep_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SWEEP=0;VBC_SWEEP=-1;VBC_SWEEP=-1,VBC_SWEEP_TILE=16"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --trans 0 --variants "$V" > gpurun_out/sw6_f64.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f32 --trans 0 --variants "$V" > gpurun_out/sw6_f32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns-mixed --dtype f64 --trans 0 --variants "$V" > gpurun_out/sw6_m64.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/sw6_f64.log gpurun_out/sw6_f32.log gpurun_out/sw6_m64.log
