set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SWEEP=0;VBC_SWEEP=1,VBC_SWEEP_EQ=0;VBC_SWEEP=1"
timeout -k 10 400 python tools/ab.py --workload ns-mixed --dtype f64 --variants "$V" > gpurun_out/sw4_nsm.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab.py --workload ns-mixed --dtype f32 --variants "$V" > gpurun_out/sw4_nsm32.log 2>&1 || exit $?
V="VBC_SWEEP=0;VBC_SWEEP=-1"
timeout -k 10 400 python tools/ab.py --workload ns --dtype f64 --copies 2 --variants "$V" > gpurun_out/sw4_ns.log 2>&1 || exit $?
timeout -k 10 400 python tools/ab.py --workload fe --dtype f64 --variants "$V" > gpurun_out/sw4_fe.log 2>&1 || exit $?
cat gpurun_out/sw4_nsm.log gpurun_out/sw4_nsm32.log gpurun_out/sw4_ns.log gpurun_out/sw4_fe.log | grep -v amdgpu.ids
