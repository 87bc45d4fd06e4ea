set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sweep_tests.log; [ $rc -ne 0 ] && exit $rc
V="@lib=tools/prevlib/libvbc.so;VBC_SWEEP=-1;VBC_SWEEP_TILE=16;VBC_SWEEP_TILE=8;VBC_SWEEP_TILE=16,VBC_SWEEP_DIAG=1"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --variants "$V" > gpurun_out/sw9_t64.log 2>&1 || exit $?
V="@lib=tools/prevlib/libvbc.so;VBC_SWEEP=-1;VBC_SWEEP_TILE=32;VBC_SWEEP_TILE=8"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f32 --variants "$V" > gpurun_out/sw9_t32.log 2>&1 || exit $?
V="@lib=tools/prevlib/libvbc.so;VBC_SWEEP=-1;VBC_SWEEP_TILE=16"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --trans 0 --variants "$V" > gpurun_out/sw9_f64.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns-mixed --dtype f64 --variants "$V" > gpurun_out/sw9_m64.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/sw9_t64.log gpurun_out/sw9_t32.log gpurun_out/sw9_f64.log gpurun_out/sw9_m64.log
