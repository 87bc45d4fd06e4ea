set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SLOT_NARROW=0;VBC_SLOT_NARROW=1"
timeout -k 10 300 python tools/ab.py --workload ldoor-csc --dtype f32 --copies 2 --variants "$V" > gpurun_out/ab13_c4.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --copies 2 --variants "$V" > gpurun_out/ab13_fe32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f64 --copies 2 --variants "$V" > gpurun_out/ab13_fe64.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench13.log 2>&1 || exit $?
cat gpurun_out/ab13_c4.log gpurun_out/ab13_fe32.log gpurun_out/ab13_fe64.log gpurun_out/bench13.log | grep -v amdgpu.ids
