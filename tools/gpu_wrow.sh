set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SLOT_WROW=0;VBC_SLOT_WROW=1"
timeout -k 10 300 python tools/ab.py --workload ldoor --dtype f64 --copies 2 --variants "$V" > gpurun_out/wrow_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ct20stif --dtype f64 --variants "$V" > gpurun_out/wrow_c2.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wrow_c3.log gpurun_out/wrow_c2.log
