set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="@lib=tools/prevlib/libvbc.so;VBC_SLOT_PAIR=0;VBC_SLOT_PAIR=1"
timeout -k 10 300 python tools/ab.py --workload fe --dtype f64 --copies 2 --variants "$V" > gpurun_out/pair_fe64.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor --dtype f64 --variants "$V" > gpurun_out/pair_c3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/pair_fe64.log gpurun_out/pair_c3.log
