set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_slots.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -2 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="@lib=tools/prevlib/libvbc.so;VBC_SLOTS=-1"
timeout -k 10 300 python tools/ab.py --workload fe --dtype f64 --copies 3 --variants "$V" > gpurun_out/hdr_fe64.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --copies 2 --variants "$V" > gpurun_out/hdr_fe32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f64 --trans 0 --variants "$V" > gpurun_out/hdr_fef.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor-csc --dtype f32 --variants "$V" > gpurun_out/hdr_c4.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor --dtype f64 --variants "$V" > gpurun_out/hdr_c3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/hdr_fe64.log gpurun_out/hdr_fe32.log gpurun_out/hdr_fef.log gpurun_out/hdr_c4.log gpurun_out/hdr_c3.log
