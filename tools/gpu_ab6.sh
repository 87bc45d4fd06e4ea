set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_slots.py -x -q --timeout 120 --timeout-method thread > gpurun_out/slots.log 2>&1; rc=$?; tail -3 gpurun_out/slots.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SLOTS=0;VBC_SLOT_KEYS16=0;VBC_SLOT_KEYS16=1"
timeout -k 10 300 python tools/ab.py --workload fe --variants "$V" > gpurun_out/ab6_fe_t.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --trans 0 --variants "$V" > gpurun_out/ab6_fe_f.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --variants "$V" > gpurun_out/ab6_fe_t32.log 2>&1 || exit $?
cat gpurun_out/ab6_fe_t.log gpurun_out/ab6_fe_f.log gpurun_out/ab6_fe_t32.log | grep -v amdgpu.ids
