set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sweep_tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SWEEP=-1,VBC_SWEEP_BANKS=0;VBC_SWEEP=-1"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --copies 2 --variants "$V" > gpurun_out/sw7_t64.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f32 --variants "$V" > gpurun_out/sw7_t32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --trans 0 --variants "$V" > gpurun_out/sw7_f64.log 2>&1 || exit $?
VBC_SWEEP=0 timeout -k 10 500 python tools/pmc_traffic.py --workload ns --dtype f64 --kernel spmv_slots --read-factor 1 \
  --counters "TCC_HIT_sum,TCC_MISS_sum" > gpurun_out/pmc_ns_slots.log 2>&1 || exit $?
cp gpurun_out/pmc_ns_f64.json gpurun_out/pmc_ns_slots_f64.json
grep -v amdgpu.ids gpurun_out/sw7_t64.log gpurun_out/sw7_t32.log gpurun_out/sw7_f64.log
