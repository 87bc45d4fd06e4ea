set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns -o run -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --workload ns --dtype f64 > gpurun_out/prof_ns.log 2>&1 || exit $?
timeout -k 10 500 python tools/pmc_traffic.py --workload ns --dtype f64 --kernel spmv_sweep --read-factor 1 \
  --counters "TCC_HIT_sum,TCC_MISS_sum" > gpurun_out/pmc_ns.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --trans 0 --variants "VBC_SWEEP=0;VBC_SWEEP=-1" > gpurun_out/ab_nsfwd.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f32 --trans 0 --variants "VBC_SWEEP=0;VBC_SWEEP=-1" > gpurun_out/ab_nsfwd32.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_r01b.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_nsfwd.log gpurun_out/ab_nsfwd32.log; tail -1 gpurun_out/bench_r01b.log
