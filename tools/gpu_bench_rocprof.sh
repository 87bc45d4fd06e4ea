set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
# the bench line and the kernel statistics of the SAME process (the default bench command)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
    python bench.py > gpurun_out/bench_prof.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_prof.log | tail -1 | cut -c1-400
cut -c1-150 gpurun_out/prof_bench/run_kernel_stats.csv | head -6
