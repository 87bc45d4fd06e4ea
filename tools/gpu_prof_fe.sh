set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
WORKLOADS=fe bash tools/gpu_prof.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_fe2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_fe2.log
grep -A3 '"AverageNs"' gpurun_out/prof_fe/run_kernel_stats.csv | head -3
