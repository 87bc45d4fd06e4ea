set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench3.log 2>&1 || exit $?
tail -1 gpurun_out/bench3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fe3 -o run -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --workload fe --dtype f64 > gpurun_out/prof_fe3.log 2>&1 || exit $?
head -2 gpurun_out/prof_fe3/run_kernel_stats.csv; grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/prof_fe3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns3 -o run -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --workload ns --dtype f64 > gpurun_out/prof_ns3.log 2>&1 || exit $?
head -2 gpurun_out/prof_ns3/run_kernel_stats.csv; grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/prof_ns3.log
