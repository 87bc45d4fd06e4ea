set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_bp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fe4 -o run -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --workload fe --dtype f64 > gpurun_out/prof_fe4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ns4 -o run -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --workload ns --dtype f64 > gpurun_out/prof_ns4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c54 -o run -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --workload c5 --dtype f32 > gpurun_out/prof_c54.log 2>&1 || exit $?
grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/bench_bp.log gpurun_out/prof_fe4.log gpurun_out/prof_ns4.log gpurun_out/prof_c54.log
for d in fe4 ns4 c54; do sed -n 2p gpurun_out/prof_$d/run_kernel_stats.csv | cut -c1-160; done
