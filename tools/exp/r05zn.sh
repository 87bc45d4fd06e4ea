# the bench's own C5 fp32 line alone, default vs 4096 ranges
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "" "VBC_TARGET_RANGES_M=4096"; do
env $v timeout -k 10 300 python -u bench.py --workload c5 --dtype f32 --no-cpu-baseline --no-secondary > gpurun_out/r05zn_bench_c5.log 2>&1 || { tail -5 gpurun_out/r05zn_bench_c5.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r05zn_bench_c5.log') if l.startswith('{')][-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['dtype'])"
done
