# C5 panel: default range count vs explicit counts, more rounds; then the bench's own c5 line
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab.py --workload c5 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 5 --variants "@multi;@multi,VBC_TARGET_RANGES_M=2048;@multi,VBC_TARGET_RANGES_M=4096;@multi" > gpurun_out/r05zm_c5.log 2>&1 || { tail -20 gpurun_out/r05zm_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zm_c5.log | tail -4
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/r05zm_bench_c5.log 2>&1 || { tail -5 gpurun_out/r05zm_bench_c5.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r05zm_bench_c5.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
