# C5 panel range count with placement spread (--copies 3) and the bench line twice per setting
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u tools/ab.py --workload c5 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --copies 3 --variants "@multi,VBC_TARGET_RANGES_M=2048;@multi,VBC_TARGET_RANGES_M=4096" > gpurun_out/r05zo_c5.log 2>&1 || { tail -20 gpurun_out/r05zo_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zo_c5.log | tail -6
for v in "VBC_TARGET_RANGES_M=2048" "VBC_TARGET_RANGES_M=4096" "VBC_TARGET_RANGES_M=2048" "VBC_TARGET_RANGES_M=4096"; do
env $v timeout -k 10 300 python -u bench.py --workload c5 --dtype f32 --no-cpu-baseline --no-secondary > gpurun_out/r05zo_bench_c5.log 2>&1 || { tail -5 gpurun_out/r05zo_bench_c5.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r05zo_bench_c5.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
