# Round 6: chunk interleave with LDS-staged y writes (one store per staged chunk) vs contiguous ranges
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab.py --workload fe --dtype f64 --graph --reps 20 --rounds 5 --copies 2 --variants "VBC_SLOT_ILV=0;VBC_SLOT_ILV=1" > gpurun_out/r06t_fe_ilv.log 2>&1 || { tail -20 gpurun_out/r06t_fe_ilv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06t_fe_ilv.log | tail -4
timeout -k 10 400 python -u tools/ab.py --workload fe --dtype f32 --graph --reps 20 --rounds 5 --variants "VBC_SLOT_ILV=0;VBC_SLOT_ILV=1" > gpurun_out/r06t_fe32_ilv.log 2>&1 || { tail -20 gpurun_out/r06t_fe32_ilv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06t_fe32_ilv.log | tail -2
VBC_SLOT_ILV=1 timeout -k 10 300 python -u bench.py --workload fe --no-secondary --no-cpu-baseline --steps 20 > gpurun_out/r06t_fe_ilv_bench.log 2>&1 || { tail -20 gpurun_out/r06t_fe_ilv_bench.log; exit 1; }
tail -1 gpurun_out/r06t_fe_ilv_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench ilv', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['parity']['pass'], d['parity']['bitwise_equal'])"
