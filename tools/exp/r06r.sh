# Round 6: FE-2D's x re-fetch (EA reads 1.006e9 B per product = 0.80e9 values + ~0.19e9 x: x fetched ~2.4x).
# (1) chunk interleave (VBC_SLOT_ILV=1: range r takes chunks r, r + R, ...) against contiguous ranges, in one
# process, bitwise check; the bench line (oracle parity) with it; (2) EA read requests of both; (3) the
# range-count sweep on the ablation build (several rounds of waves = a narrower active window).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab.py --workload fe --dtype f64 --graph --reps 20 --rounds 5 --copies 2 --variants "VBC_SLOT_ILV=0,VBC_VERBOSE=1;VBC_SLOT_ILV=1,VBC_VERBOSE=1" > gpurun_out/r06r_fe_ilv.log 2>&1 || { tail -20 gpurun_out/r06r_fe_ilv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06r_fe_ilv.log | grep "slot bin\|rel-diff" | tail -8
VBC_SLOT_ILV=1 timeout -k 10 300 python -u bench.py --workload fe --no-secondary --no-cpu-baseline --steps 20 > gpurun_out/r06r_fe_ilv_bench.log 2>&1 || { tail -20 gpurun_out/r06r_fe_ilv_bench.log; exit 1; }
tail -1 gpurun_out/r06r_fe_ilv_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench ilv', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['parity'])"
for v in 0 1; do
  VBC_SLOT_ILV=$v timeout -k 10 300 python -u tools/pmc_traffic.py --workload fe --dtype f64 --kernel spmv_slots --counters "TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum;TCC_HIT_sum,TCC_MISS_sum" --tag _ilv$v > gpurun_out/r06r_pmc_ilv$v.log 2>&1 || { tail -20 gpurun_out/r06r_pmc_ilv$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/pmc_fe_f64_ilv$v.json')); print('ilv $v', d['hbm_bytes_per_launch'], d['rdreq_per_launch']['all'], round(d['l2_hit_rate'],3))"
done
A=tools/exp/libs/libvbc_ablation.so
V="@lib=$A"
for n in 8192 16384 32768; do V="$V;@lib=$A,VBC_TARGET_RANGES_S=$n"; done
timeout -k 10 400 python -u tools/ab.py --workload fe --dtype f64 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r06r_fe_ranges.log 2>&1 || { tail -20 gpurun_out/r06r_fe_ranges.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06r_fe_ranges.log | tail -4
