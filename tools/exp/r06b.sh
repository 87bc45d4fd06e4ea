# Round 6: auto-split tests, ldoor stripe / row shard timings (both directions), PMC of the 1/8 stripe shard
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_knobs.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r06b_tests.log 2>&1 || { tail -30 gpurun_out/r06b_tests.log; exit 1; }
tail -1 gpurun_out/r06b_tests.log
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --steps 100 > gpurun_out/r06b_shard_ldoor.log 2>&1 || { tail -20 gpurun_out/r06b_shard_ldoor.log; exit 1; }
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --split rows --steps 100 > gpurun_out/r06b_shard_ldoor_rows.log 2>&1 || { tail -20 gpurun_out/r06b_shard_ldoor_rows.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r06b_shard_ldoor.log", "gpurun_out/r06b_shard_ldoor_rows.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(d["split"], d["world"], d["max_us_wall"], d["speedup_vs_first"], d.get("fwd_max_us_wall"), d.get("fwd_speedup_vs_first"), d["shards"][0]["kernel"][:40], d["shards"][0].get("fwd_kernel", "")[:40])
PY
timeout -k 10 600 python -u tools/pmc_traffic.py --program tools/shard_time.py --workload ldoor --dtype f64 --kernel spmv_planar --tag _shard8 --extra "--worlds 8 --ranks 0" --counters "TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum" > gpurun_out/r06b_pmc_shard.log 2>&1 || { tail -20 gpurun_out/r06b_pmc_shard.log; exit 1; }
grep -E '"hbm_bytes_per_launch"|"l2_hit_rate"|"all"' gpurun_out/pmc_ldoor_f64_shard8.json
