# Round 6: rank-local handles rebased (stripe split) / trimmed (row split) to what the shard touches
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_bench.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r06j_tests.log 2>&1 || { tail -40 gpurun_out/r06j_tests.log; exit 1; }
tail -2 gpurun_out/r06j_tests.log
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --steps 100 > gpurun_out/r06j_shard_ldoor.log 2>&1 || { tail -20 gpurun_out/r06j_shard_ldoor.log; exit 1; }
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --split rows --steps 100 > gpurun_out/r06j_shard_ldoor_rows.log 2>&1 || { tail -20 gpurun_out/r06j_shard_ldoor_rows.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r06j_shard_ldoor.log", "gpurun_out/r06j_shard_ldoor_rows.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(d["split"], d["world"], d["max_us_wall"], d["speedup_vs_first"], d.get("fwd_max_us_wall"), d.get("fwd_speedup_vs_first"), d["shards"][0]["kernel"][:40], d["shards"][0].get("fwd_kernel", "")[:40])
PY
