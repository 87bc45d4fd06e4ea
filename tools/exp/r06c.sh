# Round 6: row-split shards aligned to node runs (both directions), then the reference's table at HEAD
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_sharded.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || { tail -30 gpurun_out/r06c_tests.log; exit 1; }
tail -1 gpurun_out/r06c_tests.log
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --split rows --steps 100 > gpurun_out/r06c_shard_ldoor_rows.log 2>&1 || { tail -20 gpurun_out/r06c_shard_ldoor_rows.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06c_shard_ldoor_rows.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["split"], d["world"], d["max_us_wall"], d["speedup_vs_first"], d.get("fwd_max_us_wall"), d.get("fwd_speedup_vs_first"), d["model_e2e_us"]["main"], d.get("fwd_model_e2e_us"), d["shards"][0]["kernel"][:40], d["shards"][0].get("fwd_kernel", "")[:40])
PY
bash tools/exp/r06_table.sh r06_table
