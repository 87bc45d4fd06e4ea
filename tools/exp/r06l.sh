# Round 6: partial-output shard products with one fill launch (N = 1, 2, 4, 8)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --steps 100 > gpurun_out/r06l_shard_ldoor.log 2>&1 || { tail -20 gpurun_out/r06l_shard_ldoor.log; exit 1; }
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --split rows --steps 100 > gpurun_out/r06l_shard_ldoor_rows.log 2>&1 || { tail -20 gpurun_out/r06l_shard_ldoor_rows.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r06l_shard_ldoor.log", "gpurun_out/r06l_shard_ldoor_rows.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(d["split"], d["world"], d["max_us_wall"], d["speedup_vs_first"], d.get("fwd_max_us_wall"), d.get("fwd_speedup_vs_first"), [s.get("fwd_us_event") for s in d["shards"]])
PY
