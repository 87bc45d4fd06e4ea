mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --steps 100 --forward > gpurun_out/r05o_shard_ldoor.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/shard_time.py --workload fe --dtype f64 --worlds 1,2,4,8 --steps 50 > gpurun_out/r05o_shard_fe.log 2>&1 || exit $?
python - <<'P'
import json
for f in ("gpurun_out/r05o_shard_ldoor.log","gpurun_out/r05o_shard_fe.log"):
    for l in open(f):
        if l.startswith("{"):
            d=json.loads(l); print(d["workload"], d["world"], d["max_us_wall"], d["speedup_vs_first"], d.get("fwd_max_us_wall"), d.get("fwd_speedup_vs_first"))
P
