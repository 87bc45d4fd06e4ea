# Round 6: fp64 runs of 3 gathered by lane pairs (ld_xrun): the one-gather-per-lane build (-DVBC_XRUN_SINGLE,
# tools/exp/build_variant.sh) vs the product, FE-3D both directions and the ldoor shards (split kernels)
mkdir -p gpurun_out; export TMPDIR=/tmp
A=tools/exp/libs/libvbc_xrun1.so
for t in 1 0; do
timeout -k 10 400 python -u tools/ab.py --workload fe3d --trans $t --graph --reps 20 --rounds 3 --variants "@lib=$A;@x" > gpurun_out/r06o_fe3d_t$t.log 2>&1 || { tail -20 gpurun_out/r06o_fe3d_t$t.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06o_fe3d_t$t.log | tail -2
done
for v in old new; do
if [ $v = old ]; then export VBC_LIBRARY=$PWD/$A; else unset VBC_LIBRARY; fi
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --forward --steps 100 > gpurun_out/r06o_shard_ldoor_$v.log 2>&1 || { tail -20 gpurun_out/r06o_shard_ldoor_$v.log; exit 1; }
python - $v <<'PY'
import json, sys
for l in open(f"gpurun_out/r06o_shard_ldoor_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["split"], d["world"], d["max_us_wall"], d["speedup_vs_first"], d.get("fwd_max_us_wall"), d.get("fwd_speedup_vs_first"), [s["us_event"] for s in d["shards"]][:3])
PY
done
