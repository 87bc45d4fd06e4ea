# Round 6: the same SQ / TA / TCP / TCC counter passes for the tile kernel (c5-mesh, never recorded with
# them) and for FE-3D / FE-2D at HEAD, to compare their L1-side request rates (gpurun_out/pmc_*_r06v.json)
set -u -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
G="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU;TA_TA_BUSY_sum,TA_BUSY_avr,TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum;SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_VMEM_WR;TCC_EA0_RDREQ_sum;TCC_HIT_sum,TCC_MISS_sum"
run() { timeout -k 10 600 python -u tools/pmc_traffic.py --counters "$G" --tag _r06v "$@" >> gpurun_out/r06v_pmc.log 2>&1; }
run --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 &&
run --workload fe3d --dtype f64 --kernel spmv_planar_lanes &&
run --workload fe --dtype f64 --kernel spmv_slots || { tail -30 gpurun_out/r06v_pmc.log; exit 1; }
python3 - <<'PY'
import json
for w, dt in (("c5-mesh", "f32"), ("fe3d", "f64"), ("fe", "f64")):
    d = json.load(open(f"gpurun_out/pmc_{w}_{dt}_r06v.json"))
    c = {k: v["mean"] for k, v in d["counters"].items()}
    print(w, {k: f"{v:.4g}" for k, v in c.items()})
PY
