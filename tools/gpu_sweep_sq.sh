set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_LDS_BANK_CONFLICT;TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum;TA_BUSY_avr,TA_TA_BUSY_sum"
for d in 1 0; do
  VBC_SWEEP_TILE=16 VBC_SWEEP_DIAG=$d timeout -k 10 300 python tools/pmc_traffic.py --workload ns --dtype f64 --kernel spmv_sweep --read-factor 1 --counters "$C" > gpurun_out/sq_sweep_d$d.log 2>&1 || exit $?
  cp gpurun_out/pmc_ns_f64.json gpurun_out/sq_sweep_d$d.json
done
python - <<'PY'
import json
for d in (1, 0):
    j = json.load(open(f"gpurun_out/sq_sweep_d{d}.json"))
    print("DIAG", d, {k: round(v["mean"]) for k, v in j["counters"].items()})
PY
