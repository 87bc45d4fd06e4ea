set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export VBC_SWEEP_TILE=16
timeout -k 10 500 python tools/pmc_traffic.py --workload ns --dtype f64 --kernel spmv_sweep --read-factor 1 \
  --counters "TCC_HIT_sum,TCC_MISS_sum;SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_LDS,SQ_BUSY_CYCLES;SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU" > gpurun_out/sq_sweep.log 2>&1 || exit $?
grep -v "^pass" gpurun_out/sq_sweep.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['mean'])) for k,v in d['counters'].items()]; print({k:v for k,v in d.items() if k!='counters'})"
