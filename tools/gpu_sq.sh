set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/pmc_traffic.py --workload c5 --dtype f32 --kernel spmm_panel --read-factor 1 \
  --counters "SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_LDS;SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_WR,SQ_BUSY_CYCLES,SQ_INSTS_MFMA" > gpurun_out/sq_c5.log 2>&1 || exit $?
grep -v "^pass" gpurun_out/sq_c5.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['mean'])) for k,v in d['counters'].items()]"
