#!/bin/bash
# PMC passes for the panel kernel (one counter group per pass, --kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
WL=${WL:-c5}; DT=${DT:-f32}
i=0
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp_stats -o run -- python tools/exp/panel_run.py --workload $WL --dtype $DT > gpurun_out/pp_stats.log 2>&1 || exit 1
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE" "WRITE_SIZE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  echo "pass $i: $grp"
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pp_$i -o pmc -- python tools/exp/panel_run.py --workload $WL --dtype $DT > gpurun_out/pp_$i.log 2>&1 || echo "pass $i failed rc=$?"
  i=$((i+1))
done
exit 0
