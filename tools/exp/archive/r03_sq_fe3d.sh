# SQ / TA / TCP counters of the FE-3D lane-stream kernel (and its L2-confined-gather ablation, VBC_DIAG=2)
export TMPDIR=/tmp; mkdir -p gpurun_out
G="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VMEM,SQ_BUSY_CYCLES,SQ_WAVES,SQ_INSTS_VMEM_RD;TA_BUSY_avr,TA_TA_BUSY_sum,TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum"
timeout -k 10 400 python -u tools/pmc_traffic.py --counters "$G" --workload fe3d --dtype f64 --kernel spmv_planar_lanes --tag _sq > gpurun_out/sq_fe3d.log 2>&1 &&
VBC_DIAG=2 timeout -k 10 400 python -u tools/pmc_traffic.py --counters "$G" --workload fe3d --dtype f64 --kernel spmv_planar_lanes --tag _sq_diag2 > gpurun_out/sq_fe3d_diag2.log 2>&1 &&
timeout -k 10 400 python -u tools/pmc_traffic.py --counters "$G" --workload fe --dtype f64 --kernel spmv_slots --tag _sq > gpurun_out/sq_fe.log 2>&1
ls gpurun_out/*_sq*.json
