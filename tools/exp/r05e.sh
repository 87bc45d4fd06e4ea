# PMC of the c5-mesh multi-RHS kernels: the tile layout (default) and the MFMA panel (VBC_PANEL_TILES=0)
mkdir -p gpurun_out; export TMPDIR=/tmp
G="SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU;TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum,TA_TA_BUSY_sum,TA_BUSY_avr,TCC_HIT_sum,TCC_MISS_sum;TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_BUBBLE_sum"
timeout -k 10 900 python -u tools/pmc_traffic.py --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 --counters "$G" > gpurun_out/r05e_pmc_tiles.log 2>&1 || exit $?
VBC_PANEL_TILES=0 timeout -k 10 900 python -u tools/pmc_traffic.py --workload c5-mesh --dtype f32 --kernel spmm_panel --read-factor 1 --tag _panel --counters "$G" > gpurun_out/r05e_pmc_panel.log 2>&1 || exit $?
tail -5 gpurun_out/r05e_pmc_panel.log
