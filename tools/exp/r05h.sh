# L2 behaviour of the tile kernel vs its stripes per range (the XCD's front of concurrent stripes)
mkdir -p gpurun_out; export TMPDIR=/tmp
for spr in 4 8 32; do
VBC_TILE_SPR=$spr timeout -k 10 600 python -u tools/pmc_traffic.py --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 --tag _spr$spr --counters "TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum;SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU" > gpurun_out/r05h_pmc_$spr.log 2>&1 || exit $?
done
grep -h '"l2_hit_rate"\|"all"' gpurun_out/pmc_c5-mesh_f32_spr*.json
