mkdir -p gpurun_out; export TMPDIR=/tmp
V="@multi;@multi,VBC_TILE_ORDER=1,VBC_TILE_SPR=8;@multi,VBC_TILE_ORDER=1,VBC_TILE_SPR=16;@multi,VBC_TILE_ORDER=1,VBC_TILE_SPR=32;@multi,VBC_TILE_ORDER=1,VBC_TILE_SPR=16,VBC_TILE_BLOB=128;@multi,VBC_TILE_ORDER=1,VBC_TILE_SPR=16,VBC_TILE_BLOB=2048"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05p_ab.log 2>&1 || exit $?
tail -6 gpurun_out/r05p_ab.log
for v in "VBC_TILE_ORDER=0" "VBC_TILE_ORDER=1 VBC_TILE_SPR=16"; do
env $v timeout -k 10 600 python -u tools/pmc_traffic.py --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 --tag _r05p_$(echo $v | tr ' =' '__') --counters "TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum" > gpurun_out/r05p_pmc.log 2>&1 || exit $?
done
grep -h '"l2_hit_rate"\|"all"' gpurun_out/pmc_c5-mesh_f32_r05p*.json
