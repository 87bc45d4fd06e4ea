# round-5 confirmation at HEAD + the c5-mesh tile kernel's PMC record
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_confirm.sh r05q || exit $?
timeout -k 10 600 python -u tools/pmc_traffic.py --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 --counters "TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum" > gpurun_out/r05q_pmc_c5mesh.log 2>&1 || exit $?
tail -3 gpurun_out/r05q_pmc_c5mesh.log
