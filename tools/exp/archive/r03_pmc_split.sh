#!/bin/bash
set -u -o pipefail
export TMPDIR=/tmp
G="TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum"
timeout -k 10 600 python -u tools/pmc_traffic.py --steps 50 --counters "$G" --workload ct20stif --dtype f64 --kernel spmv_planar_split --read-factor 1 > gpurun_out/pmc_split.log 2>&1 &&
VBC_DIAG=4 timeout -k 10 600 python -u tools/pmc_traffic.py --steps 50 --counters "$G" --workload ct20stif --dtype f64 --kernel spmv_planar_split --read-factor 1 --tag _nt >> gpurun_out/pmc_split.log 2>&1
