# PMC records of the masked planar layout (FE-3D fp64 / fp32; the length-sorted layout as _sorted)
set -u -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G="TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum"
run() { timeout -k 10 600 python -u tools/pmc_traffic.py --counters "$G" "$@" >> gpurun_out/pmc_mask.log 2>&1; }
run --workload fe3d --dtype f64 --kernel spmv_planar &&
VBC_PLANAR_MASK=0 run --workload fe3d --dtype f64 --kernel spmv_planar --tag _sorted &&
run --workload fe3d --dtype f32 --kernel spmv_planar
