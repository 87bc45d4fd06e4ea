#!/bin/bash
# PMC traffic records for the bench's kernels (gpurun -- 'bash tools/pmc_suite.sh'): every counter group
# its own rocprofv3 pass (tools/pmc_traffic.py), each pass under its own time limit; stops at the
# first failure.  Output: gpurun_out/pmc_<workload>_<dtype>[tag].json
set -u -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G="TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum"
run() { timeout -k 10 600 python -u tools/pmc_traffic.py --counters "$G" "$@" >> gpurun_out/pmc_suite.log 2>&1; }
# round 3: the kernels the bench reports (lanes for FE-3D, masked lane pairs for ldoor fp64, the forward
# panel for c5-fwd); SUITE=short runs the three that changed this round
if [ "${SUITE:-all}" = short ]; then
run --workload fe3d --dtype f64 --kernel spmv_planar_lanes &&
run --workload ldoor --dtype f64 --kernel spmv_planar_pair &&
run --workload fe --dtype f64 --kernel spmv_slots
else
run --workload fe --dtype f64 --kernel spmv_slots &&
run --workload fe3d --dtype f64 --kernel spmv_planar_lanes &&
run --workload ldoor --dtype f64 --kernel spmv_planar_pair &&
run --workload ldoor --dtype f32 --kernel spmv_planar &&
run --workload c5 --dtype f32 --kernel spmm_panel --read-factor 1 &&
run --workload c5-fwd --dtype f32 --kernel spmm_panel --read-factor 1 &&
VBC_PANEL_DIAG=4 run --workload c5 --dtype f32 --kernel spmm_panel --read-factor 1 --tag _xcached &&
run --workload ns --dtype f64 --kernel spmv_sweep --read-factor 1
fi
