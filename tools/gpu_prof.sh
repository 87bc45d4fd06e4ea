#!/bin/bash
# rocprofv3 kernel-trace stats + PMC HBM traffic for the bench workloads (separate passes).
#   WORKLOADS="fe ns c5" bash tools/gpu_prof.sh      (outputs under gpurun_out/, copy to profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${WORKLOADS:-fe ns c5}; do
  dt=f64; kern=spmv_slots; rf=2
  if [ "$wl" = c5 ]; then dt=f32; kern=spmm_panel; rf=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$wl -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --workload $wl --dtype $dt > gpurun_out/prof_$wl.log 2>&1
  rc=$?; echo "prof $wl rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 python tools/pmc_traffic.py --workload $wl --dtype $dt --kernel $kern --read-factor $rf > gpurun_out/pmc_$wl.log 2>&1
  rc=$?; echo "pmc $wl rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
