#!/bin/bash
# rocprofv3 kernel-trace stats + PMC HBM traffic for the bench workloads (separate passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${WORKLOADS:-fe ns}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$wl -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --workload $wl > gpurun_out/prof_$wl.log 2>&1
  rc=$?; echo "prof $wl rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 python tools/pmc_traffic.py --workload $wl > gpurun_out/pmc_$wl.log 2>&1
  rc=$?; echo "pmc $wl rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
