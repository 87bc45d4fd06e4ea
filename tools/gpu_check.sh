#!/bin/bash
# One GPU session: smoke -> parity tests -> bench -> rocprofv3 kernel stats.  Every GPU step has its
# own time limit; a crash/timeout (rc >= 124 or signal) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-smoke,tests,bench,prof}
[[ $STEPS == *smoke* ]] && { step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1; }
[[ $STEPS == *tests* ]] && step tests 900 python -m pytest tests -m "gpu and not slow" -x -q
[[ $STEPS == *slow* ]] && step slow 900 python -m pytest tests -m "slow" -x -q
[[ $STEPS == *bench* ]] && step bench 600 python bench.py --steps 50 --warmup 5
[[ $STEPS == *fe* ]] && step bench_fe 600 python bench.py --steps 50 --warmup 5 --workload fe --no-cpu-baseline
[[ $STEPS == *prof* ]] && step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary
echo "== done $(date +%T)"
