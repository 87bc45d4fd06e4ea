#!/bin/bash
# GPU-box runner (gpurun -- 'bash tools/gpu.sh STEP...'): each step under its own time limit, the
# chain stops at the first failure.  Logs go to gpurun_out/.
#   tests [PYTEST-ARGS]   python -m pytest -m gpu (all GPU tests by default)
#   smoke                 __graft_entry__.smoke()
#   bench [ARGS]          python bench.py ARGS
#   prof  [ARGS]          rocprofv3 --kernel-trace --stats -- python bench.py ARGS
#   ab    [ARGS]          python tools/ab.py ARGS
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${GPU_TAG:-run}
step=$1; shift
case "$step" in
  tests) timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread "$@" \
           > gpurun_out/${tag}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${tag}_tests.log; exit $rc ;;
  smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
         rc=$?; tail -2 gpurun_out/${tag}_smoke.log; exit $rc ;;
  bench) timeout -k 10 900 python -u bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1; rc=$?
         tail -c 3000 gpurun_out/${tag}_bench.log; exit $rc ;;
  prof)  rm -rf gpurun_out/${tag}_prof
         timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python -u bench.py "$@" \
           > gpurun_out/${tag}_prof.log 2>&1; rc=$?; tail -c 2000 gpurun_out/${tag}_prof.log; exit $rc ;;
  ab)    timeout -k 10 900 python -u tools/ab.py "$@" > gpurun_out/${tag}_ab.log 2>&1; rc=$?
         tail -40 gpurun_out/${tag}_ab.log; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
