# Round-end style confirmation on one MI355X: GPU tests, smoke, bench, rocprofv3 kernel statistics.
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_confirm.sh [TAG]'   (logs: gpurun_out/TAG_*)
# Test failures (pytest rc 1) are reported and the rest still runs; any other failure ends the script.
tag=${1:-confirm}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/${tag}_gpu_tests.log | tail -20
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 420 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -c 1500 gpurun_out/${tag}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
    python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_prof_bench.log 2>&1 || exit $?
exit $rc
