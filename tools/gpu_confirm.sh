# Round-end style confirmation on one MI355X: GPU tests, smoke, bench, rocprofv3 kernel statistics.
# Usage: gpurun --timeout 1200 -- 'bash tools/gpu_confirm.sh'
set -e -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python -u bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
