mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05l_gpu_tests.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r05l_gpu_tests.log | tail -15
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r05l_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r05l_bench.log
