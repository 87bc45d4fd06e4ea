set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/pmc_traffic.py --workload fe --dtype f64 --kernel spmv_slots --read-factor 2 > gpurun_out/pmc_fe.log 2>&1 || exit $?
tail -5 gpurun_out/pmc_fe.log
