# forward multi-RHS on matrix cores: tests, bench line, PMC traffic (C5 shape)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma_fwd.py tests/test_gpu_mfma.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03f_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5-fwd --dtype f32 --no-secondary --no-cpu-baseline > gpurun_out/r03f_bench_c5fwd.log 2>&1; rc=$?; tail -c 1500 gpurun_out/r03f_bench_c5fwd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/pmc_traffic.py --workload c5-fwd --dtype f32 --kernel spmm_panel --read-factor 1 > gpurun_out/r03f_pmc.log 2>&1; rc=$?; tail -5 gpurun_out/r03f_pmc.log; exit $rc
