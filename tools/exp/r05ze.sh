# staged-X forms at their final defaults: the multi-RHS tests (all four layouts)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ze_tests.log 2>&1 || { tail -30 gpurun_out/r05ze_tests.log; exit 1; }
tail -1 gpurun_out/r05ze_tests.log
