# Round 6: x spans of the sharded handle (vbc_sharded_xspan) -- the multi-GPU tests incl. the span test
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_sharded.py tests/test_abi.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r06g_tests.log 2>&1 || { tail -40 gpurun_out/r06g_tests.log; exit 1; }
tail -2 gpurun_out/r06g_tests.log
