# Round 6: the clustered-order test and the tile tests at HEAD
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py tests/test_gpu_knobs.py > gpurun_out/r06zc_tests.log 2>&1 || { tail -30 gpurun_out/r06zc_tests.log; exit 1; }
tail -1 gpurun_out/r06zc_tests.log
