# C5 panel at the new default range count: tests, then default vs the old count
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05zl_tests.log 2>&1 || { tail -30 gpurun_out/r05zl_tests.log; exit 1; }
tail -1 gpurun_out/r05zl_tests.log
timeout -k 10 600 python -u tools/ab.py --workload c5 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "@multi;@multi,VBC_TARGET_RANGES_M=4096" > gpurun_out/r05zl_c5.log 2>&1 || { tail -20 gpurun_out/r05zl_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zl_c5.log | tail -2
