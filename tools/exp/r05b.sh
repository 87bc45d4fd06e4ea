mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05b_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r05b_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 5 --variants "@multi,VBC_PANEL_TILES=0;@multi,VBC_PANEL_TILES=1" > gpurun_out/r05b_ab.log 2>&1 || exit $?
cat gpurun_out/r05b_ab.log | tail -5
