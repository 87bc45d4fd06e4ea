mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05d_tests.log 2>&1; rc=$?
tail -12 gpurun_out/r05d_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 5 --variants "@multi,VBC_PANEL_TILES=0;@multi,VBC_PANEL_TILES=1,VBC_TILE_NBT=4;@multi,VBC_PANEL_TILES=1,VBC_TILE_NBT=8" > gpurun_out/r05d_ab.log 2>&1 || exit $?
tail -4 gpurun_out/r05d_ab.log
timeout -k 10 400 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --trans 0 --graph --reps 20 --rounds 5 --variants "@multifwd,VBC_PANEL_TILES=0;@multifwd,VBC_PANEL_TILES=1,VBC_TILE_NBT=4" > gpurun_out/r05d_abf.log 2>&1 || exit $?
tail -3 gpurun_out/r05d_abf.log
