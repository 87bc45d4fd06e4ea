mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05j_tests.log 2>&1 || { tail -30 gpurun_out/r05j_tests.log; exit 1; }
tail -2 gpurun_out/r05j_tests.log
V="@multi,VBC_PANEL_TILES=0;@multi,VBC_TILE_SPR=8;@multi,VBC_TILE_SPR=14;@multi,VBC_TILE_SPR=14,VBC_TILE_NBT=8;@multi,@lib=tools/exp/libvbc_reducedpp.so,VBC_TILE_SPR=32;@multi,@lib=tools/exp/libvbc_reducedpp.so,VBC_TILE_SPR=32,VBC_TILE_NBT=8"
timeout -k 10 500 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05j_ab.log 2>&1 || exit $?
tail -6 gpurun_out/r05j_ab.log
