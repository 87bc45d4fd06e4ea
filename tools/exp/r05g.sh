mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05g_tests.log 2>&1 || { tail -30 gpurun_out/r05g_tests.log; exit 1; }
tail -2 gpurun_out/r05g_tests.log
V="@multi,VBC_PANEL_TILES=0;@multi,VBC_TILE_X4=0,VBC_TILE_SPR=32"
for spr in 8 16 32; do for nb in 4 8; do V="$V;@multi,VBC_TILE_SPR=$spr,VBC_TILE_NBT=$nb"; done; done
timeout -k 10 500 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05g_ab.log 2>&1 || exit $?
tail -8 gpurun_out/r05g_ab.log
