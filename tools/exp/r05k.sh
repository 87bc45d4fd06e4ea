mkdir -p gpurun_out; export TMPDIR=/tmp
VBC_TILE_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -m gpu -q -x -k "tiles or c5" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k_tests.log 2>&1 || { tail -30 gpurun_out/r05k_tests.log; exit 1; }
tail -2 gpurun_out/r05k_tests.log
V="@multi,VBC_TILE_SPR=14;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=256;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=1024;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=4096;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=1024,VBC_TILE_X4=0,VBC_TILE_SPR=32;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=1024,VBC_TILE_X4=0,VBC_TILE_SPR=32,VBC_TILE_NBT=8"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05k_ab.log 2>&1 || exit $?
tail -6 gpurun_out/r05k_ab.log
