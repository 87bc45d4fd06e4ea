mkdir -p gpurun_out; export TMPDIR=/tmp
V="@multi,VBC_TILE_SPR=32;@multi,VBC_TILE_SPR=32,VBC_TILE_DIAG=1;@multi,VBC_TILE_SPR=32,VBC_TILE_DIAG=2;@multi,VBC_TILE_SPR=32,VBC_TILE_DIAG=3"
timeout -k 10 500 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05i_ab.log 2>&1 || exit $?
tail -4 gpurun_out/r05i_ab.log
