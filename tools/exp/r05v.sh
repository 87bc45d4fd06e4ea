# staged-X tile form: ablations (no staging / no stores) and cluster sizes
mkdir -p gpurun_out; export TMPDIR=/tmp
V="@multi,VBC_TILE_STAGE=0;@multi,VBC_TILE_STAGE=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_DIAG=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_DIAG=2;@multi,VBC_TILE_STAGE=1,VBC_TILE_DIAG=3;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=24,VBC_TILE_UMAX=96,VBC_TILE_DIAG=3"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05v_ab.log 2>&1 || { tail -20 gpurun_out/r05v_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05v_ab.log | grep -v "^\[vbc\]" | tail -6
