# staged-X tile form: ablations (no staging / no stores) and cluster sizes
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "staged" > gpurun_out/r05w_tests.log 2>&1 || { tail -30 gpurun_out/r05w_tests.log; exit 1; }
mkdir -p gpurun_out; export TMPDIR=/tmp
V="@multi,VBC_TILE_STAGE=0;@multi,VBC_TILE_STAGE=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_DIAG=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_DIAG=2;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=80,VBC_TILE_UMAX=224;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=48,VBC_TILE_UMAX=160"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05w_ab.log 2>&1 || { tail -20 gpurun_out/r05w_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05w_ab.log | grep -v "^\[vbc\]" | tail -6
