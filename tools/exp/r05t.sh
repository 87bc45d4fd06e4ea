# staged-X tile form, round 2: parallel X staging, per-wave stream lengths
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "staged" > gpurun_out/r05t_tests.log 2>&1 || { tail -30 gpurun_out/r05t_tests.log; exit 1; }
tail -2 gpurun_out/r05t_tests.log
V="@multi,VBC_TILE_STAGE=0;@multi,VBC_TILE_STAGE=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=32,VBC_TILE_UMAX=128;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=48,VBC_TILE_UMAX=160;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=24,VBC_TILE_UMAX=96"
VBC_VERBOSE=1 timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05t_ab.log 2>&1 || { tail -20 gpurun_out/r05t_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05t_ab.log | grep -v "^\[vbc\]" | tail -5
grep "staged X, w" gpurun_out/r05t_ab.log | sort | uniq | head
