# staged-X tile form with 8 compute waves per cluster workgroup (two 80 KB workgroups per CU)
mkdir -p gpurun_out; export TMPDIR=/tmp
VBC_VERBOSE=1 VBC_TILE_PERSIST=0 timeout -k 10 120 python -u tools/exp/xp_smoke.py 0.002 > gpurun_out/r05zd_smoke.log 2>&1 || { tail -20 gpurun_out/r05zd_smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zd_smoke.log | tail -4
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "staged" > gpurun_out/r05zd_tests.log 2>&1 || { tail -30 gpurun_out/r05zd_tests.log; exit 1; }
tail -1 gpurun_out/r05zd_tests.log
V="@multi,VBC_TILE_STAGE=0;@multi,VBC_TILE_STAGE=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=96,VBC_TILE_UMAX=192;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=160,VBC_TILE_UMAX=320;@multi,VBC_TILE_STAGE=1,VBC_TILE_WAVES=4"
VBC_VERBOSE=1 timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zd_ab.log 2>&1 || { tail -20 gpurun_out/r05zd_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zd_ab.log | grep -v "^\[vbc\]" | tail -5
grep "staged X, w" gpurun_out/r05zd_ab.log | sort | uniq | head
