# dword tile kernel with the per-stripe 16-B epilogue: blob order revisited
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "blob or tiles_mixed or node_runs" > gpurun_out/r05zg_tests.log 2>&1 || { tail -30 gpurun_out/r05zg_tests.log; exit 1; }
tail -1 gpurun_out/r05zg_tests.log
V="@multi;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=512;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=128;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=2048;@multi,VBC_TILE_ORDER=1,VBC_TILE_BLOB=512,VBC_TILE_SPR=16"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zg_ab.log 2>&1 || { tail -20 gpurun_out/r05zg_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zg_ab.log | tail -5
