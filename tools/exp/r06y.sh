# Round 6: tile ranges launched as BFS balls of one XCD's resident waves (VBC_TILE_CLUSTER=1, X rows of a
# ball fit the XCD's L2) vs natural stripe order; tile tests with both; c5-mesh both directions; c5 random
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py > gpurun_out/r06y_tests.log 2>&1 || { tail -30 gpurun_out/r06y_tests.log; exit 1; }
tail -1 gpurun_out/r06y_tests.log
for t in 1 0; do
  m=$([ $t = 1 ] && echo @multi || echo @multifwd)
  timeout -k 10 400 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --trans $t --graph --reps 20 --rounds 5 --copies 2 --variants "$m,VBC_TILE_CLUSTER=0;$m,VBC_TILE_CLUSTER=1,VBC_VERBOSE=1" > gpurun_out/r06y_ab_t$t.log 2>&1 || { tail -20 gpurun_out/r06y_ab_t$t.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r06y_ab_t$t.log | grep "tiles:\|TFLOP" | tail -5
done
