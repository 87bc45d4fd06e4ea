# Round 6: padding tiles' X loads pointed at row 0's block vs past X (-DVBC_TILE_PAD_OOB build); tile tests
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py > gpurun_out/r06z2_tests.log 2>&1 || { tail -30 gpurun_out/r06z2_tests.log; exit 1; }
tail -1 gpurun_out/r06z2_tests.log
A=tools/exp/libs/libvbc_padoob.so
for t in 1 0; do
  m=$([ $t = 1 ] && echo @multi || echo @multifwd)
  timeout -k 10 400 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --trans $t --graph --reps 20 --rounds 5 --copies 2 --variants "$m;$m,@lib=$A" > gpurun_out/r06z2_ab_t$t.log 2>&1 || { tail -20 gpurun_out/r06z2_ab_t$t.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r06z2_ab_t$t.log | tail -4
done
