# Round 6: tile kernel value loads -- lanes past the batch's values read lane 0's address (one segment
# instead of four for the second load) vs every lane its own 16 B (-DVBC_TILE_VALS_ALL build); tile tests
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfma.py tests/test_gpu_mfma_fwd.py > gpurun_out/r06w_tests.log 2>&1 || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
tail -1 gpurun_out/r06w_tests.log
A=tools/exp/libs/libvbc_valsall.so
timeout -k 10 300 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --trans 1 --graph --reps 20 --rounds 5 --copies 2 --variants "@multi;@multi,@lib=$A" > gpurun_out/r06w_ab_t1.log 2>&1 || { tail -20 gpurun_out/r06w_ab_t1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06w_ab_t1.log | tail -4
timeout -k 10 300 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --trans 0 --graph --reps 20 --rounds 5 --copies 2 --variants "@multifwd;@multifwd,@lib=$A" > gpurun_out/r06w_ab_t0.log 2>&1 || { tail -20 gpurun_out/r06w_ab_t0.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06w_ab_t0.log | tail -4
