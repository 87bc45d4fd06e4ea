# Round 6: lane-stream values grouped by run (fp64 3 x 3: 4 x 16 B + 8 B per run) vs one planar row per stored
# row (-DVBC_LANES_ROWMAJOR build); the planar / lanes GPU tests; FE-3D both directions
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planar.py tests/test_gpu_configs.py -k "lanes or fe3d or planar" > gpurun_out/r06zd_tests.log 2>&1 || { tail -30 gpurun_out/r06zd_tests.log; exit 1; }
tail -1 gpurun_out/r06zd_tests.log
A=tools/exp/libs/libvbc_rowmajor.so
for t in 1 0; do
  timeout -k 10 400 python -u tools/ab.py --workload fe3d --dtype f64 --trans $t --graph --reps 20 --rounds 5 --copies 2 --variants "@x;@lib=$A" > gpurun_out/r06zd_ab_t$t.log 2>&1 || { tail -20 gpurun_out/r06zd_ab_t$t.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r06zd_ab_t$t.log | tail -4
done
