# Round 6: tile-kernel pipeline depth on c5-mesh (D = 3 ring vs the D = 2 ping-pong; NBT 4 / 8), parity first
mkdir -p gpurun_out; export TMPDIR=/tmp
A=tools/exp/libs/libvbc_ablation.so
VBC_LIBRARY=$A VBC_TILE_DEPTH=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -q -x --timeout 120 --timeout-method thread -k "c5_mesh or tiles" > gpurun_out/r06d_tests_d3.log 2>&1 || { tail -30 gpurun_out/r06d_tests_d3.log; exit 1; }
tail -1 gpurun_out/r06d_tests_d3.log
VBC_LIBRARY=$A VBC_TILE_DEPTH=3 VBC_TILE_NBT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -q -x --timeout 120 --timeout-method thread -k "c5_mesh or tiles" > gpurun_out/r06d_tests_d3n4.log 2>&1 || { tail -30 gpurun_out/r06d_tests_d3n4.log; exit 1; }
tail -1 gpurun_out/r06d_tests_d3n4.log
V="@lib=$A,@multi;@lib=$A,@multi,VBC_TILE_DEPTH=3;@lib=$A,@multi,VBC_TILE_DEPTH=3,VBC_TILE_NBT=4;@lib=$A,@multi,VBC_TILE_NBT=4"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r06d_ab.log 2>&1 || { tail -20 gpurun_out/r06d_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06d_ab.log | tail -8
