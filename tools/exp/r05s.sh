# staged-X tile form: parity (mfma tests) then c5-mesh A/B both directions
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "staged" > gpurun_out/r05s_tests.log 2>&1 || { tail -30 gpurun_out/r05s_tests.log; exit 1; }
tail -3 gpurun_out/r05s_tests.log
V="@multi,VBC_TILE_STAGE=0;@multi,VBC_TILE_STAGE=1;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=32,VBC_TILE_UMAX=128;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=96,VBC_TILE_UMAX=224;@multi,VBC_TILE_STAGE=1,VBC_TILE_SMAX=48,VBC_TILE_UMAX=160"
VBC_VERBOSE=1 timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05s_ab.log 2>&1 || { tail -20 gpurun_out/r05s_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05s_ab.log | grep -v "^\[vbc\]" | tail -6
grep "staged X" gpurun_out/r05s_ab.log | sort | uniq | head
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --trans 0 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "@multifwd,VBC_TILE_STAGE=0;@multifwd,VBC_TILE_STAGE=1" > gpurun_out/r05s_abf.log 2>&1 || { tail -20 gpurun_out/r05s_abf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05s_abf.log | tail -3
