# C5 MFMA panel: ranges per product (VBC_TARGET_RANGES_M), both directions, fp32 and fp64
mkdir -p gpurun_out; export TMPDIR=/tmp
V="@multi;@multi,VBC_TARGET_RANGES_M=1024;@multi,VBC_TARGET_RANGES_M=1536;@multi,VBC_TARGET_RANGES_M=2048;@multi,VBC_TARGET_RANGES_M=3072"
timeout -k 10 600 python -u tools/ab.py --workload c5 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zk_c5.log 2>&1 || { tail -20 gpurun_out/r05zk_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zk_c5.log | tail -5
VF="@multifwd;@multifwd,VBC_TARGET_RANGES_M=1024;@multifwd,VBC_TARGET_RANGES_M=1536;@multifwd,VBC_TARGET_RANGES_M=2048;@multifwd,VBC_TARGET_RANGES_M=3072"
timeout -k 10 600 python -u tools/ab.py --workload c5 --trans 0 --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$VF" > gpurun_out/r05zk_c5f.log 2>&1 || { tail -20 gpurun_out/r05zk_c5f.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zk_c5f.log | tail -5
timeout -k 10 600 python -u tools/ab.py --workload c5 --dtype f64 --nrhs 16 --graph --reps 10 --rounds 3 --variants "@multi;@multi,VBC_TARGET_RANGES_M=2048" > gpurun_out/r05zk_c5d.log 2>&1 || { tail -20 gpurun_out/r05zk_c5d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zk_c5d.log | tail -2
