# FE-3D lane tiles sized for half the resident waves (VBC_LANES_RDIV, default 2): both directions
mkdir -p gpurun_out; export TMPDIR=/tmp
V="VBC_LANES_RDIV=1;VBC_LANES_RDIV=2;VBC_LANES_RDIV=4"
timeout -k 10 600 python -u tools/ab.py --workload fe3d --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zi_ab.log 2>&1 || { tail -20 gpurun_out/r05zi_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zi_ab.log | tail -3
timeout -k 10 600 python -u tools/ab.py --workload fe3d --trans 0 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zi_abf.log 2>&1 || { tail -20 gpurun_out/r05zi_abf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zi_abf.log | tail -3
timeout -k 10 600 python -u tools/ab.py --workload fe3d --dtype f32 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zi_ab32.log 2>&1 || { tail -20 gpurun_out/r05zi_ab32.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zi_ab32.log | tail -3
