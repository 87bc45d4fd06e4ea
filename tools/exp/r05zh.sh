# FE-3D lane streams: range count / deep pipeline / XCD order knobs at HEAD
mkdir -p gpurun_out; export TMPDIR=/tmp
V="VBC_NONE=0;VBC_TARGET_RANGES_L=12288;VBC_TARGET_RANGES_L=16384;VBC_LANES_DEEP=1;VBC_XCD=0;VBC_TARGET_RANGES_L=2048"
VBC_VERBOSE=1 timeout -k 10 600 python -u tools/ab.py --workload fe3d --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zh_ab.log 2>&1 || { tail -20 gpurun_out/r05zh_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zh_ab.log | grep -v "^\[vbc\]" | tail -6
grep "lanes bin" gpurun_out/r05zh_ab.log | sort | uniq | cut -c1-200 | head
