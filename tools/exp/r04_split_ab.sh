# Fused small-matrix split: pipelined slice loop and P, on the stand-ins' table partitions (graph-timed A/B)
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 50 "$@" > gpurun_out/r04_ab4_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab4_$tag.log | tail -6; }
V="VBC_SPLIT_PIPE=-1;VBC_SPLIT_PIPE=0;VBC_SPLIT_NT_MB=100000;VBC_SPLIT_NT_MB=0;VBC_SMALL_FUSE=0"
ab ct20_strict --workload ct20stif --variants "$V" &&
ab ct20_blocks --workload ct20stif --method blocks --variants "$V" &&
ab ct20_ov2d --workload ct20stif --method overlap2d07 --variants "$V" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "$V" &&
ab ldoor32_memory --workload ldoor --dtype f32 --method memory --variants "$V" &&
ab tube_blocks --workload 3dtube --method blocks --variants "$V" &&
ab thermal_blocks --workload thermal1 --method blocks --variants "$V"
