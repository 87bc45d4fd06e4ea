# Single-width fused split (VBC_SMALL_FUSE=2) on stripe shards: ldoor fp64 / fp32 1/8 and 1/4, FE 1/8.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab15_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab15_$tag.log | grep -v "^\[vbc\]" | tail -3; }
ab ldoor64_s8 --workload ldoor --dtype f64 --shard 7/8 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab ldoor32_s8 --workload ldoor --dtype f32 --shard 7/8 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab ldoor64_s4 --workload ldoor --dtype f64 --shard 3/4 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab fe_s8 --workload fe --dtype f64 --shard 7/8 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab ct20_strict --workload ct20stif --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab ldoorcsc --workload ldoor-csc --dtype f32 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2"
