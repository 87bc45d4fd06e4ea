# ldoor's 1/8 and 1/4 stripe shards (single-bucket planar split): slice loop plain / pipelined / batched.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab22_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab22_$tag.log | grep -v "^\[vbc\]" | tail -4; grep "slot bin" gpurun_out/r04_ab22_$tag.log | head -2; }
V="VBC_SPLIT_PIPE=-1;VBC_SPLIT_PIPE=0;VBC_SPLIT_PIPE=1;VBC_SPLIT_PIPE=2"
ab ldoor64_s8_0 --workload ldoor --dtype f64 --shard 0/8 --variants "$V" &&
ab ldoor64_s4_0 --workload ldoor --dtype f64 --shard 0/4 --variants "$V"
