# Per-kernel times of the ldoor fp64 'min blocks' product: default (dominant 6-wide bucket beside the
# fused side launch) against VBC_SMALL_FUSE=0 (every bucket its own layout); single-width auto-fuse check.
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "VBC_SMALL_FUSE=1" "VBC_SMALL_FUSE=0" "VBC_FORK=0"; do
  tag=$(echo $v | tr '=,' '__')
  VBC_VERBOSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_bprof_$tag -o run -- \
    python -u tools/ab.py --graph --rounds 2 --reps 20 --workload ldoor --dtype f64 --method blocks --variants "$v" \
    > gpurun_out/r04_bprof_$tag.log 2>&1 || exit $?
  echo "--- $v"; grep -v amdgpu.ids gpurun_out/r04_bprof_$tag.log | grep -v "^\[vbc\]" | tail -1
done
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab16_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab16_$tag.log | grep -v "^\[vbc\]" | tail -3; }
ab tube_overlap --workload 3dtube --method overlap --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=0" &&
ab ldoor64_s8 --workload ldoor --dtype f64 --shard 7/8 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=0"
