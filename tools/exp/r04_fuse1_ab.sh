# Single-width small matrices through the fused split (VBC_SMALL_FUSE=2) against the single-bucket
# planar split: 3dtube 'overlap' (15,110 3-wide stripes, 35 MB), ct20stif 'overlap', 3dtube strict (3 buckets, unchanged).
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab13_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab13_$tag.log | grep -v "^\[vbc\]" | tail -4; }
ab tube_overlap --workload 3dtube --method overlap --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab tube_overlap32 --workload 3dtube --dtype f32 --method overlap --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab ct20_overlap --workload ct20stif --method overlap --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab thermal_strict --workload thermal1 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2" &&
ab tube_strict --workload 3dtube --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=2"
