# ldoor stand-in 'min blocks' (150,920 6-wide stripes + 3/7/8-wide sides; 352 MB fp32 / 564 MB fp64):
# the fused split against per-bucket layouts, and every stripe cut into 3-wide column pieces.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 20 "$@" > gpurun_out/r04_ab14_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab14_$tag.log | grep -v "^\[vbc\]" | tail -6; }
V="VBC_COLSPLIT_W=0;VBC_COLSPLIT_W=3;VBC_SMALL_FUSE=0;VBC_SLOT_PLANAR=0;VBC_COLSPLIT_W=3,VBC_SMALL_FUSE=0;VBC_COLSPLIT_W=6"
ab ldoor64_blocks --workload ldoor --dtype f64 --method blocks --variants "$V" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "$V"
