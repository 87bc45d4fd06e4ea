# Medium matrices with mixed widths (ldoor fp32 'min blocks', 300 MB): the fused split against the
# streaming planar kernel forced (chunk-atomic ranges), natural / sorted order, waves per SIMD.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab5_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab5_$tag.log | tail -8; }
V="VBC_SMALL_FUSE=1;VBC_PLANAR_SPLIT=8;VBC_SMALL_FUSE=0,VBC_SLOTS=1;VBC_SMALL_FUSE=0,VBC_SLOTS=1,VBC_SLOTS_SORT=2;VBC_SMALL_FUSE=0,VBC_SLOTS=1,VBC_SLOTS_SORT=2,VBC_PLANAR_WPS=1;VBC_SMALL_FUSE=0,VBC_SLOTS=1,VBC_SLOTS_SORT=2,VBC_PLANAR_WPS=4"
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "$V" &&
ab ct20_holes --workload ct20stif --variants "VBC_SLOT_RUNS=1;VBC_SLOT_RUNS=0;VBC_SMALL_FUSE=0"
