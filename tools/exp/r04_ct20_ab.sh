# ct20stif 'min blocks' / 'min memory' / strict on the fused split with cut long stripes: P and slice
# loop variants (graph-timed, one process).
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab9_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab9_$tag.log | tail -6; }
V="VBC_KSPLIT=1.0;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=8;VBC_SPLIT_PIPE=0;VBC_SMALL_ROWS=4"
ab ct20_blocks --workload ct20stif --method blocks --variants "$V" &&
ab ct20_strict --workload ct20stif --variants "$V" &&
ab thermal_strict --workload thermal1 --variants "VBC_SMALL_FUSE=1;VBC_SMALL_FUSE=0" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "VBC_KSPLIT=1.0;VBC_PLANAR_SPLIT=4;VBC_PLANAR_SPLIT=8"
