# The split slice loop's batched form: auto threshold (VBC_SPLIT_DEEP steps per wave) on the table
# partitions after the long-stripe cut.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab10_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab10_$tag.log | tail -5; }
V="VBC_SPLIT_DEEP=2;VBC_SPLIT_DEEP=4;VBC_SPLIT_DEEP=8;VBC_SPLIT_PIPE=0"
ab ct20_strict --workload ct20stif --variants "$V" &&
ab ct20_blocks --workload ct20stif --method blocks --variants "$V" &&
ab ct20_ov2d --workload ct20stif --method overlap2d07 --variants "$V" &&
ab tube_blocks --workload 3dtube --method blocks --variants "$V" &&
ab thermal_blocks --workload thermal1 --method blocks --variants "$V" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "$V"
