# Long stripes cut into lane parts (SlotBin::ks, VBC_KSPLIT threshold x the mean chunk; 0 = off) on the
# table partitions with heavy-tailed stripes, and the fused split's P on the medium ldoor 'min blocks'.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab7_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab7_$tag.log | tail -6; }
K="VBC_KSPLIT=1.0;VBC_KSPLIT=0.75;VBC_KSPLIT=0.5;VBC_KSPLIT=0"
ab ct20_blocks --workload ct20stif --method blocks --variants "$K" &&
ab ct20_strict --workload ct20stif --variants "$K" &&
ab ct20_ov2d --workload ct20stif --method overlap2d07 --variants "$K" &&
ab tube_blocks --workload 3dtube --method blocks --variants "$K" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "VBC_KSPLIT=1.0;VBC_KSPLIT=0.5;VBC_PLANAR_SPLIT=8"
