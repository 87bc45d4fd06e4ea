# The long-stripe cut capped at a CU's share of the work: ldoor fp32 'min blocks' (2550 chunks: no cut)
# and the ct20stif partitions (cut) against VBC_KSPLIT=0.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab8_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab8_$tag.log | tail -3; }
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "VBC_KSPLIT=1.0;VBC_KSPLIT=0;VBC_PLANAR_SPLIT=8" &&
ab ct20_blocks --workload ct20stif --method blocks --variants "VBC_KSPLIT=1.0;VBC_KSPLIT=0"
