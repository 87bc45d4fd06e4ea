# Long-stripe cut threshold on the few-chunk filled partitions (fewer chunks than CUs): 1.0 (default) / 0.5 / 0.25 / 0.1.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab21_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab21_$tag.log | grep -v "^\[vbc\]" | tail -4; grep "small fused" gpurun_out/r04_ab21_$tag.log | head -4; }
V="VBC_KSPLIT=1.0;VBC_KSPLIT=0.5;VBC_KSPLIT=0.25;VBC_KSPLIT=0.1"
ab ct20_blocks --workload ct20stif --method blocks --variants "$V" &&
ab tube_blocks --workload 3dtube --method blocks --variants "$V" &&
ab thermal_blocks --workload thermal1 --method blocks --variants "$V" &&
ab ct20_blocks2d --workload ct20stif --method blocks2d --variants "$V" &&
ab thermal_blocks2d --workload thermal1 --method blocks2d --variants "$V" &&
ab ct20_strict --workload ct20stif --variants "$V" &&
ab ct20_overlap2d --workload ct20stif --method overlap2d07 --variants "$V"
