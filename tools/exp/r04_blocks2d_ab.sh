# The reference table's 'dynamic blocks 2D' rows (2D VBC, tiles up to 8x8, 2.3x fill; ct20stif 14.5 us,
# 3dtube 17.4 us): long-stripe cut threshold, forced P, fewer rows per wave.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab19_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab19_$tag.log | grep -v "^\[vbc\]" | tail -7; }
V="VBC_KSPLIT=1.0;VBC_KSPLIT=0.5;VBC_KSPLIT=0.25;VBC_PLANAR_SPLIT=4;VBC_SMALL_ROWS=4;VBC_SMALL_ROWS=2;VBC_KSPLIT=0"
ab ct20_blocks2d --workload ct20stif --method blocks2d --variants "$V" &&
ab tube_blocks2d --workload 3dtube --method blocks2d --variants "$V"
