# Fused split with up to 16 waves per chunk (VBC_FUSE_PMAX=16, with fewer rows per wave allowed) on the
# few-chunk filled partitions: 'dynamic blocks 2D' (ct20stif 191 chunks, 3dtube 159), 'min blocks'.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab20_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab20_$tag.log | grep -v "^\[vbc\]" | tail -5; }
V="VBC_FUSE_PMAX=8;VBC_FUSE_PMAX=16,VBC_SMALL_ROWS=2;VBC_FUSE_PMAX=16,VBC_SMALL_ROWS=4;VBC_FUSE_PMAX=16,VBC_SMALL_ROWS=2,VBC_KSPLIT=0.5"
ab ct20_blocks2d --workload ct20stif --method blocks2d --variants "$V" &&
ab tube_blocks2d --workload 3dtube --method blocks2d --variants "$V" &&
ab ct20_blocks --workload ct20stif --method blocks --variants "$V" &&
ab tube_blocks --workload 3dtube --method blocks --variants "$V" &&
ab ct20_strict --workload ct20stif --variants "$V"
