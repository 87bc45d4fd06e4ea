# Fork rule (no side streams beside a >= 90 % group when the rest exceeds VBC_FORK_SIDE_KB) and
# layout options for the dominant 6-wide fp64 bucket of the ldoor stand-in's 'min blocks'.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 20 "$@" > gpurun_out/r04_ab17_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab17_$tag.log | grep -v "^\[vbc\]" | tail -6; }
ab ldoor64_blocks --workload ldoor --dtype f64 --method blocks --variants "VBC_FORK_SIDE_KB=1024;VBC_FORK_SIDE_KB=1e9;VBC_TARGET_RANGES_P=8192;VBC_SLOTS=1;VBC_SIDE_FUSE=0,VBC_TARGET_RANGES_P=8192" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "VBC_FORK_SIDE_KB=1024;VBC_FORK_SIDE_KB=1e9" &&
timeout -k 10 300 python -u tools/exp/fork_ab.py > gpurun_out/r04_fork_ab4.log 2>&1 && grep -v "^\[vbc\]\|amdgpu" gpurun_out/r04_fork_ab4.log | tail -8
