# A large dominant bucket plus a tiny side bucket (the ldoor stand-in's 'min memory': 317,337 3-wide
# stripes + 32 six-wide): forked launch groups against one stream, and the layouts' verbose decisions.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab11_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab11_$tag.log | grep -v "^\[vbc\]" | tail -3; }
ab ldoor32_memory --workload ldoor --dtype f32 --method memory --variants "VBC_FORK=1;VBC_FORK=0" &&
ab ldoor32_strict --workload ldoor --dtype f32 --variants "VBC_FORK=1"
