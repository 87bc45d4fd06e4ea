# A dominant bucket headed for the merge layout fused with its side buckets (ldoor fp64 'min blocks'),
# against the forced larger fused launch and the side-fuse rule; guards: ldoor strict / min memory, ct20stif.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 20 "$@" > gpurun_out/r04_ab18_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab18_$tag.log | grep -v "^\[vbc\]" | tail -4; }
ab ldoor64_blocks --workload ldoor --dtype f64 --method blocks --variants "VBC_SIDE_FUSE=-1;VBC_TARGET_RANGES_P=8192;VBC_SIDE_FUSE=1" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "VBC_SIDE_FUSE=-1;VBC_SIDE_FUSE=1" &&
ab ldoor64_memory --workload ldoor --dtype f64 --method memory --variants "VBC_COLSPLIT=1;VBC_COLSPLIT=0" &&
ab tube_blocks --workload 3dtube --method blocks --variants "VBC_SIDE_FUSE=-1;VBC_SIDE_FUSE=0" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_planar.py tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_slots.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_tests.log 2>&1; tail -3 gpurun_out/r04f_tests.log
