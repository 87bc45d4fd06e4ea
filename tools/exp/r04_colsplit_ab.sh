# Column pieces (side stripes of a multiple of the dominant width as dominant-width stripes) and the
# side-bucket fused split forced on: ldoor fp32 'min memory' / 'min blocks' / strict, ct20stif 'min blocks'.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 "$@" > gpurun_out/r04_ab12_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_ab12_$tag.log | grep -v "^\[vbc\]" | tail -4; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_planar.py -q -k column_pieces --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_ab12_test.log 2>&1 || { tail -30 gpurun_out/r04_ab12_test.log; exit 1; }
tail -1 gpurun_out/r04_ab12_test.log
ab ldoor32_memory --workload ldoor --dtype f32 --method memory --variants "VBC_COLSPLIT=1;VBC_COLSPLIT=0" &&
ab ldoor32_blocks --workload ldoor --dtype f32 --method blocks --variants "VBC_SIDE_FUSE=-1;VBC_SIDE_FUSE=1;VBC_SIDE_FUSE=1,VBC_PLANAR_WPS=0" &&
ab ldoor64_blocks --workload ldoor --dtype f64 --method blocks --variants "VBC_SIDE_FUSE=-1;VBC_SIDE_FUSE=1" &&
ab ct20_blocks --workload ct20stif --method blocks --variants "VBC_SIDE_FUSE=-1;VBC_SIDE_FUSE=1"
