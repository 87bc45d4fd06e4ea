# ldoor stripe shards: launch-shape knobs (waves per SIMD, lane pairs, split)
mkdir -p gpurun_out; export TMPDIR=/tmp
for sh in 0/1 0/2 1/2 0/4 3/4 0/8; do
echo "== shard $sh"
timeout -k 10 300 python -u tools/ab.py --workload ldoor --dtype f64 --graph --reps 50 --rounds 3 --shard $sh --variants "VBC_VERBOSE=1;VBC_PLANAR_WPS=1;VBC_PLANAR_WPS=3;VBC_PLANAR_WPS=4;VBC_PLANAR_PAIR=0;VBC_PLANAR_SPLIT=2;VBC_PLANAR_MASK=0" 2>&1 | grep -v "amdgpu.ids" || exit 1
done
