mkdir -p gpurun_out; export TMPDIR=/tmp
for sh in 0/4 0/8; do
echo "== shard $sh"
timeout -k 10 300 python -u tools/ab.py --workload ldoor --dtype f64 --graph --reps 50 --rounds 3 --shard $sh --variants "VBC_VERBOSE=0;VBC_SPLIT_NT_MB=8;VBC_PLANAR_SPLIT=0,VBC_PLANAR_WPS=1;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=2,VBC_SPLIT_NT_MB=8;VBC_PLANAR_SPLIT=8;VBC_SPLIT_ROWS=24;VBC_SPLIT_ROWS=6" 2>&1 | grep -v "amdgpu.ids" || exit 1
done
for wl in "ldoor --dtype f32" "ldoor-csc --dtype f32" "fe3d --dtype f64"; do
echo "== $wl"
timeout -k 10 300 python -u tools/ab.py --workload $wl --graph --reps 20 --rounds 3 --variants "VBC_PLANAR_WPS=2;VBC_PLANAR_WPS=1" 2>&1 | grep -v "amdgpu.ids" || exit 1
done
