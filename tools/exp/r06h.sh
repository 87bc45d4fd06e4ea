# Round 6: FE-3D layout families at HEAD (lane streams vs the masked planar chunks vs lane pairs), both directions
mkdir -p gpurun_out; export TMPDIR=/tmp
V="@x;VBC_PLANAR_LANES=0;VBC_PLANAR_LANES=0,VBC_PLANAR_PAIR=2"
for t in 1 0; do
VBC_VERBOSE=1 timeout -k 10 400 python -u tools/ab.py --workload fe3d --trans $t --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r06h_fe3d_t$t.log 2>&1 || { tail -20 gpurun_out/r06h_fe3d_t$t.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06h_fe3d_t$t.log | tail -3
done
