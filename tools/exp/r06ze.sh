# Round 6: stripes per tile range (VBC_TILE_SPR, ablation build) with the value-load fix and clustered order
mkdir -p gpurun_out; export TMPDIR=/tmp
A=tools/exp/libs/libvbc_ablation.so
V="@multi,@lib=$A,VBC_VERBOSE=1"
for n in 24 40 42; do V="$V;@multi,@lib=$A,VBC_TILE_SPR=$n"; done
timeout -k 10 500 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --trans 1 --graph --reps 20 --rounds 4 --variants "$V" > gpurun_out/r06ze_spr.log 2>&1 || { tail -20 gpurun_out/r06ze_spr.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06ze_spr.log | grep "tiles:\|TFLOP" | tail -5
