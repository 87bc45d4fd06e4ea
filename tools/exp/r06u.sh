# Round 6: C4 (TrSpMV! on the ldoor stand-in, fp32, 0.70) -- launch-shape knobs on the ablation build:
# waves per SIMD of the planar bin, masked order window, range count
mkdir -p gpurun_out; export TMPDIR=/tmp
A=tools/exp/libs/libvbc_ablation.so
V="@lib=$A,VBC_VERBOSE=1"
for kv in VBC_PLANAR_WPS=1 VBC_PLANAR_WPS=3 VBC_PLANAR_WPS=4 VBC_MASK_WINDOW=1 VBC_MASK_WINDOW=4 VBC_PLANAR_MASK=0; do V="$V;@lib=$A,$kv"; done
timeout -k 10 400 python -u tools/ab.py --workload ldoor-csc --dtype f32 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r06u_c4.log 2>&1 || { tail -20 gpurun_out/r06u_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06u_c4.log | grep "slot bin\|TFLOP" | tail -9
