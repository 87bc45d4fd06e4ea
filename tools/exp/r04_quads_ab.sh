# VALU stripe quads (spmm_quads, widths <= 8) against the MFMA panels (VBC_PANEL_QUADS=0) on both C5
# inputs, fp32 16 RHS, with ablations (VBC_PANEL_DIAG 16: gathers confined to 4 X rows, 2: no Y stores);
# graph-timed in one process.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 400 python -u tools/ab.py --graph --rounds 5 --reps 20 --nrhs 16 "$@" > gpurun_out/r04_quadab2_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_quadab2_$tag.log | tail -5; }
V="@multi;@multi,VBC_PANEL_QUADS=0;@multi,VBC_PANEL_DIAG=16;@multi,VBC_PANEL_DIAG=2"
ab mesh --dtype f32 --workload c5-mesh --variants "$V" &&
ab rand --dtype f32 --workload c5 --variants "$V" &&
ab mesh64 --dtype f64 --workload c5-mesh --scale 0.5 --variants "@multi;@multi,VBC_PANEL_QUADS=0"
