# VALU stripe quads (spmm_quads, default for widths <= 8) against the MFMA panels (VBC_PANEL_QUADS=0)
# on both C5 inputs, fp32 16 RHS, and the quad batch knob; graph-timed in one process.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 400 python -u tools/ab.py --graph --rounds 5 --reps 20 --nrhs 16 "$@" > gpurun_out/r04_quadab_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_quadab_$tag.log | tail -4; }
ab mesh --dtype f32 --workload c5-mesh --variants "@multi;@multi,VBC_PANEL_QUADS=0" &&
ab rand --dtype f32 --workload c5 --variants "@multi;@multi,VBC_PANEL_QUADS=0" &&
ab mesh64 --dtype f64 --workload c5-mesh --scale 0.5 --variants "@multi;@multi,VBC_PANEL_QUADS=0"
