# Where the MFMA panel kernel's time goes on the structured c5-mesh input (3x3 node tiles) against the
# random C5 generator (8x8 tiles): ablations (VBC_PANEL_DIAG 2 no Y stores, 4 X gathers confined to
# cache, 8 value loads confined to cache), graph-timed in one process.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 400 python -u tools/ab.py --graph --rounds 5 --reps 20 --nrhs 16 --dtype f32 "$@" > gpurun_out/r04_c5ab_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_c5ab_$tag.log | tail -5; }
D="@multi;@multi,VBC_PANEL_DIAG=2;@multi,VBC_PANEL_DIAG=4;@multi,VBC_PANEL_DIAG=8;@multi,VBC_PANEL_DIAG=12"
ab mesh --workload c5-mesh --variants "$D" &&
ab rand --workload c5 --variants "$D"
