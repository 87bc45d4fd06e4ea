# Round 6: streaming (non-temporal) y stores, A/B in the ablation build (diag bit 16), on every store-heavy kernel
mkdir -p gpurun_out; export TMPDIR=/tmp
A=tools/exp/libs/libvbc_ablation.so
run() {  # name, ab.py args...
    n=$1; shift
    timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/r06f_$n.log 2>&1 || { tail -20 gpurun_out/r06f_$n.log; exit 1; }
    echo "== $n"; grep -v amdgpu.ids gpurun_out/r06f_$n.log | tail -2
}
run c5mesh --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "@lib=$A,@multi;@lib=$A,@multi,VBC_TILE_DIAG=16"
run fe3d --workload fe3d --graph --reps 20 --rounds 3 --variants "@lib=$A;@lib=$A,VBC_DIAG=16"
run fe3d_fwd --workload fe3d --trans 0 --graph --reps 20 --rounds 3 --variants "@lib=$A;@lib=$A,VBC_DIAG=16"
run fe --workload fe --graph --reps 20 --rounds 3 --variants "@lib=$A;@lib=$A,VBC_DIAG=16"
run ldoor --workload ldoor --graph --reps 20 --rounds 3 --variants "@lib=$A;@lib=$A,VBC_DIAG=16"
run ldoor_fwd --workload ldoor --trans 0 --graph --reps 20 --rounds 3 --variants "@lib=$A;@lib=$A,VBC_DIAG=16"
