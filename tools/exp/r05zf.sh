# default tile kernel (spmm_tiles) on c5-mesh: what the output stores cost
mkdir -p gpurun_out; export TMPDIR=/tmp
V="@multi;@multi,VBC_TILE_DIAG=8;@multi,VBC_TILE_SPR=64;@multi,VBC_TILE_SPR=64,VBC_TILE_DIAG=8"
timeout -k 10 600 python -u tools/ab.py --workload c5-mesh --dtype f32 --nrhs 16 --graph --reps 20 --rounds 3 --variants "$V" > gpurun_out/r05zf_ab.log 2>&1 || { tail -20 gpurun_out/r05zf_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zf_ab.log | tail -4
