# Occupancy variants (min waves per SIMD via __launch_bounds__): lanes kernel 5 (minw5), pair + planar 4 (minwB)
mkdir -p gpurun_out; export TMPDIR=/tmp
A="tools/exp/libs/libvbc_minw5.so"; B="tools/exp/libs/libvbc_minwB.so"
run() { timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 "$@"; }
run --workload fe3d --variants "VBC_X=0;@lib=$A" > gpurun_out/r03_minw_fe3d.log 2>&1 && tail -2 gpurun_out/r03_minw_fe3d.log &&
run --workload fe3d --trans 0 --variants "VBC_X=0;@lib=$A" > gpurun_out/r03_minw_fe3dfwd.log 2>&1 && tail -2 gpurun_out/r03_minw_fe3dfwd.log &&
run --workload fe3d --dtype f32 --variants "VBC_X=0;@lib=$A" > gpurun_out/r03_minw_fe3df32.log 2>&1 && tail -2 gpurun_out/r03_minw_fe3df32.log &&
run --workload ldoor --variants "VBC_X=0;@lib=$B" > gpurun_out/r03_minw_ldoor.log 2>&1 && tail -2 gpurun_out/r03_minw_ldoor.log &&
run --workload ldoor --dtype f32 --variants "VBC_X=0;@lib=$B" > gpurun_out/r03_minw_ldoorf32.log 2>&1 && tail -2 gpurun_out/r03_minw_ldoorf32.log &&
run --workload ldoor-csc --dtype f32 --variants "VBC_X=0;@lib=$B" > gpurun_out/r03_minw_ldoorcsc.log 2>&1 && tail -2 gpurun_out/r03_minw_ldoorcsc.log &&
run --workload ldoor --trans 0 --variants "VBC_X=0;@lib=$B" > gpurun_out/r03_minw_ldoorfwd.log 2>&1 && tail -2 gpurun_out/r03_minw_ldoorfwd.log
