mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 8 --copies 2 --workload fe3d --variants "VBC_PLANAR_LANES=1;@lib=tools/exp/libs/libvbc_vals36.so" > gpurun_out/r03i_ab_vals_fe3d.log 2>&1 && tail -4 gpurun_out/r03i_ab_vals_fe3d.log &&
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 8 --copies 2 --workload ldoor --variants "VBC_PLANAR_LANES=0;@lib=tools/exp/libs/libvbc_vals36.so" > gpurun_out/r03i_ab_vals_ldoor.log 2>&1 && tail -4 gpurun_out/r03i_ab_vals_ldoor.log
