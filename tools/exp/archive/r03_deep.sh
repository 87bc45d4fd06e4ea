mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 8 --copies 2 --workload fe3d --variants "VBC_LANES_DEEP=0;VBC_LANES_DEEP=1" > gpurun_out/r03j_ab_deep.log 2>&1; tail -4 gpurun_out/r03j_ab_deep.log
