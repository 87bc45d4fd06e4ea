mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 8 --workload fe3d --variants "VBC_DIAG=0;VBC_DIAG=1;VBC_DIAG=2;VBC_DIAG=3" > gpurun_out/r03j_ab_lanes_diag.log 2>&1; tail -5 gpurun_out/r03j_ab_lanes_diag.log
