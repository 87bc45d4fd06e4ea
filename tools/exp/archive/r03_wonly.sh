mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_confirm.sh r03b || exit 1
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 8 --copies 2 --workload fe --variants "VBC_SLOT_WONLY=1;VBC_SLOT_WONLY=0" > gpurun_out/r03b_ab_wonly_fe.log 2>&1 && tail -4 gpurun_out/r03b_ab_wonly_fe.log &&
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 8 --copies 2 --workload fe --dtype f32 --variants "VBC_SLOT_WONLY=1;VBC_SLOT_WONLY=0" > gpurun_out/r03b_ab_wonly_fe32.log 2>&1 && tail -4 gpurun_out/r03b_ab_wonly_fe32.log
