# Packed swept keys (one 32-bit word per entry) vs index + segment (VBC_SWEEP_PACK=0), NS both directions
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_sweeppack_tests.log 2>&1; tail -2 gpurun_out/r03_sweeppack_tests.log
run() { timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 "$@"; }
run --workload ns --variants "VBC_SWEEP_PACK=0;VBC_SWEEP_PACK=1" > gpurun_out/r03_sweeppack_ns.log 2>&1 && tail -2 gpurun_out/r03_sweeppack_ns.log &&
run --workload ns --dtype f32 --variants "VBC_SWEEP_PACK=0;VBC_SWEEP_PACK=1" > gpurun_out/r03_sweeppack_nsf32.log 2>&1 && tail -2 gpurun_out/r03_sweeppack_nsf32.log &&
run --workload ns --trans 0 --variants "VBC_SWEEP_PACK=0;VBC_SWEEP_PACK=1" > gpurun_out/r03_sweeppack_nsfwd.log 2>&1 && tail -2 gpurun_out/r03_sweeppack_nsfwd.log &&
run --workload ns-mixed --variants "VBC_SWEEP_PACK=0;VBC_SWEEP_PACK=1" > gpurun_out/r03_sweeppack_nsmixed.log 2>&1 && tail -2 gpurun_out/r03_sweeppack_nsmixed.log
