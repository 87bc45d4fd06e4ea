set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SWEEP=0;VBC_SWEEP=-1;VBC_SWEEP=-1,VBC_SWEEP_MINB=16;VBC_SWEEP=-1,VBC_SWEEP_MINB=32;VBC_SWEEP=-1,VBC_SWEEP_TILE=16"
timeout -k 10 400 python tools/ab.py --workload ns-mixed --dtype f64 --variants "$V" > gpurun_out/sw5_nsm.log 2>&1 || exit $?
V="VBC_SWEEP=0;VBC_SWEEP=-1;VBC_SWEEP=-1,VBC_SWEEP_MINB=8;VBC_SWEEP=-1,VBC_SWEEP_MINB=16"
timeout -k 10 400 python tools/ab.py --workload ns-mixed --dtype f32 --variants "$V" > gpurun_out/sw5_nsm32.log 2>&1 || exit $?
cat gpurun_out/sw5_nsm.log gpurun_out/sw5_nsm32.log | grep -v amdgpu.ids
