set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab.py --workload fe --copies 2 --variants "VBC_SLOT_STAGE=0;VBC_SLOT_STAGE=8" > gpurun_out/ab8_fe_t.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --trans 0 --copies 2 --variants "VBC_SLOT_KEYS16=1;VBC_SLOT_KEYS16=0" > gpurun_out/ab8_fe_f32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --variants "VBC_SLOTS=0;VBC_SLOTS=0,VBC_DIAG=1;VBC_SLOTS=0,VBC_DIAG=2" > gpurun_out/ab8_ns.log 2>&1 || exit $?
cat gpurun_out/ab8_*.log | grep -v amdgpu.ids
