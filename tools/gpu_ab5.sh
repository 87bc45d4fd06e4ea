set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SLOTS=1,VBC_SLOT_U=8;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_SLOT_STAGE=4;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_SLOT_STAGE=8;VBC_SLOTS=1,VBC_SLOT_STAGE=8"
timeout -k 10 300 python tools/ab.py --workload fe --variants "$V" > gpurun_out/ab5_fe_t.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --trans 0 --variants "$V" > gpurun_out/ab5_fe_f.log 2>&1 || exit $?
V="VBC_SLOTS=1,VBC_SLOT_U=16;VBC_SLOTS=1,VBC_SLOT_U=16,VBC_SLOT_STAGE=4;VBC_SLOTS=1,VBC_SLOT_U=16,VBC_SLOT_STAGE=8;VBC_SLOTS=1,VBC_SLOT_STAGE=8"
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --variants "$V" > gpurun_out/ab5_fe_t32.log 2>&1 || exit $?
cat gpurun_out/ab5_fe_t.log gpurun_out/ab5_fe_f.log gpurun_out/ab5_fe_t32.log | grep -v amdgpu.ids
