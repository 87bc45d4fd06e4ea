set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SLOTS=0;VBC_SLOTS=1,VBC_SLOT_U=8;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_TARGET_RANGES_S=4096;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_TARGET_RANGES_S=16384;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_TARGET_RANGES_S=32768;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_TARGET_RANGES_S=65536;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_TARGET_RANGES_S=131072"
timeout -k 10 300 python tools/ab.py --workload fe --variants "$V" > gpurun_out/ab2_fe_t.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --variants "VBC_SLOTS=0,VBC_DIAG=1;VBC_SLOTS=0" > gpurun_out/ab2_diag.log 2>&1 || exit $?
cat gpurun_out/ab2_fe_t.log gpurun_out/ab2_diag.log | grep -v amdgpu.ids
