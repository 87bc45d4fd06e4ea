set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SLOTS=1,VBC_SLOT_U=8;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_DIAG=4;VBC_SLOTS=1,VBC_SLOT_U=8,VBC_DIAG=1"
timeout -k 10 300 python tools/ab.py --workload fe --variants "$V" > gpurun_out/ab4_fe_t.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab4_fe_t.log
