set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SLOTS=0;VBC_SLOTS=1;VBC_SLOTS=1,VBC_SLOT_U=8;VBC_SLOTS=1,VBC_XCD=1"
timeout -k 10 300 python tools/ab.py --workload fe --variants "$V" > gpurun_out/ab_fe_t.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --trans 0 --variants "$V" > gpurun_out/ab_fe_f.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --variants "VBC_SLOTS=0;VBC_SLOTS=1;VBC_SLOTS=1,VBC_SLOT_U=16" > gpurun_out/ab_fe_t32.log 2>&1 || exit $?
cat gpurun_out/ab_fe_t.log gpurun_out/ab_fe_f.log gpurun_out/ab_fe_t32.log | grep -v amdgpu.ids
