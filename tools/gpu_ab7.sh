set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SLOT_STAGE=0;VBC_SLOT_STAGE=8;VBC_SLOT_STAGE=0,VBC_SLOT_KEYS16=0;VBC_SLOT_STAGE=8,VBC_SLOT_KEYS16=0"
timeout -k 10 300 python tools/ab.py --workload fe --variants "$V" > gpurun_out/ab7_fe_t.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --dtype f32 --variants "$V" > gpurun_out/ab7_fe_t32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --trans 0 --dtype f32 --variants "$V" > gpurun_out/ab7_fe_f32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload fe --trans 0 --variants "$V" > gpurun_out/ab7_fe_f.log 2>&1 || exit $?
cat gpurun_out/ab7_*.log | grep -v amdgpu.ids
