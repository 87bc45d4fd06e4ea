set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_PAD=3:4;VBC_PAD=3:3"
timeout -k 10 300 python tools/ab.py --workload ldoor --copies 2 --variants "$V" > gpurun_out/ab11_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor --dtype f32 --copies 2 --variants "$V" > gpurun_out/ab11_c3_32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor --trans 0 --variants "VBC_SLOTS=0;VBC_SLOTS=-1;VBC_SLOT_KEYS16=0" > gpurun_out/ab11_c3f.log 2>&1 || exit $?
cat gpurun_out/ab11_*.log | grep -v amdgpu.ids
