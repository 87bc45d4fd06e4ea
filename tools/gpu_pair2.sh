set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_SLOT_PAIR=0;VBC_SLOT_PAIR=1"
timeout -k 10 400 python tools/ab.py --workload fe --dtype f64 --copies 4 --rounds 7 --variants "$V" > gpurun_out/pair2_fe64.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/pair2_fe64.log
