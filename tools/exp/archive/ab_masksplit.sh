set -e -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
VBC_VERBOSE=1 $A --workload ldoor --shard 1/8 --variants "VBC_NOP=1;VBC_PLANAR_SPLIT=0;VBC_PLANAR_SPLIT=0,VBC_PLANAR_PAIR=0" > gpurun_out/abms_ldoor_s8.log 2>&1
VBC_VERBOSE=1 $A --workload ct20stif --variants "VBC_NOP=1;VBC_PLANAR_SPLIT=0" > gpurun_out/abms_ct20.log 2>&1
VBC_VERBOSE=1 $A --workload fe3d --shard 1/8 --variants "VBC_NOP=1;VBC_PLANAR_SPLIT=0" > gpurun_out/abms_fe3d_s8.log 2>&1
