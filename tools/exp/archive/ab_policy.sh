set -e -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
$A --workload fe --variants "VBC_XCD=0,VBC_RANGE_KB=0;VBC_NOP=1" > gpurun_out/abp_fe.log 2>&1
$A --workload fe --dtype f32 --variants "VBC_XCD=0,VBC_RANGE_KB=0;VBC_NOP=1;VBC_RANGE_KB=0" > gpurun_out/abp_fe32.log 2>&1
$A --workload fe --shard 1/4 --variants "VBC_XCD=0,VBC_RANGE_KB=0;VBC_NOP=1" > gpurun_out/abp_fe_s4.log 2>&1
$A --workload fe --shard 3/8 --variants "VBC_XCD=0,VBC_RANGE_KB=0;VBC_NOP=1" > gpurun_out/abp_fe_s8.log 2>&1
$A --workload ldoor --shard 1/4 --variants "VBC_TARGET_RANGES_P=2500;VBC_NOP=1" > gpurun_out/abp_ldoor_s4.log 2>&1
$A --workload ldoor --shard 1/8 --variants "VBC_PLANAR_SPLIT=4;VBC_NOP=1" > gpurun_out/abp_ldoor_s8.log 2>&1
$A --workload ct20stif --variants "VBC_PLANAR_SPLIT=8;VBC_NOP=1" > gpurun_out/abp_ct20.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload fe --worlds 1,2,4,8 > gpurun_out/shard_fe2.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor --worlds 1,2,4,8 > gpurun_out/shard_ldoor2.log 2>&1
