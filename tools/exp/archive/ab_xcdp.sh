set -e -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
$A --workload fe3d --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_fe3d.log 2>&1
$A --workload ldoor --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_ldoor.log 2>&1
$A --workload ldoor --dtype f32 --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_ldoor32.log 2>&1
$A --workload ldoor-csc --dtype f32 --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_ldoorcsc.log 2>&1
$A --workload ct20stif --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_ct20.log 2>&1
$A --workload ldoor --shard 1/8 --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_ldoor_s8.log 2>&1
$A --workload fe --trans 0 --variants "VBC_NOP=1;VBC_XCD_P=1" > gpurun_out/abx_fe_fwd.log 2>&1
