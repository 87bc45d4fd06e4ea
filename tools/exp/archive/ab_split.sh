set -e -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
V="VBC_NOP=1;@lib=tools/exp/libvbc_split12.so;@lib=tools/exp/libvbc_split36.so"
$A --workload ct20stif --variants "$V" > gpurun_out/abs_ct20.log 2>&1
$A --workload ct20stif --dtype f32 --variants "$V" > gpurun_out/abs_ct20_32.log 2>&1
$A --workload ldoor --shard 1/8 --variants "$V" > gpurun_out/abs_ldoor_s8.log 2>&1
