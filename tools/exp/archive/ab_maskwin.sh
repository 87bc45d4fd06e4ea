set -e -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
V="VBC_MASK_WINDOW=1;VBC_MASK_WINDOW=2;VBC_MASK_WINDOW=4;VBC_MASK_WINDOW=8;VBC_PLANAR_MASK=0"
VBC_VERBOSE=1 $A --workload fe3d --variants "$V" > gpurun_out/abw_fe3d.log 2>&1
VBC_VERBOSE=1 $A --workload fe3d --dtype f32 --variants "$V" > gpurun_out/abw_fe3d32.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor --dtype f32 --variants "$V" > gpurun_out/abw_ldoor32.log 2>&1
