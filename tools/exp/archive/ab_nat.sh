set -e -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
VBC_VERBOSE=1 $A --workload fe3d --variants "VBC_NOP=1;VBC_SLOTS_PAD=3.0,VBC_SLOTS_SORT=0" > gpurun_out/abnat_fe3d.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor --variants "VBC_NOP=1;VBC_SLOTS_PAD=3.0,VBC_SLOTS_SORT=0;VBC_SLOTS_PAD=3.0,VBC_SLOTS_SORT=0,VBC_PLANAR_PAIR=0" > gpurun_out/abnat_ldoor.log 2>&1
