set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planar.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mask_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
VBC_VERBOSE=1 $A --workload fe3d --variants "VBC_PLANAR_MASK=0;VBC_PLANAR_MASK=1" > gpurun_out/abm_fe3d.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor --variants "VBC_NOP=1;VBC_PLANAR_MASK=0,VBC_PLANAR_PAIR=0;VBC_PLANAR_MASK=1,VBC_PLANAR_PAIR=0" > gpurun_out/abm_ldoor.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor --dtype f32 --variants "VBC_PLANAR_MASK=0;VBC_PLANAR_MASK=1" > gpurun_out/abm_ldoor32.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor-csc --dtype f32 --variants "VBC_PLANAR_MASK=0;VBC_PLANAR_MASK=1" > gpurun_out/abm_ldoorcsc32.log 2>&1
VBC_VERBOSE=1 $A --workload ct20stif --variants "VBC_PLANAR_MASK=0;VBC_PLANAR_MASK=1" > gpurun_out/abm_ct20.log 2>&1
VBC_VERBOSE=1 $A --workload fe3d --dtype f32 --variants "VBC_PLANAR_MASK=0;VBC_PLANAR_MASK=1" > gpurun_out/abm_fe3d32.log 2>&1
