set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planar.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/maskpair_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
VBC_VERBOSE=1 $A --workload ldoor --variants "VBC_PLANAR_MASK_PAIR=0;VBC_NOP=1;VBC_PLANAR_MASK=0" > gpurun_out/abmp_ldoor.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor-csc --variants "VBC_PLANAR_MASK_PAIR=0;VBC_NOP=1;VBC_PLANAR_MASK=0" > gpurun_out/abmp_ldoorcsc.log 2>&1
VBC_VERBOSE=1 $A --workload ldoor --shard 1/4 --variants "VBC_PLANAR_MASK_PAIR=0;VBC_NOP=1;VBC_PLANAR_MASK=0" > gpurun_out/abmp_ldoor_s4.log 2>&1
