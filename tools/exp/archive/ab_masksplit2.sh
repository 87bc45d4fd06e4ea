set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ms2_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
VBC_VERBOSE=1 $A --workload ldoor --shard 1/8 --variants "VBC_NOP=1;VBC_PLANAR_MASK=0" > gpurun_out/abms2_ldoor_s8.log 2>&1
VBC_VERBOSE=1 $A --workload ct20stif --variants "VBC_NOP=1;VBC_PLANAR_MASK=0" > gpurun_out/abms2_ct20.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor --worlds 8 > gpurun_out/shard_ldoor8.log 2>&1
