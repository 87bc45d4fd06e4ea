set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planar.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pg_tests.log 2>&1
A="timeout -k 10 300 python -u tools/ab.py --copies 2"
$A --workload fe3d --variants "VBC_PLANAR_PG=0;VBC_PLANAR_PG=1" > gpurun_out/abpg_fe3d.log 2>&1
$A --workload ldoor --variants "VBC_PLANAR_PAIR=1;VBC_PLANAR_PAIR=0,VBC_PLANAR_PG=1;VBC_PLANAR_PAIR=0,VBC_PLANAR_PG=0" > gpurun_out/abpg_ldoor.log 2>&1
$A --workload ldoor-csc --variants "VBC_PLANAR_PAIR=1;VBC_PLANAR_PAIR=0,VBC_PLANAR_PG=1" > gpurun_out/abpg_ldoorcsc.log 2>&1
$A --workload ldoor --trans 0 --variants "VBC_PLANAR_PG=0;VBC_PLANAR_PG=1" > gpurun_out/abpg_ldoor_fwd.log 2>&1
$A --workload fe3d --trans 0 --variants "VBC_PLANAR_PG=0;VBC_PLANAR_PG=1" > gpurun_out/abpg_fe3d_fwd.log 2>&1
