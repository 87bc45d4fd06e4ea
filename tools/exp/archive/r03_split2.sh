#!/bin/bash
# new split defaults (cached loads, one run per step, P by rows per wave): tests + shard times + A/B
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planar.py tests/test_gpu_launch.py tests/test_gpu_multigpu.py tests/test_gpu_configs.py > gpurun_out/r03_split2_tests.log 2>&1
tail -3 gpurun_out/r03_split2_tests.log
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor > gpurun_out/r03_split2_shard_ldoor.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload fe > gpurun_out/r03_split2_shard_fe.log 2>&1
timeout -k 10 300 python -u tools/ab.py --graph --reps 50 --rounds 10 --workload ct20stif --variants "VBC_PLANAR_SPLIT=-1;VBC_PLANAR_SPLIT=0;VBC_CREATE_SERIAL_DUMMY=1" > gpurun_out/r03_split2_ct20.log 2>&1
VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --reps 50 --rounds 10 --workload ldoor --shard 3/4 --variants "VBC_PLANAR_SPLIT=-1;VBC_SPLIT_ROWS=1000;VBC_PLANAR_SPLIT=4" > gpurun_out/r03_split2_ldoor_s4.log 2>&1
