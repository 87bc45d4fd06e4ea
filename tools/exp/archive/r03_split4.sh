#!/bin/bash
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planar.py tests/test_gpu_launch.py tests/test_gpu_multigpu.py tests/test_gpu_configs.py tests/test_gpu_lanes.py > gpurun_out/r03_split4_tests.log 2>&1
tail -2 gpurun_out/r03_split4_tests.log
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor --steps 200 > gpurun_out/r03_split4_shard_ldoor.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor --dtype f32 --steps 200 > gpurun_out/r03_split4_shard_ldoor_f32.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload ct20stif --worlds 1 --steps 200 > gpurun_out/r03_split4_ct20.log 2>&1
timeout -k 10 300 python -u tools/shard_time.py --workload ct20stif --dtype f32 --worlds 1 --steps 200 >> gpurun_out/r03_split4_ct20.log 2>&1
