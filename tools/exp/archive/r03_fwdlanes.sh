#!/bin/bash
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planar.py tests/test_gpu_lanes.py -k "forward" > gpurun_out/r03_fwdlanes_tests.log 2>&1 || { tail -40 gpurun_out/r03_fwdlanes_tests.log; exit 1; }
tail -2 gpurun_out/r03_fwdlanes_tests.log
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --trans 0 --workload fe3d --variants "VBC_PLANAR_LANES=0;VBC_PLANAR_LANES=-1" > gpurun_out/r03_fwdlanes_fe3d.log 2>&1
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --trans 0 --workload fe3d --dtype f32 --variants "VBC_PLANAR_LANES=0;VBC_PLANAR_LANES=-1" > gpurun_out/r03_fwdlanes_fe3d_f32.log 2>&1
V="VBC_PLANAR_SPLIT=0;VBC_PLANAR_SPLIT=-1;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=4;VBC_PLANAR_SPLIT=8"
for wl in "ct20stif" "ct20stif --dtype f32" "ldoor --shard 0/8" "ldoor --shard 1/4" "ldoor"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 30 --rounds 8 --trans 0 --workload $wl --variants "$V" > gpurun_out/r03_fwdsplit_$tag.log 2>&1
done
