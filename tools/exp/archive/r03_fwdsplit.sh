#!/bin/bash
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_planar.py -k "forward" > gpurun_out/r03_fwdsplit_tests.log 2>&1 || { tail -30 gpurun_out/r03_fwdsplit_tests.log; exit 1; }
tail -2 gpurun_out/r03_fwdsplit_tests.log
V="VBC_PLANAR_SPLIT=0;VBC_PLANAR_SPLIT=-1;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=4;VBC_PLANAR_SPLIT=8"
for wl in "ct20stif" "ct20stif --dtype f32" "ldoor --shard 0/8" "ldoor --shard 1/4" "ldoor --dtype f32 --shard 0/8" "ldoor"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 30 --rounds 8 --trans 0 --workload $wl --variants "$V" > gpurun_out/r03_fwdsplit_$tag.log 2>&1
done
