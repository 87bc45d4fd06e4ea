#!/bin/bash
set -e
V="VBC_FWD_MIN_ROWS=1;VBC_FWD_MIN_ROWS=8;VBC_FWD_MIN_ROWS=16;VBC_FWD_MIN_ROWS=24;VBC_FWD_MIN_ROWS=32;VBC_FWD_MIN_ROWS=48"
for wl in "ldoor --shard 0/8" "ldoor --shard 1/4" "ldoor --shard 0/2" "ldoor" "ldoor --dtype f32" "fe3d --shard 0/8"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 5 --trans 0 --workload $wl --variants "$V" > gpurun_out/r03_fwdshard3_$tag.log 2>&1
done
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 5 --trans 0 --workload fe3d --variants "VBC_PLANAR_LANES=0,VBC_FWD_MIN_ROWS=1;VBC_PLANAR_LANES=0,VBC_FWD_MIN_ROWS=16;VBC_PLANAR_LANES=0,VBC_FWD_MIN_ROWS=32" > gpurun_out/r03_fwdshard3_fe3dmasked.log 2>&1
