#!/bin/bash
set -e
V="VBC_PLANAR_LANES=0;VBC_PLANAR_LANES=-1;VBC_PLANAR_LANES=1;VBC_PLANAR_LANES=1,VBC_TARGET_RANGES_L=2048"
for wl in "ldoor" "ldoor --dtype f32" "ldoor --shard 0/8" "ldoor --shard 1/4" "ldoor --shard 0/2" "fe3d --shard 0/8"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --trans 0 --workload $wl --variants "$V" > gpurun_out/r03_fwdlanes2_$tag.log 2>&1
done
