#!/bin/bash
set -e
V="VBC_SPLIT_ROWS=1000;VBC_PLANAR_SPLIT=-1;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=4;VBC_PLANAR_SPLIT=8"
for wl in "ldoor --dtype f32 --shard 0/2" "ldoor --dtype f32 --shard 1/4" "ldoor --shard 1/4" "fe3d --shard 0/8" "fe3d --shard 0/4"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 30 --rounds 8 --workload $wl --variants "$V" > gpurun_out/r03_split5_$tag.log 2>&1
done
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor --steps 200 > gpurun_out/r03_split5_shard_ldoor.log 2>&1
