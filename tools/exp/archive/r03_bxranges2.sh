#!/bin/bash
set -e
V="VBC_NOP=1;VBC_TARGET_RANGES_P=1536;VBC_TARGET_RANGES_P=2048;VBC_TARGET_RANGES_P=2560;VBC_TARGET_RANGES_P=3072;VBC_TARGET_RANGES_P=4096"
for wl in "ldoor-csc --dtype f32" "ldoor --dtype f32" "ldoor" "ldoor --shard 0/2" "ldoor --dtype f32 --shard 0/2" "fe3d --dtype f32"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --copies 2 --workload $wl --variants "$V" > gpurun_out/r03_bxranges2_$tag.log 2>&1
done
