#!/bin/bash
set -e
for wl in "ldoor-csc --dtype f32" "ldoor --dtype f32" "ldoor" "ldoor --shard 0/2" "fe" "ns"; do
  tag=$(echo $wl | tr -d ' /-' )
  VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --reps 10 --rounds 3 --workload $wl --variants "VBC_VERBOSE=1;VBC_TARGET_RANGES_P=2048;VBC_TARGET_RANGES_P=1024" > gpurun_out/r03_bxranges_$tag.log 2>&1
done
