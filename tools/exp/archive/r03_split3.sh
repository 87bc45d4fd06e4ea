#!/bin/bash
# auto split rule: ldoor shards 1/2, 1/4 and whole; C4 (ldoor-csc fp32) and FE-3D unchanged?
set -e
V="VBC_SPLIT_ROWS=1000;VBC_PLANAR_SPLIT=-1;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=4;VBC_PLANAR_SPLIT=8"
for wl in "ldoor --shard 0/2" "ldoor --shard 1/4" "ldoor" "ldoor --dtype f32" "ldoor --dtype f32 --shard 0/8"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 30 --rounds 8 --workload $wl --variants "$V" > gpurun_out/r03_split3_$tag.log 2>&1
done
timeout -k 10 300 python -u tools/ab.py --graph --reps 30 --rounds 8 --workload ldoor-csc --dtype f32 --variants "VBC_SPLIT_ROWS=1000;VBC_PLANAR_SPLIT=-1" > gpurun_out/r03_split3_csc.log 2>&1
timeout -k 10 300 python -u tools/ab.py --graph --reps 30 --rounds 8 --workload ct20stif --dtype f32 --variants "VBC_SPLIT_ROWS=1000;VBC_PLANAR_SPLIT=-1;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=4;VBC_PLANAR_SPLIT=8" > gpurun_out/r03_split3_ct20f32.log 2>&1
