#!/bin/bash
set -e
V="VBC_PLANAR_WPS=0;VBC_PLANAR_WPS=2;VBC_PLANAR_WPS=3"
for wl in "ldoor-csc --dtype f32" "ldoor --dtype f32" "ldoor" "ldoor --shard 0/2" "ldoor --shard 1/4" "ldoor --dtype f32 --shard 1/4" "ldoor --shard 0/8" "ct20stif" "fe3d" "fe"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 5 --copies 2 --workload $wl --variants "$V" > gpurun_out/r03_wps_$tag.log 2>&1
done
for wl in "ldoor" "ldoor --dtype f32" "ldoor --shard 0/8" "ldoor --shard 1/4" "ldoor --shard 0/2"; do
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 5 --copies 2 --trans 0 --workload $wl --variants "$V" > gpurun_out/r03_wps_fwd_$tag.log 2>&1
done
