#!/bin/bash
# split planar product (cached loads, NS = 1): rows per step (VBC_SPLIT_VALS builds) x waves per chunk
set -e
for wl in "ct20stif" "ldoor --shard 0/8" "ldoor --shard 7/8"; do
  V="VBC_PLANAR_SPLIT=-1"
  for lib in "" "@lib=tools/exp/libs/libvbc_u9.so," "@lib=tools/exp/libs/libvbc_u36.so,"; do
    for p in 2 4 8; do V="$V;${lib}VBC_PLANAR_SPLIT=$p"; done
  done
  V="$V;VBC_PLANAR_SPLIT=2,VBC_DIAG=4;VBC_PLANAR_SPLIT=0"
  tag=$(echo $wl | tr -d ' /-' )
  timeout -k 10 300 python -u tools/ab.py --graph --reps 50 --rounds 10 --workload $wl --variants "$V" > gpurun_out/r03_splitu_$tag.log 2>&1
done
