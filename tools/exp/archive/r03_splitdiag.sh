#!/bin/bash
# split planar product ablations (VBC_DIAG 1 no gathers, 2 gathers in 2 KB of x, 3 no y store, 4 cached loads)
set -e
for wl in "ct20stif" "ldoor --shard 0/8"; do
  V="VBC_PLANAR_SPLIT=2"
  for lib in "" "@lib=tools/exp/libs/libvbc_ns1.so,"; do
    for d in 0 1 2 3 4; do V="$V;${lib}VBC_PLANAR_SPLIT=2,VBC_DIAG=$d"; done
  done
  tag=$(echo $wl | cut -d' ' -f1)
  timeout -k 10 300 python -u tools/ab.py --graph --reps 50 --rounds 10 --workload $wl --variants "$V" > gpurun_out/r03_splitdiag_$tag.log 2>&1
done
