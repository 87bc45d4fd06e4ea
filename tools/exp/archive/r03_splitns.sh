#!/bin/bash
# split planar product: steps per phase (VBC_SPLIT_NS builds) x waves per chunk (VBC_PLANAR_SPLIT)
set -e
V=""
for lib in "" "@lib=tools/exp/libs/libvbc_ns1.so," "@lib=tools/exp/libs/libvbc_ns3.so," "@lib=tools/exp/libs/libvbc_ns4.so,"; do
  for p in 2 4 8; do V="$V;${lib}VBC_PLANAR_SPLIT=$p"; done
done
V="VBC_PLANAR_SPLIT=0$V"
timeout -k 10 300 python -u tools/ab.py --graph --reps 50 --rounds 10 --workload ct20stif --variants "$V" > gpurun_out/r03_splitns_ct20.log 2>&1
timeout -k 10 300 python -u tools/ab.py --graph --reps 50 --rounds 10 --workload ldoor --shard 0/8 --variants "$V" > gpurun_out/r03_splitns_ldoor_s8.log 2>&1
