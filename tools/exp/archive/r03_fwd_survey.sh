#!/bin/bash
# forward product y = B x on every bench workload (default layouts), graph-timed
set -e
for wl in fe fe3d ns ldoor ct20stif; do
  for dt in f64 f32; do
    timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 5 --workload $wl --dtype $dt --trans 0 --variants "VBC_VERBOSE=1" > gpurun_out/r03_fwd_${wl}_${dt}.log 2>&1
  done
done
