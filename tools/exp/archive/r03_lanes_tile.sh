#!/bin/bash
set -e
V="VBC_VERBOSE=1;VBC_TARGET_RANGES_L=8192;VBC_TARGET_RANGES_L=12288;VBC_TARGET_RANGES_L=16384;VBC_TARGET_RANGES_L=32768"
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --workload fe3d --variants "$V" > gpurun_out/r03_lanes_tile_fe3d.log 2>&1
timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 6 --workload fe3d --trans 0 --variants "$V" > gpurun_out/r03_lanes_tile_fe3d_fwd.log 2>&1
