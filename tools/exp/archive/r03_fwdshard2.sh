#!/bin/bash
set -e
V="VBC_VERBOSE=1;VBC_SLOT_RUNS=0;VBC_PLANAR_MASK=0;VBC_SLOTS_PAD=100;VBC_TARGET_RANGES_P=1024;VBC_TARGET_RANGES_P=8192;VBC_SLOTS=0"
VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 4 --trans 0 --workload ldoor --shard 0/8 --variants "$V" > gpurun_out/r03_fwdshard2.log 2>&1
