#!/bin/bash
set -e
export TMPDIR=/tmp
VBC_VERBOSE=1 timeout -k 10 300 python -u tools/ab.py --graph --reps 20 --rounds 4 --trans 0 --workload ldoor --shard 0/8 --variants "VBC_VERBOSE=1" > gpurun_out/r03_fwdshard_v.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_fwdshard_prof -o run -- python3 -u tools/ab.py --reps 20 --rounds 2 --trans 0 --workload ldoor --shard 0/8 --variants "VBC_VERBOSE=1" > gpurun_out/r03_fwdshard_prof.log 2>&1
