set -e -o pipefail
mkdir -p gpurun_out
for s in 0/1 1/4 1/8; do
VBC_VERBOSE=1 timeout -k 10 200 python -u tools/ab.py --workload ldoor --shard $s --rounds 1 --reps 5 --variants "VBC_NOP=1" >> gpurun_out/verbose.log 2>&1
done
VBC_VERBOSE=1 timeout -k 10 200 python -u tools/ab.py --workload ct20stif --rounds 1 --reps 5 --variants "VBC_NOP=1" >> gpurun_out/verbose.log 2>&1
VBC_VERBOSE=1 timeout -k 10 200 python -u tools/ab.py --workload fe --shard 1/8 --rounds 1 --reps 5 --variants "VBC_NOP=1" >> gpurun_out/verbose.log 2>&1
