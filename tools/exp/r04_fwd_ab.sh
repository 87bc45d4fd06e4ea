# Forward B·x on the mixed-width ct20stif stand-in (strict stripes 1..6 wide: one forward launch per
# width bucket) and the table partitions; graph-timed.
mkdir -p gpurun_out; export TMPDIR=/tmp
ab() { tag=$1; shift; timeout -k 10 300 python -u tools/ab.py --graph --rounds 5 --reps 30 --trans 0 "$@" > gpurun_out/r04_fwdab_$tag.log 2>&1 || return $?; echo "--- $tag"; grep -v amdgpu.ids gpurun_out/r04_fwdab_$tag.log | tail -3; }
ab ct20_strict --workload ct20stif --variants "VBC_FORK=1;VBC_FORK=0" &&
ab ct20_blocks --workload ct20stif --method blocks --variants "VBC_FORK=1;VBC_FORK=0" &&
ab ldoor_strict --workload ldoor --variants "VBC_FORK=1"
