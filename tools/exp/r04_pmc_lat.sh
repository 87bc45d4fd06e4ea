# Memory-side read latency by Little's law (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ: outstanding requests
# summed per cycle over the requests) and DRAM-credit stalls, for the random-gather probe with its table
# in the Infinity Cache (80 MB) and in HBM (1 GB, 4 GB), and for the NS (swept) and FE (slotted) kernels.
mkdir -p gpurun_out; export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
one() { tag=$1; shift; rm -rf gpurun_out/r04_lat_$tag
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/r04_lat_$tag -o pmc -- "$@" \
    > gpurun_out/r04_lat_$tag.log 2>&1 || return $?; echo "ok $tag"; }
one probe80 tools/exp/gather_probe3 10000000 4096 0 &&
one probe1g tools/exp/gather_probe3 125000000 4096 0 &&
one probe4g tools/exp/gather_probe3 500000000 4096 0 &&
one probe80s tools/exp/gather_probe3 10000000 4096 1 &&
one ns python -u bench.py --workload ns --no-secondary --no-cpu-baseline --no-parity --steps 5 --warmup 2 --eager &&
one fe python -u bench.py --workload fe --no-secondary --no-cpu-baseline --no-parity --steps 5 --warmup 2 --eager
