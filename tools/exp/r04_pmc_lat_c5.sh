# Memory-side read latency (Little's law, as r04_pmc_lat.sh) of the MFMA panel kernel on the random C5
# generator and on the structured c5-mesh input: where its X re-fetches are served (Infinity Cache ~1,100
# cycles, HBM ~1,600+).
mkdir -p gpurun_out; export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
one() { tag=$1; shift; rm -rf gpurun_out/r04_lat_$tag
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/r04_lat_$tag -o pmc -- "$@" \
    > gpurun_out/r04_lat_$tag.log 2>&1 || return $?; echo "ok $tag"; }
one c5 python -u bench.py --workload c5 --dtype f32 --no-secondary --no-cpu-baseline --no-parity --steps 5 --warmup 2 --eager &&
one c5mesh python -u bench.py --workload c5-mesh --dtype f32 --no-secondary --no-cpu-baseline --no-parity --steps 5 --warmup 2 --eager
