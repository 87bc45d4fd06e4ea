# NS: random-gather rate by where the table lives (L2 / Infinity Cache / HBM), and the counters the
# profiler offers on this box (for a DRAM-vs-Infinity-Cache split of the memory-side requests).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 tools/exp/gather_probe3 > gpurun_out/r04_gather_probe3.log 2>&1 || exit $?
tail -30 gpurun_out/r04_gather_probe3.log
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/r04_list_avail.log 2>&1 || true
grep -i -E "mall|dram|ea0_rd|hbm|df_|infinity" gpurun_out/r04_list_avail.log | head -60
