# Round-4 confirmation, part A: GPU tests, smoke, the bench line, its rocprofv3 kernel statistics, and the
# PMC traffic of the structured C5 input.  Logs: gpurun_out/r04c_*
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r04c}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${tag}_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -c 1200 gpurun_out/${tag}_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
    python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_prof_bench.log 2>&1 || exit $?
G="TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum"
timeout -k 10 400 python -u tools/pmc_traffic.py --counters "$G" --workload c5-mesh --dtype f32 --kernel spmm_panel \
    --read-factor 1 > gpurun_out/${tag}_pmc_c5mesh.log 2>&1 || exit $?
bash tools/exp/r04_pmc_lat_c5.sh || exit $?
exit $rc
