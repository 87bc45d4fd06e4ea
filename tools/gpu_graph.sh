set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_slots.py -x -q --timeout 120 --timeout-method thread > gpurun_out/graph_tests.log 2>&1; rc=$?; tail -3 gpurun_out/graph_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/graph_bench.py --workload ct20stif > gpurun_out/graph_c2.log 2>&1 || exit $?
timeout -k 10 300 python tools/graph_bench.py --workload ldoor > gpurun_out/graph_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/graph_bench.py --workload fe --reps 50 > gpurun_out/graph_fe.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/graph_c2.log gpurun_out/graph_c3.log gpurun_out/graph_fe.log
