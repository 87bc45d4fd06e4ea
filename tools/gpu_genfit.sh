set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sweep_tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SWEEP_GENFIT=0;VBC_SWEEP=-1"
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --copies 2 --variants "$V" > gpurun_out/gf_t64.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f32 --variants "$V" > gpurun_out/gf_t32.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ns --dtype f64 --trans 0 --variants "$V" > gpurun_out/gf_f64.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/gf_t64.log gpurun_out/gf_t32.log gpurun_out/gf_f64.log
