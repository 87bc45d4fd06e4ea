set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V="VBC_SLOTS=0;VBC_SLOTS=-1;VBC_SLOTS=1"
timeout -k 10 300 python tools/ab.py --workload ns --variants "$V" > gpurun_out/ab10_ns.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ct20stif --variants "$V" > gpurun_out/ab10_c2.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor-csc --dtype f32 --variants "$V" > gpurun_out/ab10_c4.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor --variants "$V" > gpurun_out/ab10_c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload ldoor --trans 0 --variants "$V" > gpurun_out/ab10_c3f.log 2>&1 || exit $?
cat gpurun_out/ab10_ns.log gpurun_out/ab10_c2.log gpurun_out/ab10_c4.log gpurun_out/ab10_c3.log gpurun_out/ab10_c3f.log | grep -v amdgpu.ids
