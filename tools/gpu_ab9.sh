set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_slots.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mfma.log 2>&1; rc=$?; tail -3 gpurun_out/mfma.log; [ $rc -ne 0 ] && exit $rc
P=sparsematrixvbcs.jl_amd/build/libvbc_prev.so
timeout -k 10 300 python tools/ab.py --workload c5 --dtype f32 --nrhs 16 --copies 2 --variants "@multi;@multi,@lib=$P;@multi,@lib=sparsematrixvbcs.jl_amd/build/libvbc_b8.so" > gpurun_out/ab9_c5.log 2>&1 || exit $?
timeout -k 10 300 python tools/ab.py --workload c5 --dtype f64 --nrhs 16 --variants "@multi;@multi,@lib=$P;@multi,@lib=sparsematrixvbcs.jl_amd/build/libvbc_b8.so" > gpurun_out/ab9_c5_64.log 2>&1 || exit $?
cat gpurun_out/ab9_*.log | grep -v amdgpu.ids
