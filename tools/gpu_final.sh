set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=smoke,tests,bench bash tools/gpu_check.sh || exit $?
WORKLOADS="fe ns c5" bash tools/gpu_prof.sh || exit $?
echo done
