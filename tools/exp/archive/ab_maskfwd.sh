set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_planar.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/maskfwd_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
