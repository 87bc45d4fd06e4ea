set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_slots.py -x -q --timeout 120 --timeout-method thread > gpurun_out/slots.log 2>&1; rc=$?; tail -5 gpurun_out/slots.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/b_slots.log 2>&1 || exit $?
VBC_SLOTS=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/b_merge.log 2>&1 || exit $?
VBC_XCD=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/b_noxcd.log 2>&1 || exit $?
for f in b_slots b_merge b_noxcd; do python -c "import json,sys; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"; done
