# 'min time (GPU, uniform)' on the ldoor stand-in, fp32 (1D uniform fit, no 2D rows)
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r04_tablet}
timeout -k 10 800 python -u tools/test_table.py --matrix GHS_psdef/ldoor --dtype f32 --no-2d --fit-time-model \
    --localities uniform --json gpurun_out/${tag}_ldoor_f32.json > gpurun_out/${tag}_ldoor_f32.log 2>&1 || exit $?
tail -8 gpurun_out/${tag}_ldoor_f32.log
