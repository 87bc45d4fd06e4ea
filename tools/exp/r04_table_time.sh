# The reference's table with the fitted time models ('min time' 1D rows, 'dynamic time 2D'): ct20stif
# fp64 (1D uniform + banded fits, the 2D rank-3 fit) and ldoor fp32 (1D uniform fit, no 2D rows).
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r04_tablet}
timeout -k 10 900 python -u tools/test_table.py --matrix Boeing/ct20stif --dtype f64 --fit-time-model \
    --json gpurun_out/${tag}_ct20stif_f64.json > gpurun_out/${tag}_ct20stif_f64.log 2>&1 || exit $?
tail -16 gpurun_out/${tag}_ct20stif_f64.log
timeout -k 10 700 python -u tools/test_table.py --matrix GHS_psdef/ldoor --dtype f32 --no-2d --fit-time-model \
    --localities uniform --json gpurun_out/${tag}_ldoor_f32.json > gpurun_out/${tag}_ldoor_f32.log 2>&1 || exit $?
tail -8 gpurun_out/${tag}_ldoor_f32.log
