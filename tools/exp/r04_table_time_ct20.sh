# The reference's table with the GPU-fitted time models on the ct20stif stand-in (1D uniform + banded
# fits, the 2D rank-3 fit): 'min time' and 'dynamic time 2D' rows.
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r04_tablet}
timeout -k 10 1000 python -u tools/test_table.py --matrix Boeing/ct20stif --dtype f64 --fit-time-model \
    --json gpurun_out/${tag}_ct20stif_f64.json > gpurun_out/${tag}_ct20stif_f64.log 2>&1 || exit $?
tail -16 gpurun_out/${tag}_ct20stif_f64.log
