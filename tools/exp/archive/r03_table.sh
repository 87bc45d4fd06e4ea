# The reference's bin/test_table.jl table on the stand-ins with the round-3 kernels (graph-timed GPU column)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/test_table.py --matrix Boeing/ct20stif --dtype f64 --fit-time-model \
    --json gpurun_out/r03_table_ct20stif_standin_f64.json > gpurun_out/r03_table_ct20stif.log 2>&1 && tail -14 gpurun_out/r03_table_ct20stif.log &&
timeout -k 10 500 python -u tools/test_table.py --matrix GHS_psdef/ldoor --dtype f32 --no-2d --fit-time-model \
    --json gpurun_out/r03_table_ldoor_standin_f32.json > gpurun_out/r03_table_ldoor.log 2>&1 && tail -10 gpurun_out/r03_table_ldoor.log
