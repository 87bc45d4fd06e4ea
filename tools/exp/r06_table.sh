# Round 6: the reference's bin/test_table.jl table re-measured at HEAD (GPU graph-timed, CPU reference
# schedule + 64-stripe grabs + 1 core), the stand-ins pinned to src/ref.out, and the time-model rows.
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r06_table}
for spec in "Boeing/ct20stif f64" "Rothberg/3dtube f64" "Schmid/thermal1 f64" "DIMACS10/chesapeake f64"; do
  set -- $spec
  short=$(basename $1)
  timeout -k 10 400 python -u tools/test_table.py --matrix $1 --dtype $2 \
      --json gpurun_out/${tag}_${short}_$2.json > gpurun_out/${tag}_${short}_$2.log 2>&1 || { tail -20 gpurun_out/${tag}_${short}_$2.log; exit 1; }
  tail -14 gpurun_out/${tag}_${short}_$2.log
done
timeout -k 10 500 python -u tools/test_table.py --matrix GHS_psdef/ldoor --dtype f32 --no-2d \
    --json gpurun_out/${tag}_ldoor_f32.json > gpurun_out/${tag}_ldoor_f32.log 2>&1 || { tail -20 gpurun_out/${tag}_ldoor_f32.log; exit 1; }
tail -8 gpurun_out/${tag}_ldoor_f32.log
