# The reference's bin/test_table.jl table on the recalibrated stand-ins (graph-timed GPU column), with
# the per-bucket layout decisions (VBC_VERBOSE) in a side log.
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r04_table}
for spec in "Boeing/ct20stif f64" "Rothberg/3dtube f64" "Schmid/thermal1 f64" "DIMACS10/chesapeake f64"; do
  set -- $spec
  short=$(basename $1)
  VBC_VERBOSE=1 timeout -k 10 400 python -u tools/test_table.py --matrix $1 --dtype $2 ${EXTRA:-} \
      --json gpurun_out/${tag}_${short}_$2.json > gpurun_out/${tag}_${short}_$2.log 2> gpurun_out/${tag}_${short}_$2.verbose.log || exit $?
  tail -16 gpurun_out/${tag}_${short}_$2.log
done
# ldoor (C3 / C4 size) in fp32 with the 1D methods: the large mixed-width / filled partitions
VBC_VERBOSE=1 timeout -k 10 500 python -u tools/test_table.py --matrix GHS_psdef/ldoor --dtype f32 --no-2d \
    --json gpurun_out/${tag}_ldoor_f32.json > gpurun_out/${tag}_ldoor_f32.log 2> gpurun_out/${tag}_ldoor_f32.verbose.log || exit $?
tail -8 gpurun_out/${tag}_ldoor_f32.log
