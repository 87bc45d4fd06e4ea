set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
V="VBC_ARENA_CONTIG=0;VBC_ARENA_CONTIG=1"
timeout -k 10 400 python tools/ab.py --workload fe --dtype f64 --copies 4 --variants "$V" > gpurun_out/contig_fe.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/contig_fe.log
