# Round-4 confirmation, part B: predicted strong scaling (every shard timed alone) and the reference's
# table on the four ref.out stand-ins + ldoor (logs: gpurun_out/r04c_shard_* and r04_table_*)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/shard_time.py --workload ldoor --dtype f64 --worlds 1,2,4,8 --steps 200 \
    > gpurun_out/r04c_shard_ldoor.log 2>&1 || exit $?
tail -6 gpurun_out/r04c_shard_ldoor.log
timeout -k 10 400 python -u tools/shard_time.py --workload fe --dtype f64 --worlds 1,2,4,8 --steps 100 \
    > gpurun_out/r04c_shard_fe.log 2>&1 || exit $?
tail -6 gpurun_out/r04c_shard_fe.log
bash tools/exp/r04_table.sh r04c_table
