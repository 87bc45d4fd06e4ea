mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/exp/latency_probe.py --workload fe > gpurun_out/r03g_lat_fe.log 2>&1 && cat gpurun_out/r03g_lat_fe.log | grep -v amdgpu.ids &&
timeout -k 10 300 python -u tools/exp/latency_probe.py --workload fe3d --scales 0.0005,0.002,0.005,0.01,0.02,0.05 > gpurun_out/r03g_lat_fe3d.log 2>&1 && cat gpurun_out/r03g_lat_fe3d.log | grep -v amdgpu.ids &&
timeout -k 10 300 python -u tools/shard_time.py --workload ldoor --worlds 1,8 > gpurun_out/r03g_shard_ldoor.log 2>&1 && cut -c1-400 gpurun_out/r03g_shard_ldoor.log | grep -v amdgpu.ids &&
timeout -k 10 300 python -u tools/ab.py --workload ct20stif --variants "VBC_PLANAR_SPLIT=1;VBC_PLANAR_SPLIT=0;VBC_PLANAR_SPLIT=2;VBC_PLANAR_SPLIT=8" > gpurun_out/r03g_ab_ct20.log 2>&1 && tail -4 gpurun_out/r03g_ab_ct20.log
