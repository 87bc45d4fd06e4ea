# FE-3D memory-side counters after the round-5 lane-tile sizing (the bench line's traffic source)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pmc_traffic.py --workload fe3d --dtype f64 --kernel spmv_planar_lanes --counters "TCC_EA0_RDREQ_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_DRAM_sum;TCC_HIT_sum,TCC_MISS_sum" > gpurun_out/r05zp_pmc_fe3d.log 2>&1 || { tail -20 gpurun_out/r05zp_pmc_fe3d.log; exit 1; }
grep -E '"hbm_bytes_per_launch"|"l2_hit_rate"|"all"' gpurun_out/pmc_fe3d_f64.json
