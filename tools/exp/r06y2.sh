# Round 6: EA read requests / L2 hit rate of the tile kernel with the clustered launch order
set -u -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
VBC_TILE_CLUSTER=1 timeout -k 10 400 python -u tools/pmc_traffic.py --counters "TCC_EA0_RDREQ_sum;TCC_HIT_sum,TCC_MISS_sum;TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum,TA_BUSY_avr" --tag _r06y_cluster --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 > gpurun_out/r06y2_pmc.log 2>&1 || { tail -30 gpurun_out/r06y2_pmc.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_c5-mesh_f32_r06y_cluster.json')); c={k:v['mean'] for k,v in d['counters'].items()}
print({k: f'{v:.4g}' for k,v in c.items()})"
