# Round 6: the tile kernel after the value-load masking -- its counters (segments per tile) and the bench line
set -u -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
G="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU;TA_TA_BUSY_sum,TA_BUSY_avr,TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum;TCC_EA0_RDREQ_sum;TCC_HIT_sum,TCC_MISS_sum"
timeout -k 10 600 python -u tools/pmc_traffic.py --counters "$G" --tag _r06x --workload c5-mesh --dtype f32 --kernel spmm_tiles --read-factor 1 > gpurun_out/r06x_pmc.log 2>&1 || { tail -30 gpurun_out/r06x_pmc.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_c5-mesh_f32_r06x.json')); c={k:v['mean'] for k,v in d['counters'].items()}
print({k: f'{v:.4g}' for k,v in c.items()})"
timeout -k 10 300 python -u bench.py --workload c5-mesh --dtype f32 --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/r06x_bench_c5mesh.log 2>&1 || { tail -20 gpurun_out/r06x_bench_c5mesh.log; exit 1; }
tail -1 gpurun_out/r06x_bench_c5mesh.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['parity'])"
