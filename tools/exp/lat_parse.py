"""Summarise tools/exp/r04_pmc_lat.sh: per dispatch of each run's dominant kernel, the memory-side read
requests, their mean latency by Little's law (TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ, cycles: the
outstanding requests summed each cycle over the requests) and the DRAM-credit stall cycles.
    python tools/exp/lat_parse.py gpurun_out > profiles/r04_lat.json"""
import csv
import glob
import json
import sys
from collections import defaultdict

KERN = {"probe": "probe", "ns": "spmv_sweep", "fe": "spmv_slots", "c5": "spmm_panel", "c5mesh": "spmm_panel"}
out = {}
for d in sorted(glob.glob(sys.argv[1] + "/r04_lat_*")):
    if d.endswith(".log"):
        continue
    tag = d.rsplit("r04_lat_", 1)[1]
    want = KERN["probe" if tag.startswith("probe") else tag]
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if want not in row.get("Kernel_Name", ""):
                continue
            per[row.get("Dispatch_Id", row.get("Correlation_Id"))][row["Counter_Name"]] += float(row["Counter_Value"])
    if not per:
        continue
    keys = ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_LEVEL_sum", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "GRBM_GUI_ACTIVE"]
    avg = {k: sum(v.get(k, 0.0) for v in per.values()) / len(per) for k in keys}
    out[tag] = {"kernel": want, "dispatches": len(per), **{k: round(v) for k, v in avg.items()},
                "mean_latency_cycles": round(avg["TCC_EA0_RDREQ_LEVEL_sum"] / max(avg["TCC_EA0_RDREQ_sum"], 1), 1),
                "credit_stall_per_active_cycle": round(avg["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / max(avg["GRBM_GUI_ACTIVE"], 1), 3)}
print(json.dumps(out, indent=1))
