"""Summarise rocprofv3 counter_collection CSVs: mean per launch of each counter for kernels matching a name."""
import csv
import glob
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else "spmm_panel"
vals = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if pat in row.get("Kernel_Name", ""):
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} mean {sum(v)/len(v):16.1f}  n={len(v)}")
