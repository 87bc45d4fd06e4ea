"""Collect per-launch HBM traffic of the bench's dominant kernel with rocprofv3 PMC counters.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KB) are collected in SEPARATE passes (they
do not fit one pass), with --kernel-trace only (no sys/runtime traces), and on gfx950 FETCH_SIZE
counts exactly half of the bytes of wide coalesced streaming reads, so read bytes = 2 x FETCH_SIZE.
Writes profiles/pmc_<workload>_<dtype>.json with the corrected per-launch figure (and the raw ones).

    python tools/pmc_traffic.py [--workload ns] [--dtype f64] [--extra "--scale 1.0"]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL = "spmv_ranges"  # --kernel overrides


def run_pass(counters, outdir, bench_args, kernel=KERNEL, program="bench.py"):
    cmd = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "--output-format", "csv", "-d", str(outdir),
           "-o", "pmc", "--", sys.executable, str(ROOT / program), *bench_args]
    print("pass:", " ".join(counters), flush=True)
    subprocess.run(cmd, check=True, cwd=ROOT, timeout=180)
    files = glob.glob(str(outdir / "**" / "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                name = row["Counter_Name"]
                vals.setdefault(name, []).append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ns")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--extra", default="")
    ap.add_argument("--counters", default="", help="extra counter passes, ';'-separated groups")
    ap.add_argument("--kernel", default=KERNEL, help="kernel name substring to attribute counters to")
    ap.add_argument("--tag", default="", help="suffix of the output file name (ablation runs)")
    ap.add_argument("--program", default="", help="run this script with --extra's arguments instead of bench.py "
                    "(e.g. tools/shard_time.py for one shard of a split)")
    ap.add_argument("--read-factor", type=float, default=2.0,
                    help="FETCH_SIZE correction: 2 for 16-B/lane streaming reads (gfx950 half-count), 1 for "
                         "dword loads and gathers")
    args = ap.parse_args()
    out = ROOT / "gpurun_out" / "pmc"
    if args.program:
        bench_args = ["--steps", str(args.steps), "--warmup", "2", "--workload", args.workload, "--dtype",
                      args.dtype] + args.extra.split()
    else:
        bench_args = ["--steps", str(args.steps), "--warmup", "2", "--no-cpu-baseline", "--no-secondary", "--no-parity",
                      "--workload", args.workload, "--dtype", args.dtype] + args.extra.split()
    res = {}
    passes = [["FETCH_SIZE"], ["WRITE_SIZE"]] + [g.split(",") for g in args.counters.split(";") if g]
    for i, counters in enumerate(passes):
        try:
            vals = run_pass(counters, out / f"pass{i}", bench_args, args.kernel, args.program or "bench.py")
        except subprocess.SubprocessError as e:  # a counter set the profiler cannot serve
            print("pass failed:", counters, e, flush=True)
            if i < 2:
                raise
            continue
        for k, v in vals.items():
            res[k] = dict(mean=sum(v) / len(v), n=len(v), min=min(v), max=max(v))
    fetch_kb = res["FETCH_SIZE"]["mean"]
    write_kb = res["WRITE_SIZE"]["mean"]
    summary = {
        "workload": args.workload, "dtype": args.dtype, "kernel": args.kernel,
        "program": (args.program + " " + args.extra).strip() or None,
        "method": "rocprofv3 --kernel-trace --pmc, FETCH_SIZE and WRITE_SIZE in separate passes; "
                  f"read bytes = {args.read_factor:g} x FETCH_SIZE (gfx950 counts 16-B/lane streaming reads "
                  "at half, MI355X_MICROARCH.md §HBM; dword loads and gathers are counted in full)",
        "fetch_size_kb_per_launch": fetch_kb, "write_size_kb_per_launch": write_kb,
        "hbm_bytes_per_launch": int(args.read_factor * fetch_kb * 1024 + write_kb * 1024),
        "raw_bytes_per_launch": int(fetch_kb * 1024 + write_kb * 1024),
        "counters": res,
    }
    if "TCC_EA0_RDREQ_sum" in res:
        rq = res["TCC_EA0_RDREQ_sum"]["mean"]
        bub = res.get("TCC_BUBBLE_sum", {}).get("mean", 0.0)
        r32 = res.get("TCC_EA0_RDREQ_32B_sum", {}).get("mean", 0.0)
        summary["rdreq_per_launch"] = {"all": rq, "bubble_128B": bub, "32B": r32,
                                       "dram": res.get("TCC_EA0_RDREQ_DRAM_sum", {}).get("mean")}
    if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
        h, m = res["TCC_HIT_sum"]["mean"], res["TCC_MISS_sum"]["mean"]
        summary["l2_hit_rate"] = h / max(h + m, 1.0)
    if os.environ.get("VBC_PANEL_DIAG") or os.environ.get("VBC_DIAG"):
        summary["ablation_env"] = {k: v for k, v in os.environ.items() if k.startswith("VBC_")}
    p = ROOT / "profiles" / f"pmc_{args.workload}_{args.dtype}{args.tag}.json"
    p.write_text(json.dumps(summary, indent=1) + "\n")
    (ROOT / "gpurun_out" / p.name).write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
