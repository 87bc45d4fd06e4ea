"""Fixed cost per product: graph-replayed product time against matrix size (fe / fe3d / ldoor scales),
fitted as t = t0 + bytes / BW.  python tools/exp/latency_probe.py --workload fe3d --scales 0.001,0.01,0.1"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fe")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--scales", default="0.0005,0.002,0.005,0.01,0.02,0.05")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch

    import bench
    import sparsematrixvbcs_amd as V
    dtype = np.float64 if args.dtype == "f64" else np.float32
    esz = np.dtype(dtype).itemsize
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    pts = []
    for sc in (float(v) for v in args.scales.split(",")):
        B = bench.build_matrix(args.workload, dtype, sc)
        x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, B.m).astype(dtype)).to(dev)
        y = torch.empty(B.n, dtype=x.dtype, device=dev)
        Bt = B.T
        with torch.cuda.stream(stream):
            B.handle(0, True)
            for _ in range(5):
                V.mul_(y, Bt, x)
        torch.cuda.synchronize(dev)
        _, ev_ms, _ = bench.timed_products(lambda: V.mul_(y, Bt, x), args.steps, dev, stream, 1)
        nb = bench.algorithmic_bytes(B, esz)
        inf = B.info(0, True)
        pts.append((nb, ev_ms * 1e3))
        print(json.dumps({"scale": sc, "bytes": nb, "us": round(ev_ms * 1e3, 2), "kernel": bench.kernel_name(B, 0, 1),
                          "planar_split": inf["planar_split"], "GBs": round(nb / ev_ms / 1e6, 1)}), flush=True)
        B.release()
    b = np.array([p[0] for p in pts], float)
    t = np.array([p[1] for p in pts], float)
    A = np.stack([np.ones_like(b), b], 1)
    (t0, inv), *_ = np.linalg.lstsq(A, t, rcond=None)
    print(json.dumps({"fit_t0_us": round(t0, 2), "fit_GBs": round(1e-3 / inv, 1)}))


if __name__ == "__main__":
    main()
