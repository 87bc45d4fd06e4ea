"""HIP-graph replay of a product sequence vs eager launches (launch-bound small operators).

An iterative solver calls mul! on the same handle every iteration; for a matrix that sits in L2/MALL
(the ct20stif stand-in, 2.6e6 nnz) the launch path (Python -> ctypes -> vbc_mul -> hipLaunchKernel)
is a visible part of each product.  libvbc launches on the caller's stream with no allocation, sync
or host copy on the VBC_MEM_DEVICE path, so a product sequence can be captured once into a HIP graph
(torch.cuda.CUDAGraph is hipGraph on ROCm) and replayed.

    python tools/graph_bench.py [--workload ct20stif|fe] [--reps 100]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ct20stif")
    ap.add_argument("--reps", type=int, default=100)
    args = ap.parse_args()
    import torch

    import sparsematrixvbcs_amd as V

    if args.workload == "fe":
        B = V.synthetic.fe_grid_2d(2236, dof=2)
    else:
        name = {"ct20stif": "Boeing/ct20stif", "ldoor": "GHS_psdef/ldoor"}[args.workload]
        B = V.SparseMatrix1DVBC[8](V.synthetic.standin(name).T.tocsc(), V.StrictChunker(8))
    rng = np.random.default_rng(0xC0FFEE)
    x = torch.from_numpy(rng.uniform(-1, 1, B.m)).cuda()
    y = torch.empty(B.n, dtype=torch.float64, device="cuda")
    Bt = B.T
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(5):
            V.mul_(y, Bt, x)  # builds the handle and warms up outside the capture
    torch.cuda.synchronize()
    res = {}
    for mode in ("eager", "graph"):
        if mode == "graph":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(args.reps):
                    V.mul_(y, Bt, x)
        times = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record(s)
                if mode == "graph":
                    g.replay()
                else:
                    for _ in range(args.reps):
                        V.mul_(y, Bt, x)
                e1.record(s)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / args.reps)
        res[mode] = float(np.median(times))
        print(f"{args.workload} {mode:6s} {res[mode]:8.2f} us per product (median of 7 x {args.reps})", flush=True)
    print(f"graph speed-up {res['eager'] / res['graph']:.2f}x")


if __name__ == "__main__":
    main()
