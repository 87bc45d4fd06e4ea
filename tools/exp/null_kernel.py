"""Per-launch floor of back-to-back kernels in one HIP-graph replay on this box: a one-element torch
kernel, and libvbc's product on a tiny matrix (64 stripes).  python tools/exp/null_kernel.py"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    import sparsematrixvbcs_amd as V
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    t = torch.zeros(1, device=dev)
    _, ms, _ = bench.timed_products(lambda: t.add_(1.0), 500, dev, s, 1)
    print(json.dumps({"what": "torch one-element add_, graph of 500", "us_per_launch": round(ms * 1e3, 3)}))
    for L, q in ((64, 64), (1024, 4096), (8192, 65536)):
        B = V.synthetic.vbr_1dvbc(4096, L, q, 3, W=8, seed=1)
        x = torch.rand(B.m, dtype=torch.float64, device=dev)
        y = torch.empty(B.n, dtype=torch.float64, device=dev)
        with torch.cuda.stream(s):
            V.mul_(y, B.T, x)
        torch.cuda.synchronize()
        _, ms, _ = bench.timed_products(lambda: V.mul_(y, B.T, x), 500, dev, s, 1)
        print(json.dumps({"what": f"libvbc B'x, {L} stripes, {q} rows", "kernel": bench.kernel_name(B, 0, 1),
                          "us_per_launch": round(ms * 1e3, 3)}))


if __name__ == "__main__":
    main()
