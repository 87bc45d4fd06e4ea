"""Probe (round 6): the forward product B_g x_g of a stripe shard writes all m rows of y (zeros where its
stripes store nothing).  Rebased to the span of rows it stores (vbc_sharded_xspan's span), the shard is
(hi - lo) x n_g and its product writes only that span.  Times both forms of every 1/N ldoor shard
(graph-replayed, both directions) and checks the rebased products against the plain ones bit for bit."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="ldoor")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch

    import bench
    import sparsematrixvbcs_amd as V
    from sparsematrixvbcs_amd import distributed as D
    from sparsematrixvbcs_amd.matrices import SparseMatrix1DVBC
    B = bench.build_matrix(args.workload, np.float64)
    cuts = D.stripe_split(B, args.world)
    rng = np.random.default_rng(3)
    dev = torch.device("cuda", 0)

    def graph_us(fn):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        return min(bench.timed_products(fn, args.reps, dev, s, 1)[1] for _ in range(3)) * 1e3

    for r in range(args.world):
        S, col0 = D.shard(B, int(cuts[r]), int(cuts[r + 1]))
        lo, hi = int(S.idx.min()) - 1, int(S.idx.max())
        Rb = SparseMatrix1DVBC(S.W, hi - lo, S.n, S.Phi, S.pos, (S.idx - lo).astype(S.idx.dtype), S.ofs, S.val)
        xf = torch.from_numpy(rng.uniform(-1, 1, S.n)).to(dev)
        xt = torch.from_numpy(rng.uniform(-1, 1, S.m)).to(dev)
        y_full = torch.empty(S.m, dtype=torch.float64, device=dev)
        y_span = torch.empty(hi - lo, dtype=torch.float64, device=dev)
        yt = torch.empty(S.n, dtype=torch.float64, device=dev)
        yt2 = torch.empty(S.n, dtype=torch.float64, device=dev)
        out = {"shard": r, "rows": [lo, hi], "m": S.m,
               "fwd_plain_us": graph_us(lambda: V.mul_(y_full, S, xf)),
               "fwd_rebased_us": graph_us(lambda: V.mul_(y_span, Rb, xf)),
               "t_plain_us": graph_us(lambda: V.mul_(yt, S.T, xt)),
               "t_rebased_us": graph_us(lambda: V.mul_(yt2, Rb.T, xt[lo:hi]))}
        V.mul_(y_full, S, xf)
        V.mul_(y_span, Rb, xf)
        V.mul_(yt, S.T, xt)
        V.mul_(yt2, Rb.T, xt[lo:hi])
        torch.cuda.synchronize()
        out["fwd_bitwise"] = bool(torch.equal(y_full[lo:hi], y_span))
        out["fwd_outside_zero"] = bool((y_full[:lo] == 0).all()) and bool((y_full[hi:] == 0).all())
        out["t_bitwise"] = bool(torch.equal(yt, yt2))
        out = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}
        print(json.dumps(out), flush=True)
        S.release()
        Rb.release()


if __name__ == "__main__":
    main()
