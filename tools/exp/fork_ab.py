"""B'x with several launch groups: forked side streams (default) vs one stream (VBC_FORK=0), graph-replayed.
Matrices: the ct20stif / ldoor stand-ins under the 'min blocks' partition (mixed widths), ldoor TrSpMV! (CSC
column blocking), the golden-free mixed-width generator."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import os  # noqa: E402

import sparsematrixvbcs_amd as V  # noqa: E402


def graph_time(fn, reps=50, rounds=5):
    s = torch.cuda.Stream()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return float(np.median(ts))


def main():
    W = 8
    lim = lambda mdl: V.ConstrainedCost(mdl, V.VertexCount(), W)
    cases = []
    for name in ("Boeing/ct20stif", "GHS_psdef/ldoor"):
        A = V.synthetic.standin(name).T.tocsc()
        cases.append((name + " min blocks", lambda A=A: V.SparseMatrix1DVBC[W](A, V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks())))))
        cases.append((name + " strict", lambda A=A: V.SparseMatrix1DVBC[W](A, V.StrictChunker(W))))
    cases.append(("mixed w 1..8, 2e5 stripes", lambda: V.synthetic.vbr_1dvbc(400000, 200000, 2000000, np.arange(200000) % 8 + 1, W=8, seed=1)))
    for label, make in cases:
        B = make()
        x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, B.m)).cuda()
        res = []
        for fork in ("1", "0", "L0"):
            os.environ["VBC_FORK"] = fork[-1]
            os.environ["VBC_SLOTS_LONG"] = "0" if fork == "L0" else "2"
            Bv = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
            inf = Bv.info(trans=True)
            y = torch.zeros(B.n, dtype=torch.float64, device="cuda")
            res.append((graph_time(lambda: V.mul_(y, Bv.T, x)), y.clone(), inf))
            Bv.release()
        os.environ.pop("VBC_FORK")
        os.environ.pop("VBC_SLOTS_LONG")
        same = torch.equal(res[0][1], res[1][1])
        inf = res[0][2]
        print(f"{label:40s} fork {res[0][0]:7.2f} us  one stream {res[1][0]:7.2f} us  old rule, one stream "
              f"{res[2][0]:7.2f} us (planar {res[2][2]['planar_bins']} merge {res[2][2]['bins_t']})  bitwise {same}  "
              f"planar {inf['planar_bins']} slot {inf['slot_bins']} sweep {inf['sweep_bins']} merge {inf['bins_t']}", flush=True)


if __name__ == "__main__":
    main()
