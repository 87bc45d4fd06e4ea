"""Layout choices and graph-timed B'x of the ct20stif stand-in under the 'min blocks' partition
(mixed widths 3 / 6 / 7 / 8 with fill), with layout knobs set per variant (VBC_* env, read at create)."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import sparsematrixvbcs_amd as V  # noqa: E402
from tools.exp.fork_ab import graph_time  # noqa: E402


def main():
    W = 8
    lim = V.ConstrainedCost(V.model_SparseMatrix1DVBC_blocks(), V.VertexCount(), W)
    name = sys.argv[1] if len(sys.argv) > 1 else "Boeing/ct20stif"
    A = V.synthetic.standin(name).T.tocsc()
    B0 = V.SparseMatrix1DVBC[W](A, V.DynamicTotalChunker(lim))
    x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, B0.m)).cuda()
    ref = None
    for var in sys.argv[2:]:
        env = dict(kv.split("=") for kv in var.split(",") if "=" in kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        os.environ["VBC_VERBOSE"] = "1"
        B = V.SparseMatrix1DVBC(B0.W, B0.m, B0.n, B0.Phi, B0.pos, B0.idx, B0.ofs, B0.val)
        inf = B.info(trans=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        y = torch.zeros(B.n, dtype=torch.float64, device="cuda")
        t = graph_time(lambda: V.mul_(y, B.T, x))
        ref = y.clone() if ref is None else ref
        d = (y - ref).norm().item() / ref.norm().item()
        print(f"{var:40s} {t:8.2f} us  planar {inf['planar_bins']} slot {inf['slot_bins']} merge {inf['bins_t']} "
              f"split {inf['planar_split']} rel-diff {d:.1e}", flush=True)
        B.release()


if __name__ == "__main__":
    main()
