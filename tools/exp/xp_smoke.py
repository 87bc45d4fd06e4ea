"""Quick check of the persistent staged-X tile kernel on a small c5-mesh (B'X and B X, 16 RHS) vs the oracle."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
import sparsematrixvbcs_amd as V
from oracle import oracle as O
os.environ.setdefault("VBC_TILE_STAGE", "1")
B = bench.build_matrix("c5-mesh", np.float32, float(sys.argv[1]) if len(sys.argv) > 1 else 0.002)
B.val[:] = np.random.default_rng(3).integers(-8, 9, B.val.shape)
print("info", B.info(multi=True)["planar_mask"], flush=True)
Rd = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
rng = np.random.default_rng(1)
for trans in (True, False):
    nx, ny = (B.m, B.n) if trans else (B.n, B.m)
    X = rng.integers(-8, 9, (nx, 16)).astype(np.float32)
    Y = torch.full((ny, 16), float("nan"), dtype=torch.float32, device="cuda:0")
    V.mul_(Y, B.T if trans else B, torch.from_numpy(X).to("cuda:0"), engine="mfma")
    torch.cuda.synchronize()
    want = np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64), np.zeros(ny), trans=trans) for j in range(16)], axis=1)
    got = Y.cpu().numpy()
    print("trans", trans, "bitwise", np.array_equal(got, want.astype(np.float32)), "maxdiff", np.nanmax(np.abs(got - want)), flush=True)
