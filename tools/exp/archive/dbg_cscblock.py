import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import sparsematrixvbcs_amd as V
from oracle import oracle as O
os.environ["VBC_PLANAR_SPLIT"] = "0"
A = V.synthetic.fe_stiffness_3d(90000, 2_000_000, 3, np.float64).tocsc()
A.sort_indices()
m, n = A.shape
x = np.random.default_rng(23).uniform(-1, 1, m)
ref = O.trspmv(A, x, np.zeros(n))
for blk in ("0", "1"):
    os.environ["VBC_CSC_BLOCK"] = blk
    C = V.SparseMatrixCSC(A)
    y = torch.zeros(n, dtype=torch.float64, device="cuda:0")
    V.TrSpMV_(y, C, torch.from_numpy(x).cuda())
    g = y.cpu().numpy()
    inf = C.info(trans=True)
    bad = np.nonzero(g != ref)[0]
    print(blk, {k: inf[k] for k in ("L", "slot_bins", "planar_bins", "sweep_bins", "bins_t", "planar_run", "planar_split")},
          "ndiff", len(bad), bad[:10], np.abs(g - ref).max())
    C.release()
