import sys; sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch
import sparsematrixvbcs_amd as V
from test_gpu_mfma import ref_1d, ref_cols, as_dev
for dtype in (np.float64, np.float32):
    B = V.synthetic.vbr_1dvbc(300, 64, 600, 2, W=2, dtype=dtype, seed=11)
    R = ref_1d(B)
    X = np.random.default_rng(5).uniform(-1, 1, (B.m, 16)).astype(dtype)
    X[17, 3] = np.inf; X[101, 0] = np.nan; X[250, 9] = -np.inf
    for eng in ("mfma", "vector"):
        Yd = as_dev(np.zeros((B.n, 16), dtype), "R")
        V.mul_(Yd, B.T, as_dev(X, "R"), engine=eng)
        got = Yd.cpu().numpy()
        ref = ref_cols(R, X, np.zeros((B.n, 16), dtype), 1.0, 0.0)
        print(dtype.__name__, eng, "got nan at", np.argwhere(np.isnan(got)).tolist(), "ref nan at", np.argwhere(np.isnan(ref)).tolist())
        print("  got inf", np.argwhere(np.isinf(got)).tolist(), "ref inf", np.argwhere(np.isinf(ref)).tolist())
    for r in (17, 101, 250):
        st = [l for l in range(64) if r + 1 in B.idx[B.pos[l]-1:B.pos[l+1]-1]]
        print("row", r, "in stripes", st)
