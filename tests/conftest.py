import os
import sys
from pathlib import Path

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden" / "matrices.npz"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvbc's HIP kernels)")
    config.addinivalue_line("markers", "slow: large sizes")


def golden_matrices():
    """The six SuiteSparse matrices of the reference's test/matrices.jl, expanded to full
    (runtests.jl:18 `SparseMatrixCSC(A)`), with their committed scipy probes."""
    d = np.load(GOLDEN, allow_pickle=False)
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_shape")})
    out = {}
    for k in keys:
        m, n = d[k + "_shape"]
        A = sp.csc_matrix((d[k + "_V"], (d[k + "_I"] - 1, d[k + "_J"] - 1)), shape=(m, n))
        if d[k + "_sym"][0]:
            T = sp.tril(A)
            A = (T + sp.tril(T, -1).T).tocsc()
        A.sort_indices()
        out[k] = dict(A=A, xf=d[k + "_xf"], yf=d[k + "_yf"], xt=d[k + "_xt"], yt=d[k + "_yt"])
    return out


SIZES = [1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17]  # runtests.jl:14-16


def sprand_family(trials=4, seed=0xDEADBEEF, kinds=("f64", "bool", "i32")):
    """Restatement of the runtests.jl:14-16 corpus with our own seeded generator (Julia's RNG stream
    is not reproducible here): sprand(m, n, 0.2) for m, n in SIZES, Float64 / Bool / Int32 values."""
    rng = np.random.default_rng(seed)
    mats = []
    for kind in kinds:
        for m in SIZES:
            for n in SIZES:
                for t in range(trials):
                    mask = rng.random((m, n)) < 0.2
                    if kind == "f64":
                        vals = rng.random((m, n))
                    elif kind == "bool":
                        vals = np.ones((m, n))
                    else:
                        vals = rng.integers(-2**31, 2**31, (m, n)).astype(np.float64)
                    A = sp.csc_matrix(np.where(mask, vals, 0.0))
                    # keep explicit structure exactly as sampled (no zero values drawn in practice)
                    mats.append((f"{kind}_{m}x{n}_{t}", A))
    return mats


@pytest.fixture(scope="session")
def golden():
    return golden_matrices()


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
