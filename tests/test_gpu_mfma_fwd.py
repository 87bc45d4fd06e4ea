"""GPU parity of the matrix-core multi-RHS FORWARD product Y = α·B·X + β·Y (VBC_CREATE_MULTI_FORWARD:
the panel layout of Bᵀ -- output row groups as stripes, tile columns as stored rows -- run by the same
spmm_panel kernel, so the matrix is read once for all right-hand sides).

The reference has no matrix mul! (multiply_1DVBC.jl:184-185, multiply_VBC.jl:196-197), so parity is
column by column against the oracle's forward products (multiply_1DVBC.jl:13-83, multiply_VBC.jl:7-87).
Tolerances as test_gpu_mfma.py: one-hot probes exact; random X normwise 1e-12 (fp64) / 1e-5 (fp32)."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.test_gpu_mfma import TOL32, TOL64, as_dev, ref_1d, ref_2d, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(autouse=True, params=["tiles", "0"], ids=["tiles", "panels"])
def multi_layout(request, monkeypatch):
    """Every test on the two multi-RHS layouts (test_gpu_mfma.py): MFMA panels, and the tile-granular layout
    of C = Bᵀ's small tiles (VBC_PANEL_TILES=1)."""
    monkeypatch.setenv("VBC_PANEL_TILES", "1" if request.param == "tiles" else "0")
    return request.param


def ref_cols_fwd(R, X, Y0, alpha, beta):
    Rd = R
    if R.val.dtype != np.float64:
        Rd = type(R).__new__(type(R))
        Rd.__dict__.update(R.__dict__)
        Rd.val = R.val.astype(np.float64)
    return np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64),
                           np.ascontiguousarray(Y0[:, j], dtype=np.float64), alpha, beta, trans=False,
                           ref_semantics=False) for j in range(X.shape[1])], axis=1)


def multi_fwd_info(B):
    return B.info(0, trans=False, multi=True)


def test_golden_one_hot_forward(golden):
    """B·E over identity blocks of 16 columns gives exactly the columns of A (runtests.jl:29-40)."""
    for key, g in golden.items():
        A = g["A"]
        m, n = A.shape
        D = A.toarray()
        for B in (V.SparseMatrix1DVBC[4](A, V.StrictChunker(4)),
                  V.SparseMatrixVBC[4, 4](A, V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)))):
            for layout in ("R", "C"):
                for j0 in range(0, n, 16):
                    k = min(16, n - j0)
                    X = np.zeros((n, k))
                    X[np.arange(j0, j0 + k), np.arange(k)] = 1.0
                    Y = as_dev(np.full((m, k), np.nan), layout)
                    V.mul_(Y, B, as_dev(X, layout), engine="mfma")
                    assert np.array_equal(Y.cpu().numpy(), D[:, j0:j0 + k]), (key, type(B).__name__, layout)
            assert multi_fwd_info(B)["bins_m"] > 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("nrhs", [2, 16, 33, 64, 70])
def test_forward_1dvbc_random(nrhs, dtype):
    """Widths 1..16 and a w > 16 stripe, empty stripes and rows, α / β, both layouts, vs the oracle."""
    tol = TOL64 if dtype == np.float64 else TOL32
    rng = np.random.default_rng(300 + nrhs)
    for widths, q in ((list(range(1, 17)), 2000), ([1, 20, 7, 33], 150)):
        L = 60
        w = np.array([widths[i % len(widths)] for i in range(L)])
        B = V.synthetic.vbr_1dvbc(900, L, q, w, W=40, dtype=dtype, seed=nrhs * 5 + int(w.sum()))
        R = ref_1d(B)
        for layout in ("R", "C"):
            X = rng.uniform(-1, 1, (B.n, nrhs)).astype(dtype)
            Y0 = rng.uniform(-1, 1, (B.m, nrhs)).astype(dtype)
            for alpha, beta in ((1.0, 0.0), (-1.5, 0.5)):
                Yd = as_dev(Y0, layout)
                V.mul_(Yd, B, as_dev(X, layout), alpha, beta, engine="mfma")
                assert rel(Yd.cpu().numpy(), ref_cols_fwd(R, X, Y0, alpha, beta)) <= tol, (widths, layout, alpha)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("uw", [(8, 8), (4, 16), (16, 4), (3, 5), (1, 1), (20, 3)])
def test_forward_vbc2d_random(uw, dtype):
    """C5 shape at small size (costs.jl:200-220 generator): u x w tiles, block rows as output groups
    (u = 20 > 16: cut into 16 + 4), 16 RHS."""
    u, w = uw
    tol = TOL64 if dtype == np.float64 else TOL32
    B = V.synthetic.vbr_2d(40, 30, 200, u, w, dtype=dtype, seed=u * 17 + w)
    R = ref_2d(B)
    rng = np.random.default_rng(u * w)
    X = rng.uniform(-1, 1, (B.n, 16)).astype(dtype)
    Y0 = rng.uniform(-1, 1, (B.m, 16)).astype(dtype)
    for layout in ("R", "C"):
        Yd = as_dev(Y0, layout)
        V.mul_(Yd, B, as_dev(X, layout), 2.0, 0.25, engine="mfma")
        assert rel(Yd.cpu().numpy(), ref_cols_fwd(R, X, Y0, 2.0, 0.25)) <= tol, layout


def test_forward_node_runs_and_bytes():
    """A 3-dof stiffness operator: rows grouped in node runs of 3 (identical stripe lists); the
    forward panel layout streams the matrix once -- its bytes are those of one pass, not 16."""
    B = V.synthetic.fe_stiffness_3d_1dvbc(30000, 300000)
    R = ref_1d(B)
    rng = np.random.default_rng(8)
    X = rng.uniform(-1, 1, (B.n, 16))
    Y = torch.zeros((B.m, 16), dtype=torch.float64, device="cuda:0")
    V.mul_(Y, B, torch.from_numpy(X).cuda())
    assert rel(Y.cpu().numpy(), ref_cols_fwd(R, X, np.zeros((B.m, 16)), 1.0, 0.0)) <= TOL64
    inf = multi_fwd_info(B)
    nv = int(B.ofs[-1] - 1)
    assert nv * 8 <= inf["bytes_m"] <= 1.6 * nv * 8 + 4 * len(B.idx) * 3  # one pass (+ keys, panel padding)


def test_forward_nonfinite_x():
    """Inf / NaN in X reach exactly the outputs the reference's forward loop gives them."""
    B = V.synthetic.vbr_2d(30, 20, 120, 4, 4, dtype=np.float64, seed=5)
    R = ref_2d(B)
    X = np.random.default_rng(2).uniform(-1, 1, (B.n, 16))
    X[3, 0], X[17, 5] = np.inf, np.nan
    Y = torch.zeros((B.m, 16), dtype=torch.float64, device="cuda:0")
    V.mul_(Y, B, torch.from_numpy(X).cuda())
    ref = ref_cols_fwd(R, X, np.zeros((B.m, 16)), 1.0, 0.0)
    got = Y.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = np.isfinite(ref)
    assert np.array_equal(np.isinf(got), np.isinf(ref))
    assert rel(got[fin], ref[fin]) <= TOL64


def test_forward_duplicate_row_in_stripe_adds_both():
    """A hand-built 1DVBC whose stripe stores one row twice (the reference's constructors never do, but
    its forward loop y[idx[Q]] += ... takes both, multiply_1DVBC.jl:33-36): the forward panel layout
    must add the two copies, not keep the last one."""
    W = 4
    spl = np.array([1, 3, 5], np.int64)            # two stripes of width 2
    pos = np.array([1, 4, 6], np.int64)            # stripe 1: rows 2, 2, 5; stripe 2: rows 1, 5
    idx = np.array([2, 2, 5, 1, 5], np.int64)
    ofs = np.array([1, 7, 11], np.int64)
    val = np.zeros(10 + 8)
    val[:10] = np.random.default_rng(4).uniform(-1, 1, 10)
    B = V.SparseMatrix1DVBC(W, 6, 4, V.SplitPartition(spl), pos, idx, ofs, val)
    R = ref_1d(B)
    X = np.random.default_rng(5).uniform(-1, 1, (4, 16))
    ref = ref_cols_fwd(R, X, np.zeros((6, 16)), 1.0, 0.0)
    for layout in ("R", "C"):
        Y = as_dev(np.zeros((6, 16)), layout)
        V.mul_(Y, B, as_dev(X, layout), engine="mfma")
        assert rel(Y.cpu().numpy(), ref) <= TOL64, layout
