"""GPU parity of the row-swept layout (csrc/vbc_sweep.hip) against the oracle, both directions.

The library picks the swept layout for a width bucket (w <= 8) whose neighbouring segments gather
from unrelated places of a large x (the costs.jl:63-83 generator); VBC_SWEEP=1 forces it for every
bucket of width <= 8, so the reference's own corpus (golden matrices, sprand grid, ragged / empty
stripes) runs through it too.  Each segment still folds its entries in stored (reference) order --
B'x: a stripe's rows in row order; Bx: an output row's blocks in stripe order -- so the one-hot probes
are bit-exact; random x: tolerances of test_gpu_parity.py (1e-12 fp64, 1e-5 fp32).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.conftest import sprand_family
from tests.test_gpu_parity import METHODS_1D, TOL32, TOL64, dev, oracle_ref, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


@pytest.fixture(params=["8k", "16k", "16k-unpacked"])
def forced(request, monkeypatch):
    """Handles created inside the test use the swept layout for every B'x bucket of width <= 8, with
    8 KB or 16 KB of LDS accumulators per wave; keys packed (one 32-bit word: segment and the gather
    index's delta to the step's base) or, with VBC_SWEEP_PACK=0, the 32-bit index + 16-bit segment."""
    monkeypatch.setenv("VBC_SWEEP", "1")
    monkeypatch.setenv("VBC_SWEEP_TILE", "8" if request.param == "8k" else "16")
    monkeypatch.setenv("VBC_SWEEP_PACK", "0" if request.param.endswith("unpacked") else "1")
    return request.param


def sweep_bins(B, trans=True):
    return B.info(trans=trans)["sweep_bins"]


def one_hot_t(B, A):
    """Every e_i through mul!(y, B', x) and every e_j through mul!(y, B, x): the rows / columns of A,
    exactly (runtests.jl:29-53, 63-87)."""
    m, n = A.shape
    D = A.toarray()
    for trans, nin, nout, ref in ((True, m, n, D), (False, n, m, D.T)):
        E = torch.eye(nin, dtype=torch.float64, device=DEV)
        Y = torch.full((nin, nout), float("nan"), dtype=torch.float64, device=DEV)
        for i in range(nin):
            V.mul_(Y[i], V.adjoint(B) if trans else B, E[i])
        got = Y.cpu().numpy()
        assert np.array_equal(got, ref), (trans, np.argwhere(got != ref)[:5])


def test_forced_golden_one_hot(golden, forced):
    for key, g in golden.items():
        for meth in METHODS_1D:
            B = V.SparseMatrix1DVBC[4](g["A"], meth())
            one_hot_t(B, g["A"])
            assert sweep_bins(B) > 0 and sweep_bins(B, trans=False) > 0, key
        B = V.SparseMatrixVBC[4, 4](g["A"], V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)))
        one_hot_t(B, g["A"])


def test_forced_sprand_grid_one_hot(forced):
    for name, A in sprand_family(trials=1):
        one_hot_t(V.SparseMatrix1DVBC[4](A, METHODS_1D[1]()), A)


@pytest.mark.parametrize("widths", [[1], [2], [3], [4], [5, 6, 7, 8], [2, 9], [3, 17, 64]])
def test_forced_widths_tiles(forced, widths):
    """Every compile-time width, buckets mixing swept (w <= 8) and merged / slotted (w > 8) stripes,
    several tiles per bucket with a partial last tile, alpha / beta, both dtypes, both directions
    (forward with several buckets: beta scaling first, then one accumulating launch per bucket)."""
    rng = np.random.default_rng(sum(widths) + 11)
    L = 2600
    w = np.array([widths[i % len(widths)] for i in range(L)])
    B = V.synthetic.vbr_1dvbc(3000, L, 12000, w, W=max(64, w.max()), seed=int(w.sum()) + 3)
    for dtype, tol in ((np.float64, TOL64), (np.float32, TOL32)):
        Bd = B if dtype == np.float64 else V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs,
                                                               B.val.astype(np.float32))
        nsw = len([v for v in set(widths) if v <= 8])
        assert sweep_bins(Bd) == nsw and sweep_bins(Bd, trans=False) == nsw
        for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
            x = rng.uniform(-1, 1, nx).astype(dtype)
            y0 = rng.uniform(-1, 1, ny).astype(dtype)
            for alpha, beta in ((1.0, 0.0), (0.5, -1.5)):
                yd = dev(y0)
                V.mul_(yd, V.adjoint(Bd) if trans else Bd, dev(x), alpha, beta)
                yr = oracle_ref(B, x.astype(np.float64), y0.astype(np.float64), alpha, beta, trans)
                assert rel(yd.cpu().numpy(), yr) <= tol, (widths, dtype, trans, alpha, beta)


def test_forced_summation_order_bitwise(forced):
    """Integer-valued data whose partial sums exceed 2^53: only the reference's per-stripe row order
    reproduces the oracle bit for bit."""
    rng = np.random.default_rng(12)
    B = V.synthetic.vbr_1dvbc(5000, 700, 9000, 4, W=8, seed=99)
    B.val[:] = rng.integers(-2**20, 2**20, B.val.size).astype(np.float64)
    x = rng.integers(-2**33, 2**33, B.m).astype(np.float64)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert np.array_equal(y.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True))
    xf = rng.integers(-2**33, 2**33, B.n).astype(np.float64)
    y = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(xf))
    assert np.array_equal(y.cpu().numpy(), O.mul(R, xf, np.zeros(B.m), trans=False))


def test_forced_nonfinite_x_stays_in_place(forced):
    """Padding lanes are skipped: an Inf / NaN of x reaches exactly the stripes that store its row."""
    rng = np.random.default_rng(8)
    B = V.synthetic.vbr_1dvbc(300, 60, 700, np.arange(60) % 4 + 1, W=8, seed=77)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    x = rng.uniform(-1, 1, B.m)
    x[0] = np.nan
    x[17] = np.inf
    x[101] = -np.inf
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    got, ref = y.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert rel(got[fin], ref[fin]) <= TOL64
    xf = rng.uniform(-1, 1, B.n)
    xf[0] = np.nan
    xf[5] = np.inf
    y = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(xf))
    got, ref = y.cpu().numpy(), O.mul(R, xf, np.zeros(B.m), trans=False)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(np.isinf(got), np.isinf(ref))


def test_forced_edge_cases(forced):
    """Empty matrices, empty stripes (zeroed / beta-scaled), one 20000-row stripe in a tile of short ones."""
    for (m, n) in ((0, 0), (0, 5), (5, 0), (1, 1)):
        A = sp.csc_matrix((m, n))
        B = V.SparseMatrix1DVBC[4](A, V.EquiChunker(2))
        y = torch.full((n,), 7.0, dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, torch.ones(m, dtype=torch.float64, device=DEV))
        assert torch.all(y == 0)
    rng = np.random.default_rng(1)
    D = np.zeros((20000, 12))
    D[:, 3] = rng.random(20000)
    D[rng.integers(0, 20000, 50), 7] = 1.0
    A = sp.csc_matrix(D)
    for meth in (V.EquiChunker(1), V.EquiChunker(4), V.StrictChunker(8)):
        B = V.SparseMatrix1DVBC[8](A, meth)
        assert sweep_bins(B) > 0
        x = rng.uniform(-1, 1, 20000)
        for beta in (0.0, 2.0):
            y0 = rng.uniform(-1, 1, 12)
            y = dev(y0)
            V.mul_(y, B.T, dev(x), 1.0, beta)
            assert rel(y.cpu().numpy(), D.T @ x + beta * y0) <= TOL64
            xf = rng.uniform(-1, 1, 12)
            y0 = rng.uniform(-1, 1, 20000)
            y = dev(y0)
            V.mul_(y, B, dev(xf), 1.0, beta)
            assert rel(y.cpu().numpy(), D @ xf + beta * y0) <= TOL64


def test_forced_trspmv_and_multi_rhs(golden, forced):
    """TrSpMV! on CSC (w = 1 buckets) and the per-column multi-RHS path over a swept handle."""
    for key, g in golden.items():
        A = g["A"]
        y = torch.full((A.shape[1],), float("nan"), dtype=torch.float64, device=DEV)
        V.TrSpMV_(y, A, dev(g["xt"]))
        assert rel(y.cpu().numpy(), O.trspmv(A, g["xt"], np.zeros(A.shape[1]))) <= TOL64, key
    rng = np.random.default_rng(4)
    B = V.synthetic.vbr_1dvbc(800, 300, 2500, 4, W=8, seed=5)
    X = rng.uniform(-1, 1, (B.m, 5))
    Y = torch.zeros((B.n, 5), dtype=torch.float64, device=DEV)
    V.mul_(Y, B.T, dev(X))
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    ref = np.stack([O.mul(R, X[:, j], np.zeros(B.n), trans=True) for j in range(5)], axis=1)
    assert rel(Y.cpu().numpy(), ref) <= TOL64


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_auto_uniform_rows_use_sweep(dtype):
    """Auto mode: the uniform-row generator at an x beyond L2 (m = 4e6) is laid out swept; the FE
    mesh operator of a similar size is not.  Parity against the oracle on the swept one."""
    B = V.synthetic.north_star(dtype=dtype, scale=0.4)
    assert sweep_bins(B) == 1 and sweep_bins(B, trans=False) == 1
    rng = np.random.default_rng(0xC0FFEE)
    x = rng.uniform(-1, 1, B.m).astype(dtype)
    y = torch.zeros(B.n, dtype=torch.from_numpy(x).dtype, device=DEV)
    V.mul_(y, B.T, dev(x))
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    yr = O.mul(R, x.astype(np.float64), np.zeros(B.n), trans=True)
    assert rel(y.cpu().numpy(), yr) <= (TOL64 if dtype == np.float64 else TOL32)
    xf = rng.uniform(-1, 1, B.n).astype(dtype)
    y = torch.zeros(B.m, dtype=torch.from_numpy(xf).dtype, device=DEV)
    V.mul_(y, B, dev(xf))
    yr = O.mul(R, xf.astype(np.float64), np.zeros(B.m), trans=False)
    assert rel(y.cpu().numpy(), yr) <= (TOL64 if dtype == np.float64 else TOL32)
    F = V.synthetic.fe_grid_2d(1000, dof=2, dtype=dtype)
    assert sweep_bins(F) == 0 and sweep_bins(F, trans=False) == 0


def test_packed_keys_bytes_and_fallback(monkeypatch):
    """Packed swept keys move 4 instead of 6 index bytes per entry (bytes_t) with the same y bit for bit;
    a step whose gather indices span more than the delta field (2^21 rows at 1024 segments per tile)
    keeps the unpacked form, and both forms match the oracle."""
    monkeypatch.setenv("VBC_SWEEP", "1")
    rng = np.random.default_rng(11)

    def build(pack, A):
        monkeypatch.setenv("VBC_SWEEP_PACK", pack)
        B = V.SparseMatrix1DVBC[8](A, V.EquiChunker(1))
        B.info(trans=True)  # the handle (and its layout) is made now, under this setting
        return B

    def run(B, x):
        y = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, dev(x))
        return y.cpu().numpy()

    # dense enough: every step's 64 rows lie within a few thousand rows
    A = sp.random(200000, 4096, density=2e-3, format="csc", random_state=3, dtype=np.float64)
    Bp, Bu = build("1", A), build("0", A)
    assert sweep_bins(Bp) == 1 and sweep_bins(Bu) == 1
    assert Bp.info(trans=True)["bytes_t"] < Bu.info(trans=True)["bytes_t"]
    x = rng.uniform(-1, 1, A.shape[0])
    yp, yu = run(Bp, x), run(Bu, x)
    assert np.array_equal(yp, yu)
    R = O.Ref1DVBC(Bp.m, Bp.n, Bp.W, Bp.Phi.spl, Bp.pos, Bp.idx, Bp.ofs, Bp.val)
    assert np.array_equal(yp, O.mul(R, x, np.zeros(Bp.n), trans=True))
    # sparse: 64 one-row stripes spread over 5e6 rows -- one step spans more than 2^21 rows
    m = 5_000_000
    rows = np.sort(rng.choice(m, 64, replace=False))
    A2 = sp.csc_matrix((rng.uniform(-1, 1, 64), (rows, np.arange(0, 1024, 16))), shape=(m, 1024))
    Bp2, Bu2 = build("1", A2), build("0", A2)
    assert Bp2.info(trans=True)["bytes_t"] == Bu2.info(trans=True)["bytes_t"]  # fell back
    x2 = rng.uniform(-1, 1, m)
    y2 = run(Bp2, x2)
    R2 = O.Ref1DVBC(Bp2.m, Bp2.n, Bp2.W, Bp2.Phi.spl, Bp2.pos, Bp2.idx, Bp2.ofs, Bp2.val)
    assert np.array_equal(y2, O.mul(R2, x2, np.zeros(Bp2.n), trans=True))
