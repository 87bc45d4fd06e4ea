"""GPU parity of the slotted-segment layout (csrc/vbc_slots.h) against the oracle.

The library picks the slotted layout per width bucket when segment lengths are near-uniform
(mesh operators); VBC_SLOTS=1 forces it for every representable bucket, so the reference's own
corpus (golden matrices, sprand grid, ragged/empty stripes, w up to 64) runs through it too.
Tolerances as in test_gpu_parity.py: one-hot probes bit-exact, random x <= 1e-12 (fp64) / 1e-5 (fp32).
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.conftest import sprand_family
from tests.test_gpu_parity import METHODS_1D, METHODS_2D, TOL32, TOL64, dev, one_hot_probes, oracle_ref, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


@pytest.fixture
def forced(monkeypatch):
    """Handles created inside the test use the slotted layout wherever it is representable."""
    monkeypatch.setenv("VBC_SLOTS", "1")
    yield
    monkeypatch.delenv("VBC_SLOTS", raising=False)


def slot_bins(B, trans=True):
    return B.info(trans=trans)["slot_bins"]


def test_forced_golden_one_hot(golden, forced, order):
    for key, g in golden.items():
        for meth in METHODS_1D:
            B = V.SparseMatrix1DVBC[4](g["A"], meth())
            one_hot_probes(B, g["A"])
            assert slot_bins(B) > 0 and slot_bins(B, trans=False) > 0, key
        for meth in METHODS_2D:
            one_hot_probes(V.SparseMatrixVBC[4, 4](g["A"], meth()), g["A"])


def test_forced_golden_one_hot_full_keys(golden, forced, monkeypatch):
    """The 32-bit key form of the slotted layout (compression off) under the one-hot protocol."""
    monkeypatch.setenv("VBC_SLOT_KEYS16", "0")
    for key, g in golden.items():
        one_hot_probes(V.SparseMatrix1DVBC[4](g["A"], METHODS_1D[1]()), g["A"])


@pytest.mark.parametrize("dedup", ["0", "1"])
def test_shared_delta_patterns(monkeypatch, dedup):
    """Compressed rows with identical delta patterns are stored once (VBC_SLOT_DEDUP=1, the default):
    the FE operator's interior chunks share one pattern, its boundary chunks keep their own; results
    are identical with and without sharing."""
    monkeypatch.setenv("VBC_SLOT_DEDUP", dedup)
    B = V.synthetic.fe_grid_2d(200, dof=2)
    assert slot_bins(B) == 1
    rng = np.random.default_rng(17)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
        x = rng.uniform(-1, 1, nx)
        yd = torch.zeros(ny, dtype=torch.float64, device=DEV)
        V.mul_(yd, V.adjoint(B) if trans else B, dev(x))
        assert rel(yd.cpu().numpy(), O.mul(R, x, np.zeros(ny), trans=trans)) <= TOL64, trans
    shared = B.info(trans=True)["bytes_t"]
    monkeypatch.setenv("VBC_SLOT_DEDUP", "0" if dedup == "1" else "1")
    C = V.synthetic.fe_grid_2d(200, dof=2)
    other = C.info(trans=True)["bytes_t"]
    assert (shared < other) if dedup == "1" else (shared > other)


def test_fe_nonfinite_and_unaligned_x():
    """The production FE layout (slotted, shared delta patterns): Inf / NaN of x stay where the
    reference puts them, and an x view that is only 8-B aligned gives the same bits."""
    B = V.synthetic.fe_grid_2d(120, dof=2)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(23)
    x = rng.uniform(-1, 1, B.m)
    x[[0, 7, 501, B.m - 1]] = [np.nan, np.inf, -np.inf, np.nan]
    ref = O.mul(R, x, np.zeros(B.n), trans=True)
    for off in (0, 1):
        buf = torch.zeros(B.m + 1, dtype=torch.float64, device=DEV)
        buf[off:off + B.m] = dev(x)
        y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, buf[off:off + B.m])
        got = y.cpu().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isinf(got), np.isinf(ref)), off
        fin = np.isfinite(ref)
        assert np.array_equal(got[fin], ref[fin]), off


def test_keys16_falls_back_on_wide_deltas(monkeypatch):
    """Rows whose keys span more than int16 keep 32-bit keys (and stay exact)."""
    monkeypatch.setenv("VBC_SLOTS", "1")
    monkeypatch.setenv("VBC_SLOT_KEYS16", "2")
    rng = np.random.default_rng(5)
    m, n = 200000, 64
    D = sp.random(m, n, density=4e-5, random_state=5, format="csc")
    B = V.SparseMatrix1DVBC[1](D, V.EquiChunker(1))
    x = rng.uniform(-1, 1, m)
    y = torch.zeros(n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert rel(y.cpu().numpy(), D.T @ x) <= TOL64


def test_forced_sprand_grid_one_hot(forced):
    for name, A in sprand_family(trials=1):
        one_hot_probes(V.SparseMatrix1DVBC[4](A, METHODS_1D[1]()), A)


@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (2.5, 0.0), (1.0, 1.0), (-0.5, 2.0)])
def test_forced_random_alpha_beta(golden, forced, order, alpha, beta):
    rng = np.random.default_rng(21)
    for key, g in golden.items():
        A = g["A"]
        m, n = A.shape
        for B in (V.SparseMatrix1DVBC[8](A, V.DynamicTotalChunker(V.model_SparseMatrix1DVBC_memory(), 8)),
                  V.SparseMatrixVBC[3, 5](A, V.AlternatingPacker(V.EquiChunker(5), V.EquiChunker(3)))):
            for trans, nx, ny in ((False, n, m), (True, m, n)):
                x = rng.uniform(-1, 1, nx)
                y0 = rng.uniform(-1, 1, ny)
                yd = dev(y0)
                V.mul_(yd, V.adjoint(B) if trans else B, dev(x), alpha, beta)
                yr = oracle_ref(B, x, y0.copy(), alpha, beta, trans)
                assert rel(yd.cpu().numpy(), yr) <= TOL64, (key, trans)
        B = V.SparseMatrix1DVBC[4](A, V.OverlapChunker(0.9, 4))
        for trans, nx, ny in ((False, n, m), (True, m, n)):
            x, y0 = rng.uniform(-1, 1, nx), rng.uniform(-1, 1, ny)
            yd = dev(y0)
            V.mul_(yd, V.adjoint(B) if trans else B, dev(x), alpha, beta, quirks=True)
            assert rel(yd.cpu().numpy(), oracle_ref(B, x, y0.copy(), alpha, beta, trans, quirks=True)) <= TOL64


@pytest.fixture(params=["natural", "sorted"])
def order(request, monkeypatch):
    """Slotted segment order: natural (affine y map where possible) or sorted by length (y offsets
    from the table, staged in LDS per range)."""
    monkeypatch.setenv("VBC_SLOTS_SORT", "2" if request.param == "sorted" else "0")
    return request.param


@pytest.mark.parametrize("widths", [[1], [2], [3], [4], [2, 3], [5, 6, 7, 8], [9, 12, 16], [17, 31, 33, 64]])
def test_forced_widths(forced, order, widths):
    """Every width variant of the slotted kernel (compile-time 1..8, runtime w > 8), both dtypes,
    several buckets (non-affine segment maps, multi-bucket forward accumulation)."""
    rng = np.random.default_rng(sum(widths) + 5)
    L = 70
    w = np.array([widths[i % len(widths)] for i in range(L)])
    B = V.synthetic.vbr_1dvbc(400, L, 1400, w, W=max(64, w.max()), seed=int(w.sum()) + 1)
    for dtype, tol in ((np.float64, TOL64), (np.float32, TOL32)):
        Bd = B if dtype == np.float64 else V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs,
                                                               B.val.astype(np.float32))
        for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
            x = rng.uniform(-1, 1, nx).astype(dtype)
            y0 = rng.uniform(-1, 1, ny).astype(dtype)
            for alpha, beta in ((1.0, 0.0), (0.5, -1.5)):
                yd = dev(y0)
                V.mul_(yd, V.adjoint(Bd) if trans else Bd, dev(x), alpha, beta)
                yr = oracle_ref(B, x.astype(np.float64), y0.astype(np.float64), alpha, beta, trans)
                assert rel(yd.cpu().numpy(), yr) <= tol, (widths, trans, dtype, alpha, beta)


def test_forced_nonfinite_x_stays_in_place(forced):
    """Padding rows take x as 0: an Inf / NaN of x reaches exactly the outputs whose segments store
    that row, as in the reference's per-stripe loop (multiply_1DVBC.jl:101-104)."""
    rng = np.random.default_rng(8)
    B = V.synthetic.vbr_1dvbc(300, 60, 700, np.arange(60) % 4 + 1, W=8, seed=77)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    x = rng.uniform(-1, 1, B.m)
    x[0] = np.nan          # padding rows gather x[0]
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


def test_forced_edge_cases(forced, order):
    """Empty matrices, empty stripes, one 20000-row stripe in a chunk of short ones."""
    for (m, n) in ((0, 0), (0, 5), (5, 0), (1, 1)):
        A = sp.csc_matrix((m, n))
        B = V.SparseMatrix1DVBC[4](A, V.EquiChunker(2))
        y = torch.full((n,), 7.0, dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, torch.ones(m, dtype=torch.float64, device=DEV))
        assert torch.all(y == 0)
        y = torch.full((m,), 7.0, dtype=torch.float64, device=DEV)
        V.mul_(y, B, torch.ones(n, dtype=torch.float64, device=DEV))
        assert torch.all(y == 0)
    rng = np.random.default_rng(1)
    D = np.zeros((20000, 12))
    D[:, 3] = rng.random(20000)
    D[rng.integers(0, 20000, 50), 7] = 1.0
    A = sp.csc_matrix(D)
    for meth in (V.EquiChunker(1), V.EquiChunker(4), V.StrictChunker(8)):
        B = V.SparseMatrix1DVBC[8](A, meth)
        x = rng.uniform(-1, 1, 20000)
        for beta in (0.0, 2.0):
            y0 = rng.uniform(-1, 1, 12)
            y = dev(y0)
            V.mul_(y, B.T, dev(x), 1.0, beta)
            assert rel(y.cpu().numpy(), D.T @ x + beta * y0) <= TOL64
        xf = rng.uniform(-1, 1, 12)
        y = torch.zeros(20000, dtype=torch.float64, device=DEV)
        V.mul_(y, B, dev(xf))
        assert rel(y.cpu().numpy(), D @ xf) <= TOL64


def test_forced_integer_exact(forced):
    rng = np.random.default_rng(9)
    D = np.where(rng.random((300, 200)) < 0.1, rng.integers(-1000, 1000, (300, 200)), 0).astype(np.float64)
    A = sp.csc_matrix(D)
    B = V.SparseMatrix1DVBC[8](A, V.DynamicTotalChunker(V.model_SparseMatrix1DVBC_memory(), 8))
    x = rng.integers(-100, 100, 300).astype(np.float64)
    y = torch.zeros(200, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert np.array_equal(y.cpu().numpy(), D.T @ x)
    xf = rng.integers(-100, 100, 200).astype(np.float64)
    y = torch.zeros(300, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(xf))
    assert np.array_equal(y.cpu().numpy(), D @ xf)


def test_forced_trspmv(golden, forced):
    for key, g in golden.items():
        A = g["A"]
        y = torch.full((A.shape[1],), float("nan"), dtype=torch.float64, device=DEV)
        V.TrSpMV_(y, A, dev(g["xt"]))
        assert rel(y.cpu().numpy(), O.trspmv(A, g["xt"], np.zeros(A.shape[1]))) <= TOL64, key


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_auto_fe_grid_uses_slots(dtype):
    """Auto mode: the FE operator (uniform 10-row stripes, 5-block rows) is laid out slotted in both
    directions, and matches the oracle."""
    B = V.synthetic.fe_grid_2d(150, dof=2, dtype=dtype)
    assert slot_bins(B) == 1 and slot_bins(B, trans=False) == 1
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    rng = np.random.default_rng(3)
    tol = TOL64 if dtype == np.float64 else TOL32
    for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
        x = rng.uniform(-1, 1, nx).astype(dtype)
        yd = torch.zeros(ny, dtype=torch.from_numpy(x).dtype, device=DEV)
        V.mul_(yd, V.adjoint(B) if trans else B, dev(x))
        yr = O.mul(R, x.astype(np.float64), np.zeros(ny), trans=trans)
        assert rel(yd.cpu().numpy(), yr) <= tol, trans


def test_auto_sorted_slots_for_standin():
    """A SuiteSparse-like stand-in (3D stiffness, ragged stripe lengths) is laid out slotted in sorted
    order in auto mode (padding ~1 %) and matches the oracle in both directions and both dtypes."""
    A = V.synthetic.fe_stiffness_3d(3000, 150000, 3, seed=4)
    B = V.SparseMatrix1DVBC[8](A, V.StrictChunker(8))
    assert slot_bins(B) == 1
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(6)
    for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
        x = rng.uniform(-1, 1, nx)
        y0 = rng.uniform(-1, 1, ny)
        for alpha, beta in ((1.0, 0.0), (2.0, -0.5)):
            yd = dev(y0)
            V.mul_(yd, V.adjoint(B) if trans else B, dev(x), alpha, beta)
            assert rel(yd.cpu().numpy(), O.mul(R, x, y0.copy(), alpha, beta, trans=trans, ref_semantics=False)) <= TOL64, trans
    C = V.SparseMatrixCSC(A.astype(np.float32))
    y = torch.zeros(A.shape[1], dtype=torch.float32, device=DEV)
    xs = rng.uniform(-1, 1, A.shape[0]).astype(np.float32)
    V.TrSpMV_(y, C, dev(xs))
    assert rel(y.cpu().numpy(), A.T @ xs.astype(np.float64)) <= TOL32


def test_auto_ns_sorted_slots_vs_oracle():
    """Uniform-random rows (Poisson stripe lengths, costs.jl:63-83): auto mode sorts the stripes by
    length inside windows (padding ~3 %), y offsets come from the table; parity both directions."""
    B = V.synthetic.north_star(scale=0.01)
    assert slot_bins(B) == 1
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(0xC0FFEE)
    for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
        x = rng.uniform(-1, 1, nx)
        yd = torch.zeros(ny, dtype=torch.float64, device=DEV)
        V.mul_(yd, V.adjoint(B) if trans else B, dev(x))
        assert rel(yd.cpu().numpy(), O.mul(R, x, np.zeros(ny), trans=trans)) <= TOL64, trans


def test_slots_deterministic_and_matches_merge(monkeypatch):
    """Same matrix, slotted vs merged layout: both within tolerance of each other; slotted runs are
    bitwise reproducible."""
    B1 = V.synthetic.fe_grid_2d(120, dof=2)
    monkeypatch.setenv("VBC_SLOTS", "0")
    B0 = V.synthetic.fe_grid_2d(120, dof=2)
    assert slot_bins(B0) == 0
    monkeypatch.delenv("VBC_SLOTS")
    assert slot_bins(B1) == 1
    x = torch.rand(B1.m, dtype=torch.float64, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    ya, yb, y0 = (torch.empty(B1.n, dtype=torch.float64, device=DEV) for _ in range(3))
    V.mul_(ya, B1.T, x)
    V.mul_(yb, B1.T, x)
    V.mul_(y0, B0.T, x)
    assert torch.equal(ya, yb)
    assert (torch.linalg.norm(ya - y0) / torch.linalg.norm(y0)).item() <= 1e-14


@pytest.mark.parametrize("keys16", ["0", "2"])
@pytest.mark.parametrize("stage", ["0", "8"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_staged_writes(monkeypatch, stage, dtype, keys16):
    """LDS-staged y writes (VBC_SLOT_STAGE) and both key forms (32-bit keys / per-row base + int16
    deltas): single-width matrices of every width (contiguous chunk outputs), a partial last chunk,
    and a y that is not 16-B aligned (element-wise write path)."""
    monkeypatch.setenv("VBC_SLOTS", "1")
    monkeypatch.setenv("VBC_SLOT_STAGE", stage)
    monkeypatch.setenv("VBC_SLOT_KEYS16", keys16)
    tol = TOL64 if dtype == np.float64 else TOL32
    rng = np.random.default_rng(int(stage) + np.dtype(dtype).itemsize)
    cases = [V.synthetic.fe_grid_2d(37, dof=2, dtype=dtype)]
    for w in (1, 2, 3, 4, 8, 12):
        L = 1000 // w + 3
        Bw = V.synthetic.vbr_1dvbc(900, L, 6 * L, w, W=16, seed=w)
        cases.append(V.SparseMatrix1DVBC(Bw.W, Bw.m, Bw.n, Bw.Phi, Bw.pos, Bw.idx, Bw.ofs, Bw.val.astype(dtype)))
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    for B in cases:
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
        for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
            x = rng.uniform(-1, 1, nx).astype(dtype)
            yr = O.mul(R, x.astype(np.float64), np.zeros(ny), trans=trans)
            for off in (0, 1):
                buf = torch.full((ny + 1,), float("nan"), dtype=tdt, device=DEV)
                yd = buf[off:off + ny]
                V.mul_(yd, V.adjoint(B) if trans else B, dev(x))
                assert rel(yd.cpu().numpy(), yr) <= tol, (B.n, trans, off)
                if off == 1:
                    assert torch.isnan(buf[0])  # nothing written outside y
                else:
                    assert torch.isnan(buf[ny])
