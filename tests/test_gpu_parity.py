"""GPU parity: libvbc's HIP kernels (through the C ABI, via the Python mirror) against the oracle.

Tolerances (stated per BASELINE.md §2): one-hot probes are bit-exact (the reference's own protocol,
runtests.jl:29-53, `==`); random x: normwise relative error <= 1e-12 in fp64 (BASELINE target 1e-10)
and <= 1e-5 in fp32 against the fp64 product.  Integer-valued inputs with small integer x are exact.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.conftest import sprand_family

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"

TOL64, TOL32 = 1e-12, 1e-5

METHODS_1D = [
    lambda: V.StrictChunker(4),
    lambda: V.OverlapChunker(0.9, 4),
    lambda: V.DynamicTotalChunker(V.ConstrainedCost(V.model_SparseMatrix1DVBC_blocks(), V.VertexCount(), 4)),
    lambda: V.DynamicTotalChunker(V.ConstrainedCost(V.model_SparseMatrix1DVBC_memory(np.float64, np.int64), V.VertexCount(), 4)),
]
METHODS_2D = [
    lambda: V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)),
    lambda: V.AlternatingPacker(V.OverlapChunker(0.9, 4), V.OverlapChunker(0.9, 4)),
]


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    d = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (d if d else 1.0)


def one_hot_probes(B, A, dtype=np.float64):
    """Every e_j through mul!(y, B, x) and every e_i through mul!(y, B', x); results must equal the
    columns / rows of A exactly (runtests.jl:29-53)."""
    m, n = A.shape
    D = A.toarray().astype(dtype)
    for trans, nin, nout, ref in ((False, n, m, D.T), (True, m, n, D)):
        E = torch.eye(nin, dtype=torch.from_numpy(np.zeros(0, dtype)).dtype, device=DEV) if nin else None
        Y = torch.full((nin, nout), float("nan"), dtype=E.dtype if E is not None else torch.float64, device=DEV)
        op = V.adjoint(B) if trans else B
        for j in range(nin):
            V.mul_(Y[j], op, E[j], True, False)
        got = Y.cpu().numpy()
        assert np.array_equal(got, ref), ("trans" if trans else "fwd", np.argwhere(got != ref)[:5])


def test_golden_one_hot_1dvbc(golden):
    for key, g in golden.items():
        for meth in METHODS_1D:
            B = V.SparseMatrix1DVBC[4](g["A"], meth())
            one_hot_probes(B, g["A"])


def test_golden_one_hot_vbc(golden):
    for key, g in golden.items():
        for meth in METHODS_2D:
            B = V.SparseMatrixVBC[4, 4](g["A"], meth())
            one_hot_probes(B, g["A"])


def test_sprand_grid_one_hot():
    for name, A in sprand_family(trials=1):
        for meth in (METHODS_1D[0], METHODS_1D[1], METHODS_1D[3]):
            one_hot_probes(V.SparseMatrix1DVBC[4](A, meth()), A)
        one_hot_probes(V.SparseMatrixVBC[4, 4](A, METHODS_2D[1]()), A)


def oracle_ref(B, x, y, alpha, beta, trans, quirks=False):
    if isinstance(B, V.SparseMatrixVBC):
        R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    else:
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    return O.mul(R, x, y, alpha, beta, trans=trans, ref_semantics=quirks)


@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (2.5, 0.0), (1.0, 1.0), (-0.5, 2.0)])
def test_golden_random_vs_oracle(golden, alpha, beta):
    rng = np.random.default_rng(11)
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
        # the committed scipy products (tests/golden) directly
        B = V.SparseMatrix1DVBC[4](A, V.StrictChunker(4))
        yd = torch.zeros(m, dtype=torch.float64, device=DEV)
        V.mul_(yd, B, dev(g["xf"]))
        assert rel(yd.cpu().numpy(), g["yf"]) <= TOL64
        yd = torch.zeros(n, dtype=torch.float64, device=DEV)
        V.mul_(yd, B.T, dev(g["xt"]))
        assert rel(yd.cpu().numpy(), g["yt"]) <= TOL64


def test_reference_quirks_bitwise_semantics(golden):
    A = golden["LPnetlib__lp_etamacro"]["A"]
    m, n = A.shape
    B = V.SparseMatrix1DVBC[4](A, V.OverlapChunker(0.9, 4))
    rng = np.random.default_rng(3)
    for trans, nx, ny in ((False, n, m), (True, m, n)):
        x, y0 = rng.uniform(-1, 1, nx), rng.uniform(-1, 1, ny)
        yd = dev(y0)
        V.mul_(yd, V.adjoint(B) if trans else B, dev(x), 2.0, 3.0, quirks=True)
        yr = oracle_ref(B, x, y0.copy(), 2.0, 3.0, trans, quirks=True)
        assert rel(yd.cpu().numpy(), yr) <= TOL64


def test_fp32(golden):
    for key, g in golden.items():
        A = g["A"]
        B = V.SparseMatrix1DVBC[8](A, V.OverlapChunker(0.5, 8), dtype=np.float32)
        one_hot_probes(B, A, np.float32)
        yd = torch.zeros(A.shape[1], dtype=torch.float32, device=DEV)
        V.mul_(yd, B.T, dev(g["xt"].astype(np.float32)))
        assert rel(yd.cpu().numpy(), g["yt"]) <= TOL32, key
        yd = torch.zeros(A.shape[0], dtype=torch.float32, device=DEV)
        V.mul_(yd, B, dev(g["xf"].astype(np.float32)))
        assert rel(yd.cpu().numpy(), g["yf"]) <= TOL32, key


def test_host_memory_path(golden):
    g = golden["HB__west0132"]
    B = V.SparseMatrix1DVBC[4](g["A"], V.EquiChunker(3))
    y = np.zeros(g["A"].shape[1])
    V.mul_(y, B.T, g["xt"])
    assert rel(y, g["yt"]) <= TOL64
    y = np.zeros(g["A"].shape[0])
    V.mul_(y, B, g["xf"])
    assert rel(y, g["yf"]) <= TOL64


def test_trspmv(golden):
    for key, g in golden.items():
        A = g["A"]
        y = torch.full((A.shape[1],), float("nan"), dtype=torch.float64, device=DEV)
        V.TrSpMV_(y, A, dev(g["xt"]))
        yr = O.trspmv(A, g["xt"], np.zeros(A.shape[1]))
        assert rel(y.cpu().numpy(), yr) <= TOL64, key


@pytest.mark.parametrize("widths", [[1], [2, 3], [5, 6, 7, 8], [9, 12, 16], [17, 31, 33, 64]])
def test_widths_and_generic_path(widths):
    """Every width bucket, including the runtime-width variant (w > 8) up to the 64 limit."""
    rng = np.random.default_rng(sum(widths))
    L = 40
    w = np.array([widths[i % len(widths)] for i in range(L)])
    B = V.synthetic.vbr_1dvbc(300, L, 900, w, W=max(64, w.max()), seed=int(w.sum()))
    for dtype, tol in ((np.float64, TOL64), (np.float32, TOL32)):
        Bd = B if dtype == np.float64 else V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs,
                                                               B.val.astype(np.float32))
        for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
            x = rng.uniform(-1, 1, nx).astype(dtype)
            yd = torch.zeros(ny, dtype=torch.from_numpy(x).dtype, device=DEV)
            V.mul_(yd, V.adjoint(Bd) if trans else Bd, dev(x))
            yr = oracle_ref(B, x.astype(np.float64), np.zeros(ny), 1.0, 0.0, trans)
            assert rel(yd.cpu().numpy(), yr) <= tol, (widths, trans, dtype)


def test_edge_cases():
    # empty matrices / empty stripes / long stripes (G = 64 loop) / one dense column
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
    D[:, 3] = rng.random(20000)                      # one dense column: 20000 rows in one stripe
    D[rng.integers(0, 20000, 50), 7] = 1.0           # sparse neighbours, empty stripes elsewhere
    A = sp.csc_matrix(D)
    for meth in (V.EquiChunker(1), V.EquiChunker(4), V.StrictChunker(8)):
        B = V.SparseMatrix1DVBC[8](A, meth)
        x = rng.uniform(-1, 1, 20000)
        y = torch.zeros(12, dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, dev(x))
        assert rel(y.cpu().numpy(), D.T @ x) <= TOL64
        xf = rng.uniform(-1, 1, 12)
        y = torch.zeros(20000, dtype=torch.float64, device=DEV)
        V.mul_(y, B, dev(xf))
        assert rel(y.cpu().numpy(), D @ xf) <= TOL64
    with pytest.raises(V.DimensionMismatch):
        V.mul_(torch.zeros(11, dtype=torch.float64, device=DEV), B.T, dev(x))
    # eltype(y) = Float32 with a Float64 matrix computes in Float32 (multiply_1DVBC.jl:102 converts)
    y32 = torch.zeros(12, dtype=torch.float32, device=DEV)
    V.mul_(y32, B.T, dev(x))
    assert rel(y32.cpu().numpy().astype(np.float64), D.T @ x) <= 1e-5
    with pytest.raises(V.UnsupportedDtype):    # no GPU product into a Float16 y
        V.mul_(torch.zeros(12, dtype=torch.float16, device=DEV), B.T, dev(x))


def test_integer_valued_exact():
    """Int32-valued matrices (runtests.jl:16) with small-integer x: every partial sum is an exact
    integer < 2^53, so GPU == oracle bit for bit in fp64 regardless of summation order."""
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


def test_multi_rhs_columnwise(golden):
    A = golden["LPnetlib__lp_blend"]["A"]
    m, n = A.shape
    B = V.SparseMatrix1DVBC[4](A, V.StrictChunker(4))
    rng = np.random.default_rng(4)
    X = np.asfortranarray(rng.uniform(-1, 1, (m, 16)))
    Y = np.asfortranarray(np.zeros((n, 16)))
    V.mul_(Y, B.T, X)
    R = O.Ref1DVBC(m, n, 4, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    Yr = O.mulmat_t(R, X, np.asfortranarray(np.zeros((n, 16))))
    assert rel(Y, Yr) <= TOL64
    Xd = torch.from_numpy(np.ascontiguousarray(X.T)).to(DEV).T   # column-major view
    Yd = torch.zeros((16, n), dtype=torch.float64, device=DEV).T
    V.mul_(Yd, B.T, Xd)
    assert rel(Yd.cpu().numpy(), Yr) <= TOL64


def test_synthetic_medium_vs_oracle():
    """costs.jl:63-83 generator at 1e6 x 1e6 (mixed widths): GPU vs oracle, both directions."""
    B = V.synthetic.north_star(scale=0.1, mixed=True)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(0xC0FFEE)
    for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
        x = rng.uniform(-1, 1, nx)
        yd = torch.zeros(ny, dtype=torch.float64, device=DEV)
        V.mul_(yd, V.adjoint(B) if trans else B, dev(x))
        yr = O.mul(R, x, np.zeros(ny), trans=trans, nthreads=8)
        assert rel(yd.cpu().numpy(), yr) <= TOL64


@pytest.mark.slow
def test_north_star_size_independent_properties():
    """At the benchmark's full size (1e7 x 1e7, 1e8 nnz), properties that need no CPU product:
    (1) 1ᵀ(B'x) = (B·1)ᵀx (transposed kernel vs forward kernel, checksum of checksums);
    (2) linearity B'(x1 + 2 x2) = B'x1 + 2 B'x2;  (3) determinism: two runs are bitwise equal."""
    B = V.synthetic.north_star()
    g = torch.Generator(device=DEV).manual_seed(0xC0FFEE)
    x1 = torch.rand(B.m, dtype=torch.float64, device=DEV, generator=g) * 2 - 1
    x2 = torch.rand(B.m, dtype=torch.float64, device=DEV, generator=g) * 2 - 1
    y1 = torch.empty(B.n, dtype=torch.float64, device=DEV)
    y2 = torch.empty_like(y1)
    y3 = torch.empty_like(y1)
    V.mul_(y1, B.T, x1)
    V.mul_(y2, B.T, x2)
    V.mul_(y3, B.T, x1 + 2 * x2)
    assert (torch.linalg.norm(y3 - (y1 + 2 * y2)) / torch.linalg.norm(y3)).item() <= 1e-13
    y1b = torch.empty_like(y1)
    V.mul_(y1b, B.T, x1)
    assert torch.equal(y1, y1b)
    ones = torch.ones(B.n, dtype=torch.float64, device=DEV)
    r = torch.empty(B.m, dtype=torch.float64, device=DEV)
    V.mul_(r, B, ones)
    lhs, rhs = y1.sum().item(), torch.dot(r, x1).item()
    assert abs(lhs - rhs) <= 1e-9 * torch.linalg.norm(r).item() * torch.linalg.norm(x1).item()


@pytest.mark.parametrize("nrhs", [2, 3, 16, 17, 40, 70])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_multi_rhs_rowmajor(nrhs, dtype):
    """Fused multi-RHS kernel (row-major X / Y) vs the oracle applied column by column, with
    alpha/beta, mixed widths 1..8 (fused) and a w > 8 bucket (per-column fallback), both directions."""
    tol = TOL64 if dtype == np.float64 else TOL32
    rng = np.random.default_rng(nrhs)
    for widths in ([1, 2, 3, 4, 5, 6, 7, 8], [4], [2, 12]):
        L = 48
        w = np.array([widths[i % len(widths)] for i in range(L)])
        B = V.synthetic.vbr_1dvbc(700, L, 1500, w, W=16, seed=nrhs + int(w.sum()))
        if dtype == np.float32:
            B = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val.astype(np.float32))
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
        for trans, nx, ny in ((True, B.m, B.n), (False, B.n, B.m)):
            X = rng.uniform(-1, 1, (nx, nrhs)).astype(dtype)
            Y0 = rng.uniform(-1, 1, (ny, nrhs)).astype(dtype)
            Yd = dev(Y0)
            V.mul_(Yd, V.adjoint(B) if trans else B, dev(X), 1.5, 0.5)
            ref = np.stack([O.mul(R, X[:, j].astype(np.float64), Y0[:, j].astype(np.float64), 1.5, 0.5,
                                  trans=trans, ref_semantics=False) for j in range(nrhs)], axis=1)
            assert rel(Yd.cpu().numpy(), ref) <= tol, (widths, trans, nrhs)


def test_multi_rhs_vbc2d_golden(golden):
    """2D VBC, 16 right-hand sides (config C5 shape), one-hot identity blocks: exact."""
    for key, g in golden.items():
        A = g["A"]
        m, n = A.shape
        B = V.SparseMatrixVBC[4, 4](A, V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)))
        D = A.toarray()
        for j0 in range(0, m, 16):
            k = min(16, m - j0)
            X = np.zeros((m, k))
            X[np.arange(j0, j0 + k), np.arange(k)] = 1.0
            Y = torch.zeros((n, k), dtype=torch.float64, device=DEV)
            V.mul_(Y, B.T, dev(X))
            assert np.array_equal(Y.cpu().numpy(), D[j0:j0 + k, :].T), key
