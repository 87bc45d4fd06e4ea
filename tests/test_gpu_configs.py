"""BASELINE.json configs on the GPU against the CPU oracle, at their own sizes.

  C1  sprand(10_000, 10_000, 1e-3) Float64 (runtests.jl:14-16 scaled up), B*x and B'*x, strict and
      width-1 stripes, plus Base.:* (multiply_1DVBC.jl:182-185) on vectors and matrices;
  C2  Boeing/ct20stif stand-in: tests/test_io_costs.py and test_gpu_slots.py;
  C3  ldoor block-row split: tests/test_gpu_sharded.py;
  C4  TrSpMV! and 1DVBC B'x on the GHS_psdef/ldoor stand-in (952203^2, 42.5M nnz), Float32;
  C5  2D VBC 16-RHS: tests/test_gpu_mfma.py;
  north star: the 10^7 x 10^7, 1e8-nnz bench matrices (FE 2D, FE 3D irregular, NS uniform) at full
      size against the oracle, normwise rel-err <= 1e-10 (BASELINE.json), forward and transposed.
Tolerances: fp64 normwise 1e-10 at full size (BASELINE), 1e-12 at C1; fp32 1e-5 normwise against
the fp64 oracle product of the same fp32 data.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import sparsematrixvbcs_amd as V
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    d = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (d if d else 1.0)


def ref_of(B):
    return O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)


def threads():
    from oracle import simd
    return simd.host_threads()


def c1_matrix():
    rng = np.random.default_rng(0xDEADBEEF)
    return sp.random(10_000, 10_000, density=1e-3, format="csc", random_state=rng, dtype=np.float64)


@pytest.mark.parametrize("method", ["strict8", "equi1", "default"])
def test_c1_sprand_1e4(method):
    A = c1_matrix()
    meth = {"strict8": V.StrictChunker(8), "equi1": V.EquiChunker(1), "default": None}[method]
    B = V.SparseMatrix1DVBC[8](A, meth)
    R = ref_of(B)
    rng = np.random.default_rng(5)
    xt, xf = rng.uniform(-1, 1, B.m), rng.uniform(-1, 1, B.n)
    yt = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    yf = torch.full((B.m,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(yt, B.T, dev(xt))
    V.mul_(yf, B, dev(xf))
    ref_t = O.mul(R, xt, np.zeros(B.n), trans=True)
    ref_f = O.mul(R, xf, np.zeros(B.m))
    assert rel(yt.cpu().numpy(), ref_t) <= 1e-12
    assert rel(yf.cpu().numpy(), ref_f) <= 1e-12
    # one-hot probes of a column sample: exact columns / rows of A (runtests.jl:29-53)
    D = A.tocsr()
    for j in rng.choice(B.n, 20, replace=False):
        e = np.zeros(B.n)
        e[j] = 1.0
        V.mul_(yf, B, dev(e), True, False)
        assert np.array_equal(yf.cpu().numpy(), A[:, j].toarray().ravel())
    for i in rng.choice(B.m, 20, replace=False):
        e = np.zeros(B.m)
        e[i] = 1.0
        V.mul_(yt, B.T, dev(e), True, False)
        assert np.array_equal(yt.cpu().numpy(), D[i, :].toarray().ravel())


def test_base_star_vectors_and_matrices():
    """Base.:*(A, x) (multiply_1DVBC.jl:182-185): y = similar(x, T, size(A, 1)), mul!(y, A, x, true,
    false), for B, B', torch and numpy vectors, and matrix right-hand sides (column by column)."""
    A = c1_matrix()
    B = V.SparseMatrix1DVBC[8](A, V.StrictChunker(8))
    R = ref_of(B)
    rng = np.random.default_rng(9)
    xt, xf = rng.uniform(-1, 1, B.m), rng.uniform(-1, 1, B.n)
    ref_t = O.mul(R, xt, np.zeros(B.n), trans=True)
    ref_f = O.mul(R, xf, np.zeros(B.m))
    assert rel((B.T @ dev(xt)).cpu().numpy(), ref_t) <= 1e-12
    assert rel((B @ dev(xf)).cpu().numpy(), ref_f) <= 1e-12
    assert rel(B.T @ xt, ref_t) <= 1e-12          # host vectors: staged through HBM
    assert rel(V.matmul(B, xf), ref_f) <= 1e-12
    X = rng.uniform(-1, 1, (B.m, 5))
    Yg = (B.T @ dev(X)).cpu().numpy()
    Yh = B.T @ np.asfortranarray(X)
    for c in range(5):
        rc = O.mul(R, np.ascontiguousarray(X[:, c]), np.zeros(B.n), trans=True)
        assert rel(Yg[:, c], rc) <= 1e-12
        assert rel(Yh[:, c], rc) <= 1e-12


def test_host_staging_reuse_and_views():
    """Host-pointer products reuse the handle's staging buffers and, for a column-major view with
    ld > rows, never touch the parent's padding rows (only the logical extent moves)."""
    A = c1_matrix()
    B = V.SparseMatrix1DVBC[8](A, V.StrictChunker(8))
    R = ref_of(B)
    rng = np.random.default_rng(13)
    for _ in range(3):
        x = rng.uniform(-1, 1, B.m)
        assert rel(V.mul_(np.zeros(B.n), B.T, x), O.mul(R, x, np.zeros(B.n), trans=True)) <= 1e-12
    X = np.asfortranarray(rng.uniform(-1, 1, (B.m, 3)))
    parent = np.asfortranarray(np.full((B.n + 7, 3), 123.0))
    Yv = parent[:B.n, :]  # F-ordered view, ld = n + 7
    V.mul_(Yv, B.T, X, 1.0, 0.0, engine="vector")
    assert np.all(parent[B.n:, :] == 123.0)
    for c in range(3):
        assert rel(Yv[:, c], O.mul(R, np.ascontiguousarray(X[:, c]), np.zeros(B.n), trans=True)) <= 1e-12


@pytest.fixture(scope="module")
def ldoor_f32():
    A = V.synthetic.standin("GHS_psdef/ldoor", dtype=np.float32)
    return A


def test_c4_trspmv_ldoor_f32(ldoor_f32):
    """C4: TrSpMV!(y, A, x) (TrSpMV.jl:1-20) on the ldoor stand-in, Float32, vs the oracle."""
    A = ldoor_f32
    m, n = A.shape
    x = np.random.default_rng(17).uniform(-1, 1, m).astype(np.float32)
    y = torch.full((n,), float("nan"), dtype=torch.float32, device=DEV)
    V.TrSpMV_(y, A, dev(x))
    ref = O.trspmv(A, x, np.zeros(n, np.float32), nthreads=threads())
    exact = O.trspmv(A.astype(np.float64), x.astype(np.float64), np.zeros(n), nthreads=threads())
    got = y.cpu().numpy()
    assert rel(got, exact) <= 1e-5
    assert rel(got, ref) <= 1e-5


def test_c4_1dvbc_transposed_ldoor_f32(ldoor_f32):
    """C4 in 1DVBC form: B = SparseMatrix1DVBC{8}(permutedims(A), StrictChunker(8)) (test_table.jl:27),
    mul!(y, B', x) Float32 vs the oracle; also forward."""
    A = ldoor_f32
    B = V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))
    R = ref_of(B)
    rng = np.random.default_rng(19)
    x = rng.uniform(-1, 1, B.m).astype(np.float32)
    y = torch.full((B.n,), float("nan"), dtype=torch.float32, device=DEV)
    V.mul_(y, B.T, dev(x))
    ref = O.mul(R, x, np.zeros(B.n, np.float32), trans=True, nthreads=threads())
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    exact = O.mul(R64, x.astype(np.float64), np.zeros(B.n), trans=True, nthreads=threads())
    assert rel(y.cpu().numpy(), exact) <= 1e-5
    assert rel(y.cpu().numpy(), ref) <= 1e-5
    xf = rng.uniform(-1, 1, B.n).astype(np.float32)
    yf = torch.full((B.m,), float("nan"), dtype=torch.float32, device=DEV)
    V.mul_(yf, B, dev(xf))
    exact_f = O.mul(R64, xf.astype(np.float64), np.zeros(B.m))
    assert rel(yf.cpu().numpy(), exact_f) <= 1e-5


@pytest.mark.slow
@pytest.mark.parametrize("workload", ["fe", "fe3d", "ns"])
def test_north_star_full_size_vs_oracle(workload):
    """The 10^7 x 10^7, ~1e8-nnz bench matrices: GPU y against the oracle on the same input,
    normwise rel-err <= 1e-10 (BASELINE.json north star), both directions."""
    import bench
    B = bench.build_matrix(workload, np.float64)
    R = ref_of(B)
    rng = np.random.default_rng(0xC0FFEE)
    xt, xf = rng.uniform(-1, 1, B.m), rng.uniform(-1, 1, B.n)
    y = torch.empty(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(xt))
    ref = O.mul(R, xt, np.zeros(B.n), trans=True, nthreads=threads())
    assert rel(y.cpu().numpy(), ref) <= 1e-10
    if workload == "fe3d":  # the automatic layout choice reaches the lane-stream family (vbc_info planar_mask bit 2)
        assert B.info(0, True)["planar_mask"] & 4
    B.release()
    yf = torch.empty(B.m, dtype=torch.float64, device=DEV)
    V.mul_(yf, B, dev(xf))
    ref_f = O.mul(R, xf, np.zeros(B.m))
    assert rel(yf.cpu().numpy(), ref_f) <= 1e-10
    B.release()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("ragged", [False, True])
def test_trspmv_column_blocking(monkeypatch, dtype, ragged):
    """vbc_csc_create groups consecutive columns with identical row patterns (a node's dof columns)
    into one stripe.  Each y[j] still sums its column in stored row order (TrSpMV.jl:10-16): on the
    3-dof operator every bucket is slotted / planar and TrSpMV! equals the unit-stripe layout bit for
    bit; with a few triples broken (ragged: 1- and 2-wide groups, whose small buckets may take the
    merge layout) it matches within tolerance.  Forward product on the blocked handle too."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")  # one wave per chunk: per-column serial order
    A = V.synthetic.fe_stiffness_3d(90000, 2_000_000, 3, dtype).tocsc()
    if ragged:
        D = A.tolil()
        D[5, 7] = 1.5
        D[11, 300] = -2.0
        A = D.tocsc().astype(dtype)
    A.sort_indices()
    m, n = A.shape
    rng = np.random.default_rng(23)
    x = rng.uniform(-1, 1, m).astype(dtype)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    tol = 1e-12 if dtype == np.float64 else 1e-5
    outs = {}
    for blk in ("1", "0"):
        monkeypatch.setenv("VBC_CSC_BLOCK", blk)
        C = V.SparseMatrixCSC(A)
        y = torch.full((n,), float("nan"), dtype=tdt, device=DEV)
        V.TrSpMV_(y, C, dev(x))
        outs[blk] = y.cpu().numpy()
        assert (C.info(trans=True)["L"] < n) == (blk == "1")
        C.release()
    exact = O.trspmv(A.astype(np.float64), x.astype(np.float64), np.zeros(n), nthreads=threads())
    assert rel(outs["1"], exact) <= tol
    if ragged:
        assert rel(outs["1"], outs["0"]) <= tol
    else:
        assert np.array_equal(outs["1"], outs["0"])
    monkeypatch.setenv("VBC_CSC_BLOCK", "1")
    C = V.SparseMatrixCSC(A)
    xf = rng.uniform(-1, 1, n).astype(dtype)
    yf = torch.zeros(m, dtype=tdt, device=DEV)
    V.mul_(yf, C, dev(xf))
    assert rel(yf.cpu().numpy(), A.astype(np.float64) @ xf.astype(np.float64)) <= tol


@pytest.mark.slow
@pytest.mark.parametrize("workload", ["c5", "c5-mesh"])
def test_c5_full_size_four_columns(workload):
    """BASELINE C5 at the bench's full size (2D VBC, 1e8 fp32 values, 16 row-major right-hand sides): the
    multi-RHS product in both directions (B'X on B's layout, B·X on Bᵀ's), 4 of the 16 columns against the
    oracle's per-column product in fp64 (the reference has no matrix mul!, multiply_VBC.jl:194-197, so its
    semantics is column by column), normwise 1e-5."""
    import bench
    B = bench.build_matrix(workload, np.float32)
    Rd = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    rng = np.random.default_rng(0xC0FFEE)
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        X = rng.uniform(-1, 1, (nx, 16)).astype(np.float32)
        Y = torch.full((ny, 16), float("nan"), dtype=torch.float32, device=DEV)
        V.mul_(Y, B.T if trans else B, dev(X))
        got = Y.cpu().numpy()
        for j in (0, 5, 10, 15):
            ref = O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64), np.zeros(ny), trans=trans,
                        nthreads=threads())
            assert rel(got[:, j], ref) <= 1e-5, (workload, trans, j)
        B.release()
