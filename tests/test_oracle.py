"""Pin the CPU oracle (oracle/vbc_oracle.c) against the reference's own fixtures and protocol.

- one-hot probes (runtests.jl:29-53,63-87) must reproduce A's columns / rows EXACTLY;
- random probes must match the committed scipy products (tests/golden/matrices.npz) within the
  reference's isapprox tolerance √eps (bin/test_table.jl:42,84,126) -- we use 1e-13 normwise;
- hand-derived layout KATs follow constructors_1DVBC.jl / constructors_VBC.jl by hand.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle as O
from tests.conftest import sprand_family


def equi(n, w):
    return np.r_[np.arange(1, n + 1, w), n + 1].astype(np.int64)


def one_hot_1d(B, A, trans):
    m, n = A.shape
    D = A.toarray()
    nin = m if trans else n
    for j in range(nin):
        x = np.zeros(nin)
        x[j] = 1.0
        y = np.zeros(n if trans else m)
        O.mul(B, x, y, 1.0, 0.0, trans=trans)
        ref = D[j, :] if trans else D[:, j]
        assert np.array_equal(y, ref), (j, trans)


def rel(a, b):
    d = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (d if d else 1.0)


@pytest.mark.parametrize("w", [1, 2, 3, 4])
def test_oracle_one_hot_golden(golden, w):
    for key, g in golden.items():
        A = g["A"]
        B = O.build_1dvbc(A, equi(A.shape[1], w), 4, pad=8)
        assert np.array_equal(O.vbc_to_dense(B), A.toarray()), key
        one_hot_1d(B, A, False)
        one_hot_1d(B, A, True)


@pytest.mark.parametrize("u,w", [(1, 1), (2, 3), (4, 4)])
def test_oracle_vbc_one_hot_golden(golden, u, w):
    for key, g in golden.items():
        A = g["A"]
        m, n = A.shape
        B = O.build_vbc(A, equi(m, u), equi(n, w), 4, 4, pad=32)
        assert np.array_equal(O.vbc_to_dense(B), A.toarray()), key
        one_hot_1d(B, A, False)
        one_hot_1d(B, A, True)


def test_oracle_random_vs_committed_scipy(golden):
    for key, g in golden.items():
        A = g["A"]
        m, n = A.shape
        for B in (O.build_1dvbc(A, equi(n, 3), 4), O.build_vbc(A, equi(m, 2), equi(n, 4), 4, 4)):
            y = np.full(m, np.nan)
            O.mul(B, g["xf"], y, 1.0, 0.0)
            assert rel(y, g["yf"]) < 1e-13, key
            y = np.full(n, np.nan)
            O.mul(B, g["xt"], y, 1.0, 0.0, trans=True)
            assert rel(y, g["yt"]) < 1e-13, key
        y = np.full(n, np.nan)
        O.trspmv(A, g["xt"], y)
        assert rel(y, g["yt"]) < 1e-13, key


def test_oracle_kat_1dvbc_layout():
    # A = [1 0 2; 0 3 0; 4 5 0; 0 0 6], Φ = [1, 3, 4]  (derived by hand from constructors_1DVBC.jl)
    A = sp.csc_matrix(np.array([[1, 0, 2], [0, 3, 0], [4, 5, 0], [0, 0, 6]], dtype=np.float64))
    B = O.build_1dvbc(A, np.array([1, 3, 4]), 2, pad=8)
    assert B.pos.tolist() == [1, 4, 6]
    assert B.ofs.tolist() == [1, 7, 9]
    assert B.idx.tolist() == [1, 2, 3, 1, 4]
    assert B.val.tolist() == [1, 0, 0, 3, 4, 5, 2, 6] + [0] * 8
    # W = 1 < w = 2 must trip @assert w <= W (constructors_1DVBC.jl:46)
    with pytest.raises(O.OracleError, match="Assertion"):
        O.build_1dvbc(A, np.array([1, 3, 4]), 1)


def test_oracle_kat_vbc_layout():
    A = sp.csc_matrix(np.array([[1, 0, 2], [0, 3, 0], [4, 5, 0], [0, 0, 6]], dtype=np.float64))
    B = O.build_vbc(A, np.array([1, 3, 5]), np.array([1, 3, 4]), 2, 2, pad=0)
    assert B.pos.tolist() == [1, 3, 5]
    assert B.ofs.tolist() == [1, 9, 13]
    assert B.idx.tolist() == [1, 2, 1, 2]
    assert B.val.tolist() == [1, 0, 0, 3, 4, 5, 0, 0, 2, 0, 0, 6]


def test_oracle_strict_fast_path_matches_generic(golden):
    import sparsematrixvbcs_amd as V
    for key, g in golden.items():
        A = g["A"]
        spl = V.StrictChunker(4).partition(A).spl
        a = O.build_1dvbc(A, spl, 4, pad=8)
        b = O.build_1dvbc(A, spl, 4, pad=8, strict=True)
        for f in ("pos", "idx", "ofs", "val"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), (key, f)


def test_oracle_reference_quirks():
    rng = np.random.default_rng(7)
    A = sp.random(30, 20, 0.3, random_state=3, format="csc")
    B = O.build_1dvbc(A, equi(20, 3), 4)
    D = A.toarray()
    x, y0 = rng.random(20), rng.random(30)
    # forward: α dropped (multiply_1DVBC.jl:48), β applied (:50-52)
    y = y0.copy(); O.mul(B, x, y, 2.0, 3.0, ref_semantics=True)
    assert np.allclose(y, 3 * y0 + D @ x)
    y = y0.copy(); O.mul(B, x, y, 2.0, 3.0, ref_semantics=False)
    assert np.allclose(y, 3 * y0 + 2 * D @ x)
    # transposed: overwrite (multiply_1DVBC.jl:114-116)
    xt, yt0 = rng.random(30), rng.random(20)
    y = yt0.copy(); O.mul(B, xt, y, 2.0, 3.0, trans=True, ref_semantics=True)
    assert np.allclose(y, D.T @ xt)
    y = yt0.copy(); O.mul(B, xt, y, 2.0, 3.0, trans=True, ref_semantics=False)
    assert np.allclose(y, 3 * yt0 + 2 * D.T @ xt)
    # DimensionMismatch (multiply_1DVBC.jl:44-45)
    with pytest.raises(O.OracleError, match="DimensionMismatch"):
        O.mul(B, np.zeros(19), np.zeros(30))


def test_oracle_sprand_grid_one_hot():
    """runtests.jl:14-16 size grid (own RNG), one trial per size and kind, W = 4 equi stripes."""
    for name, A in sprand_family(trials=1):
        m, n = A.shape
        for w in (1, 3, 4):
            B = O.build_1dvbc(A, equi(n, w), 4, pad=8)
            assert np.array_equal(O.vbc_to_dense(B), A.toarray()), name
        one_hot_1d(B, A, False)
        one_hot_1d(B, A, True)


def test_oracle_fp32_and_threads(golden):
    g = golden["LPnetlib__lp_etamacro"]
    A = g["A"]
    B = O.build_1dvbc(A, equi(A.shape[1], 4), 4, dtype=np.float32)
    x = g["xt"].astype(np.float32)
    y1 = np.zeros(A.shape[1], np.float32)
    y4 = np.zeros(A.shape[1], np.float32)
    O.mul(B, x, y1, trans=True, nthreads=1)
    O.mul(B, x, y4, trans=True, nthreads=4)
    assert np.array_equal(y1, y4)  # per-stripe order is thread-independent
    assert rel(y1.astype(np.float64), g["yt"]) < 1e-5
