"""GPU parity of the matrix-core multi-RHS product Y = α·B'X + β·Y (vbc_panel.h, VBC_CREATE_MULTI).

The reference has no matrix mul! (multiply_1DVBC.jl:184-185), so parity is column by column against
the oracle's transposed products (multiply_1DVBC.jl:90-134, multiply_VBC.jl:93-147).  Tolerances as
test_gpu_parity.py: one-hot probes bit-exact; random X normwise 1e-12 (fp64) / 1e-5 (fp32 vs the
fp64 product).
"""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"
TOL64, TOL32 = 1e-12, 1e-5


@pytest.fixture(autouse=True, params=["tiles", "0"], ids=["tiles", "panels"])
def multi_layout(request, monkeypatch):
    """Every test on the two multi-RHS layouts: every width on the MFMA panels (VBC_PANEL_TILES=0), and every
    bucket of width <= 4 whose tiles are <= 4 rows in the tile-granular layout (VBC_PANEL_TILES=1, spmm_tiles --
    the default for such buckets when their rows come in tiles).  (Round 6: the VALU stripe-quad layout and the
    staged-X / persistent / 16-B tile forms, which lost their A/B in rounds 4-5, left the library.)"""
    monkeypatch.setenv("VBC_PANEL_TILES", "1" if request.param == "tiles" else "0")
    return request.param


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    d = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (d if d else 1.0)


def as_dev(M, layout):
    """Device copy of M in row-major ("R") or column-major ("C") storage."""
    if layout == "R":
        return torch.from_numpy(np.ascontiguousarray(M)).to(DEV)
    return torch.from_numpy(np.ascontiguousarray(M.T)).to(DEV).T


def ref_cols(R, X, Y0, alpha, beta):
    """Oracle B'X + β Y0, one transposed product per column, in fp64."""
    Rd = R
    if R.val.dtype != np.float64:
        Rd = type(R).__new__(type(R))
        Rd.__dict__.update(R.__dict__)
        Rd.val = R.val.astype(np.float64)
    return np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64),
                           np.ascontiguousarray(Y0[:, j], dtype=np.float64), alpha, beta, trans=True,
                           ref_semantics=False) for j in range(X.shape[1])], axis=1)


def ref_1d(B):
    return O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)


def ref_2d(B):
    return O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)


def test_golden_one_hot_mfma(golden):
    """Every matrix of test/matrices.jl as 1DVBC and 2D VBC: identity blocks of 16 columns through
    the panel product give exactly the rows of A (runtests.jl:63-87 protocol, 16 at a time)."""
    for key, g in golden.items():
        A = g["A"]
        m, n = A.shape
        D = A.toarray()
        mats = [V.SparseMatrix1DVBC[4](A, V.StrictChunker(4)),
                V.SparseMatrixVBC[4, 4](A, V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)))]
        for B in mats:
            for layout in ("R", "C"):
                for j0 in range(0, m, 16):
                    k = min(16, m - j0)
                    X = np.zeros((m, k))
                    X[np.arange(j0, j0 + k), np.arange(k)] = 1.0
                    Y = as_dev(np.full((n, k), np.nan), layout)
                    V.mul_(Y, B.T, as_dev(X, layout), engine="mfma")
                    assert np.array_equal(Y.cpu().numpy(), D[j0:j0 + k, :].T), (key, type(B).__name__, layout)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("nrhs", [1, 2, 5, 16, 17, 33, 64, 70])
def test_mfma_1dvbc_random(nrhs, dtype):
    """Widths 1..16 (every panel packing S = 16/w), a w > 16 stripe (cut into 16-column pieces),
    empty stripes (fill list), alpha/beta, row- and column-major operands vs the oracle."""
    tol = TOL64 if dtype == np.float64 else TOL32
    rng = np.random.default_rng(100 + nrhs)
    for widths, q in ((list(range(1, 17)), 2000), ([2], 100), ([16], 900), ([1, 20, 7, 33], 150)):
        L = 60
        w = np.array([widths[i % len(widths)] for i in range(L)])
        B = V.synthetic.vbr_1dvbc(900, L, q, w, W=40, dtype=dtype, seed=nrhs * 7 + int(w.sum()))
        if q <= 150:
            assert (np.diff(B.pos) == 0).any()  # some stripes empty: the fill list writes them
        R = ref_1d(B)
        for layout in ("R", "C"):
            X = rng.uniform(-1, 1, (B.m, nrhs)).astype(dtype)
            Y0 = rng.uniform(-1, 1, (B.n, nrhs)).astype(dtype)
            for alpha, beta in ((1.0, 0.0), (1.5, 0.5), (-2.0, 1.0)):
                Yd = as_dev(Y0, layout)
                V.mul_(Yd, B.T, as_dev(X, layout), alpha, beta, engine="mfma")
                assert rel(Yd.cpu().numpy(), ref_cols(R, X, Y0, alpha, beta)) <= tol, (widths, layout, alpha, beta)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("uw", [(8, 8), (4, 16), (16, 4), (3, 5), (1, 1)])
def test_mfma_vbc2d_random(uw, dtype):
    """C5 shape at small size: 2D VBC u x w tiles (costs.jl:200-220 generator), 16 RHS."""
    u, w = uw
    tol = TOL64 if dtype == np.float64 else TOL32
    B = V.synthetic.vbr_2d(40, 30, 200, u, w, dtype=dtype, seed=u * 31 + w)
    R = ref_2d(B)
    rng = np.random.default_rng(u + w)
    X = rng.uniform(-1, 1, (B.m, 16)).astype(dtype)
    Y0 = rng.uniform(-1, 1, (B.n, 16)).astype(dtype)
    for layout in ("R", "C"):
        Yd = as_dev(Y0, layout)
        V.mul_(Yd, B.T, as_dev(X, layout), 1.0, 0.25, engine="mfma")
        assert rel(Yd.cpu().numpy(), ref_cols(R, X, Y0, 1.0, 0.25)) <= tol, layout


def test_mfma_matches_vector_engine_and_is_deterministic():
    """Same product through the matrix-core and the vector engines; repeated runs bitwise equal."""
    B = V.synthetic.vbr_1dvbc(5000, 900, 20000, np.arange(900) % 8 + 1, W=8, dtype=np.float64, seed=3)
    X = torch.rand((B.m, 16), dtype=torch.float64, device=DEV)
    Y1 = torch.empty((B.n, 16), dtype=torch.float64, device=DEV)
    Y2 = torch.empty_like(Y1)
    Y3 = torch.empty_like(Y1)
    V.mul_(Y1, B.T, X, engine="mfma")
    V.mul_(Y2, B.T, X, engine="vector")
    V.mul_(Y3, B.T, X, engine="mfma")
    assert rel(Y1.cpu().numpy(), Y2.cpu().numpy()) <= 1e-13
    assert torch.equal(Y1, Y3)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_mfma_nonfinite_confined_to_own_stripe(dtype):
    """An Inf / NaN in X reaches exactly the columns whose stripes store that row (as in the
    reference's per-stripe loop), never the other stripes sharing its panel."""
    B = V.synthetic.vbr_1dvbc(300, 64, 600, 2, W=2, dtype=dtype, seed=11)
    R = ref_1d(B)
    rng = np.random.default_rng(5)
    X = rng.uniform(-1, 1, (B.m, 16)).astype(dtype)
    X[17, 3] = np.inf
    X[101, 0] = np.nan
    X[250, 9] = -np.inf
    Yd = as_dev(np.zeros((B.n, 16), dtype), "R")
    V.mul_(Yd, B.T, as_dev(X, "R"), engine="mfma")
    got = Yd.cpu().numpy()
    ref = ref_cols(R, X, np.zeros((B.n, 16), dtype), 1.0, 0.0)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert rel(got[fin], ref[fin]) <= (TOL64 if dtype == np.float64 else TOL32)


def test_mfma_quirks_and_errors():
    """Reference α/β quirks (transposed overwrites y) and the boundary errors of vbc_mul_mat."""
    B = V.synthetic.vbr_1dvbc(200, 40, 300, 4, W=4, seed=2)
    R = ref_1d(B)
    X = np.random.default_rng(0).uniform(-1, 1, (B.m, 8))
    Y0 = np.ones((B.n, 8))
    Yd = as_dev(Y0, "R")
    V.mul_(Yd, B.T, as_dev(X, "R"), 3.0, 2.0, quirks=True, engine="mfma")
    assert rel(Yd.cpu().numpy(), ref_cols(R, X, Y0, 1.0, 0.0)) <= TOL64
    with pytest.raises(V.DimensionMismatch):
        V.mul_(torch.zeros((B.n + 1, 8), dtype=torch.float64, device=DEV), B.T, as_dev(X, "R"), engine="mfma")
    # round 3: the forward product runs on matrix cores too (panel layout of B'); forward quirks drop α
    Xf = np.random.default_rng(1).uniform(-1, 1, (B.n, 8))
    Yf = as_dev(np.ones((B.m, 8)), "R")
    V.mul_(Yf, B, as_dev(Xf, "R"), 3.0, 2.0, quirks=True, engine="mfma")
    want = np.stack([O.mul(R, Xf[:, j].copy(), np.ones(B.m), 1.0, 2.0, trans=False, ref_semantics=False)
                     for j in range(8)], axis=1)
    assert rel(Yf.cpu().numpy(), want) <= TOL64


def test_mfma_host_memory_and_info():
    """numpy operands (staged through HBM) and the panel layout's vbc_info fields."""
    B = V.synthetic.vbr_2d(20, 20, 80, 4, 4, dtype=np.float64, seed=9)
    R = ref_2d(B)
    X = np.random.default_rng(1).uniform(-1, 1, (B.m, 16))
    Y = np.zeros((B.n, 16))
    V.mul_(Y, B.T, X, engine="mfma")
    assert rel(Y, ref_cols(R, X, np.zeros((B.n, 16)), 1.0, 0.0)) <= TOL64
    inf = B.info(multi=True)
    assert inf["bins_m"] == 1 and inf["bins_t"] == 0 and inf["bytes_m"] > 0


@pytest.mark.parametrize("workload,scale", [("c5", 0.1), ("c5-mesh", 0.05)])
def test_c5_panels_scaled_every_column(workload, scale):
    """The bench's C5 inputs at reduced scale (the random 8x8-tile generator, costs.jl:200-220, 1e7 values;
    the structured 3x3 node-tile mesh, 5e6), 16 row-major right-hand sides through the matrix-core panel
    product, B'X and B X: every column against the oracle (fp32 vs the fp64 product, normwise 1e-5)."""
    import bench
    B = bench.build_matrix(workload, np.float32, scale)
    rng = np.random.default_rng(47)
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        X = rng.uniform(-1, 1, (nx, 16)).astype(np.float32)
        Y = torch.empty((ny, 16), dtype=torch.float32, device=DEV)
        V.mul_(Y, B.T if trans else B, torch.from_numpy(X).to(DEV))
        got = Y.cpu().numpy()
        Rd = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
        for j in range(16):
            ref = O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64), np.zeros(ny), trans=trans)
            assert rel(got[:, j], ref) <= TOL32, (trans, j)


def test_mixed_widths_tiles_and_panels(multi_layout):
    """A matrix with widths 3 and 12 runs both multi-RHS kernels in one product (with VBC_PANEL_TILES=1 the
    tile kernel for the 3-wide stripes, whose rows come in runs; MFMA panels for the 12-wide ones) and matches
    the oracle on every column; vbc_info planar_mask bits 7 and 10 (the removed stripe-quad and staged-X
    layouts) stay clear."""
    B = V.synthetic.vbr_1dvbc(700, 80, 900, np.where(np.arange(80) % 2 == 0, 3, 12), W=16, dtype=np.float32, seed=12)
    inf = B.info(multi=True)
    assert inf["planar_mask"] & (128 | 1024) == 0
    assert inf["bins_m"] == 2
    R = ref_1d(B)
    X = np.random.default_rng(2).uniform(-1, 1, (B.m, 16)).astype(np.float32)
    Yd = as_dev(np.zeros((B.n, 16), np.float32), "R")
    V.mul_(Yd, B.T, as_dev(X, "R"), engine="mfma")
    assert rel(Yd.cpu().numpy(), ref_cols(R, X, np.zeros((B.n, 16)), 1.0, 0.0)) <= TOL32


def _vbc2d_mixed_heights(rng, K, L, q, heights, widths, dtype):
    """A SparseMatrixVBC whose block rows have the given heights (cycled) and stripes the given widths:
    q distinct random (k, l) tiles, dense u_k x w_l blocks (constructors_VBC.jl:95-105 layout)."""
    u = np.array([heights[i % len(heights)] for i in range(K)])
    w = np.array([widths[i % len(widths)] for i in range(L)])
    pspl = np.concatenate([[1], 1 + np.cumsum(u)])
    spl = np.concatenate([[1], 1 + np.cumsum(w)])
    keys = np.unique(rng.integers(0, K * L, q))
    l, k = keys // K, keys % K  # sorted by stripe, then block row
    cnt = np.bincount(l, minlength=L)
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)])
    sizes = u[k] * w[l]
    ofs = np.concatenate([[1], 1 + np.cumsum(np.bincount(l, weights=sizes, minlength=L).astype(np.int64))])
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + 64, dtype)
    val[:nv] = rng.uniform(-1, 1, nv)
    return V.SparseMatrixVBC(4, 4, int(pspl[-1] - 1), int(spl[-1] - 1), V.SplitPartition(pspl), V.SplitPartition(spl),
                             pos, k + 1, ofs, val)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_tiles_mixed_heights_widths_every_column(dtype, multi_layout):
    """Tile layout (spmm_tiles): block rows of heights 1..4 in one stripe (slot rows past a tile's height
    masked), widths 1..4 (one bucket each, non-affine columns), empty stripes, 5 / 16 / 21 right-hand sides,
    row- and column-major operands, alpha / beta, both directions -- every column against the oracle, and
    with VBC_PANEL_TILES=1 the layout flag (vbc_info planar_mask bit 9)."""
    rng = np.random.default_rng(61)
    tol = TOL64 if dtype == np.float64 else TOL32
    B = _vbc2d_mixed_heights(rng, 300, 400, 1200, (3, 1, 4, 2, 3), (1, 3, 2, 4, 3), dtype)
    assert (np.diff(B.pos) == 0).any()
    if multi_layout == "tiles":
        assert B.info(multi=True)["planar_mask"] & 512
        assert B.info(trans=False, multi=True)["planar_mask"] & 512
    R = ref_2d(B)
    for nrhs in (5, 16, 21):
        for layout in ("R", "C"):
            for trans in (True, False):
                nx, ny = (B.m, B.n) if trans else (B.n, B.m)
                X = rng.uniform(-1, 1, (nx, nrhs)).astype(dtype)
                Y0 = rng.uniform(-1, 1, (ny, nrhs)).astype(dtype)
                alpha, beta = (1.0, 0.0) if nrhs == 16 else (0.5, -1.25)
                Yd = as_dev(Y0, layout)
                V.mul_(Yd, B.T if trans else B, as_dev(X, layout), alpha, beta, engine="mfma")
                Rd = R
                if dtype != np.float64:
                    Rd = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
                want = np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64),
                                       np.ascontiguousarray(Y0[:, j], dtype=np.float64), alpha, beta, trans=trans,
                                       ref_semantics=False) for j in range(nrhs)], axis=1)
                assert rel(Yd.cpu().numpy(), want) <= tol, (nrhs, layout, trans)


def test_tiles_node_runs_with_holes_exact_and_nonfinite(multi_layout):
    """A 1DVBC whose stripes store node runs of 3 rows, some missing one row (the hole is a masked slot row
    of its tile): integer data bit for bit on all 16 columns (each column is the reference's fma chain);
    an Inf / NaN in X at a hole row reaches no stripe that does not store it."""
    rng = np.random.default_rng(62)
    N, L = 500, 300
    rows, cnt = [], []
    for l in range(L):
        nodes = np.sort(rng.choice(N, 10, replace=False))
        r = (nodes[:, None] * 3 + np.arange(3)[None, :]).reshape(-1)
        if l % 4 == 0:
            r = np.delete(r, rng.integers(0, len(r)))
        rows.append(r)
    widths = 1 + np.arange(L) % 3
    cnt = np.array([len(r) for r in rows])
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)])
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * widths)])
    spl = np.concatenate([[1], 1 + np.cumsum(widths)])
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + 8)
    val[:nv] = rng.integers(-8, 9, nv)
    B = V.SparseMatrix1DVBC(8, 3 * N, int(spl[-1] - 1), V.SplitPartition(spl), pos, np.concatenate(rows) + 1, ofs, val)
    if multi_layout == "tiles":
        assert B.info(multi=True)["planar_mask"] & 512
    R = ref_1d(B)
    X = rng.integers(-8, 9, (B.m, 16)).astype(np.float64)
    Yd = as_dev(np.full((B.n, 16), np.nan), "R")
    V.mul_(Yd, B.T, as_dev(X, "R"), engine="mfma")
    assert np.array_equal(Yd.cpu().numpy(), ref_cols(R, X, np.zeros((B.n, 16)), 1.0, 0.0))
    hole = [r for r in range(3 * (rows[0][0] // 3), 3 * (rows[0][-1] // 3) + 3)
            if r not in set(rows[0].tolist()) and (r // 3) in set((rows[0] // 3).tolist())]
    assert hole
    X[hole[0], :] = np.nan
    X[hole[0], 5] = np.inf
    V.mul_(Yd, B.T, as_dev(X, "R"), engine="mfma")
    got, ref = Yd.cpu().numpy(), ref_cols(R, X, np.zeros((B.n, 16)), 1.0, 0.0)
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert np.array_equal(got[fin], ref[fin])


def test_tiles_clustered_launch_order_bitwise(multi_layout, monkeypatch):
    """The tile layout's clustered launch order (VBC_TILE_CLUSTER: ranges taken as BFS balls over shared X row
    groups) changes only which wave folds which range when: at small scale, forced on
    (2) against off (0), both directions, the products are bit-identical and equal the oracle's on integer data."""
    import bench
    B = bench.build_matrix("c5-mesh", np.float32, 0.01)
    B.val[:] = np.random.default_rng(5).integers(-8, 9, B.val.shape)
    Rd = ref_2d(B)
    Rd.val = Rd.val.astype(np.float64)
    rng = np.random.default_rng(12)
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        X = rng.integers(-8, 9, (nx, 16)).astype(np.float32)
        got = {}
        for mode in ("0", "2"):
            monkeypatch.setenv("VBC_TILE_CLUSTER", mode)
            Bm = bench.build_matrix("c5-mesh", np.float32, 0.01)  # a fresh handle per mode (create-time knob)
            Bm.val[:] = B.val
            Yd = torch.empty((ny, 16), dtype=torch.float32, device=DEV)
            V.mul_(Yd, Bm.T if trans else Bm, torch.from_numpy(X).to(DEV), engine="mfma")
            got[mode] = Yd.cpu().numpy()
            Bm.release()
        want = np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64), np.zeros(ny), 1.0, 0.0, trans=trans,
                               ref_semantics=False) for j in range(16)], axis=1)
        assert np.array_equal(got["0"], got["2"]), trans
        assert np.array_equal(got["2"], want.astype(np.float32)), trans


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_c5_mesh_integer_bitwise(dtype, multi_layout):
    """The structured C5 input (3 x 3 node tiles) at small scale, 16 row-major right-hand sides, both directions
    (B·X on Bᵀ's layout): integer data, so every column equals the oracle bit for bit (each column is the
    reference's fma chain, multiply_VBC.jl:126-135); then random data with alpha / beta, 7 right-hand sides,
    column-major operands (the element path of the epilogue)."""
    import bench
    B = bench.build_matrix("c5-mesh", dtype, 0.002)
    B.val[:] = np.random.default_rng(3).integers(-8, 9, B.val.shape)
    if multi_layout == "tiles":
        assert B.info(multi=True)["planar_mask"] & 512 and B.info(trans=False, multi=True)["planar_mask"] & 512
    Rd = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    rng = np.random.default_rng(11)
    tdt = torch.float32 if dtype == np.float32 else torch.float64
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        X = rng.integers(-8, 9, (nx, 16)).astype(dtype)
        Y0 = rng.integers(-8, 9, (ny, 16)).astype(dtype)
        for alpha, beta in ((1.0, 0.0), (2.0, -1.0)):
            Yd = torch.from_numpy(Y0.copy()).to(DEV)
            V.mul_(Yd, B.T if trans else B, torch.from_numpy(X).to(DEV), alpha, beta, engine="mfma")
            want = np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64),
                                   np.ascontiguousarray(Y0[:, j], dtype=np.float64), alpha, beta, trans=trans,
                                   ref_semantics=False) for j in range(16)], axis=1)
            assert Yd.dtype == tdt and np.array_equal(Yd.cpu().numpy(), want.astype(dtype)), (trans, alpha, beta)
        X = rng.uniform(-1, 1, (nx, 7)).astype(dtype)
        Y0 = rng.uniform(-1, 1, (ny, 7)).astype(dtype)
        Yd = as_dev(Y0, "C")
        V.mul_(Yd, B.T if trans else B, as_dev(X, "C"), 0.5, -1.25, engine="mfma")
        want = np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64),
                               np.ascontiguousarray(Y0[:, j], dtype=np.float64), 0.5, -1.25, trans=trans,
                               ref_semantics=False) for j in range(7)], axis=1)
        assert rel(Yd.cpu().numpy(), want) <= (TOL64 if dtype == np.float64 else TOL32), trans
