"""GPU parity of the planar slotted layout (csrc/vbc_planar.h: one stripe per lane, column-group-major
chunk rows) for mul!(y, B', x) with stripes 3..8 wide, against the oracle.  The library picks it for
those widths automatically (fp64 w >= 3, fp32 w = 3 and w >= 5); VBC_SLOT_PLANAR=0 / 1 force the
previous slotted form / planar.  Tolerances as test_gpu_parity.py: one-hot probes bit-exact (the
reference's protocol, runtests.jl:29-53), random x <= 1e-12 (fp64) / 1e-5 (fp32)."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.test_gpu_parity import TOL32, TOL64, dev, one_hot_probes, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


def ref_of(B):
    return O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)


def planar_bins(B):
    return B.info(trans=True)["planar_bins"]


@pytest.mark.parametrize("planar", ["0", "1"])
def test_golden_one_hot_w8(golden, monkeypatch, planar):
    """The reference corpus cut into 3-, 5- and 8-wide stripes (EquiChunker; the corpus' own column
    patterns give Strict/Overlap chunkers stripes of at most 2 columns)."""
    monkeypatch.setenv("VBC_SLOTS", "1")
    monkeypatch.setenv("VBC_SLOT_PLANAR", planar)
    seen = 0
    for key, g in golden.items():
        for meth in (V.EquiChunker(3), V.EquiChunker(5), V.EquiChunker(8)):
            B = V.SparseMatrix1DVBC[8](g["A"], meth)
            one_hot_probes(B, g["A"])
            seen += planar_bins(B)
    assert (seen > 0) == (planar == "1")


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w", [3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("keys16", ["0", "1"])
def test_widths_random_x(monkeypatch, dtype, w, keys16):
    """Every planar width, both key forms, natural (affine, LDS-staged writes) and length-sorted
    (table-mapped) segment orders, alpha / beta."""
    monkeypatch.setenv("VBC_SLOT_KEYS16", keys16)
    rng = np.random.default_rng(w)
    for ragged in (False, True):
        L = 5000
        q = 40000 if not ragged else 25000
        B = V.synthetic.vbr_1dvbc(30000, L, q, w, W=8, dtype=dtype, seed=w + 7 * ragged)
        if not ragged:  # near-uniform rows per stripe: natural order
            pass
        R = ref_of(B)
        x = rng.uniform(-1, 1, B.m).astype(dtype)
        y0 = rng.uniform(-1, 1, B.n).astype(dtype)
        tol = TOL64 if dtype == np.float64 else TOL32
        for alpha, beta in ((1.0, 0.0), (0.5, 2.0)):
            y = dev(y0.copy())
            V.mul_(y, B.T, dev(x), alpha, beta)
            R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
            ref = O.mul(R64, x.astype(np.float64), y0.astype(np.float64), alpha, beta, trans=True,
                        ref_semantics=False)
            assert rel(y.cpu().numpy(), ref) <= tol, (w, ragged, alpha, beta)
        exp_planar = w >= 3 and not (dtype == np.float32 and w == 4)
        assert (planar_bins(B) > 0) == exp_planar or B.info(trans=True)["sweep_bins"] > 0


@pytest.mark.parametrize("stage", ["0", "8"])
def test_fe3d_planar_matches_oracle_bitwise(monkeypatch, stage):
    """The irregular 3D stiffness operator (w = 3): planar result equals the oracle bit for bit
    (same per-lane FMA order as multiply_1DVBC.jl:101-104), staged and direct y writes."""
    monkeypatch.setenv("VBC_SLOT_STAGE", stage)
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")  # one wave per chunk: the reference's summation order
    B = V.synthetic.fe_stiffness_3d_1dvbc(300000, 3_000_000)
    assert planar_bins(B) == 1
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, B.m)
    y = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    ref = O.mul(ref_of(B), x, np.zeros(B.n), trans=True)
    assert np.array_equal(y.cpu().numpy(), ref)


def test_planar_nonfinite_x(monkeypatch):
    """Inf / NaN in x land exactly where the reference puts them (padding rows take x as 0)."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    B = V.synthetic.fe_stiffness_3d_1dvbc(30000, 300000)
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, B.m)
    x[[0, 17, 999]] = [np.inf, np.nan, -np.inf]
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    ref = O.mul(ref_of(B), x, np.zeros(B.n), trans=True)
    got = y.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert np.array_equal(got[fin], ref[fin])


def test_planar_quirks_and_forward_unaffected():
    """quirks mode (transposed overwrites y) and the forward product (not planar) on the same matrix."""
    B = V.synthetic.fe_stiffness_3d_1dvbc(60000, 600000, dtype=np.float32)
    R = ref_of(B)
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, B.m).astype(np.float32)
    y = dev(rng.uniform(-1, 1, B.n).astype(np.float32))
    V.mul_(y, B.T, dev(x), 3.0, 7.0, quirks=True)
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    assert rel(y.cpu().numpy(), O.mul(R64, x.astype(np.float64), np.zeros(B.n), trans=True)) <= TOL32
    xf = rng.uniform(-1, 1, B.n).astype(np.float32)
    yf = torch.zeros(B.m, dtype=torch.float32, device=DEV)
    V.mul_(yf, B, dev(xf))
    assert rel(yf.cpu().numpy(), O.mul(R64, xf.astype(np.float64), np.zeros(B.m))) <= TOL32


def expand_runs(B, R, seed, break_one=False):
    """B with every stored row i replaced by the run of R consecutive rows R(i-1)+1 .. R(i-1)+R (fresh
    values): the node-dof row structure of a stiffness operator.  break_one: the first stripe's first
    run gets a gap, so the bucket has no aligned runs."""
    rng = np.random.default_rng(seed)
    w = np.diff(B.Phi.spl)
    cnt = np.diff(B.pos) * R
    idx = ((B.idx[:, None] - 1) * R + np.arange(R)[None, :]).reshape(-1) + 1
    if break_one:  # first run of the first non-empty stripe: rows r, r, r+2 (a repeated row, no run)
        q0 = int(np.sum(cnt[:int(np.argmax(cnt > 0))]))
        idx[q0 + 1] = idx[q0]
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)]).astype(np.int64)
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * w)]).astype(np.int64)
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + len(B.val) - int(B.ofs[-1] - 1), B.val.dtype)
    val[:nv] = rng.uniform(-1, 1, nv).astype(B.val.dtype)
    return V.SparseMatrix1DVBC(B.W, R * B.m, B.n, V.SplitPartition(B.Phi.spl.copy()), pos, idx.astype(np.int64),
                               ofs, val)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("R", [2, 3])
@pytest.mark.parametrize("w", [3, 5, 8])
def test_row_runs(monkeypatch, dtype, R, w):
    """Row runs (SlotBin::run): one key and one R-wide x gather per run of R consecutive rows.  The
    result equals the oracle bit for bit (fp64: same per-lane FMA order) and the run-free planar layout
    (VBC_SLOT_RUNS=0); a bucket whose rows are not all in aligned runs falls back to run = 1."""
    rng = np.random.default_rng(R * 10 + w)
    base = V.synthetic.vbr_1dvbc(7000, 3000, 20000, w, W=8, dtype=dtype, seed=w)
    B = expand_runs(base, R, seed=w + R)
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    x = rng.uniform(-1, 1, B.m).astype(dtype)
    x[[5, 1234]] = [np.inf, np.nan]  # non-finite x inside runs: they land where the oracle puts them
    outs = {}
    for runs in ("1", "0"):
        monkeypatch.setenv("VBC_SLOT_RUNS", runs)
        monkeypatch.setenv("VBC_SLOT_PLANAR", "1")
        monkeypatch.setenv("VBC_SLOTS", "1")
        monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
        Bc = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)  # fresh handle cache
        inf = Bc.info(trans=True)
        assert inf["planar_bins"] == 1 and inf["planar_run"] == (R if runs == "1" else 1)
        y = torch.full((B.n,), 7.0, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
        V.mul_(y, Bc.T, dev(x))
        outs[runs] = y.cpu().numpy()
        Bc.release()
    ref = O.mul(R64, x.astype(np.float64), np.zeros(B.n), trans=True)
    got = outs["1"]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    if dtype == np.float64:
        assert np.array_equal(got[fin], ref[fin])
    else:
        assert rel(np.nan_to_num(got[fin], posinf=0, neginf=0), np.nan_to_num(ref[fin], posinf=0, neginf=0)) <= TOL32
    assert np.array_equal(outs["1"], outs["0"], equal_nan=True)


def test_row_runs_fallback(monkeypatch):
    """One stripe whose first two rows repeat an x row: not runs -> the bucket keeps run = 1."""
    monkeypatch.setenv("VBC_SLOT_PLANAR", "1")
    monkeypatch.setenv("VBC_SLOTS", "1")
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    base = V.synthetic.vbr_1dvbc(5000, 2000, 12000, 3, W=8, seed=3)
    B = expand_runs(base, 3, seed=4, break_one=True)
    assert B.info(trans=True)["planar_run"] == 1
    rng = np.random.default_rng(6)
    x = rng.uniform(-1, 1, B.m)
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert np.array_equal(y.cpu().numpy(), O.mul(ref_of(B), x, np.zeros(B.n), trans=True))


def test_fe3d_uses_runs():
    """The 3-dof stiffness stand-in (one stripe per node) is laid out with runs of 3."""
    B = V.synthetic.fe_stiffness_3d_1dvbc(30000, 300000)
    inf = B.info(trans=True)
    assert inf["planar_bins"] == 1 and inf["planar_run"] == 3


@pytest.mark.parametrize("P", ["2", "4", "8"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w,R", [(3, 3), (5, 1), (8, 2), (4, 1)])
def test_split_chunks(monkeypatch, P, dtype, w, R):
    """Split planar product (SlotBin::split): P waves per chunk, partials summed in LDS.  Random x
    within tolerance of the oracle (normwise, 1e-12 fp64 / 1e-5 fp32), alpha / beta, affine (natural
    order) and table-mapped (sorted) outputs; integer-valued data bit for bit."""
    if dtype == np.float32 and w == 4:
        pytest.skip("fp32 w = 4 is not planar")
    monkeypatch.setenv("VBC_PLANAR_SPLIT", P)
    monkeypatch.setenv("VBC_SLOTS", "1")
    rng = np.random.default_rng(int(P) * 100 + w)
    for sort in ("0", "2"):
        monkeypatch.setenv("VBC_SLOTS_SORT", sort)
        base = V.synthetic.vbr_1dvbc(4000, 700, 30000, w, W=8, dtype=dtype, seed=w + int(P))
        B = expand_runs(base, R, seed=w) if R > 1 else base
        inf = B.info(trans=True)
        assert inf["planar_bins"] == 1 and inf["planar_split"] == int(P) and inf["planar_run"] == R
        R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
        x = rng.uniform(-1, 1, B.m).astype(dtype)
        y0 = rng.uniform(-1, 1, B.n).astype(dtype)
        tol = TOL64 if dtype == np.float64 else TOL32
        for alpha, beta in ((1.0, 0.0), (-0.5, 3.0)):
            y = dev(y0.copy())
            V.mul_(y, B.T, dev(x), alpha, beta)
            ref = O.mul(R64, x.astype(np.float64), y0.astype(np.float64), alpha, beta, trans=True, ref_semantics=False)
            assert rel(y.cpu().numpy(), ref) <= tol, (sort, alpha)
        # integer-valued: every partial sum exact, so any summation order gives the oracle's bits
        Bi = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs,
                                 rng.integers(-50, 50, len(B.val)).astype(dtype))
        xi = rng.integers(-20, 20, B.m).astype(dtype)
        y = torch.zeros(B.n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
        V.mul_(y, Bi.T, dev(xi))
        refi = O.mul(O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, Bi.val.astype(np.float64)),
                     xi.astype(np.float64), np.zeros(B.n), trans=True)
        assert np.array_equal(y.cpu().numpy().astype(np.float64), refi)
        B.release()
        Bi.release()


def test_split_auto_small_matrix():
    """A one-width 3-dof operator of ct20stif's size (17443 stripes, 273 planar chunks: the rounds 1-3
    stand-in) picks the split product."""
    A = V.synthetic.fe_stiffness_3d(52329, 2600295, 3, np.float64)
    B = V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))
    inf = B.info(trans=True)
    assert inf["planar_bins"] >= 1 and inf["planar_split"] > 1
    x = np.random.default_rng(1).uniform(-1, 1, B.m)
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert rel(y.cpu().numpy(), O.mul(ref_of(B), x, np.zeros(B.n), trans=True)) <= TOL64


@pytest.mark.parametrize("sort", ["0", "2"])
@pytest.mark.parametrize("keys16", ["0", "1"])
@pytest.mark.parametrize("stage", ["0", "8"])
def test_pair_layout(monkeypatch, sort, keys16, stage):
    """Lane-pair planar layout (SlotBin::pair: fp64, 3-wide stripes, runs of 3): one 16-B gather per
    lane, DPP exchange, each column folded serially by one lane -> the oracle's bits, and the same
    bits as the plain planar layout (VBC_PLANAR_PAIR=0); alpha / beta; non-finite x."""
    monkeypatch.setenv("VBC_SLOTS", "1")
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    monkeypatch.setenv("VBC_SLOTS_SORT", sort)
    monkeypatch.setenv("VBC_SLOT_KEYS16", keys16)
    monkeypatch.setenv("VBC_SLOT_STAGE", stage)
    base = V.synthetic.vbr_1dvbc(9000, 4000, 30000, 3, W=8, seed=31)
    B = expand_runs(base, 3, seed=32)
    R = ref_of(B)
    rng = np.random.default_rng(33)
    x = rng.uniform(-1, 1, B.m)
    x[[4, 2001, 17000]] = [np.inf, np.nan, -np.inf]
    y0 = rng.uniform(-1, 1, B.n)
    outs = {}
    for pair in ("2", "0"):
        monkeypatch.setenv("VBC_PLANAR_PAIR", pair)
        Bc = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
        inf = Bc.info(trans=True)
        assert inf["planar_bins"] == 1 and inf["planar_run"] == 3 and inf["planar_pair"] == (pair == "2")
        y = torch.full((B.n,), 5.0, dtype=torch.float64, device=DEV)
        V.mul_(y, Bc.T, dev(x))
        outs[pair] = y.cpu().numpy()
        yb = dev(y0.copy())
        V.mul_(yb, Bc.T, dev(np.nan_to_num(x, posinf=1.0, neginf=-1.0, nan=0.5)), -0.5, 2.0)
        outs[pair + "ab"] = yb.cpu().numpy()
        Bc.release()
    ref = O.mul(R, x, np.zeros(B.n), trans=True)
    got = outs["2"]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert np.array_equal(got[fin], ref[fin])
    assert np.array_equal(outs["2"], outs["0"], equal_nan=True)
    xf = np.nan_to_num(x, posinf=1.0, neginf=-1.0, nan=0.5)
    refab = O.mul(R, xf, y0.copy(), -0.5, 2.0, trans=True, ref_semantics=False)
    assert rel(outs["2ab"], refab) <= TOL64
    assert np.array_equal(outs["2ab"], outs["0ab"])


def test_pair_auto_selection(monkeypatch):
    """Auto selection: long 3-run segments (ldoor-like, ~15 runs per stripe) take the pair layout, also
    as a blocked CSC (TrSpMV!); FE-3D's ~3 runs per stripe keep the plain planar layout (small
    matrices take the split product instead; kept out here)."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    B = V.synthetic.fe_stiffness_3d_1dvbc(60000, 600000)
    assert B.info(trans=True)["planar_pair"] == 0
    A = V.synthetic.fe_stiffness_3d(60000, 2_700_000, 3, np.float64).tocsc()
    A.sort_indices()
    C = V.SparseMatrixCSC(A)
    assert C.info(trans=True)["planar_pair"] == 1
    x = np.random.default_rng(4).uniform(-1, 1, A.shape[0])
    y = torch.zeros(A.shape[1], dtype=torch.float64, device=DEV)
    V.TrSpMV_(y, C, dev(x))
    assert np.array_equal(y.cpu().numpy(), O.trspmv(A, x, np.zeros(A.shape[1])))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_vbc2d_3x3_tiles_runs(monkeypatch, dtype):
    """SparseMatrixVBC{3,3} with 3x3 tiles (multiply_VBC.jl:93-147): B'x expands each tile into its
    three rows (constructors_VBC.jl:95-105), which are runs of 3 consecutive x rows -> the planar
    layout with row runs (fp64: lane pairs when forced).  Equals the oracle bit for bit in fp64
    (per-column serial order); both directions, alpha / beta."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    monkeypatch.setenv("VBC_SLOTS", "1")  # small and long-striped: auto would pick the merge layout
    import scipy.sparse as sp
    rng = np.random.default_rng(41)
    nb = 3000
    blocks = sp.random(nb, nb, density=0.004, random_state=rng, format="csr")
    A = sp.kron(blocks, np.ones((3, 3))).tocsc()
    A.data = rng.uniform(-1, 1, A.nnz)
    A = A.astype(dtype)
    B = V.SparseMatrixVBC[3, 3](A, V.AlternatingPacker(V.EquiChunker(3), V.EquiChunker(3)))
    R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    for pair in ("0", "2"):
        if pair == "2" and dtype == np.float32:
            continue
        monkeypatch.setenv("VBC_PLANAR_PAIR", pair)
        Bc = V.SparseMatrixVBC(B.U, B.W, B.m, B.n, B.Pi, B.Phi, B.pos, B.idx, B.ofs, B.val)
        inf = Bc.info(trans=True)
        assert inf["planar_bins"] >= 1 and inf["planar_run"] == 3
        assert inf["planar_pair"] == (1 if pair == "2" else 0)
        x = rng.uniform(-1, 1, B.m).astype(dtype)
        y = torch.zeros(B.n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
        V.mul_(y, Bc.T, dev(x))
        ref = O.mul(R, x.astype(np.float64), np.zeros(B.n), trans=True)
        if dtype == np.float64:
            assert np.array_equal(y.cpu().numpy(), ref)
        else:
            assert rel(y.cpu().numpy(), ref) <= TOL32
        y0 = rng.uniform(-1, 1, B.n).astype(dtype)
        y = dev(y0.copy())
        V.mul_(y, Bc.T, dev(x), 2.0, -1.0)
        refab = O.mul(R, x.astype(np.float64), y0.astype(np.float64), 2.0, -1.0, trans=True, ref_semantics=False)
        assert rel(y.cpu().numpy(), refab) <= (TOL64 if dtype == np.float64 else TOL32)
        xf = rng.uniform(-1, 1, B.n).astype(dtype)
        yf = torch.zeros(B.m, dtype=y.dtype, device=DEV)
        V.mul_(yf, Bc, dev(xf))
        assert rel(yf.cpu().numpy(), O.mul(R, xf.astype(np.float64), np.zeros(B.m))) <= (TOL64 if dtype == np.float64 else TOL32)
        Bc.release()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w,R", [(3, 3), (2, 2), (2, 3), (3, 2), (4, 3), (4, 2)])
@pytest.mark.parametrize("stage", ["0", "8"])
def test_forward_row_runs(monkeypatch, dtype, w, R, stage):
    """Forward mul!(y, B, x) with node-blocked rows (R consecutive output rows with identical stripe
    lists): the planar forward layout, one w-wide x gather per R rows.  Against the oracle's forward
    product (multiply_1DVBC.jl:9-83) within tolerance, alpha / beta, quirks (alpha dropped); integer
    values bit for bit; the layout falls back when one row breaks its run."""
    monkeypatch.setenv("VBC_SLOT_STAGE", stage)
    rng = np.random.default_rng(100 * w + R)
    base = V.synthetic.vbr_1dvbc(6000, 1500, 30000, w, W=8, dtype=dtype, seed=w + R)
    # forward runs: rows of the TRANSPOSE (stripes of A^T) in runs -> build B from a blocked matrix
    At = sp_blocked(base, R, rng, dtype)
    B = V.SparseMatrix1DVBC[8](At, V.EquiChunker(w))
    assert B.info(trans=False)["fwd_run"] == R
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    tol = TOL64 if dtype == np.float64 else TOL32
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    for alpha, beta in ((1.0, 0.0), (0.5, -1.5)):
        x = rng.uniform(-1, 1, B.n).astype(dtype)
        y0 = rng.uniform(-1, 1, B.m).astype(dtype)
        y = dev(y0.copy())
        V.mul_(y, B, dev(x), alpha, beta)
        ref = O.mul(R64, x.astype(np.float64), y0.astype(np.float64), alpha, beta, ref_semantics=False)
        assert rel(y.cpu().numpy(), ref) <= tol, (alpha, beta)
    y = dev(y0.copy())
    V.mul_(y, B, dev(x), 3.0, 0.0, quirks=True)  # forward quirks: alpha dropped
    assert rel(y.cpu().numpy(), O.mul(R64, x.astype(np.float64), np.zeros(B.m))) <= tol
    Bi = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs,
                             rng.integers(-30, 30, len(B.val)).astype(dtype))
    xi = rng.integers(-20, 20, B.n).astype(dtype)
    yi = torch.zeros(B.m, dtype=tdt, device=DEV)
    V.mul_(yi, Bi, dev(xi))
    Ri = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, Bi.val.astype(np.float64))
    assert np.array_equal(yi.cpu().numpy().astype(np.float64), O.mul(Ri, xi.astype(np.float64), np.zeros(B.m)))


def sp_blocked(base, R, rng, dtype):
    """A CSC matrix whose rows come in runs of R with identical patterns: row r of `base`'s pattern
    (as a CSC of its m x n shape) expanded into R rows with fresh values."""
    import scipy.sparse as sp
    D = sp.csr_matrix(base.to_csc() if hasattr(base, "to_csc") else _to_csc(base))
    Dk = sp.kron(D, np.ones((R, 1))).tocsc()
    Dk.data = rng.uniform(-1, 1, Dk.nnz).astype(dtype)
    return Dk.astype(dtype)


def _to_csc(B):
    import scipy.sparse as sp
    rows, cols, vals = [], [], []
    for l in range(len(B.Phi)):
        j0, w = B.Phi.spl[l] - 1, B.Phi.spl[l + 1] - B.Phi.spl[l]
        for k, Q in enumerate(range(B.pos[l] - 1, B.pos[l + 1] - 1)):
            for c in range(w):
                rows.append(B.idx[Q] - 1)
                cols.append(j0 + c)
                vals.append(1.0)
    return sp.csc_matrix((vals, (rows, cols)), shape=(B.m, B.n))


@pytest.mark.parametrize("P", ["2", "4", "8"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w,R", [(3, 3), (2, 2), (4, 3)])
def test_forward_split(monkeypatch, P, dtype, w, R):
    """Split planar forward product (spmv_planar_fwd_split, planar_mask bit 3): P waves per chunk of
    node-blocked output rows, partial sums met in LDS.  Random x within tolerance of the oracle's
    forward product (multiply_1DVBC.jl:9-83), alpha / beta, quirks; integer values bit for bit (any
    summation order is exact)."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", P)
    monkeypatch.setenv("VBC_SLOTS_PAD", "100")  # keep the natural order (the split product needs it)
    rng = np.random.default_rng(10 * w + R + int(P))
    base = V.synthetic.vbr_1dvbc(3000, 900, 20000, w, W=8, dtype=dtype, seed=w * R)
    B = V.SparseMatrix1DVBC[8](sp_blocked(base, R, rng, dtype), V.EquiChunker(w))
    inf = B.info(trans=False)
    assert inf["fwd_run"] == R and inf["planar_mask"] & 8
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    tol = TOL64 if dtype == np.float64 else TOL32
    for alpha, beta in ((1.0, 0.0), (0.5, -1.5)):
        x = rng.uniform(-1, 1, B.n).astype(dtype)
        y0 = rng.uniform(-1, 1, B.m).astype(dtype)
        y = dev(y0.copy())
        V.mul_(y, B, dev(x), alpha, beta)
        ref = O.mul(R64, x.astype(np.float64), y0.astype(np.float64), alpha, beta, ref_semantics=False)
        assert rel(y.cpu().numpy(), ref) <= tol, (alpha, beta)
    y = dev(y0.copy())
    V.mul_(y, B, dev(x), 3.0, 0.0, quirks=True)
    assert rel(y.cpu().numpy(), O.mul(R64, x.astype(np.float64), np.zeros(B.m))) <= tol
    Bi = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs,
                             rng.integers(-30, 30, len(B.val)).astype(dtype))
    xi = rng.integers(-20, 20, B.n).astype(dtype)
    yi = torch.zeros(B.m, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
    V.mul_(yi, Bi, dev(xi))
    Ri = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, Bi.val.astype(np.float64))
    assert np.array_equal(yi.cpu().numpy().astype(np.float64), O.mul(Ri, xi.astype(np.float64), np.zeros(B.m)))


def test_forward_split_auto_small_matrix(monkeypatch):
    """A one-width 3-dof operator of ct20stif's size (273 chunks of node rows: the rounds 1-3 stand-in)
    picks the split forward product by default and matches the oracle; VBC_CREATE_SERIAL
    (serial=True) keeps one wave per chunk."""
    A = V.synthetic.fe_stiffness_3d(52329, 2600295, 3, np.float64)
    B = V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))
    assert B.info(trans=False)["planar_mask"] & 8
    x = np.random.default_rng(2).uniform(-1, 1, B.n)
    y = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(x))
    ref = O.mul(ref_of(B), x, np.zeros(B.m))
    assert rel(y.cpu().numpy(), ref) <= TOL64
    B.release()
    B.serial = True
    assert not B.info(trans=False)["planar_mask"] & 8
    V.mul_(y, B, dev(x))
    assert rel(y.cpu().numpy(), ref) <= TOL64


def test_forward_row_runs_fallback():
    """One row outside its run's pattern: the forward product keeps the row-by-row layout."""
    import scipy.sparse as sp
    rng = np.random.default_rng(7)
    A = sp.kron(sp.random(2000, 2000, density=0.003, random_state=rng, format="csr"), np.ones((3, 1))).tocsc()
    A = A.tolil()
    A[4, 1999] = 1.0  # row 4 (run 1) gains a column its run-mates lack
    A = A.tocsc()
    B = V.SparseMatrix1DVBC[8](A, V.EquiChunker(3))
    assert B.info(trans=False)["fwd_run"] == 1
    x = rng.uniform(-1, 1, B.n)
    y = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(x))
    assert rel(y.cpu().numpy(), A @ x) <= TOL64


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w,R", [(3, 3), (5, 1), (6, 3)])
@pytest.mark.parametrize("keys16,win", [("0", "1"), ("1", "2"), ("1", "3")])
def test_masked_chunk_order(monkeypatch, dtype, w, R, keys16, win):
    """Masked planar layout (SlotBin::mask): each natural chunk's 64 stripes in decreasing length
    order, dead lanes of a chunk row reading lane 0's lines and folding nothing.  Every stripe still
    folds its rows serially in stored order, so the result equals the length-sorted layout
    (VBC_PLANAR_MASK=0) bit for bit and, in fp64, the oracle bit for bit -- Inf/NaN in x land where
    the reference's loop puts them; alpha / beta."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    monkeypatch.setenv("VBC_PLANAR_PAIR", "0")
    monkeypatch.setenv("VBC_SLOT_KEYS16", keys16)
    monkeypatch.setenv("VBC_MASK_WINDOW", win)  # stripes sorted by length inside windows of `win` chunks
    base = V.synthetic.vbr_1dvbc(7000, 5000, 20000, w, W=8, dtype=dtype, seed=71 + w)
    B = expand_runs(base, R, seed=72) if R > 1 else base
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    rng = np.random.default_rng(73)
    x = rng.uniform(-1, 1, B.m).astype(dtype)
    x[[3, 1500, B.m - 2]] = [np.inf, np.nan, -np.inf]
    xf = np.nan_to_num(x, posinf=1.0, neginf=-1.0, nan=0.5)
    y0 = rng.uniform(-1, 1, B.n).astype(dtype)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    outs = {}
    for mk in ("1", "0"):
        monkeypatch.setenv("VBC_PLANAR_MASK", mk)
        Bc = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
        inf = Bc.info(trans=True)
        assert inf["planar_bins"] == 1 and inf["planar_run"] == R and inf["planar_mask"] == int(mk)
        y = torch.full((B.n,), 7.0, dtype=tdt, device=DEV)
        V.mul_(y, Bc.T, dev(x))
        outs[mk] = y.cpu().numpy()
        yb = dev(y0.copy())
        V.mul_(yb, Bc.T, dev(xf), 1.5, -0.5)
        outs[mk + "ab"] = yb.cpu().numpy()
        Bc.release()
    assert np.array_equal(outs["1"], outs["0"], equal_nan=True)
    assert np.array_equal(outs["1ab"], outs["0ab"])
    ref = O.mul(R64, x.astype(np.float64), np.zeros(B.n), trans=True)
    got = outs["1"].astype(np.float64)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    if dtype == np.float64:
        assert np.array_equal(got[fin], ref[fin])
    else:
        assert np.array_equal(np.isinf(got[fin]), np.isinf(ref[fin]))
    refab = O.mul(R64, xf.astype(np.float64), y0.astype(np.float64), 1.5, -0.5, trans=True, ref_semantics=False)
    assert rel(outs["1ab"].astype(np.float64), refab) <= (TOL64 if dtype == np.float64 else TOL32)


@pytest.mark.parametrize("keys16", ["0", "1"])
@pytest.mark.parametrize("win", ["1", "2"])
def test_masked_pair_layout(monkeypatch, keys16, win):
    """Lane-pair layout (fp64, 3-wide stripes, runs of 3) in the masked chunk-local order: padding
    stripe slots of a run-row read pair 0's lines and fold nothing.  Same bits as the unmasked pair
    kernel on the same order (VBC_PLANAR_MASK_PAIR=0), as the plain planar layout, and as the oracle;
    Inf/NaN in x; alpha / beta."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    monkeypatch.setenv("VBC_PLANAR_PAIR", "2")
    monkeypatch.setenv("VBC_SLOT_KEYS16", keys16)
    monkeypatch.setenv("VBC_MASK_WINDOW", win)
    base = V.synthetic.vbr_1dvbc(9000, 4000, 16000, 3, W=8, seed=81)  # ~4 runs per stripe: pads naturally
    B = expand_runs(base, 3, seed=82)
    R = ref_of(B)
    rng = np.random.default_rng(83)
    x = rng.uniform(-1, 1, B.m)
    x[[5, 3001, 20000]] = [np.inf, np.nan, -np.inf]
    xf = np.nan_to_num(x, posinf=1.0, neginf=-1.0, nan=0.5)
    y0 = rng.uniform(-1, 1, B.n)
    outs = {}
    for tag, env in (("mask", {}), ("nomask", {"VBC_PLANAR_MASK_PAIR": "0"}), ("plain", {"VBC_PLANAR_PAIR": "0"})):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        Bc = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
        inf = Bc.info(trans=True)
        assert inf["planar_pair"] == (tag != "plain") and inf["planar_mask"] == (tag != "nomask")
        y = torch.full((B.n,), 3.0, dtype=torch.float64, device=DEV)
        V.mul_(y, Bc.T, dev(x))
        outs[tag] = y.cpu().numpy()
        yb = dev(y0.copy())
        V.mul_(yb, Bc.T, dev(xf), 0.75, -1.25)
        outs[tag + "ab"] = yb.cpu().numpy()
        Bc.release()
        for k in env:
            monkeypatch.delenv(k)
    ref = O.mul(R, x, np.zeros(B.n), trans=True)
    got = outs["mask"]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert np.array_equal(got[fin], ref[fin])
    for t in ("nomask", "plain"):
        assert np.array_equal(outs[t], got, equal_nan=True)
        assert np.array_equal(outs[t + "ab"], outs["maskab"])
    refab = O.mul(R, xf, y0.copy(), 0.75, -1.25, trans=True, ref_semantics=False)
    assert rel(outs["maskab"], refab) <= TOL64


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w,R", [(3, 3), (2, 2)])
def test_forward_masked_order(monkeypatch, dtype, w, R):
    """Forward planar product with row runs in the masked chunk-local order (rows with uneven block
    counts): same bits as the length-sorted layout (VBC_PLANAR_MASK=0) -- each output row still sums
    its blocks in stripe order -- and the oracle's forward product (multiply_1DVBC.jl:9-83); integer
    data bit for bit."""
    rng = np.random.default_rng(90 + w + R)
    base = V.synthetic.vbr_1dvbc(6000, 1500, 9000, w, W=8, dtype=dtype, seed=91 + w)
    At = sp_blocked(base, R, rng, dtype)
    B = V.SparseMatrix1DVBC[8](At, V.EquiChunker(w))
    vi = rng.integers(-30, 30, len(B.val)).astype(dtype)
    x = rng.uniform(-1, 1, B.n).astype(dtype)
    xi = rng.integers(-20, 20, B.n).astype(dtype)
    tdt = torch.float64 if dtype == np.float64 else torch.float32
    outs = {}
    for mk in ("1", "0"):
        monkeypatch.setenv("VBC_PLANAR_MASK", mk)
        Bc = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
        inf = Bc.info(trans=False)
        assert ((inf["planar_mask"] >> 1) & 1) == int(mk)
        if mk == "1":
            assert inf["fwd_run"] == R
        runs0 = inf["fwd_run"] == R  # mk = 0: the sorted run layout, or the row-by-row fallback
        y = torch.zeros(B.m, dtype=tdt, device=DEV)
        V.mul_(y, Bc, dev(x))
        outs[mk] = y.cpu().numpy()
        Bc.release()
        Bi = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, vi)
        yi = torch.zeros(B.m, dtype=tdt, device=DEV)
        V.mul_(yi, Bi, dev(xi))
        outs[mk + "i"] = yi.cpu().numpy()
        Bi.release()
    if runs0:  # same per-row block order and per-block dot product
        assert np.array_equal(outs["1"], outs["0"])
    assert np.array_equal(outs["1i"], outs["0i"])
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    assert rel(outs["0"].astype(np.float64), O.mul(R64, x.astype(np.float64), np.zeros(B.m))) <= \
        (TOL64 if dtype == np.float64 else TOL32)
    assert rel(outs["1"].astype(np.float64), O.mul(R64, x.astype(np.float64), np.zeros(B.m))) <= \
        (TOL64 if dtype == np.float64 else TOL32)
    Ri = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, vi.astype(np.float64))
    assert np.array_equal(outs["1i"].astype(np.float64), O.mul(Ri, xi.astype(np.float64), np.zeros(B.m)))


def test_small_mixed_widths_fused_split(golden, monkeypatch):
    """A small matrix with several width buckets (the ct20stif stand-in's strict stripes are 1..6 wide,
    calibrated to src/ref.out) runs every bucket planar and split, in ONE launch (vbc_info planar_mask
    bit 5): the product matches the oracle (the P slices reorder a chunk's sum: normwise 1e-12),
    bit-for-bit on one-hot probes of the reference corpus cut into mixed widths, with non-finite x where
    the reference puts it, alpha / beta, fp32; VBC_SMALL_FUSE=0 and serial=True keep the unfused
    layouts and the oracle's bits."""
    import bench
    B = bench.build_matrix("ct20stif", np.float64)
    inf = B.info(trans=True)
    assert inf["planar_mask"] & 32 and inf["planar_split"] > 1 and inf["bins_t"] == 0
    rng = np.random.default_rng(21)
    R = ref_of(B)
    for alpha, beta in ((1.0, 0.0), (0.5, -1.5)):
        x = rng.uniform(-1, 1, B.m)
        y0 = rng.uniform(-1, 1, B.n)
        y = dev(y0.copy())
        V.mul_(y, B.T, dev(x), alpha, beta)
        ref = O.mul(R, x, y0.copy(), alpha, beta, trans=True, ref_semantics=False)
        assert rel(y.cpu().numpy(), ref) <= TOL64, (alpha, beta)
    x = rng.uniform(-1, 1, B.m)
    x[[3, 999]] = [np.inf, np.nan]
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    ref = O.mul(R, x, np.zeros(B.n), trans=True)
    got = y.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert rel(got[fin], ref[fin]) <= TOL64
    B.serial = True  # VBC_CREATE_SERIAL: no split, the oracle's bits
    yS = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    x = rng.uniform(-1, 1, B.m)
    V.mul_(yS, B.T, dev(x))
    assert not B.info(trans=True)["planar_mask"] & 32
    assert np.array_equal(yS.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True))
    B32 = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val.astype(np.float32))
    assert B32.info(trans=True)["planar_mask"] & 32
    x32 = x.astype(np.float32)
    y32 = torch.zeros(B.n, dtype=torch.float32, device=DEV)
    V.mul_(y32, B32.T, dev(x32))
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B32.val.astype(np.float64))
    assert rel(y32.cpu().numpy(), O.mul(R64, x32.astype(np.float64), np.zeros(B.n), trans=True)) <= TOL32
    # one-hot probes (runtests.jl:42-53, exact) on the corpus cut into mixed widths 1..8 (P forced: the
    # corpus' chunks are too short for the automatic rule to split them)
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "4")
    seen = 0
    for key, g in golden.items():
        A = g["A"]
        n = A.shape[1]
        w, tot = [], 0
        while tot < n:
            w.append(min(len(w) % 8 + 1, n - tot))
            tot += w[-1]
        Bm = V.SparseMatrix1DVBC[8](A, V.SplitPartition(np.concatenate([[1], 1 + np.cumsum(w)])))
        seen += bool(Bm.info(trans=True)["planar_mask"] & 32)
        one_hot_probes(Bm, A)
    assert seen > 0


def test_fused_split_runs_with_holes_nonfinite(monkeypatch):
    """Runs with holes (SlotBin::holes): rows that almost come in node runs of 3 are padded to whole
    runs inside the fused small split; a padded row's x is taken as 0, so a NaN / Inf in x at a row a
    stripe does NOT store never reaches that stripe's outputs (the reference only visits stored rows,
    multiply_1DVBC.jl:101-104), and the stored rows fold in their order (bit-exact on integer data)."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "4")
    rng = np.random.default_rng(44)
    N, L = 400, 300
    widths = np.where(np.arange(L) % 2 == 0, 1, 2)  # two width buckets: the fused path
    rows, cnt = [], []
    for l in range(L):
        nodes = np.sort(rng.choice(N, 12, replace=False))
        r = (nodes[:, None] * 3 + np.arange(3)[None, :]).reshape(-1)
        if l % 5 == 0:  # every fifth stripe misses one row of one of its runs: a hole
            r = np.delete(r, rng.integers(0, len(r)))
        rows.append(r)
        cnt.append(len(r))
    cnt = np.array(cnt)
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)])
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * widths)])
    spl = np.concatenate([[1], 1 + np.cumsum(widths)])
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + 8)
    val[:nv] = rng.integers(-8, 9, nv)
    B = V.SparseMatrix1DVBC(8, 3 * N, int(spl[-1] - 1), V.SplitPartition(spl), pos, np.concatenate(rows) + 1, ofs, val)
    inf = B.info(trans=True)
    assert inf["planar_mask"] & 32 and inf["planar_run"] == 3
    R = ref_of(B)
    x = rng.integers(-8, 9, B.m).astype(np.float64)
    y = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert np.array_equal(y.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True))  # integer data: exact
    stored = set(np.concatenate(rows).tolist())
    holes = [r for l in range(0, L, 5) for r in range(3 * (rows[l][0] // 3), 3 * (rows[l][-1] // 3) + 3)
             if r not in set(rows[l].tolist()) and (r // 3) in set((rows[l] // 3).tolist())]
    assert holes
    x[holes[0]] = np.nan
    x[holes[-1]] = np.inf
    V.mul_(y, B.T, dev(x))
    ref = O.mul(R, x, np.zeros(B.n), trans=True)
    got = y.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert np.array_equal(got[fin], ref[fin])


def _holey_matrix(rng, N, L, widths, m=None, last_row_every=0):
    """Stripes of 12 node runs of 3 rows each, every fifth missing one row (a hole); m rows (default 3 N).
    last_row_every > 0: every such stripe also stores row m - 1 (m % 3 != 0: a run past the operand)."""
    m = 3 * N if m is None else m
    rows = []
    for l in range(L):
        nodes = np.sort(rng.choice(N, 12, replace=False))
        r = (nodes[:, None] * 3 + np.arange(3)[None, :]).reshape(-1)
        if l % 5 == 0:
            r = np.delete(r, rng.integers(0, len(r)))
        if last_row_every and l % last_row_every == 0:
            r = np.append(r, m - 1)
        rows.append(r)
    cnt = np.array([len(r) for r in rows])
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)])
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * widths)])
    spl = np.concatenate([[1], 1 + np.cumsum(widths)])
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + 8)
    val[:nv] = rng.integers(-8, 9, nv)
    return V.SparseMatrix1DVBC(8, m, int(spl[-1] - 1), V.SplitPartition(spl), pos, np.concatenate(rows) + 1, ofs, val)


@pytest.mark.parametrize("env", [{"VBC_PLANAR_LANES": "1"}, {"VBC_SIDE_FUSE": "1"},
                                 {"VBC_PLANAR_LANES": "1", "VBC_SIDE_FUSE": "1"}])
def test_holey_rows_outside_the_fused_split(monkeypatch, env):
    """runs with holes are built only for the buckets of the fused launch, whose bins run
    the split product; a side bucket (VBC_SIDE_FUSE=1 leaves the dominant width out of the launch) and a
    lane-stream layout (VBC_PLANAR_LANES=1) keep the plain rows.  Exact on integer data; create succeeds."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "4")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(47)
    L = 900
    # dominant 3-wide bucket (>= 80 % of the stripes) beside 1- and 2-wide side stripes
    widths = np.where(np.arange(L) % 10 == 0, 1, np.where(np.arange(L) % 10 == 5, 2, 3))
    B = _holey_matrix(rng, 500, L, widths)
    R = ref_of(B)
    x = rng.integers(-8, 9, B.m).astype(np.float64)
    y = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert np.array_equal(y.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True))
    xr = rng.uniform(-1, 1, B.m)
    V.mul_(y, B.T, dev(xr))
    assert rel(y.cpu().numpy(), O.mul(R, xr, np.zeros(B.n), trans=True)) <= TOL64


def test_holey_runs_never_pass_the_operand(monkeypatch):
    """a run of R rows is gathered by one R-wide load, so hole_runs rejects an R whose
    last group would run past m (m % 3 != 0, the last row stored): no load beyond x, exact result."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "4")
    rng = np.random.default_rng(48)
    L = 300
    widths = np.where(np.arange(L) % 2 == 0, 1, 2)
    for m in (3 * 400 + 1, 3 * 400 + 2):
        B = _holey_matrix(rng, 400, L, widths, m=m, last_row_every=7)
        assert B.info(trans=True)["planar_mask"] & 32
        R = ref_of(B)
        x = rng.integers(-8, 9, B.m).astype(np.float64)
        y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, dev(x))
        assert np.array_equal(y.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True)), m
        xn = x.copy()
        xn[-1] = np.nan  # the stored last row: NaN reaches exactly the stripes storing it
        V.mul_(y, B.T, dev(xn))
        ref = O.mul(R, xn, np.zeros(B.n), trans=True)
        got = y.cpu().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        assert np.array_equal(got[~np.isnan(ref)], ref[~np.isnan(ref)])


def _node_stripes(rng, N, L, widths, nodes_of, hole_every):
    """Stripes of node runs (rows 3 k .. 3 k + 2 of each chosen node), every hole_every-th missing one row."""
    rows = []
    for l in range(L):
        nodes = np.sort(rng.choice(N, nodes_of(l), replace=False))
        r = (nodes[:, None] * 3 + np.arange(3)[None, :]).reshape(-1)
        if l % hole_every == 0:
            r = np.delete(r, rng.integers(0, len(r)))
        rows.append(r)
    cnt = np.array([len(r) for r in rows])
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)])
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * widths)])
    spl = np.concatenate([[1], 1 + np.cumsum(widths)])
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + 8)
    val[:nv] = rng.integers(-8, 9, nv)
    B = V.SparseMatrix1DVBC(8, 3 * N, int(spl[-1] - 1), V.SplitPartition(spl), pos, np.concatenate(rows) + 1, ofs, val)
    return B, rows


def test_fused_split_long_stripes_cut(monkeypatch):
    """Long stripes of the fused split (SlotBin::ks, vbc_info planar_mask bit 6): a stripe whose rows x
    width exceed 1.5x the mean chunk's is cut into 2 / 4 parts of whole runs, laid in the lanes of one
    chunk and summed across the lanes before the store.  Exact on integer data (runs with holes, a NaN /
    Inf at rows a long stripe does not store), the same bits on every call, and VBC_KSPLIT=0 keeps every
    stripe whole with the same exact result."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "4")
    rng = np.random.default_rng(45)
    N, L = 600, 400
    widths = 1 + np.arange(L) % 3
    B, rows = _node_stripes(rng, N, L, widths, lambda l: 80 if l % 29 == 0 else (30 if l % 13 == 0 else 8), 7)
    inf = B.info(trans=True)
    assert inf["planar_mask"] & 32 and inf["planar_mask"] & 64 and inf["planar_run"] == 3
    R = ref_of(B)
    x = rng.integers(-8, 9, B.m).astype(np.float64)
    ref = O.mul(R, x, np.zeros(B.n), trans=True)
    y = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert np.array_equal(y.cpu().numpy(), ref)
    y2 = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    xr = rng.uniform(-1, 1, B.m)
    V.mul_(y, B.T, dev(xr))
    V.mul_(y2, B.T, dev(xr))
    assert np.array_equal(y.cpu().numpy(), y2.cpu().numpy())  # deterministic
    assert rel(y.cpu().numpy(), O.mul(R, xr, np.zeros(B.n), trans=True)) <= TOL64
    # a NaN / Inf in a hole of a long stripe's run reaches nothing that stripe writes
    long_holes = [r for l in range(0, L, 7 * 29) for r in range(3 * (rows[l][0] // 3), 3 * (rows[l][-1] // 3) + 3)
                  if r not in set(rows[l].tolist()) and (r // 3) in set((rows[l] // 3).tolist())]
    assert long_holes
    xn = x.copy()
    xn[long_holes[0]] = np.nan
    xn[long_holes[-1]] = np.inf
    V.mul_(y, B.T, dev(xn))
    refn = O.mul(R, xn, np.zeros(B.n), trans=True)
    got = y.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(refn)) and np.array_equal(np.isinf(got), np.isinf(refn))
    assert np.array_equal(got[np.isfinite(refn)], refn[np.isfinite(refn)])
    # alpha / beta on the cut stripes
    y0 = rng.integers(-8, 9, B.n).astype(np.float64)
    yb = dev(y0.copy())
    V.mul_(yb, B.T, dev(x), 2.0, -1.0)
    assert np.array_equal(yb.cpu().numpy(), O.mul(R, x, y0.copy(), 2.0, -1.0, trans=True, ref_semantics=False))
    monkeypatch.setenv("VBC_KSPLIT", "0")
    Bw = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
    assert Bw.info(trans=True)["planar_mask"] & 32 and not Bw.info(trans=True)["planar_mask"] & 64
    yw = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(yw, Bw.T, dev(x))
    assert np.array_equal(yw.cpu().numpy(), ref)


def test_fused_split_min_blocks_partition():
    """The ct20stif stand-in under the reference's 'min blocks' partition (bin/test_table.jl:67-69: widths
    1..8, its widest stripes the fullest) cuts its long stripes (planar_mask bit 6) and matches the oracle
    in fp64 and fp32."""
    A = V.synthetic.standin("Boeing/ct20stif", np.float64)
    meth = V.DynamicTotalChunker(V.ConstrainedCost(V.model_SparseMatrix1DVBC_blocks(), V.VertexCount(), 8))
    B = V.SparseMatrix1DVBC[8](A, meth)
    inf = B.info(trans=True)
    assert inf["planar_mask"] & 32 and inf["planar_mask"] & 64
    rng = np.random.default_rng(46)
    R = ref_of(B)
    x = rng.uniform(-1, 1, B.m)
    y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert rel(y.cpu().numpy(), O.mul(R, x, np.zeros(B.n), trans=True)) <= TOL64
    B32 = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val.astype(np.float32))
    x32 = x.astype(np.float32)
    y32 = torch.zeros(B.n, dtype=torch.float32, device=DEV)
    V.mul_(y32, B32.T, dev(x32))
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B32.val.astype(np.float64))
    assert rel(y32.cpu().numpy(), O.mul(R64, x32.astype(np.float64), np.zeros(B.n), trans=True)) <= TOL32


def test_fused_side_buckets_beside_a_dominant_width():
    """A large matrix whose chunks overflow one fused launch, with one dominant width (300,000 3-wide
    stripes) and small side buckets (1-, 4- and 5-wide stripes, as a time-model partition leaves them):
    the dominant bucket keeps its own planar layout and the side buckets run as one fused split launch
    (planar_mask bit 5 with planar_bins >= 2); the product matches the oracle, fp64 and fp32."""
    L = 301500
    widths = np.full(L, 3)
    widths[100::601] = 4
    widths[200::601] = 5
    widths[300::601] = 1
    for dtype, tol in ((np.float64, TOL64), (np.float32, TOL32)):
        B = V.synthetic.vbr_1dvbc(200000, L, 6 * L, widths, W=8, dtype=dtype, seed=48)
        inf = B.info(trans=True)
        assert inf["planar_mask"] & 32 and inf["planar_bins"] >= 2, inf
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
        x = np.random.default_rng(49).uniform(-1, 1, B.m).astype(dtype)
        y = torch.zeros(B.n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
        V.mul_(y, B.T, dev(x))
        assert rel(y.cpu().numpy(), O.mul(R, x.astype(np.float64), np.zeros(B.n), trans=True)) <= tol


def test_forward_mixed_widths_on_transposed_layout(monkeypatch):
    """B·x of a matrix whose stripes have several widths (the ct20stif stand-in's strict stripes, 1..6
    wide) runs as the transposed product of C = Bᵀ (vbc_info planar_mask bit 8: C's stripes are B's row
    groups, one fused launch): it matches the oracle's forward product (normwise 1e-12) with alpha /
    beta, a NaN / Inf in x reaches exactly the rows the reference's stripes touch, fp32 agrees at 1e-5,
    and VBC_FWD_T=0 (the per-width forward launches) and serial=True give the same result."""
    import bench
    B = bench.build_matrix("ct20stif", np.float64)
    assert B.info(trans=False)["planar_mask"] & 256
    R = ref_of(B)
    rng = np.random.default_rng(50)
    x = rng.uniform(-1, 1, B.n)
    y0 = rng.uniform(-1, 1, B.m)
    for alpha, beta in ((1.0, 0.0), (0.5, -1.5)):
        y = dev(y0.copy())
        V.mul_(y, B, dev(x), alpha, beta)
        ref = O.mul(R, x, y0.copy(), alpha, beta, trans=False, ref_semantics=False)
        assert rel(y.cpu().numpy(), ref) <= TOL64, (alpha, beta)
    xn = x.copy()
    xn[[7, 4001]] = [np.nan, np.inf]
    y = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(xn))
    ref = O.mul(R, xn, np.zeros(B.m), trans=False)
    got = y.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isinf(got), np.isinf(ref))
    assert rel(got[np.isfinite(ref)], ref[np.isfinite(ref)]) <= TOL64
    yt = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(yt, B, dev(x))
    monkeypatch.setenv("VBC_FWD_T", "0")
    Bw = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
    assert not Bw.info(trans=False)["planar_mask"] & 256
    yw = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(yw, Bw, dev(x))
    assert rel(yw.cpu().numpy(), yt.cpu().numpy()) <= TOL64
    monkeypatch.delenv("VBC_FWD_T")
    B32 = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val.astype(np.float32))
    y32 = torch.zeros(B.m, dtype=torch.float32, device=DEV)
    V.mul_(y32, B32, dev(x.astype(np.float32)))
    R64 = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B32.val.astype(np.float64))
    assert rel(y32.cpu().numpy(), O.mul(R64, x.astype(np.float32).astype(np.float64), np.zeros(B.m), trans=False)) <= TOL32


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_column_pieces_side_stripes(dtype, monkeypatch):
    """One dominant width (3) with a few 6-wide side stripes (the ldoor stand-in's 'min memory' shape):
    the side stripes run as pairs of 3-wide column pieces in the dominant bucket (one planar bin
    instead of two), bitwise equal to VBC_COLSPLIT=0 and to the oracle in the reference's serial order."""
    L = 60000
    widths = np.full(L, 3)
    widths[7::997] = 6
    widths[11::1999] = 9
    B = V.synthetic.vbr_1dvbc(120000, L, 8 * L, widths, W=9, dtype=dtype, seed=71)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
    x = np.random.default_rng(72).uniform(-1, 1, B.m).astype(dtype)
    want = O.mul(R, x.astype(np.float64), np.zeros(B.n), trans=True)
    ys, bins = [], []
    for cs in ("1", "0"):
        monkeypatch.setenv("VBC_COLSPLIT", cs)
        Bc = V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)
        Bc.serial = True
        bins.append(Bc.info(trans=True)["planar_bins"])
        y = torch.zeros(B.n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
        V.mul_(y, Bc.T, dev(x))
        ys.append(y.cpu().numpy())
        assert rel(ys[-1], want) <= (TOL64 if dtype == np.float64 else TOL32)
    assert bins[0] < bins[1], bins
    assert np.array_equal(ys[0], ys[1])


def test_ldoor_min_blocks_and_min_memory_partitions():
    """The ldoor stand-in under the reference's 'min blocks' partition (150,920 6-wide stripes beside 3-, 7-
    and 8-wide ones; fp64 its dominant bucket is merge-bound, so it is fused with the side buckets: one
    fused split launch, planar_mask bit 5) and 'min memory' (32 6-wide stripes beside 317,337 3-wide ones,
    run as 3-wide column pieces: one planar bin): both match the oracle (bin/test_table.jl:67-69)."""
    A = V.synthetic.standin("GHS_psdef/ldoor", np.float64).T.tocsc()
    lim = lambda mdl: V.ConstrainedCost(mdl, V.VertexCount(), 8)
    rng = np.random.default_rng(81)
    for name, meth in (("blocks", V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks()))),
                       ("memory", V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_memory(np.float64, np.int64))))):
        B = V.SparseMatrix1DVBC[8](A, meth)
        inf = B.info(trans=True)
        if name == "blocks":
            assert inf["planar_mask"] & 32, inf
        else:
            assert inf["planar_bins"] == 1, inf
        x = rng.uniform(-1, 1, B.m)
        y = torch.zeros(B.n, dtype=torch.float64, device=DEV)
        V.mul_(y, B.T, dev(x))
        assert rel(y.cpu().numpy(), O.mul(ref_of(B), x, np.zeros(B.n), trans=True)) <= TOL64, name


@pytest.mark.parametrize("keys16", ["0", "2"])
@pytest.mark.parametrize("mask", ["0", "1"])
def test_forward_lane_pairs_bitwise(monkeypatch, keys16, mask):
    """Forward lane pairs (round 6, vbc_planar.h run_pair DOT, vbc_info planar_mask bit 11): fp64 3 x 3 node
    blocks (an ldoor-like operator, ~15 blocks per node) laid out as the B'x lane pairs of the transposed
    blocks, each output row adding its per-block dot product (the reference's forward order,
    multiply_1DVBC.jl:34, :62-71).  Random x: bit for bit against the oracle and against the forward row-run
    layout (VBC_PLANAR_PAIR=0); alpha / beta; both key forms; natural and masked chunk order; a node with no
    block (empty output rows: beta * y)."""
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    monkeypatch.setenv("VBC_SLOT_KEYS16", keys16)
    monkeypatch.setenv("VBC_PLANAR_MASK", mask)
    A = V.synthetic.fe_stiffness_3d(90000, 4_000_000, 3, np.float64).tocsc()
    A = A.tolil()
    A[30:33, :] = 0.0  # node 10 couples to nothing: empty output rows
    A = A.tocsc()
    A.eliminate_zeros()
    B = V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))  # bin/test_table.jl:27
    R = ref_of(B)
    rng = np.random.default_rng(31)
    outs = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("VBC_PLANAR_PAIR", pair)
        B.release()
        inf = B.info(trans=False)
        assert bool(inf["planar_mask"] & 2048) == (pair == "1") and inf["fwd_run"] == 3, inf["planar_mask"]
        x = rng.uniform(-1, 1, B.n)
        y = torch.full((B.m,), float("nan"), dtype=torch.float64, device=DEV)
        V.mul_(y, B, dev(x))
        ref = O.mul(R, x, np.zeros(B.m))
        assert np.array_equal(y.cpu().numpy(), ref), pair
        outs[pair] = y.cpu().numpy()
        y0 = rng.uniform(-1, 1, B.m)
        yb = dev(y0.copy())
        V.mul_(yb, B, dev(x), 0.5, -1.5)
        assert rel(yb.cpu().numpy(), O.mul(R, x, y0.copy(), 0.5, -1.5, ref_semantics=False)) <= 1e-14
        outs[pair + "ab"] = yb.cpu().numpy()
        rng = np.random.default_rng(31)  # the same x / y0 for the other layout
    assert np.array_equal(outs["1"], outs["0"]) and np.array_equal(outs["1ab"], outs["0ab"])
