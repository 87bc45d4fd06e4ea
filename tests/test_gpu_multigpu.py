"""The single-process multi-GPU handle (include/vbc.h vbc1d_create_sharded / vbc_sharded_mul, SURVEY.md
§8e) against the oracle.  On a one-GPU box: devices=[0] runs the RCCL code path with one rank, and
devices=[0, 0, 0] runs three shards on one device (no communicator) -- the split, the per-shard
handles and the exchange pattern of every (split, direction) pair, fp64 normwise <= 1e-12 against the
oracle.  Disjoint outputs (stripes: B'x, rows: Bx) of a layout with per-segment serial summation
(slotted, planar, swept) equal the single-GPU product bit for bit; reduced outputs (stripes: Bx,
rows: B'x) reorder the addition of the shards' partial sums."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from sparsematrixvbcs_amd import distributed as D
from tests.test_gpu_parity import TOL64, dev, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


def ref_of(B):
    return O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)


@pytest.fixture(scope="module")
def mat():
    rng = np.random.default_rng(11)
    return V.synthetic.vbr_1dvbc(9000, 2500, 60000, rng.integers(1, 9, 2500), W=8, seed=12)


@pytest.mark.parametrize("split", ["stripes", "rows"])
@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0]])
def test_sharded_products(mat, split, devices):
    B = mat
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=devices, split=split)
    R = ref_of(B)
    rng = np.random.default_rng(len(devices))
    # the shards' ranges are distributed.py's byte-balanced cuts
    cuts = D.stripe_split(B, len(devices)) if split == "stripes" else D.row_split(B, len(devices))
    ranges = [(lo, hi) for lo, hi, _ in S.shards()]
    if split == "stripes":
        assert ranges == [(int(B.Phi.spl[a] - 1), int(B.Phi.spl[b] - 1)) for a, b in zip(cuts[:-1], cuts[1:])]
    else:
        assert ranges == [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        disjoint = (split == "stripes") == trans
        for alpha, beta in ((1.0, 0.0), (0.5, -2.0)):
            x = rng.uniform(-1, 1, nx)
            y0 = rng.uniform(-1, 1, ny)
            ref = O.mul(R, x, y0.copy(), alpha, beta, trans=trans, ref_semantics=False)
            y = dev(y0.copy())
            V.mul_(y, S.T if trans else S, dev(x), alpha, beta)
            got = y.cpu().numpy()
            assert rel(got, ref) <= TOL64, (split, devices, trans, disjoint, alpha)
            yh = y0.copy()  # host operands: staged on devices[0]
            V.mul_(yh, S.T if trans else S, x, alpha, beta)
            assert rel(yh, ref) <= TOL64
    S.release()


def test_sharded_disjoint_equals_single_gpu_fe():
    """A 2D FE operator split over 4 shards: B'x equals the single-GPU handle's result bit for bit."""
    B = V.synthetic.fe_grid_2d(300, dof=2)
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0, 0, 0, 0], split="stripes", forward=False)
    x = dev(np.random.default_rng(3).uniform(-1, 1, B.m))
    y1 = torch.empty(B.n, dtype=torch.float64, device=DEV)
    y4 = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y1, B.T, x)
    V.mul_(y4, S.T, x)
    assert torch.equal(y1, y4)
    S.release()


def test_sharded_quirks_and_errors(mat):
    B = mat
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0, 0], split="rows")
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, B.m)
    y = dev(rng.uniform(-1, 1, B.n))
    V.mul_(y, S.T, dev(x), 3.0, 9.0, quirks=True)  # transposed quirks: overwrite, alpha ignored
    assert rel(y.cpu().numpy(), O.mul(ref_of(B), x, np.zeros(B.n), trans=True)) <= TOL64
    with pytest.raises(V.DimensionMismatch):
        V.mul_(dev(np.zeros(B.n + 1)), S.T, dev(x))
    with pytest.raises(V.UnsupportedDtype):
        V.mul_(torch.zeros(B.n, dtype=torch.float32, device=DEV), S.T, dev(x))
    S.release()
    with pytest.raises(V.ArgumentError):
        D.MultiGPUSparseMatrix1DVBC(B, devices=[999])
    with pytest.raises(V.ArgumentError):
        D.MultiGPUSparseMatrix1DVBC(B, devices=[])


def test_sharded_more_shards_than_stripes():
    """Shards with no stripes / no rows (cuts collapse) are valid empty handles."""
    A = np.zeros((40, 6))
    A[::3, 1] = 1.0
    A[5, 4] = 2.0
    import scipy.sparse as sp
    B = V.SparseMatrix1DVBC[4](sp.csc_matrix(A), V.EquiChunker(2))
    for split in ("stripes", "rows"):
        S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0] * 8, split=split)
        x = np.arange(40, dtype=np.float64)
        y = dev(np.zeros(6))
        V.mul_(y, S.T, dev(x))
        assert np.allclose(y.cpu().numpy(), A.T @ x)
        xf = np.arange(6, dtype=np.float64)
        yf = dev(np.zeros(40))
        V.mul_(yf, S, dev(xf))
        assert np.allclose(yf.cpu().numpy(), A @ xf)
        S.release()
