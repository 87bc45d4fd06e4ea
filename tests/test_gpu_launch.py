"""GPU checks of the launch-shape rules: the XCD-contiguous workgroup order of the slotted
and planar kernels, the halved range count of small slotted buckets and the split / pair choice for
few chunks.  None of them may change a result: a segment is folded by one wave in stored (reference)
row order whichever workgroup runs it, so every variant must equal the identity order bit for bit, and
the oracle (multiply_1DVBC.jl:90-180) within the suite's tolerances."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.test_gpu_parity import TOL64, dev, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def product(B, x, trans=True):
    y = torch.zeros(B.n if trans else B.m, dtype=torch.float64, device="cuda:0")
    V.mul_(y, B.T if trans else B, dev(x))
    return y.cpu().numpy()


def oracle(B, x, trans=True):
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    return O.mul(R, x, np.zeros(B.n if trans else B.m), trans=trans)


def variants(monkeypatch, B, x, envs, trans=True):
    out = []
    for env in envs:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        B.release()
        out.append(product(B, x, trans))
        for k in env:
            monkeypatch.delenv(k)
    B.release()
    return out


@pytest.mark.parametrize("trans", [True, False])
def test_xcd_order_slotted_bitwise(monkeypatch, trans):
    """FE-2D (slotted layout, hundreds of workgroups): XCD-contiguous order == identity order."""
    B = V.synthetic.fe_grid_2d(300, dof=2, dtype=np.float64, seed=5)
    x = np.random.default_rng(1).uniform(-1, 1, B.m if trans else B.n)
    a, b = variants(monkeypatch, B, x, [{"VBC_XCD": "0", "VBC_XCD_P": "0"}, {"VBC_XCD": "1", "VBC_XCD_P": "1"}], trans)
    assert np.array_equal(a, b)
    assert rel(a, oracle(B, x, trans)) <= TOL64


@pytest.mark.parametrize("pair", ["0", "2"])
def test_xcd_order_planar_bitwise(monkeypatch, pair):
    """FE-3D stand-in (planar layout with runs of 3; pair = 2 forces the lane-pair kernel): the XCD
    order of the planar kernels is bit-identical to the identity order and to the oracle (both fold
    each stripe serially in stored order)."""
    B = V.synthetic.fe_stiffness_3d_1dvbc(300000, 3_000_000)
    x = np.random.default_rng(2).uniform(-1, 1, B.m)
    monkeypatch.setenv("VBC_PLANAR_PAIR", pair)
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    a, b = variants(monkeypatch, B, x, [{"VBC_XCD_P": "0"}, {"VBC_XCD_P": "1"}])
    assert np.array_equal(a, b)
    assert np.array_equal(a, oracle(B, x))


def test_small_bucket_ranges_bitwise(monkeypatch):
    """A stripe shard of FE small enough for the halved range count: same bits as the full range
    count (VBC_RANGE_KB=0) and as the oracle within tolerance."""
    B = V.synthetic.fe_grid_2d(700, dof=2, dtype=np.float64, seed=6)
    cuts = V.distributed.stripe_split(B, 4)
    S, _ = V.distributed.shard(B, int(cuts[1]), int(cuts[2]))
    x = np.random.default_rng(3).uniform(-1, 1, S.m)
    a, b = variants(monkeypatch, S, x, [{"VBC_RANGE_KB": "0"}, {"VBC_RANGE_KB": "100000"}])
    assert np.array_equal(a, b)
    assert rel(a, oracle(S, x)) <= TOL64


def test_few_chunks_split_choice(monkeypatch):
    """A 3-dof stiffness matrix with a few hundred pair chunks: the split rule picks P <= 4 (chunks x P
    within half the wave slots) and the product matches the oracle; forcing the lane-pair layout gives
    the oracle's bits."""
    B = V.synthetic.fe_stiffness_3d_1dvbc(60000, 2_700_000)
    x = np.random.default_rng(4).uniform(-1, 1, B.m)
    inf = B.info(trans=True)
    assert 1 <= inf["planar_split"] <= 4
    assert rel(product(B, x), oracle(B, x)) <= TOL64
    B.release()
    monkeypatch.setenv("VBC_PLANAR_PAIR", "2")
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    assert B.info(trans=True)["planar_pair"] == 1
    assert np.array_equal(product(B, x), oracle(B, x))
