"""GPU parity of the per-lane compacted planar layout (csrc/vbc_planar.h run_planar_lanes, SlotBin::lanes)
for mul!(y, B', x) against the oracle (multiply_1DVBC.jl:90-180).

A tile of consecutive stripes is dealt to the 64 lanes as contiguous sub-blocks; each lane folds its
stripes one after another, each in stored row order, so every output is the reference's serial sum:
fp64 results (and fp32 on integer-valued data) must equal the oracle bit for bit.  VBC_PLANAR_LANES=1
forces the layout wherever it is representable (planar widths 3..8, natural contiguous outputs);
VBC_TARGET_RANGES_L shrinks the range count so one wave walks several tiles (tile switches inside the
software pipeline).  Empty stripes (one PAD | LAST zero run), dead lanes (reading lane 0's lines),
row runs and non-finite x are covered."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.test_gpu_parity import TOL32, TOL64, dev, one_hot_probes, rel
from tests.test_gpu_planar import expand_runs

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"


def ref_of(B, dtype=None):
    val = B.val if dtype is None else B.val.astype(dtype)
    return O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, val)


def lanes_on(B):
    return (B.info(trans=True)["planar_mask"] & 4) != 0


def fresh(B):
    return V.SparseMatrix1DVBC(B.W, B.m, B.n, B.Phi, B.pos, B.idx, B.ofs, B.val)


@pytest.fixture
def forced(monkeypatch):
    monkeypatch.setenv("VBC_SLOTS", "1")
    monkeypatch.setenv("VBC_PLANAR_LANES", "1")
    monkeypatch.setenv("VBC_PLANAR_SPLIT", "0")
    return monkeypatch


def test_golden_one_hot(golden, forced):
    """The reference's corpus (test/matrices.jl) in 3-, 5- and 8-wide stripes: one-hot probes exact."""
    seen = 0
    for key, g in golden.items():
        for meth in (V.EquiChunker(3), V.EquiChunker(5), V.EquiChunker(8)):
            B = V.SparseMatrix1DVBC[8](g["A"], meth)
            one_hot_probes(B, g["A"])
            seen += lanes_on(B)
    assert seen > 0


@pytest.mark.parametrize("ranges", [None, "6"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w", [3, 4, 5, 6, 7, 8])
def test_widths_integer_data_bitwise(forced, dtype, w, ranges):
    """Every width, ragged stripes with empty ones, integer-valued data (every partial sum exact in
    both precisions): the lanes product equals the oracle bit for bit; random x with α / β within
    the suite's tolerance.  ranges = 6: several tiles per wave."""
    if dtype == np.float32 and w == 4:
        pytest.skip("fp32 w = 4 rows are one 16-B lane vector: not planar")
    if ranges:
        forced.setenv("VBC_TARGET_RANGES_L", ranges)
    rng = np.random.default_rng(w)
    B = V.synthetic.vbr_1dvbc(9000, 4000, 14000, w, W=8, dtype=dtype, seed=w)
    assert np.any(np.diff(B.pos) == 0)  # empty stripes present
    nv = int(B.ofs[-1] - 1)
    B.val[:nv] = rng.integers(-4, 5, nv).astype(dtype)
    assert lanes_on(B)
    x = rng.integers(-3, 4, B.m).astype(dtype)
    y = torch.full((B.n,), float("nan"), dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
    V.mul_(y, B.T, dev(x))
    ref = O.mul(ref_of(B, np.float64), x.astype(np.float64), np.zeros(B.n), trans=True)
    assert np.array_equal(y.cpu().numpy().astype(np.float64), ref)
    xr = rng.uniform(-1, 1, B.m).astype(dtype)
    y0 = rng.uniform(-1, 1, B.n).astype(dtype)
    for alpha, beta in ((1.0, 0.0), (0.5, -2.0)):
        y = dev(y0.copy())
        V.mul_(y, B.T, dev(xr), alpha, beta)
        ref = O.mul(ref_of(B, np.float64), xr.astype(np.float64), y0.astype(np.float64), alpha, beta, trans=True,
                    ref_semantics=False)
        assert rel(y.cpu().numpy(), ref) <= (TOL64 if dtype == np.float64 else TOL32), (w, alpha)


@pytest.mark.parametrize("pair", ["0", "1"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("R", [2, 3])
def test_row_runs_nonfinite(forced, dtype, R, pair):
    """Row runs (one key and one R-wide gather per run) with Inf / NaN in x: non-finite values land
    where the oracle puts them; fp64 bit for bit."""
    forced.setenv("VBC_LANES_PAIR", pair)
    rng = np.random.default_rng(R)
    B = expand_runs(V.synthetic.vbr_1dvbc(6000, 3000, 15000, 3, W=8, dtype=dtype, seed=R), R, seed=R + 1)
    assert lanes_on(B) and B.info(trans=True)["planar_run"] == R
    # lane pairs: fp64 3-wide runs of 3 only
    assert B.info(trans=True)["planar_pair"] == (1 if (pair == "1" and R == 3 and dtype == np.float64) else 0)
    x = rng.uniform(-1, 1, B.m).astype(dtype)
    x[[0, 7, 4321]] = [np.inf, np.nan, -np.inf]  # x[0]: the address dead lanes / empty stripes touch
    y = torch.zeros(B.n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
    V.mul_(y, B.T, dev(x))
    ref = O.mul(ref_of(B, np.float64), x.astype(np.float64), np.zeros(B.n), trans=True)
    got = y.cpu().numpy().astype(np.float64)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    if dtype == np.float64:
        assert np.array_equal(got[fin], ref[fin])
    else:
        assert rel(np.nan_to_num(got[fin], posinf=0, neginf=0), np.nan_to_num(ref[fin], posinf=0, neginf=0)) <= TOL32


@pytest.mark.parametrize("pair", ["0", "1"])
@pytest.mark.parametrize("ranges", [None, "40"])
def test_fe3d_bitwise_and_equal_to_masked(forced, ranges, pair):
    """The irregular 3-dof stiffness operator: lanes (one lane or a lane pair per stream) == oracle ==
    the masked planar layout, bit for bit."""
    forced.setenv("VBC_LANES_PAIR", pair)
    if ranges:
        forced.setenv("VBC_TARGET_RANGES_L", ranges)
    B = V.synthetic.fe_stiffness_3d_1dvbc(300000, 3_000_000)
    x = np.random.default_rng(3).uniform(-1, 1, B.m)
    y = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y, B.T, dev(x))
    assert lanes_on(B)
    ref = O.mul(ref_of(B), x, np.zeros(B.n), trans=True)
    assert np.array_equal(y.cpu().numpy(), ref)
    forced.setenv("VBC_PLANAR_LANES", "0")
    forced.delenv("VBC_SLOTS")
    Bm = fresh(B)
    assert not lanes_on(Bm)
    y2 = torch.full((B.n,), float("nan"), dtype=torch.float64, device=DEV)
    V.mul_(y2, Bm.T, dev(x))
    assert torch.equal(y, y2)


def test_auto_selection_full_size_fe3d():
    """At the bench size (3.3e6 stripes) the library picks the lanes layout by itself."""
    B = V.synthetic.fe_stiffness_3d_1dvbc(3 * 3333333, int(1e8))
    assert lanes_on(B)
    B.release()


@pytest.mark.parametrize("ranges", [None, "5"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("w", [2, 3])
def test_forward_lanes(forced, dtype, w, ranges):
    """Forward mul!(y, B, x) in lane streams (planar_mask bit 4): node blocks of R = 3 output rows
    transposed into the B'x lane-stream kernel (W = 3 outputs, runs of w x rows).  Random x within
    tolerance of the oracle's forward product (multiply_1DVBC.jl:9-83), alpha / beta, forward quirks,
    rows without blocks (beta * y), several tiles per wave; integer values bit for bit."""
    from tests.test_gpu_planar import sp_blocked
    if ranges:
        forced.setenv("VBC_TARGET_RANGES_L", ranges)
    rng = np.random.default_rng(w + (7 if ranges else 0))
    base = V.synthetic.vbr_1dvbc(5000, 1500, 24000, w, W=8, dtype=dtype, seed=3 * w)
    A = sp_blocked(base, 3, rng, dtype)
    A = A.tolil()
    A[30:36, :] = 0  # two node rows without blocks
    A = A.tocsc()
    A.eliminate_zeros()
    B = V.SparseMatrix1DVBC[8](A, V.EquiChunker(w))
    inf = B.info(trans=False)
    assert inf["planar_mask"] & 16 and inf["fwd_run"] == 3
    R64 = ref_of(B, np.float64)
    tol = TOL64 if dtype == np.float64 else TOL32
    for alpha, beta in ((1.0, 0.0), (-0.5, 2.0)):
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
    yi = torch.full((B.m,), 7.0, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=DEV)
    V.mul_(yi, Bi, dev(xi))
    assert np.array_equal(yi.cpu().numpy().astype(np.float64),
                          O.mul(ref_of(Bi, np.float64), xi.astype(np.float64), np.zeros(B.m)))


def test_forward_lanes_auto_fe3d(monkeypatch):
    """The irregular 3-dof operator picks forward lane streams by default (>= 256 node rows per resident
    wave: the wave count is cut to 256 so 10^5 node rows qualify) and matches the oracle."""
    monkeypatch.setenv("VBC_TARGET_RANGES_L", "256")
    B = V.synthetic.fe_stiffness_3d_1dvbc(300000, 3_000_000)
    assert B.info(trans=False)["planar_mask"] & 16
    x = np.random.default_rng(4).uniform(-1, 1, B.n)
    y = torch.zeros(B.m, dtype=torch.float64, device=DEV)
    V.mul_(y, B, dev(x))
    assert rel(y.cpu().numpy(), O.mul(ref_of(B), x, np.zeros(B.m))) <= TOL64
