"""The AUTOMATIC layout selection driven by random structures.

Every other GPU test forces a layout with a knob or runs one of the bench's few stand-ins; a real
SuiteSparse matrix whose structure differs from them takes whatever path vbc*_create picks.  Here about
60 matrices are drawn from a seeded grid of structures -- width mixes (one width 1..8; 1..2; 1..8; 3..6;
a dominant width beside a few odd stripes), stripe-length distributions (near-constant, Poisson,
heavy-tailed, a few giant stripes, many empty stripes), row placement (banded like a mesh operator,
uniform over x like the reference's generator costs.jl:63-83, node runs of 3 or 2 with and without holes)
and sizes from a few stripes to ~3e5 (straddling the fused-split, split, lane-stream, fork and row-swept
thresholds) -- and each goes through the DEFAULT create path (no knob set) in both directions and in
both float eltypes, against the oracle:

* integer-valued data (every partial sum exact): the default layouts must equal the oracle bit for bit
  in both directions, whatever order they sum in;
* random data: normwise relative error <= 1e-12 (fp64) / 1e-5 (fp32) in both directions, and the
  VBC_CREATE_SERIAL layouts (B.serial: the reference's serial per-stripe order, multiply_1DVBC.jl:101-104)
  equal the oracle's B'x bit for bit.

The protocol is the reference's own sweep over sizes (test/runtests.jl:14-53), widened to the structure
axes the layout heuristics branch on.  The layout families the grid reached are asserted at the end so a
change of thresholds that silently stops exercising one is noticed."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O
from tests.test_gpu_parity import TOL32, TOL64, rel

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"

WIDTHS = ("1", "2", "3", "4", "6", "8", "mix12", "mix18", "mix36", "dom3")
LENGTHS = ("const", "poisson", "heavy", "giant", "empty")
PLACES = ("band", "uniform", "runs3", "runs3holes", "runs2")
SIZES = (("tiny", 40), ("small", 1500), ("medium", 20000), ("large", 150000))
MEAN_ROWS = (3, 10, 30)


def _widths(rng, kind, L):
    if kind.isdigit():
        return np.full(L, int(kind), np.int64)
    if kind == "mix12":
        return rng.integers(1, 3, L)
    if kind == "mix18":
        return rng.integers(1, 9, L)
    if kind == "mix36":
        return rng.integers(3, 7, L)
    # dom3: >= 80 % 3-wide stripes beside 1-, 2-, 6- and 7-wide ones (a time-model partition's shape)
    w = np.full(L, 3, np.int64)
    side = rng.random(L) < 0.12
    w[side] = rng.choice([1, 2, 6, 7], int(side.sum()))
    return w


def _counts(rng, kind, L, d):
    if kind == "const":
        c = np.full(L, d, np.int64)
    elif kind == "poisson":
        c = rng.poisson(d, L)
    elif kind == "heavy":  # Pareto tail, mean ~ d
        c = np.minimum((d * 0.5 * (1 + rng.pareto(1.6, L))).astype(np.int64), 50 * d + 200)
    elif kind == "giant":  # a few stripes 100x longer than the rest
        c = rng.poisson(d, L)
        g = rng.choice(L, max(1, L // 2000), replace=False)
        c[g] = 100 * d + rng.integers(0, 50, len(g))
    else:  # empty: 40 % of the stripes store nothing
        c = rng.poisson(d, L)
        c[rng.random(L) < 0.4] = 0
    return c.astype(np.int64)


def _rows(rng, place, L, m, counts):
    """Per stripe: sorted distinct 0-based rows.  Returns (stripe ids, rows) of the stored rows."""
    if place in ("runs3", "runs3holes", "runs2"):
        R = 2 if place == "runs2" else 3
        nodes_m = m // R
        nc = np.maximum(counts // R, 0)
        sid = np.repeat(np.arange(L, dtype=np.int64), nc)
        centre = sid * nodes_m // max(L, 1)
        node = np.clip(centre + rng.integers(-64, 65, len(sid)), 0, nodes_m - 1)
        keys = np.unique(sid * nodes_m + node)
        sid, node = keys // nodes_m, keys % nodes_m
        sid = np.repeat(sid, R)
        rows = (node[:, None] * R + np.arange(R)[None, :]).reshape(-1)
        if place == "runs3holes":  # ~1 row in 25 missing: the structural zeros of a node coupling
            keep = rng.random(len(rows)) >= 0.04
            sid, rows = sid[keep], rows[keep]
        return sid, rows
    sid = np.repeat(np.arange(L, dtype=np.int64), counts)
    if place == "band":
        band = 2048
        lo = np.clip(sid * m // max(L, 1) - band // 2, 0, max(m - band, 0))
        row = lo + rng.integers(0, min(band, m), len(sid))
    else:
        row = rng.integers(0, m, len(sid))
    keys = np.unique(sid * m + row)
    return keys // m, keys % m


def _matrix(seed, wk, lk, pk, L, d, m_over=None):
    rng = np.random.default_rng(seed)
    w = _widths(rng, wk, L)
    n = int(w.sum())
    m = m_over or max(n, 64)
    sid, rows = _rows(rng, pk, L, m, _counts(rng, lk, L, d))
    cnt = np.bincount(sid, minlength=L).astype(np.int64)
    spl = np.concatenate([[1], 1 + np.cumsum(w)]).astype(np.int64)
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)]).astype(np.int64)
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * w)]).astype(np.int64)
    nv = int(ofs[-1] - 1)
    return V.SparseMatrix1DVBC(8, m, n, V.SplitPartition(spl), pos, rows + 1, ofs, np.zeros(nv + 8)), rng


def _grid():
    """~60 cases from the seeded grid; every size, width, length and placement kind appears."""
    rng = np.random.default_rng(0x5E1EC7)
    cases = []
    for i in range(56):
        size, L = SIZES[i % len(SIZES)]
        wk = WIDTHS[i % len(WIDTHS)]
        lk = LENGTHS[(i // 2) % len(LENGTHS)]
        pk = PLACES[(i // 3) % len(PLACES)]
        d = int(MEAN_ROWS[int(rng.integers(0, len(MEAN_ROWS)))])
        if size == "large":
            d = min(d, 10)
        cases.append((f"{i:02d}-{size}-w{wk}-{lk}-{pk}-d{d}", 1000 + i, wk, lk, pk, L, d, None))
    # the row-swept layout: x of >= 16 MB (fp64) with rows uniform over it (costs.jl:63-83)
    cases.append(("56-sweep-w4-poisson-uniform", 1056, "4", "poisson", "uniform", 60000, 8, 2_500_000))
    cases.append(("57-sweep-mix18-heavy-uniform", 1057, "mix18", "heavy", "uniform", 40000, 8, 2_500_000))
    # large node-run operators (lane streams / lane pairs / planar) and a medium masked one
    cases.append(("58-xl-w3-poisson-runs3", 1058, "3", "poisson", "runs3", 300000, 9, None))
    cases.append(("59-xl-dom3-const-runs3holes", 1059, "dom3", "const", "runs3holes", 200000, 12, None))
    # >= 8 node runs per stripe: the fp64 lane-pair layout
    cases.append(("60-xl-w3-poisson-runs3-long", 1060, "3", "poisson", "runs3", 120000, 30, None))
    return cases


CASES = _grid()
SEEN = {}


def _families(inf, trans):
    pm = inf["planar_mask"]
    f = set()
    if trans:
        if pm & 32:
            f.add("fused-split")
        if pm & 64:
            f.add("long-stripes-cut")
        if pm & 4:
            f.add("lanes")
        if inf["planar_pair"]:
            f.add("pair")
        if inf["planar_split"] > 1 and not pm & 32:
            f.add("split")
        if inf["sweep_bins"]:
            f.add("sweep")
        if inf["planar_bins"] and not pm & (4 | 32) and inf["planar_split"] == 1:
            f.add("planar")
        if inf["slot_bins"] > inf["planar_bins"]:
            f.add("slotted")
        if inf["bins_t"] > inf["slot_bins"] + inf["sweep_bins"]:
            f.add("merge")
        if inf["planar_run"] > 1:
            f.add("runs")
    else:
        if pm & 256:
            f.add("fwd-on-C")
        if pm & 16:
            f.add("fwd-lanes")
        if pm & 8:
            f.add("fwd-split")
        if inf["fwd_run"] > 1:
            f.add("fwd-runs")
        if inf["sweep_bins"]:
            f.add("fwd-sweep")
    return f


def _check(B, R, x, trans, exact, tol):
    nx, ny = (B.m, B.n) if trans else (B.n, B.m)
    y = torch.full((ny,), float("nan"), dtype=torch.from_numpy(x).dtype, device=DEV)
    V.mul_(y, B.T if trans else B, torch.from_numpy(x).to(DEV))
    got = y.cpu().numpy()
    ref = O.mul(R, x, np.zeros(ny, x.dtype), trans=trans)
    if exact:
        assert np.array_equal(got, ref), ("not bitwise", trans)
    else:
        assert rel(got, ref) <= tol, ("rel", trans, rel(got, ref))
    return got, ref


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_auto_layout_random_structure(case):
    name, seed, wk, lk, pk, L, d, m_over = case
    B0, rng = _matrix(seed, wk, lk, pk, L, d, m_over)
    nv = int(B0.ofs[-1] - 1)
    integer = seed % 2 == 0
    fams = set()
    for dt, tol in ((np.float64, TOL64), (np.float32, TOL32)):
        val = np.zeros(nv + 8, dt)
        val[:nv] = rng.integers(-8, 9, nv) if integer else rng.uniform(-1, 1, nv)
        B = V.SparseMatrix1DVBC(8, B0.m, B0.n, B0.Phi, B0.pos, B0.idx, B0.ofs, val)
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
        for trans in (True, False):
            nx = B.m if trans else B.n
            x = (rng.integers(-8, 9, nx) if integer else rng.uniform(-1, 1, nx)).astype(dt)
            _check(B, R, x, trans, integer, tol)
            fams |= _families(B.info(0, trans), trans)
        B.release()
        # VBC_CREATE_SERIAL: the reference's per-stripe order -> B'x equals the oracle bit for bit
        Bs = V.SparseMatrix1DVBC(8, B0.m, B0.n, B0.Phi, B0.pos, B0.idx, B0.ofs, val)
        Bs.serial = True
        x = rng.uniform(-1, 1, B.m).astype(dt)
        _check(Bs, R, x, True, True, tol)
        assert not Bs.info(0, True)["planar_mask"] & 32 and Bs.info(0, True)["planar_split"] == 1
        Bs.release()
    SEEN[name] = fams


def test_auto_layout_grid_reached_every_family():
    """The grid above drove the default create path into every layout family (run after the cases)."""
    if len(SEEN) < len(CASES):
        pytest.skip("needs the whole grid in this session")
    allf = set().union(*SEEN.values())
    # (the lane-stream layout needs >= 256 stripes per resident wave, ~1e6 stripes: the bench's fe3d drives it)
    want = {"fused-split", "long-stripes-cut", "pair", "sweep", "planar", "slotted", "runs", "fwd-on-C", "fwd-runs"}
    assert want <= allf, sorted(want - allf)
