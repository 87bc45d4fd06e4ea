"""libvbc products captured into a HIP graph (torch.cuda.CUDAGraph = hipGraph on ROCm) replay to the
same bits as eager launches: the VBC_MEM_DEVICE path launches on the caller's stream and never
allocates, synchronises or copies once the handle exists (tools/graph_bench.py measures the gain)."""
import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from tests.test_gpu_parity import dev

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("layout", ["auto", "sweep", "merge"])
def test_graph_replay_matches_eager(monkeypatch, layout):
    if layout == "sweep":
        monkeypatch.setenv("VBC_SWEEP", "1")
    elif layout == "merge":
        monkeypatch.setenv("VBC_SLOTS", "0")
    rng = np.random.default_rng(31)
    B = V.synthetic.vbr_1dvbc(3000, 700, 9000, np.arange(700) % 6 + 1, W=8, seed=3)
    x = dev(rng.uniform(-1, 1, B.m))
    xf = dev(rng.uniform(-1, 1, B.n))
    s = torch.cuda.Stream()
    y_e = [torch.zeros(B.n, dtype=torch.float64, device="cuda") for _ in range(2)]
    f_e = torch.zeros(B.m, dtype=torch.float64, device="cuda")
    with torch.cuda.stream(s):  # eager reference (also builds both handles outside the capture)
        V.mul_(y_e[0], B.T, x)
        V.mul_(y_e[1], B.T, x, 0.5, 0.0)
        V.mul_(f_e, B, xf)
    torch.cuda.synchronize()
    y_g = [torch.full((B.n,), float("nan"), dtype=torch.float64, device="cuda") for _ in range(2)]
    f_g = torch.full((B.m,), float("nan"), dtype=torch.float64, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        V.mul_(y_g[0], B.T, x)
        V.mul_(y_g[1], B.T, x, 0.5, 0.0)
        V.mul_(f_g, B, xf)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for a, b in zip(y_g + [f_g], y_e + [f_e]):
        assert torch.equal(a, b)


def test_forked_groups_bitwise_eager_graph_and_two_streams(monkeypatch):
    """A B'x product with several independent launch groups (slotted narrow widths, one planar bucket
    per wide width, the merge kernel for a heavy-tailed bucket, the fill list of empty stripes) runs
    the groups after the first on side streams joined back into the caller's (Launch::fork_*).  It
    must equal the sequential launch (VBC_FORK=0) bit for bit: eagerly, replayed from a HIP graph,
    and with the same handle used from two caller streams at once, each product ordered after the
    writes of x that precede it on its own stream.  (VBC_SMALL_FUSE=0: the matrix is small enough for the
    fused split, which would run all its buckets as one launch.)"""
    monkeypatch.setenv("VBC_SMALL_FUSE", "0")
    rng = np.random.default_rng(5)
    L = 20000
    G = V.synthetic.vbr_1dvbc(40000, L, 200000, np.arange(L) % 8 + 1, W=8, seed=9)
    cnt = np.diff(G.pos).copy()
    cnt[::37] = 0  # empty stripes: the fill list
    keep = np.repeat(np.diff(G.pos) == cnt, np.diff(G.pos))
    w = np.diff(G.Phi.spl)
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)])
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * w)])
    vkeep = np.repeat(np.repeat(np.diff(G.pos) == cnt, np.diff(G.pos)), np.repeat(w, np.diff(G.pos)))
    val = np.concatenate([G.val[:int(G.ofs[-1] - 1)][vkeep], np.zeros(len(G.val) - int(G.ofs[-1] - 1))])
    B0 = V.SparseMatrix1DVBC(G.W, G.m, G.n, G.Phi, pos, G.idx[keep], ofs, val)
    Bf = V.SparseMatrix1DVBC(B0.W, B0.m, B0.n, B0.Phi, B0.pos, B0.idx, B0.ofs, B0.val)
    Bs = V.SparseMatrix1DVBC(B0.W, B0.m, B0.n, B0.Phi, B0.pos, B0.idx, B0.ofs, B0.val)
    Bf.info(trans=True)
    monkeypatch.setenv("VBC_FORK", "0")
    Bs.info(trans=True)
    monkeypatch.delenv("VBC_FORK")
    inf = Bf.info(trans=True)
    groups = inf["planar_bins"] + (inf["slot_bins"] > inf["planar_bins"]) + (inf["bins_t"] > 0) + (inf["sweep_bins"] > 0)
    assert groups >= 2  # several launch groups: the fork path runs
    x = dev(rng.uniform(-1, 1, B0.m))
    ys = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    V.mul_(ys, Bs.T, x)
    yf = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    V.mul_(yf, Bf.T, x)
    torch.cuda.synchronize()
    assert torch.equal(yf, ys)
    from oracle import oracle as O
    R = O.Ref1DVBC(B0.m, B0.n, B0.W, B0.Phi.spl, B0.pos, B0.idx, B0.ofs, B0.val)
    ref = O.mul(R, x.cpu().numpy(), np.zeros(B0.n), trans=True)
    assert np.linalg.norm(ys.cpu().numpy() - ref) <= 1e-12 * np.linalg.norm(ref)
    # graph replay of forked products
    s = torch.cuda.Stream()
    yg = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(3):
            V.mul_(yg, Bf.T, x, 1.0, 0.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(yg, ys)
    # two caller streams, each writing its own x right before its product
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    xa, xb = torch.empty_like(x), torch.empty_like(x)
    ya = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    yb = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    x2 = dev(rng.uniform(-1, 1, B0.m))
    ys2 = torch.zeros(B0.n, dtype=torch.float64, device="cuda")
    V.mul_(ys2, Bs.T, x2)
    torch.cuda.synchronize()
    for _ in range(5):
        with torch.cuda.stream(s1):
            xa.copy_(x)
            V.mul_(ya, Bf.T, xa)
        with torch.cuda.stream(s2):
            xb.copy_(x2)
            V.mul_(yb, Bf.T, xb)
    torch.cuda.synchronize()
    assert torch.equal(ya, ys) and torch.equal(yb, ys2)
    # an eager product on a second stream while a capture on the first holds the side streams: it must
    # not queue work on them (it runs its groups on its own stream), and both results stay exact
    s3 = torch.cuda.Stream()
    ye = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    yc = torch.full((B0.n,), float("nan"), dtype=torch.float64, device="cuda")
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s, capture_error_mode="relaxed"):
        V.mul_(yc, Bf.T, x)
        with torch.cuda.stream(s3):
            V.mul_(ye, Bf.T, x2)
    torch.cuda.synchronize()
    assert torch.equal(ye, ys2)
    g2.replay()
    torch.cuda.synchronize()
    assert torch.equal(yc, ys)
