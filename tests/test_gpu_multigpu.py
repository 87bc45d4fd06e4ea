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


# ---- round 3: eltypes and strides on the sharded boundary, the 2D sharded handle, RCCL over real GPUs --

def _x_as_compute(x):
    return np.asarray(x, dtype=np.float64)


@pytest.mark.parametrize("split", ["stripes", "rows"])
def test_sharded_mixed_eltypes_and_strides(mat, split):
    """vbc_sharded_mul_ex: x of another eltype is converted (multiply_1DVBC.jl:102), strided x / y
    views are read and written in place, and a y of another float eltype is refused -- host and
    device operands, both directions."""
    B = mat
    R = ref_of(B)
    rng = np.random.default_rng(21)
    for devices in ([0], [0, 0, 0]):
        S = D.MultiGPUSparseMatrix1DVBC(B, devices=devices, split=split)
        for trans in (True, False):
            nx, ny = (B.m, B.n) if trans else (B.n, B.m)
            x32 = rng.uniform(-1, 1, nx).astype(np.float32)
            xi = rng.integers(-5, 6, nx).astype(np.int32)
            y0 = rng.uniform(-1, 1, ny)
            for x in (x32, xi):
                ref = O.mul(R, _x_as_compute(x), y0.copy(), 0.5, 2.0, trans=trans, ref_semantics=False)
                yh = y0.copy()
                V.mul_(yh, S.T if trans else S, x, 0.5, 2.0)  # host, converted x
                assert rel(yh, ref) <= TOL64, (split, devices, trans, x.dtype)
                yd = dev(y0.copy())
                V.mul_(yd, S.T if trans else S, torch.from_numpy(x).to(DEV), 0.5, 2.0)  # device, converted x
                assert rel(yd.cpu().numpy(), ref) <= TOL64
            # strided views: every other element of a wider buffer; the gaps stay untouched
            xs = rng.uniform(-1, 1, 2 * nx)
            ys = np.full(3 * ny, 7.0)
            ys[::3] = y0
            ref = O.mul(R, xs[::2].copy(), y0.copy(), 1.0, -1.0, trans=trans, ref_semantics=False)
            V.mul_(ys[::3], S.T if trans else S, xs[::2], 1.0, -1.0)
            assert rel(ys[::3], ref) <= TOL64
            assert np.all(ys[1::3] == 7.0) and np.all(ys[2::3] == 7.0)
            xt = dev(xs)
            yt = dev(np.full(3 * ny, 7.0))
            yt[::3] = dev(y0)
            V.mul_(yt[::3], S.T if trans else S, xt[::2], 1.0, -1.0)
            got = yt.cpu().numpy()
            assert rel(got[::3], ref) <= TOL64
            assert np.all(got[1::3] == 7.0) and np.all(got[2::3] == 7.0)
            with pytest.raises(V.UnsupportedDtype):  # eltype(y) != the handle's compute eltype
                V.mul_(np.zeros(ny, np.float32), S.T if trans else S, x32)
            with pytest.raises(V.UnsupportedDtype):
                V.mul_(torch.zeros(ny, dtype=torch.float32, device=DEV), S.T if trans else S,
                       torch.from_numpy(x32).to(DEV))
        S.release()


def test_sharded_ex_never_reads_past_a_host_buffer(mat):
    """A Float32 x whose last element ends a page followed by an inaccessible page: the converting
    product reads exactly length(x) Float32s (the round-2 ABI read it as Float64 and overran); a
    Float32 y on the Float64 handle is refused before any access."""
    import ctypes as C
    import mmap
    B = mat
    libc = C.CDLL(None)
    libc.mprotect.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    page = mmap.PAGESIZE
    nbytes = max(B.m, B.n) * 4
    npages = (nbytes + page - 1) // page
    buf = mmap.mmap(-1, (npages + 1) * page)
    base = C.addressof(C.c_char.from_buffer(buf))
    assert libc.mprotect(base + npages * page, page, 0) == 0  # PROT_NONE guard page
    x = np.frombuffer(buf, dtype=np.float32, count=B.m, offset=npages * page - B.m * 4)
    x[:] = np.random.default_rng(4).uniform(-1, 1, B.m).astype(np.float32)
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0, 0], split="stripes")
    y = np.zeros(B.n)
    V.mul_(y, S.T, x)
    ref = O.mul(ref_of(B), x.astype(np.float64), np.zeros(B.n), trans=True)
    assert rel(y, ref) <= TOL64
    y32 = np.frombuffer(buf, dtype=np.float32, count=B.n, offset=npages * page - B.n * 4)
    L = V._lib
    st = L.lib().vbc_sharded_mul_ex(S._h, 1, x.ctypes.data, L.VBC_F32, 1, B.m, y32.ctypes.data, L.VBC_F32, 1, B.n,
                                    1.0, 0.0, L.VBC_MEM_HOST, None, 0)
    assert st == L.VBC_UNSUPPORTED_DTYPE
    S.release()
    del x, y32
    assert libc.mprotect(base + npages * page, page, 3) == 0  # PROT_READ | PROT_WRITE again


def _vbc2d(seed, dtype=np.float64):
    import scipy.sparse as sp
    A = sp.random(700, 520, density=0.02, random_state=seed, format="csc", dtype=np.float64)
    A.data = np.random.default_rng(seed).uniform(-1, 1, A.nnz)
    B = V.SparseMatrixVBC[4, 4](A.astype(dtype), V.AlternatingPacker(V.OverlapChunker(0.9, 4), V.OverlapChunker(0.9, 4)))
    return B


@pytest.mark.parametrize("split", ["stripes", "rows"])
@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_sharded_vbc2d(split, devices):
    """vbc2d_create_sharded (multiply_VBC.jl:182-189 threaded the same way): both splits, both
    directions, α/β, device and host operands, against the oracle's VBC products; the row split
    keeps Π's block rows whole."""
    B = _vbc2d(3)
    R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    S = D.MultiGPUSparseMatrix(B, devices=devices, split=split)
    assert S.is2d
    if split == "rows":
        bounds = set(int(b) - 1 for b in B.Pi.spl)
        assert all(lo in bounds and hi in bounds for lo, hi, _ in S.shards())
    rng = np.random.default_rng(9)
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        for alpha, beta in ((1.0, 0.0), (-0.5, 3.0)):
            x = rng.uniform(-1, 1, nx)
            y0 = rng.uniform(-1, 1, ny)
            ref = O.mul(R, x, y0.copy(), alpha, beta, trans=trans, ref_semantics=False)
            y = dev(y0.copy())
            V.mul_(y, S.T if trans else S, dev(x), alpha, beta)
            assert rel(y.cpu().numpy(), ref) <= TOL64, (split, devices, trans, alpha)
            yh = y0.copy()
            V.mul_(yh, S.T if trans else S, x, alpha, beta)
            assert rel(yh, ref) <= TOL64
        # one-hot probes (runtests.jl:63-87): exact on every shard layout
        for j in (0, nx // 3, nx - 1):
            e = np.zeros(nx)
            e[j] = 1.0
            ref = O.mul(R, e, np.zeros(ny), trans=trans)
            y = dev(np.zeros(ny))
            V.mul_(y, S.T if trans else S, dev(e))
            assert np.array_equal(y.cpu().numpy(), ref)
    S.release()


def test_sharded_serial_flag_bit_identical_on_split_product_sizes():
    """a small stripe shard may choose the split planar product (P slices per chunk) while
    the whole matrix does not.  With serial=True (VBC_CREATE_SERIAL) every shard keeps the
    reference's serial per-stripe order: the stripe-sharded B'x equals the single-GPU product and
    the oracle bit for bit on a 3-dof stiffness matrix of ct20stif's size, whose default layout splits."""
    A = V.synthetic.fe_stiffness_3d(52329, 2600295, 3, np.float64, seed=5)  # one-width 3-dof (rounds 1-3 stand-in)
    B = V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))
    assert B.info(0, True)["planar_split"] > 1  # the default layout folds chunks in slices
    B.release()
    B.serial = True
    assert B.info(0, True)["planar_split"] == 1
    x = np.random.default_rng(2).uniform(-1, 1, B.m)
    y1 = dev(np.zeros(B.n))
    V.mul_(y1, B.T, dev(x))
    ref = O.mul(ref_of(B), x, np.zeros(B.n), trans=True)
    assert np.array_equal(y1.cpu().numpy(), ref)
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0] * 8, split="stripes", forward=False, serial=True)
    y8 = dev(np.full(B.n, np.nan))
    V.mul_(y8, S.T, dev(x))
    assert torch.equal(y1, y8)
    S.release()
    B.release()


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two GPUs (RCCL exchange between distinct devices)")
@pytest.mark.parametrize("split", ["stripes", "rows"])
def test_sharded_distinct_devices_rccl(mat, split):
    """the RCCL exchange between distinct devices (broadcast / send-recv of x, the β slices,
    the y gather or ncclReduce) against the oracle and the single-GPU handle, both directions, β != 0."""
    B = mat
    R = ref_of(B)
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0, 1], split=split)
    rng = np.random.default_rng(33)
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        x = rng.uniform(-1, 1, nx)
        y0 = rng.uniform(-1, 1, ny)
        ref = O.mul(R, x, y0.copy(), 0.75, -1.5, trans=trans, ref_semantics=False)
        y = dev(y0.copy())
        V.mul_(y, S.T if trans else S, dev(x), 0.75, -1.5)
        torch.cuda.synchronize()
        assert rel(y.cpu().numpy(), ref) <= TOL64
        y1 = dev(y0.copy())
        V.mul_(y1, B.T if trans else B, dev(x), 0.75, -1.5)
        if (split == "stripes") == trans:  # disjoint slices: the single-GPU result bit for bit
            assert torch.equal(y, y1)
    S.release()


def test_sharded_serial_flag_forward_rows():
    """the forward counterpart.  Small forward layouts run the split forward product by
    default (P waves per chunk, partial sums meeting in LDS: vbc_info planar_mask bit 3); serial=True
    (VBC_CREATE_SERIAL) turns it off in every shard too, so each output row sums its blocks in the
    reference's stripe order (multiply_1DVBC.jl:62-71).  The row-sharded B·x -- disjoint y slices --
    matches the oracle, and equals the single-GPU serial product bit for bit wherever a shard runs the
    same forward kernel family (the slotted and planar forward kernels associate a block's w-term dot
    product differently, vbc.h VBC_SPLIT_ROWS note)."""
    A = V.synthetic.fe_stiffness_3d(52329, 2600295, 3, np.float64, seed=5)  # one-width 3-dof (rounds 1-3 stand-in)
    B = V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))
    assert B.info(0, False)["planar_mask"] & 8  # the default forward layout splits chunks
    B.release()
    B.serial = True
    whole = B.info(0, False)
    assert not whole["planar_mask"] & 8
    x = np.random.default_rng(4).uniform(-1, 1, B.n)
    y1 = dev(np.zeros(B.m))
    V.mul_(y1, B, dev(x))
    ref = O.mul(ref_of(B), x, np.zeros(B.m), trans=False)
    assert rel(y1.cpu().numpy(), ref) <= TOL64
    fam = lambda inf: (inf["fwd_run"], inf["planar_mask"] & 0b11010, inf["slot_bins"] > 0, inf["bins_f"])
    same_family_seen = False
    for nsh in (2, 8):
        S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0] * nsh, split="rows", transposed=False, serial=True)
        yk = dev(np.full(B.m, np.nan))
        V.mul_(yk, S, dev(x))
        assert rel(yk.cpu().numpy(), ref) <= TOL64
        infos = [S.shard_info(g) for g in range(nsh)]
        assert not any(i["planar_mask"] & 8 for i in infos)
        for g, (lo, hi, _) in enumerate(S.shards()):
            if fam(infos[g]) == fam(whole):
                same_family_seen = True
                assert torch.equal(y1[lo:hi], yk[lo:hi]), (nsh, g)
        S.release()
    assert same_family_seen
    B.release()


@pytest.mark.parametrize("forward,transposed,want", [(True, False, "rows"), (False, True, "stripes"),
                                                     (True, True, "stripes")])
def test_sharded_auto_split(forward, transposed, want):
    """VBC_SPLIT_AUTO (vbc.h): the split with the smaller predicted kernel + exchange time of the
    products the handle builds -- forward only: rows (disjoint y, no reduce); B'x: stripes -- reported by
    vbc_sharded_split, and the products of the chosen split match the oracle."""
    B = V.synthetic.standin("GHS_psdef/ldoor", scale=0.005).T.tocsc()
    B = V.SparseMatrix1DVBC[8](B, V.StrictChunker(8))
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0, 0, 0, 0], split="auto", forward=forward, transposed=transposed)
    assert S.split == want
    rng = np.random.default_rng(9)
    R = ref_of(B)
    for trans in ([True] if transposed else []) + ([False] if forward else []):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        x = rng.uniform(-1, 1, nx)
        y = dev(np.full(ny, np.nan))
        V.mul_(y, S.T if trans else S, dev(x))
        assert rel(y.cpu().numpy(), O.mul(R, x, np.zeros(ny), trans=trans)) <= TOL64, trans
    S.release()


@pytest.mark.parametrize("split", ["stripes", "rows"])
@pytest.mark.parametrize("which", ["ldoor", "random"])
def test_x_spans_cover_every_read(mat, split, which):
    """vbc_sharded_xspan: a shard's disjoint-output product (stripes: B'x, rows: B x) reads x only inside its
    span -- what devices[0] sends a shard on another GPU instead of broadcasting x.  Each shard's product with
    x poisoned (NaN) outside the span equals its product with the whole x bit for bit; on the mesh stand-in
    the spans are a share of x plus a halo, far narrower than x."""
    import ctypes as C
    from sparsematrixvbcs_amd import _lib as L
    if which == "ldoor":
        B = V.SparseMatrix1DVBC[8](V.synthetic.standin("GHS_psdef/ldoor", scale=0.01).T.tocsc(), V.StrictChunker(8))
    else:
        B = mat
    world = 4
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=[0] * world, split=split)
    trans = split == "stripes"
    nx = B.m if trans else B.n
    rng = np.random.default_rng(21)
    x = rng.uniform(-1, 1, nx)
    stream = torch.cuda.current_stream().cuda_stream
    spans, shards = S.x_spans(), S.shards()
    try:
        for g, ((lo, hi), (a, b, _)) in enumerate(zip(spans, shards)):
            assert 0 <= lo <= hi <= nx, (g, lo, hi)
            ny = b - a
            xp = x.copy()
            xp[:lo] = np.nan
            xp[hi:] = np.nan
            ys = []
            for xv in (x, xp):
                xd = dev(xv)
                y = torch.full((ny,), float("nan"), dtype=torch.float64, device=DEV)
                L.check(L.lib().vbc_mul(S.shard_handle(g), int(trans), xd.data_ptr(), nx, y.data_ptr(), ny, 1.0, 0.0,
                                        L.VBC_MEM_DEVICE, stream, 0))
                torch.cuda.synchronize()
                ys.append(y.cpu().numpy())
            assert not np.isnan(ys[1]).any(), (g, lo, hi)
            assert np.array_equal(ys[0], ys[1]), g
        if which == "ldoor":  # row-major 3D mesh: each shard's x is its quarter plus a halo
            assert max(hi - lo for lo, hi in spans) < 0.5 * nx, spans
        # and the sharded product as a whole (the spans are what a distinct-device exchange sends)
        y = torch.full((B.n if trans else B.m,), float("nan"), dtype=torch.float64, device=DEV)
        V.mul_(y, S.T if trans else S, dev(x))
        ny = len(y)
        assert rel(y.cpu().numpy(), O.mul(ref_of(B), x, np.zeros(ny), trans=trans)) <= TOL64
    finally:
        S.release()
