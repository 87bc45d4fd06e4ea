"""Multi-GPU products: one process per GPU, torch.distributed (RCCL over xGMI for `nccl`).

SURVEY.md §8e.  The reference's only parallel region is the threaded stripe loop of the transposed
product (multiply_1DVBC.jl:169-177, multiply_VBC.jl:182-189); here the stripes (or the rows) of the
stored matrix B (m x n) are split into contiguous ranges balanced by HBM bytes, one per rank, and
every rank builds its own libvbc handle from its slice:

  split="stripes" (block rows of A when B stores Aᵀ, as bin/test_table.jl:27 does):
    * mul!(y, B', x): each rank owns the y columns of its stripes -> no data-path collective
      (`local_mul_t`); `mul_t` replicates y with one all_gather;
    * mul!(y, B, x): each rank forms the partial α·B_r·x_r over its columns and one
      all_reduce(sum) combines them (the north star's "RCCL all-reduce of y").
  split="rows" (every stripe's stored rows filtered to the rank's row range at create time):
    * mul!(y, B, x): each rank owns y rows [r0, r1) -> no data-path collective (`local_mul`);
      `mul` replicates y with one all_gather;
    * mul!(y, B', x): partial y from the rank's rows, one all_reduce(sum).

Each rank's handle covers only what its shard touches: a stripe shard's rows are rebased to the span its
stripes store (`rebase_rows`), a row shard drops the stripes that store none of its rows (`trim_stripes`), so
the partial-output product writes that span (the rest of the partial is zero) instead of every row or column
(the ldoor 1/8 stripe shard's B x: 16.4 -> 11.9 us), and x is read from the matching slice.

`comm="cpu"` runs the collectives on host copies (gloo process groups on one GPU in tests); the
per-rank product is always libvbc's GPU kernel unless a `local_mul` is injected (CPU-only tests).
The reference has no distributed code at all; this is new in the build.
"""
import numpy as np

from .matrices import SparseMatrix1DVBC, _simd_pad
from .partition import SplitPartition


def stripe_split(B, parts):
    """Stripe boundaries l_0 = 0 < ... < l_parts = L (0-based) balancing HBM bytes per part."""
    L = len(B.Phi)
    esz = B.val.dtype.itemsize
    rows = np.diff(B.pos)
    cost = np.concatenate([[0], np.cumsum(np.diff(B.ofs) * esz + rows * 4 + 12, dtype=np.float64)])
    targets = cost[-1] * np.arange(1, parts) / parts
    cuts = np.searchsorted(cost, targets, side="left")
    cuts = np.clip(cuts, 0, L)
    return np.concatenate([[0], np.maximum.accumulate(cuts), [L]]).astype(np.int64)


def shard(B, lo, hi):
    """Stripes [lo, hi) of B as a stand-alone SparseMatrix1DVBC (m x n_local) and its first column."""
    spl = B.Phi.spl[lo:hi + 1]
    col0 = int(spl[0] - 1)
    pos, ofs = B.pos[lo:hi + 1], B.ofs[lo:hi + 1]
    idx = B.idx[pos[0] - 1:pos[-1] - 1]
    nv = int(ofs[-1] - ofs[0])
    val = np.zeros(nv + _simd_pad(B.W, B.val.dtype), B.val.dtype)  # keep the SIMD tail pad
    val[:nv] = B.val[ofs[0] - 1:ofs[-1] - 1]
    S = SparseMatrix1DVBC(B.W, B.m, int(spl[-1] - spl[0]), SplitPartition(spl - col0), pos - (pos[0] - 1), idx,
                          ofs - (ofs[0] - 1), val)
    return S, col0


def _row_widths(B):
    """Width of the stripe of every stored row (length q)."""
    w = np.diff(B.Phi.spl)
    return np.repeat(w, np.diff(B.pos))


def row_runs(B):
    """The largest R in {3, 2} such that R divides m and every stripe's stored rows come in aligned runs of
    R consecutive rows (a node's dof rows in a stiffness operator); 1 otherwise."""
    idx = B.idx.astype(np.int64) - 1
    cnt = np.diff(B.pos).astype(np.int64)
    for R in (3, 2):
        if B.m % R or np.any(cnt % R):
            continue
        if len(idx) == 0:
            return R
        ph = (np.arange(len(idx), dtype=np.int64) - np.repeat(B.pos[:-1].astype(np.int64) - 1, cnt)) % R
        if not np.all(idx % R == ph):  # the k-th stored row of a run sits at row k of its aligned group
            continue
        cont = (ph[:-1] == R - 1) | (idx[1:] == idx[:-1] + 1)  # inside a run the rows are consecutive
        if np.all(cont):
            return R
    return 1


def row_split(B, parts, align=None):
    """Row boundaries r_0 = 0 < ... < r_parts = m (0-based) balancing the stored bytes per part, each a
    multiple of `align` (default row_runs(B): a cut never splits a node's rows, so every row shard keeps
    the node-blocked layouts -- the forward lane pairs / row runs need m_local % 3 == 0)."""
    esz = B.val.dtype.itemsize
    per_row = np.bincount(B.idx - 1, weights=_row_widths(B) * esz + 4, minlength=B.m)
    cost = np.concatenate([[0.0], np.cumsum(per_row)])
    targets = cost[-1] * np.arange(1, parts) / parts
    cuts = np.clip(np.searchsorted(cost, targets, side="left"), 0, B.m)
    a = row_runs(B) if align is None else int(align)
    if a > 1:
        cuts = np.clip((cuts + a // 2) // a * a, 0, B.m)
    return np.concatenate([[0], np.maximum.accumulate(cuts), [B.m]]).astype(np.int64)


def row_shard(B, r0, r1):
    """Rows [r0, r1) of B: every stripe keeps its stored rows inside the range (in stored order, so the
    per-stripe summation order of mul!(y, B', x) is the reference's); returns an (r1-r0) x n matrix."""
    w = _row_widths(B)
    keep = (B.idx > r0) & (B.idx <= r1)
    L = len(B.Phi)
    stripe = np.repeat(np.arange(L), np.diff(B.pos))
    counts = np.bincount(stripe[keep], minlength=L).astype(np.int64)
    pos = np.concatenate([[1], 1 + np.cumsum(counts)]).astype(np.int64)
    wl = np.diff(B.Phi.spl)
    ofs = np.concatenate([[1], 1 + np.cumsum(counts * wl)]).astype(np.int64)
    # value offsets of the kept rows: ofs[l] + (Q - pos[l]) * w_l
    q0 = np.arange(len(B.idx), dtype=np.int64) - (B.pos[stripe] - 1)
    start = (B.ofs[stripe] - 1) + q0 * w
    ks, kw = start[keep], w[keep]
    nv = int(ofs[-1] - 1)
    if nv:
        elem = np.repeat(ks - np.concatenate([[0], np.cumsum(kw)[:-1]]), kw) + np.arange(nv)
    else:
        elem = np.zeros(0, np.int64)
    val = np.zeros(nv + _simd_pad(B.W, B.val.dtype), B.val.dtype)
    val[:nv] = B.val[elem]
    return SparseMatrix1DVBC(B.W, int(r1 - r0), B.n, SplitPartition(B.Phi.spl.copy()), pos, B.idx[keep] - r0, ofs,
                             val)


def rebase_rows(S):
    """S restricted to the span of rows its stripes store: (the (hi - lo) x n matrix, lo).  A shard of a mesh
    operator's stripes stores its own rows plus a halo; its forward product then writes that span only, and
    its transposed product reads x[lo:hi].  (S itself, 0 when it stores no row or spans every row.)"""
    if len(S.idx) == 0:
        return S, 0
    lo, hi = int(S.idx.min()) - 1, int(S.idx.max())
    if lo == 0 and hi == S.m:
        return S, 0
    return SparseMatrix1DVBC(S.W, hi - lo, S.n, S.Phi, S.pos, S.idx - lo, S.ofs, S.val), lo


def trim_stripes(S):
    """S without its leading and trailing stripes that store no row: (the matrix, its first column).  A row
    shard of a mesh operator keeps the stripes of its rows plus a halo."""
    nz = np.nonzero(np.diff(S.pos))[0]
    if len(nz) == 0 or (nz[0] == 0 and nz[-1] == len(S.Phi) - 1):
        return S, 0
    return shard(S, int(nz[0]), int(nz[-1]) + 1)


# --- cost model of a sharded product --------------------------------------------
# Shard kernel: a fixed launch-and-ramp cost plus its bytes at the streaming rate one MI355X sustains -- both
# MEASURED on this code (a graph-replayed near-empty product 3.1 us; tools/exp/keep_probe.hip
# streams 52-110 MB at 5.7-6.4 TB/s).  Collectives: ASSUMED, not measured (no multi-GPU box was ever
# available to this build): each MI355X has 7 xGMI links of 153.6 GB/s (bidirectional: 76.8 GB/s per
# direction); a ring collective over the node is taken to reach COLL_EFF of the 7 links' one-way rate, and
# every ring step costs COLL_STEP_US of latency.  include/vbc.h states the same constants (VBC_SPLIT_AUTO).
KERNEL_T0_US = 3.1
KERNEL_GBS = 5700.0
XGMI_LINKS, XGMI_LINK_GBS, COLL_EFF, COLL_STEP_US = 7, 76.8, 0.6, 2.0
COLL_GBS = XGMI_LINKS * XGMI_LINK_GBS * COLL_EFF  # ~323 GB/s per GPU (assumption)


def collective_us(kind, nbytes, world):
    """Predicted time of one RCCL collective over `world` GPUs of one node (the assumptions above):
    ring all-reduce 2(N-1)/N x bytes, all-gather / reduce-scatter / reduce (N-1)/N x bytes of the full
    vector, broadcast the whole vector once; plus the ring's per-step latency."""
    if world <= 1 or nbytes <= 0:
        return 0.0
    n = world
    vol, steps = {"allreduce": (2.0 * (n - 1) / n, 2 * (n - 1)), "allgather": ((n - 1) / n, n - 1),
                  "reduce": ((n - 1) / n, n - 1), "broadcast": (1.0, n - 1)}[kind]
    return vol * nbytes / (COLL_GBS * 1e3) + steps * COLL_STEP_US


def _matrix_bytes(B, ti=4):
    esz = B.val.dtype.itemsize
    return esz * int(B.ofs[-1] - 1) + ti * int(B.pos[-1] - 1) + ti * (3 * len(B.Phi) + 3)


def predict_product_us(B, world, split, trans, replicate=True):
    """Predicted wall time of one sharded product mul!(y, op(B), x) (us): the slowest shard's kernel (its
    matrix bytes, its x reads and y writes) plus the collective its exchange pattern needs --
    a disjoint output needs none (an all-gather when `replicate` asks for y on every rank), a partial
    output one all-reduce of y.  Returns (total, kernel, collective)."""
    esz = B.val.dtype.itemsize
    nx, ny = (B.m, B.n) if trans else (B.n, B.m)
    mat = _matrix_bytes(B) / world
    if split == "rows" and world > 1:
        mat += 12.0 * len(B.Phi) * (world - 1) / world  # every row shard keeps every stripe's headers
    disjoint = (split == "stripes") == bool(trans)
    xb = esz * (nx if disjoint else nx / world)
    yb = esz * (ny / world if disjoint else ny)
    kern = KERNEL_T0_US + (mat + xb + yb) / (KERNEL_GBS * 1e3)
    if disjoint:
        coll = collective_us("allgather", esz * ny, world) if replicate else 0.0
    else:
        coll = collective_us("allreduce", esz * ny, world)
    return kern + coll, kern, coll


def choose_split(B, world, directions="tf", replicate=True):
    """The split ("stripes" / "rows") with the smaller predicted time summed over the products a caller
    will run (`directions`: "t" mul!(y, B', x), "f" mul!(y, B, x)); ties go to the stripe split (the
    reference's own parallel direction, multiply_1DVBC.jl:169-177)."""
    cost = {}
    for split in ("stripes", "rows"):
        cost[split] = sum(predict_product_us(B, world, split, d == "t", replicate)[0] for d in directions)
    return "rows" if cost["rows"] < cost["stripes"] * (1 - 1e-9) else "stripes"


class ShardedSparseMatrix1DVBC:
    """A SparseMatrix1DVBC split across the ranks of `group` (torch.distributed), one libvbc handle
    per rank.  See the module docstring for the two splits and which product needs a collective."""

    def __init__(self, B, rank, world, group=None, local_mul=None, device=None, split="stripes", comm="device",
                 directions="tf"):
        if split == "auto":  # by the cost model: predicted kernel + collective time of the products to run
            split = choose_split(B, world, directions)
        if split not in ("stripes", "rows"):
            raise ValueError("split must be 'stripes', 'rows' or 'auto'")
        if comm not in ("device", "cpu"):
            raise ValueError("comm must be 'device' or 'cpu'")
        self.m, self.n, self.W = B.m, B.n, B.W
        self.rank, self.world, self.group = rank, world, group
        self.split, self.comm = split, comm
        # the local handle covers rows [row0, row0 + m_local) and columns [col0, col0 + n_local) of B
        if split == "stripes":
            self.cuts = stripe_split(B, world)
            self.splits = [int(c) for c in (B.Phi.spl[self.cuts] - 1)]  # column ranges
            sh, self.col0 = shard(B, int(self.cuts[rank]), int(self.cuts[rank + 1]))
            self.local, self.row0 = rebase_rows(sh)
        else:
            self.cuts = row_split(B, world)
            self.splits = [int(c) for c in self.cuts]  # row ranges
            self.row0 = int(self.cuts[rank])
            self.local, self.col0 = trim_stripes(row_shard(B, self.row0, int(self.cuts[rank + 1])))
        self.m_local, self.n_local = self.local.m, self.local.n
        self.col_splits = self.splits if split == "stripes" else None  # (round-1 name)
        if local_mul is None:
            from .multiply import mul_
            local_mul = mul_
        self._product = local_mul  # mul!(y, op, x, α, β) on this rank's handle
        self.device = device

    # --- collectives ----------------------------------------------------------------------------
    def _all_reduce(self, t):
        import torch.distributed as dist
        if self.comm == "cpu" and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def _gather_bufs(self, dtype, dev):
        """The padded send slice and the world x max-slice receive buffer of `gather`, allocated once
        per (eltype, device) and reused by every later call (no allocation in a solver's loop)."""
        import torch
        key = (dtype, str(dev))
        bufs = getattr(self, "_gbufs", None)
        if bufs is None:
            bufs = self._gbufs = {}
        if key not in bufs:
            ms = max(self.splits[r + 1] - self.splits[r] for r in range(self.world))
            bufs[key] = (torch.zeros(ms, dtype=dtype, device=dev), torch.empty(self.world * ms, dtype=dtype, device=dev))
        return bufs[key]

    def gather(self, y_local, out=None):
        """Replicated vector from every rank's slice of the split dimension: one all_gather of
        equal-length padded slices into a preallocated buffer; written into `out` when given (the
        product loop then allocates nothing), else into a new tensor."""
        import torch
        import torch.distributed as dist
        sizes = [self.splits[r + 1] - self.splits[r] for r in range(self.world)]
        dev = torch.device("cpu") if self.comm == "cpu" else y_local.device
        buf, flat = self._gather_bufs(y_local.dtype, dev)
        buf[:len(y_local)].copy_(y_local)
        dist.all_gather_into_tensor(flat, buf, group=self.group)
        if out is None:
            out = torch.empty(self.splits[-1] - self.splits[0], dtype=y_local.dtype, device=y_local.device)
        ms = buf.shape[0]
        for r, s in enumerate(sizes):
            out[self.splits[r] - self.splits[0]:self.splits[r] - self.splits[0] + s].copy_(flat[r * ms:r * ms + s])
        return out

    @staticmethod
    def _outside(y, lo, n, beta):
        """The entries of a full-length partial outside [lo, lo + n): beta * y (0 when beta is 0; then the
        whole vector is zeroed in one fill -- the product overwrites [lo, lo + n) -- one launch, not two)."""
        if beta == 0.0:
            y.zero_()
            return
        if beta != 1.0:
            for part in (y[:lo], y[lo + n:]):
                part.mul_(beta)

    # --- mul!(y, B', x) ---------------------------------------------------------------------------
    def local_mul_t(self, y_local, x, alpha=1.0, beta=0.0):
        """This rank's part of α·B'x + β·y (x: length m, or already its rows [row0, row0 + m_local)).
        stripes: y_local = columns col0 .. col0+n_local-1 of y (final, no collective); rows: y_local is a
        length-n partial -- the product over the rank's columns, zero elsewhere (β applied on rank 0)."""
        xs = x[self.row0:self.row0 + self.m_local] if len(x) == self.m else x
        if self.split == "stripes":
            return self._product(y_local, self.local.T, xs, alpha, beta)
        b = beta if self.rank == 0 else 0.0
        self._outside(y_local, self.col0, self.n_local, b)
        self._product(y_local[self.col0:self.col0 + self.n_local], self.local.T, xs, alpha, b)
        return y_local

    def mul_t(self, y, x, alpha=1.0, beta=0.0):
        """Replicated y (length n) = α·B'x + β·y; x replicated (length m)."""
        if self.split == "stripes":
            part = y[self.col0:self.col0 + self.n_local].clone()
            self.local_mul_t(part, x, alpha, beta)
            return self.gather(part, out=y)
        self.local_mul_t(y, x, alpha, beta)
        return self._all_reduce(y)

    # --- mul!(y, B, x) ----------------------------------------------------------------------------
    def local_mul(self, y_local, x, alpha=1.0, beta=0.0):
        """This rank's part of α·Bx + β·y (x: length n, or already its columns [col0, col0 + n_local)).
        rows: y_local = rows row0 .. row0+m_local-1 of y (final, no collective); stripes: y_local is a
        length-m partial -- the product over the rows the rank's stripes store, zero elsewhere (β applied
        on rank 0)."""
        xs = x[self.col0:self.col0 + self.n_local] if len(x) == self.n else x
        if self.split == "rows":
            return self._product(y_local, self.local, xs, alpha, beta)
        b = beta if self.rank == 0 else 0.0
        self._outside(y_local, self.row0, self.m_local, b)
        self._product(y_local[self.row0:self.row0 + self.m_local], self.local, xs, alpha, b)
        return y_local

    def mul(self, y, x, alpha=1.0, beta=0.0):
        """Replicated y (length m) = α·Bx + β·y; x replicated (length n)."""
        if self.split == "rows":
            part = y[self.row0:self.row0 + self.m_local].clone()
            self.local_mul(part, x, alpha, beta)
            return self.gather(part, out=y)
        self.local_mul(y, x, alpha, beta)
        return self._all_reduce(y)


class MultiGPUSparseMatrix1DVBC:
    """ONE process driving several GPUs: libvbc's sharded handle (include/vbc.h vbc1d_create_sharded /
    vbc2d_create_sharded, RCCL over xGMI between distinct devices).  Same splits as
    ShardedSparseMatrix1DVBC, but the exchange runs inside the library on device pointers of
    devices[0] (the Julia drop-in's configuration: one session, x and y on one device, the other GPUs
    as workers).  B may be a SparseMatrix1DVBC or a SparseMatrixVBC (the 2D transposed product is
    threaded the same way, multiply_VBC.jl:182-189; its row split keeps Π's block rows whole).

        S = MultiGPUSparseMatrix1DVBC(B, devices=[0, 1, 2, 3], split="stripes")
        mul_(y, S.T, x)      # mul!(y, B', x): each shard's x span sent, y slices gathered on devices[0]
        mul_(y, S, x)        # mul!(y, B, x): x slices, ncclReduce(sum) of y

    `devices` all equal (e.g. [0, 0, 0]) runs every shard on that device with no communicator.
    Like the single-GPU mul_, x / y may be any strided vectors of any supported eltype (converted to
    the handle's compute eltype, multiply_1DVBC.jl:9,85,102): vbc_sharded_mul_ex carries them."""

    def __init__(self, B, devices=(0,), split="stripes", transposed=True, forward=True, serial=False):
        import ctypes as C
        from . import _lib as _L
        if split not in ("stripes", "rows", "auto"):
            raise ValueError("split must be 'stripes', 'rows' or 'auto'")
        self.m, self.n, self.W = B.m, B.n, B.W
        self.val = B.val  # eltype queries (mul_ computes in eltype(y))
        self.dtype = B.val.dtype
        self.split = split
        self.is2d = hasattr(B, "Pi")
        self.devices = [int(d) for d in devices]
        flags = ((_L.VBC_CREATE_TRANSPOSED if transposed else 0) | (_L.VBC_CREATE_FORWARD if forward else 0)
                 | (_L.VBC_CREATE_SERIAL if serial else 0))
        t = _L.vbc_types(_L.dtype_code(B.val.dtype), 64, _L.compute_code(B.val.dtype), 0)
        devs = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        kind = {"stripes": _L.VBC_SPLIT_STRIPES, "rows": _L.VBC_SPLIT_ROWS, "auto": _L.VBC_SPLIT_AUTO}[split]
        if self.is2d:
            _L.check(_L.lib().vbc2d_create_sharded(
                C.byref(h), B.m, B.n, B.U, B.W, len(B.Pi), B.Pi.spl.ctypes.data, len(B.Phi), B.Phi.spl.ctypes.data,
                B.pos.ctypes.data, B.idx.ctypes.data, B.ofs.ctypes.data, B.val.ctypes.data, len(B.val), C.byref(t),
                len(self.devices), devs, kind, flags), "create_sharded (2D)")
        else:
            _L.check(_L.lib().vbc1d_create_sharded(
                C.byref(h), B.m, B.n, B.W, len(B.Phi), B.Phi.spl.ctypes.data, B.pos.ctypes.data, B.idx.ctypes.data,
                B.ofs.ctypes.data, B.val.ctypes.data, len(B.val), C.byref(t), len(self.devices), devs, kind, flags),
                "create_sharded")
        self._h = h
        self.compute = t.compute_dtype
        sp = C.c_int()
        _L.check(_L.lib().vbc_sharded_split(h, C.byref(sp)), "split")
        self.split = "stripes" if sp.value == _L.VBC_SPLIT_STRIPES else "rows"  # (what VBC_SPLIT_AUTO chose)

    @property
    def shape(self):
        return (self.m, self.n)

    @property
    def T(self):
        from .matrices import Adjoint
        return Adjoint(self)

    def shards(self):
        """[(lo, hi, device)] per shard: its 0-based range of the split dimension (columns for
        split='stripes', rows for split='rows')."""
        import ctypes as C
        from . import _lib as _L
        out = []
        for g in range(len(self.devices)):
            lo, hi, dev = C.c_int64(), C.c_int64(), C.c_int()
            _L.check(_L.lib().vbc_sharded_shard(self._h, g, None, C.byref(lo), C.byref(hi), C.byref(dev)), "shard")
            out.append((lo.value, hi.value, dev.value))
        return out

    def x_spans(self):
        """[(lo, hi)] per shard: the 0-based span of x its disjoint-output product reads (vbc_sharded_xspan) --
        what devices[0] sends it instead of broadcasting x."""
        import ctypes as C
        from . import _lib as _L
        out = []
        for g in range(len(self.devices)):
            lo, hi = C.c_int64(), C.c_int64()
            _L.check(_L.lib().vbc_sharded_xspan(self._h, g, C.byref(lo), C.byref(hi)), "xspan")
            out.append((lo.value, hi.value))
        return out

    def shard_handle(self, g):
        """Shard g's single-GPU handle (a raw vbc_handle pointer owned by this object)."""
        import ctypes as C
        from . import _lib as _L
        h = C.c_void_p()
        _L.check(_L.lib().vbc_sharded_shard(self._h, g, C.byref(h), None, None, None), "shard")
        return h

    def shard_info(self, g):
        """vbc_get_info of shard g's single-GPU handle (its layouts: planar_split, planar_mask, ...)."""
        import ctypes as C
        from . import _lib as _L
        h = C.c_void_p()
        lo, hi, dev = C.c_int64(), C.c_int64(), C.c_int()
        _L.check(_L.lib().vbc_sharded_shard(self._h, g, C.byref(h), C.byref(lo), C.byref(hi), C.byref(dev)), "shard")
        inf = _L.vbc_info()
        _L.check(_L.lib().vbc_get_info(h, C.byref(inf)), "info")
        return {f: getattr(inf, f) for f, _ in _L.vbc_info._fields_}

    def _mul(self, y, x, trans, alpha, beta, stream, quirks):
        from . import _lib as _L
        from .multiply import _mem_device_stream, _stride
        if len(x.shape) != 1 or len(y.shape) != 1:
            raise _L.ArgumentError("the multi-GPU product takes vectors")
        nx, ny = x.shape[0], y.shape[0]
        if (nx, ny) != ((self.m, self.n) if trans else (self.n, self.m)):
            raise _L.DimensionMismatch(f"size(A)={self.shape}, length(x)={nx}, length(y)={ny}")
        xdt, ydt = _L.dtype_code(x.dtype), _L.dtype_code(y.dtype)
        mem, dev, stream = _mem_device_stream(x, y, stream)
        if mem == _L.VBC_MEM_DEVICE and dev != self.devices[0]:
            raise _L.ArgumentError(f"x and y must live on devices[0] = cuda:{self.devices[0]}")
        flags = _L.VBC_MUL_REFERENCE_QUIRKS if quirks else 0
        _L.check(_L.lib().vbc_sharded_mul_ex(self._h, int(trans), _L.ptr(x), xdt, _stride(x), nx, _L.ptr(y), ydt,
                                             _stride(y), ny, float(alpha), float(beta), mem, stream, flags),
                 "mul! (sharded)")
        return y

    def release(self):
        from . import _lib as _L
        if getattr(self, "_h", None):
            _L.lib().vbc_sharded_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


MultiGPUSparseMatrix = MultiGPUSparseMatrix1DVBC  # either format (1DVBC or VBC)
