"""Multi-GPU products: one process per GPU, torch.distributed (RCCL over xGMI for `nccl`).

SURVEY.md §8e.  The stored matrix B (m x n, column stripes) is split into contiguous stripe ranges
balanced by bytes (a stripe's share = w·|rows|·sizeof(Tv) + 4·|rows| + 12), one per rank:
  * mul!(y, B', x): each rank owns the y columns of its stripes -> no data-path collective; the
    optional `gather` assembles the full y with one all_gather;
  * mul!(y, B, x):  each rank forms the partial α·B_r·x_r over its columns, one all_reduce(sum)
    combines them and β·y is applied once.
The reference has no distributed code at all; this is new in the build.
"""
import numpy as np

from .matrices import SparseMatrix1DVBC
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
    val = B.val[ofs[0] - 1:ofs[-1] - 1]
    S = SparseMatrix1DVBC(B.W, B.m, int(spl[-1] - spl[0]), SplitPartition(spl - col0), pos - (pos[0] - 1), idx,
                          ofs - (ofs[0] - 1), val)
    return S, col0


class ShardedSparseMatrix1DVBC:
    """Stripe-sharded SparseMatrix1DVBC across the ranks of `group` (torch.distributed).

    `local_mul(y, op, x, alpha, beta)` performs this rank's product; it defaults to the libvbc GPU
    path (sparsematrixvbcs.mul_) and exists so the collective logic can be exercised with gloo on CPU
    tests (there is no CPU fallback in the product path)."""

    def __init__(self, B, rank, world, group=None, local_mul=None, device=None):
        self.m, self.n, self.W = B.m, B.n, B.W
        self.rank, self.world, self.group = rank, world, group
        self.cuts = stripe_split(B, world)
        self.col_splits = [int(B.Phi.spl[c] - 1) for c in self.cuts]
        self.local, self.col0 = shard(B, int(self.cuts[rank]), int(self.cuts[rank + 1]))
        self.n_local = self.local.n
        if local_mul is None:
            from .multiply import mul_
            local_mul = mul_
        self.local_mul = local_mul
        self.device = device

    # --- mul!(y, B', x): no data-path collective -------------------------------------------------
    def mul_t(self, y_local, x, alpha=1.0, beta=0.0):
        """y_local (length n_local: columns col0 .. col0+n_local-1 of y) = α·B_rᵀ x + β·y_local."""
        return self.local_mul(y_local, self.local.T, x, alpha, beta)

    def gather(self, y_local):
        """Full y (length n) from every rank's slice: one all_gather of equal-length padded slices."""
        import torch
        import torch.distributed as dist
        sizes = [self.col_splits[r + 1] - self.col_splits[r] for r in range(self.world)]
        mx = max(sizes)
        buf = torch.zeros(mx, dtype=y_local.dtype, device=y_local.device)
        buf[:self.n_local] = y_local
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf, group=self.group)
        return torch.cat([o[:s] for o, s in zip(outs, sizes)])

    # --- mul!(y, B, x): one all_reduce -----------------------------------------------------------
    def mul(self, y, x, alpha=1.0, beta=0.0):
        """y (length m, replicated) = α·B x + β·y; x is the full (replicated) vector of length n."""
        import torch
        import torch.distributed as dist
        part = torch.empty_like(y)
        self.local_mul(part, self.local, x[self.col0:self.col0 + self.n_local], alpha, 0.0)
        dist.all_reduce(part, op=dist.ReduceOp.SUM, group=self.group)
        if beta == 0.0:
            y.copy_(part)
        else:
            y.mul_(beta).add_(part)
        return y
