"""Synthetic variable-block matrices for parity tests and the benchmark.

Follows the reference's own VBR generator (costs.jl:63-83): draw q distinct (row i, stripe l) pairs
uniformly and store a full w-wide dense row for each, values rand(Tv) ~ U[0, 1).  The fields are
produced directly in the reference layout (1-based Int64 spl/pos/idx/ofs + val), exactly what
`SparseMatrix1DVBC{W}(sparse(I, J, V, m, n), pack_stripe(A, EquiChunker(w)))` would hold for that
matrix (constructors_1DVBC.jl:9-92), without materialising the CSC.
"""
import numpy as np

from .matrices import SparseMatrix1DVBC, SparseMatrixVBC, _simd_pad
from .partition import SplitPartition


def vbr_1dvbc(m, L, q, widths, W=8, dtype=np.float64, seed=0xDEADBEEF, pad=True):
    """m rows, L stripes with widths `widths` (int or length-L array), ~q stored rows.

    Returns a SparseMatrix1DVBC whose stripe l has the distinct sorted rows drawn for it."""
    rng = np.random.default_rng(seed)
    w = np.broadcast_to(np.asarray(widths, dtype=np.int64), (L,)).copy()
    if w.max(initial=1) > W:
        raise ValueError("stripe width exceeds W")
    keys = np.unique(rng.integers(0, np.int64(m) * L, size=int(q), dtype=np.int64))  # sorted by (l, i)
    stripe = keys // m
    row = keys - stripe * m
    counts = np.bincount(stripe, minlength=L).astype(np.int64)
    spl = np.empty(L + 1, np.int64)
    spl[0] = 1
    np.cumsum(w, out=spl[1:])
    spl[1:] += 1
    pos = np.empty(L + 1, np.int64)
    pos[0] = 1
    np.cumsum(counts, out=pos[1:])
    pos[1:] += 1
    ofs = np.empty(L + 1, np.int64)
    ofs[0] = 1
    np.cumsum(counts * w, out=ofs[1:])
    ofs[1:] += 1
    nv = int(ofs[-1] - 1)
    padn = _simd_pad(W, dtype) if pad else 0
    val = np.empty(nv + padn, dtype)
    val[:nv] = rng.random(nv, dtype=np.float64 if dtype == np.float64 else np.float32)
    val[nv:] = 0
    n = int(spl[-1] - 1)
    return SparseMatrix1DVBC(W, m, n, SplitPartition(spl), pos, row + 1, ofs, val)


def vbr_1dvbc_banded(m, L, q, widths, band, W=8, dtype=np.float64, seed=0xDEADBEEF):
    """vbr_1dvbc with x locality: stripe l draws its rows from a window of `band` rows centred on its
    own position scaled to m (row l * m / L), as a mesh operator's column block does -- the GPU
    kernels then stream the layout instead of gathering from all of x (costs.py, locality="banded")."""
    rng = np.random.default_rng(seed)
    w = np.broadcast_to(np.asarray(widths, dtype=np.int64), (L,)).copy()
    if w.max(initial=1) > W:
        raise ValueError("stripe width exceeds W")
    band = int(max(1, min(band, m)))
    stripe = rng.integers(0, L, size=int(q), dtype=np.int64)
    lo = np.clip(stripe * m // max(L, 1) - band // 2, 0, m - band)
    row = lo + rng.integers(0, band, size=int(q), dtype=np.int64)
    keys = np.unique(stripe * m + row)  # sorted by (l, i), distinct
    stripe = keys // m
    row = keys - stripe * m
    counts = np.bincount(stripe, minlength=L).astype(np.int64)
    spl = np.concatenate([[1], 1 + np.cumsum(w)]).astype(np.int64)
    pos = np.concatenate([[1], 1 + np.cumsum(counts)]).astype(np.int64)
    ofs = np.concatenate([[1], 1 + np.cumsum(counts * w)]).astype(np.int64)
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + _simd_pad(W, dtype), dtype)
    val[:nv] = rng.random(nv, dtype=np.float64 if dtype == np.float64 else np.float32)
    return SparseMatrix1DVBC(W, m, int(spl[-1] - 1), SplitPartition(spl), pos, row + 1, ofs, val)


def north_star(dtype=np.float64, scale=1.0, seed=0xDEADBEEF, mixed=False):
    """NS-1DVBC: 10^7 x 10^7, W = 8, w = 4, 2.5e6 stripes, 10 row-blocks per stripe
    on average -> q = 2.5e7 stored rows, nnz = 1.0e8, no fill.  `mixed`: w ~ U{1..8} per stripe with
    the row count chosen so that nnz is still ~1e8.  `scale` shrinks every dimension (tests)."""
    m = int(round(1e7 * scale))
    if mixed:
        rng = np.random.default_rng(seed ^ 0x5EED)
        L = int(round(1e7 * scale / 4.5))  # E[w] = 4.5 -> n ~ 1e7
        w = rng.integers(1, 9, L)
        q = int(round(1e8 * scale / w.mean()))
        return vbr_1dvbc(m, L, q, w, 8, dtype, seed)
    L = m // 4
    return vbr_1dvbc(m, L, int(round(2.5e7 * scale)), 4, 8, dtype, seed)


def fe_grid_2d(N, dof=2, W=8, dtype=np.float64, seed=0xDEADBEEF):
    """SuiteSparse-like finite-element operator: the 5-point stencil on an N x N node grid with
    `dof` unknowns per node (dense dof x dof coupling blocks), as a 1DVBC whose stripes are the node
    columns (what StrictChunker finds: the dof columns of a node share one pattern).  N = 2236,
    dof = 2 gives 1.0e7 x 1.0e7 with 1.0e8 stored values, no fill -- the 'SuiteSparse-like'
    north-star size of BASELINE.json with the locality of a mesh (x gathers hit cache)."""
    rng = np.random.default_rng(seed)
    nodes = N * N
    node = np.arange(nodes, dtype=np.int64)
    a, b = node // N, node % N
    offs = np.array([-N, -1, 0, 1, N], dtype=np.int64)  # ascending neighbour order
    valid = np.stack([a > 0, b > 0, np.ones(nodes, bool), b < N - 1, a < N - 1], axis=1)
    nb = (node[:, None] + offs[None, :])[valid]          # neighbours, row-major by node: sorted
    cnt = valid.sum(axis=1).astype(np.int64)             # neighbour blocks per stripe
    rows = (nb[:, None] * dof + np.arange(dof)[None, :]).reshape(-1)  # 0-based x rows
    L = nodes
    spl = 1 + np.arange(L + 1, dtype=np.int64) * dof
    pos = np.empty(L + 1, np.int64)
    pos[0] = 1
    np.cumsum(cnt * dof, out=pos[1:])
    pos[1:] += 1
    ofs = np.empty(L + 1, np.int64)
    ofs[0] = 1
    np.cumsum(cnt * dof * dof, out=ofs[1:])
    ofs[1:] += 1
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + _simd_pad(W, dtype), dtype)
    val[:nv] = rng.random(nv, dtype=np.float64 if dtype == np.float64 else np.float32)
    m = nodes * dof
    return SparseMatrix1DVBC(W, m, m, SplitPartition(spl), pos, rows + 1, ofs, val)


def vbr_2d(K, L, q, u, w, U=None, W=None, dtype=np.float32, seed=0xDEADBEEF, pad=True):
    """The reference's 2D VBR generator (costs.jl:200-220): q distinct (block row k, stripe l) pairs
    drawn uniformly from K x L, each a dense u x w tile of rand(Tv); m = u*K, n = w*L.  Fields are
    produced directly in the SparseMatrixVBC{U,W} layout (constructors_VBC.jl:95-105: per stripe,
    blocks in ascending k, tile row-major, idx = block-row id) -- what
    SparseMatrixVBC{U,W}(A, pack_stripe(A', EquiChunker(u)), pack_stripe(A, EquiChunker(w))) holds."""
    U = u if U is None else U
    W = w if W is None else W
    rng = np.random.default_rng(seed)
    keys = np.unique(rng.integers(0, np.int64(K) * L, size=int(q), dtype=np.int64))  # sorted by (l, k)
    stripe = keys // K
    krow = keys - stripe * K
    counts = np.bincount(stripe, minlength=L).astype(np.int64)
    pspl = 1 + np.arange(K + 1, dtype=np.int64) * u
    spl = 1 + np.arange(L + 1, dtype=np.int64) * w
    pos = np.empty(L + 1, np.int64)
    pos[0] = 1
    np.cumsum(counts, out=pos[1:])
    pos[1:] += 1
    ofs = 1 + np.concatenate([[0], np.cumsum(counts * (u * w))]).astype(np.int64)
    nv = int(ofs[-1] - 1)
    padn = _simd_pad(W, dtype) if pad else 0
    val = np.empty(nv + padn, dtype)
    val[:nv] = rng.random(nv, dtype=np.float64 if dtype == np.float64 else np.float32)
    val[nv:] = 0
    return SparseMatrixVBC(U, W, u * K, w * L, SplitPartition(pspl), SplitPartition(spl), pos, krow + 1, ofs, val)


def c5(dtype=np.float32, scale=1.0, u=8, w=8, seed=0xDEADBEEF):
    """Config C5 (BASELINE.json): 2D SparseMatrixVBC, dense u x w tiles, for the 16-RHS product.
    Full size: K = L = 2^18 block rows / stripes (m = n = 2,097,152 at u = w = 8), 6 tiles per stripe
    on average (q = 1,572,864) -> 1.0e8 stored values."""
    K = max(4, int(round(2 ** 18 * scale)))
    L = max(4, int(round(2 ** 18 * scale * 8 / w)))
    q = int(round(6 * L * 64 / (u * w)))
    return vbr_2d(K, L, q, u, w, dtype=dtype, seed=seed)


# SuiteSparse matrices of BASELINE.json's configs C2-C4 (not available offline): (n, nnz) from the
# reference's own output (ct20stif: src/ref.out:29-32) and the SuiteSparse index (ldoor).
STANDINS = {"Boeing/ct20stif": (52329, 2600295), "GHS_psdef/ldoor": (952203, 42493817)}


def _stiffness_blocks(n, nnz, dof, seed):
    """Block structure of fe_stiffness_3d: node pairs (bi, bj) -- the N diagonal blocks, then each kept
    neighbour pair in both orientations -- and their dof x dof values (symmetric overall)."""
    if n % dof:
        raise ValueError("n must be a multiple of dof")
    rng = np.random.default_rng(seed)
    N = n // dof
    g = int(np.ceil(N ** (1 / 3)))
    node = np.arange(N, dtype=np.int64)
    a, b, c = node // (g * g), (node // g) % g, node % g
    offs = [(da, db, dc) for da in (-1, 0, 1) for db in (-1, 0, 1) for dc in (-1, 0, 1)
            if 0 < abs(da) + abs(db) + abs(dc) <= 2]
    pairs = []
    for da, db, dc in offs:
        if (da, db, dc) <= (0, 0, 0):  # each unordered pair once (lexicographically positive offsets)
            continue
        aa, bb, cc = a + da, b + db, c + dc
        ok = (aa >= 0) & (aa < g) & (bb >= 0) & (bb < g) & (cc >= 0) & (cc < g)
        nb = aa * g * g + bb * g + cc
        ok &= nb < N
        pairs.append(np.stack([node[ok], nb[ok]], axis=1))
    pairs = np.concatenate(pairs)
    want = int(round(nnz / (dof * dof)))  # blocks: N diagonal + 2 per kept pair
    keep = max(0, min(len(pairs), (want - N) // 2))
    pairs = pairs[np.sort(rng.choice(len(pairs), keep, replace=False))]
    bi = np.concatenate([node, pairs[:, 0], pairs[:, 1]])
    bj = np.concatenate([node, pairs[:, 1], pairs[:, 0]])
    blk = rng.uniform(-1, 1, (N + keep, dof, dof))
    diag = (blk[:N] + np.transpose(blk[:N], (0, 2, 1))) / 2
    vals = np.concatenate([diag, blk[N:], np.transpose(blk[N:], (0, 2, 1))])
    return N, bi, bj, vals


def fe_stiffness_3d(n, nnz, dof=3, dtype=np.float64, seed=0xDEADBEEF):
    """A symmetric 3D finite-element stiffness stand-in with exactly n rows and nnz within 9 of the
    target: n/dof mesh nodes on a near-cubic grid (row-major), each node coupled to itself and to a
    random symmetric subset of its 18 face/edge neighbours, every coupling a dense dof x dof block of
    U[-1, 1) values (symmetric: block(j, i) = block(i, j)').  Returns a sorted scipy CSC matrix."""
    import scipy.sparse as sp
    N, bi, bj, vals = _stiffness_blocks(n, nnz, dof, seed)
    r = (bi[:, None, None] * dof + np.arange(dof)[None, :, None]).repeat(dof, axis=2)
    cidx = (bj[:, None, None] * dof + np.arange(dof)[None, None, :]).repeat(dof, axis=1)
    A = sp.csc_matrix((vals.reshape(-1).astype(dtype), (r.reshape(-1), cidx.reshape(-1))), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    return A


def fe_stiffness_3d_1dvbc(n, nnz, dof=3, W=8, dtype=np.float64, seed=0xDEADBEEF):
    """fe_stiffness_3d(n, nnz, dof) directly as SparseMatrix1DVBC{W} with one stripe per mesh node
    (= SparseMatrix1DVBC{W}(A, EquiChunker(dof)) on that matrix, without materialising the CSC):
    stripe j holds, for every coupled node i in ascending order, the dof rows i*dof .. i*dof+dof-1,
    each the dof-wide row of block(i, j).  Irregular rows per stripe (1 + a random subset of 18
    neighbours) -- the SuiteSparse-like 3D counterpart of fe_grid_2d at any size."""
    N, bi, bj, vals = _stiffness_blocks(n, nnz, dof, seed)
    order = np.lexsort((bi, bj))  # by stripe (node column j), then row node i
    bi, bj, vals = bi[order], bj[order], vals[order]
    cnt = np.bincount(bj, minlength=N).astype(np.int64)  # blocks per stripe
    spl = 1 + np.arange(N + 1, dtype=np.int64) * dof
    pos = np.concatenate([[1], 1 + np.cumsum(cnt * dof)]).astype(np.int64)
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * dof * dof)]).astype(np.int64)
    rows = (bi[:, None] * dof + np.arange(dof)[None, :]).reshape(-1) + 1
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + _simd_pad(W, dtype), dtype)
    val[:nv] = vals.reshape(-1)  # block row-major == dof stored rows of dof values each
    return SparseMatrix1DVBC(W, n, n, SplitPartition(spl), pos, rows, ofs, val)


def standin(name, dtype=np.float64, seed=0xDEADBEEF):
    """fe_stiffness_3d with the n and nnz of a SuiteSparse matrix of BASELINE.json (C2-C4)."""
    n, nnz = STANDINS[name]
    return fe_stiffness_3d(n, nnz, 3, dtype, seed)
