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


# SuiteSparse matrices of BASELINE.json's configs C2-C4 and of the reference's recorded benchmark
# (src/ref.out), not available offline: (n, nnz) from the reference's own output (ct20stif :29-32,
# chesapeake :58-60, thermal1 :108-110, 3dtube :157-159) and the SuiteSparse index (ldoor).
STANDINS = {"Boeing/ct20stif": (52329, 2600295), "GHS_psdef/ldoor": (952203, 42493817),
            "DIMACS10/chesapeake": (39, 340), "Schmid/thermal1": (82654, 574458),
            "Rothberg/3dtube": (45330, 3213618)}

# How each stand-in is generated, calibrated (at the default seed) so that the reference's memory
# column of src/ref.out -- structure only: 24·(L+1) + 8·q + 8·|val| (io.memory_bytes) -- comes out
# right for StrictChunker(8) (tests/test_io_costs.py asserts within 1 %) and, softer, for the optimal
# min-memory partition:
#   ct20stif: 3D mesh, 83 % 3-dof / 17 % 6-dof nodes, all 26 neighbours reachable, 2.8 % of the node
#             pairs with one structural zero -> strict 0.999, min memory 0.999 of ref.out :40,:45;
#   thermal1: 2D mesh of 1-dof nodes, 8 neighbours, numbered at random inside windows of 3 ->
#             strict 1.000 (every strict stripe but one is one column; ref.out :123 has all of them),
#             min memory 0.983;
#   3dtube:   3D mesh of 3-dof nodes, 26 neighbours, 0.1 % of the pairs with a structural zero ->
#             strict 1.001, min memory 0.995 (:172,:177);
#   chesapeake: a graph (no diagonal) of 39 vertices and 170 edges drawn with weight exp(-|i-j|/2)
#             -> strict exact, min memory 1.001 (:71,:76);
#   ldoor:    the pure 3-dof stiffness stand-in of rounds 1-3 (no recorded reference numbers).
STANDIN_MODEL = {
    "Boeing/ct20stif": dict(kind="mesh", dims=3, dof_probs=(0, 0, 0.83, 0, 0, 0.17), reach=3, drop=0.028),
    "Schmid/thermal1": dict(kind="mesh", dims=2, dof_probs=(1,), reach=2, shuffle=3),
    "Rothberg/3dtube": dict(kind="mesh", dims=3, dof_probs=(0, 0, 1), reach=3, drop=0.001),
    "DIMACS10/chesapeake": dict(kind="graph", lam=2.0, structure_seed=1),
    "GHS_psdef/ldoor": dict(kind="stiffness3"),
}


def banded_graph(n, nnz, lam, seed=0, value_seed=0xDEADBEEF, dtype=np.float64):
    """Symmetric graph adjacency without a diagonal: nnz/2 distinct edges {i, j} drawn with weight
    exp(-|i - j| / lam) (a numbering with locality), values U[-1, 1) symmetric."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    i, j = np.triu_indices(n, 1)
    p = np.exp(-(j - i) / lam)
    e = rng.choice(len(i), nnz // 2, replace=False, p=p / p.sum())
    r = np.concatenate([i[e], j[e]])
    c = np.concatenate([j[e], i[e]])
    A = sp.csc_matrix((_sym_uniform(r, c, value_seed).astype(dtype), (r, c)), shape=(n, n))
    A.sort_indices()
    return A


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


def fe_stiffness_3d_vbc(n, nnz, dof=3, U=8, W=8, dtype=np.float32, seed=0xDEADBEEF):
    """fe_stiffness_3d(n, nnz, dof) directly as SparseMatrixVBC{U,W} with dof x dof node tiles: block
    row k = mesh node k's rows, stripe l = node l's columns (what AlternatingPacker(StrictChunker,
    StrictChunker) finds on that matrix -- a node's dof columns share a pattern, and so do its dof
    rows -- unless two consecutive nodes happen to share theirs).  Per stripe the coupled nodes'
    tiles in ascending block row, each tile row-major (constructors_VBC.jl:95-105).  The structured
    (mesh) counterpart of c5's random tiles: neighbouring stripes gather neighbouring X block rows."""
    N, bi, bj, vals = _stiffness_blocks(n, nnz, dof, seed)
    order = np.lexsort((bi, bj))
    bi, bj, vals = bi[order], bj[order], vals[order]
    cnt = np.bincount(bj, minlength=N).astype(np.int64)
    spl = 1 + np.arange(N + 1, dtype=np.int64) * dof
    pos = np.concatenate([[1], 1 + np.cumsum(cnt)]).astype(np.int64)
    ofs = np.concatenate([[1], 1 + np.cumsum(cnt * dof * dof)]).astype(np.int64)
    nv = int(ofs[-1] - 1)
    val = np.zeros(nv + _simd_pad(W, dtype, U), dtype)
    val[:nv] = vals.reshape(-1)
    return SparseMatrixVBC(U, W, n, n, SplitPartition(spl.copy()), SplitPartition(spl), pos, bi + 1, ofs, val)


def c5_mesh(dtype=np.float32, scale=1.0, seed=0xDEADBEEF):
    """C5 on a STRUCTURED input: the 3D stiffness stand-in of c5's size (2,097,152 rows, 1.0e8
    stored values) as a SparseMatrixVBC of 3 x 3 node tiles (fe_stiffness_3d_vbc)."""
    n = 3 * int(round(699051 * scale))
    return fe_stiffness_3d_vbc(n, int(round(1e8 * scale)), 3, dtype=dtype, seed=seed)


def _sym_uniform(r, c, seed):
    """U[-1, 1) value of entry (r, c), symmetric in (r, c): a 64-bit mix of (min, max, seed)."""
    lo = np.minimum(r, c).astype(np.uint64)
    hi = np.maximum(r, c).astype(np.uint64)
    with np.errstate(over="ignore"):
        h = lo * np.uint64(0x9E3779B97F4A7C15) ^ (hi + np.uint64(seed & 0xFFFFFFFF)) * np.uint64(0xC2B2AE3D27D4EB4F)
        h ^= h >> np.uint64(31)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(29)
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 / 2 ** 53) - 1.0


def fe_mixed_dof(n, nnz, dims=3, dof_probs=(0.0, 0.0, 1.0), reach=3, diag=True, drop=0.0, shuffle=1,
                 seed=0xDEADBEEF, dtype=np.float64):
    """A symmetric finite-element stand-in with a MIXED number of unknowns per mesh node, exactly n rows
    and exactly nnz stored entries (when the parities allow; else within one block).
    * mesh nodes on a near-square (dims = 2) / near-cubic (dims = 3) grid, row-major; node k has d_k
      dofs drawn from dof_probs (d = 1, 2, ...), the last node trimmed so the d_k sum to n -- a real
      stiffness matrix's nodes lose dofs to constraints and carry different element types, so its
      strict stripes are of mixed widths (ct20stif: 2.4 columns on average, from src/ref.out);
    * node pairs: the grid neighbours whose offsets have |offset|_1 <= reach (3D: reach 2 = the 18
      face / edge neighbours, 3 = all 26; 2D: 1 or 2), a random subset kept in a random order until
      the stored entries reach nnz (every node keeps its diagonal block when `diag`);
    * every coupling a d_i x d_j block, values U[-1, 1) symmetric in (row, col); a `drop` fraction of
      the node pairs lose one entry of their block (and its mirror) -- the exact zeros of element
      couplings that make a node's columns differ slightly, so StrictChunker splits the node while a
      fill-tolerant partition (min memory, overlap) merges it back;
    * `shuffle` > 1 numbers the nodes in a random order inside windows of that many grid positions (an
      unstructured mesh's numbering: consecutive nodes are near, but not grid neighbours).
    Returns a sorted scipy CSC matrix."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    probs = np.asarray(dof_probs, dtype=np.float64)
    probs = probs / probs.sum()
    ds = np.arange(1, len(probs) + 1)
    est = int(n / float(probs @ ds)) + 64
    d = rng.choice(ds, size=est, p=probs).astype(np.int64)
    cs = np.cumsum(d)
    while cs[-1] < n:  # (never at these sizes)
        d = np.concatenate([d, rng.choice(ds, size=64, p=probs)])
        cs = np.cumsum(d)
    N = int(np.searchsorted(cs, n) + 1)
    d = d[:N]
    d[-1] -= int(cs[N - 1] - n)
    off = np.concatenate([[0], np.cumsum(d)])
    g = int(np.ceil(N ** (1.0 / dims) - 1e-9))
    while g ** dims < N:
        g += 1
    node = np.arange(N, dtype=np.int64)
    coords = [(node // g ** (dims - 1 - k)) % g for k in range(dims)]
    import itertools
    offs = [o for o in itertools.product((-1, 0, 1), repeat=dims) if 0 < sum(map(abs, o)) <= reach and o > (0,) * dims]
    pi, pj = [], []
    for o in offs:
        ok = np.ones(N, bool)
        nb = np.zeros(N, np.int64)
        for k in range(dims):
            c = coords[k] + o[k]
            ok &= (c >= 0) & (c < g)
            nb = nb * g + c
        ok &= nb < N
        pi.append(node[ok])
        pj.append(nb[ok])
    pi, pj = np.concatenate(pi), np.concatenate(pj)
    if shuffle > 1:  # relabel grid positions within windows of `shuffle` consecutive nodes
        lab = np.arange(N, dtype=np.int64)
        for w0 in range(0, N, shuffle):
            lab[w0:w0 + shuffle] = w0 + rng.permutation(min(shuffle, N - w0))
        pi, pj = lab[pi], lab[pj]

    def entries(bi, bj):
        sz = d[bi] * d[bj]
        start = np.concatenate([[0], np.cumsum(sz)])
        blk = np.repeat(np.arange(len(bi)), sz)
        loc = np.arange(int(start[-1])) - start[blk]
        return blk, off[bi][blk] + loc // d[bj][blk], off[bj][blk] + loc % d[bj][blk]
    # the upper-triangle entries of every candidate pair; the dropped ones (structural zeros) go away
    pblk, prow, pcol = entries(pi, pj)
    live = np.ones(len(prow), bool)
    if drop > 0:  # a `drop` fraction of the couplings lose one entry (and its mirror): a structural zero
        hit = np.flatnonzero(rng.random(len(pi)) < drop)
        sz = d[pi] * d[pj]
        first = np.concatenate([[0], np.cumsum(sz)])[:-1]
        live[first[hit] + (rng.random(len(hit)) * sz[hit]).astype(np.int64)] = False
    contrib = 2 * np.bincount(pblk[live], minlength=len(pi))
    base = int(np.sum(d * d)) if diag else 0
    want = nnz - base
    perm = rng.permutation(len(pi))
    cum = np.cumsum(contrib[perm])
    k = int(np.searchsorted(cum, want, side="left")) + 1  # the first prefix reaching `want`
    k = min(k, len(perm))
    sel = np.zeros(len(pi), bool)
    sel[perm[:k]] = True
    keep = live & sel[pblk]
    excess = (int(cum[k - 1]) if k else 0) - want
    if excess > 0:  # trim the last coupling's entries (two stored entries each) to land on nnz exactly
        last = np.flatnonzero(keep & (pblk == perm[k - 1]))
        keep[last[:excess // 2]] = False
    drows, dcols = (entries(node, node)[1:] if diag else (np.zeros(0, np.int64), np.zeros(0, np.int64)))
    rows = np.concatenate([drows, prow[keep], pcol[keep]])
    cols = np.concatenate([dcols, pcol[keep], prow[keep]])
    vals = _sym_uniform(rows, cols, seed).astype(dtype)
    A = sp.csc_matrix((vals, (rows, cols)), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    return A


def standin(name, dtype=np.float64, seed=0xDEADBEEF, scale=1.0):
    """The synthetic stand-in of a SuiteSparse matrix (STANDINS: its n and nnz; STANDIN_MODEL: its
    structure, calibrated against src/ref.out at the default seed); `scale` shrinks n and nnz (tests
    only: the structural KATs hold at scale 1)."""
    n, nnz = STANDINS[name]
    spec = dict(STANDIN_MODEL[name])
    kind = spec.pop("kind")
    if kind == "graph":
        return banded_graph(n, nnz, spec["lam"], spec["structure_seed"] if seed == 0xDEADBEEF else seed,
                            value_seed=seed, dtype=dtype)
    if scale != 1.0:
        n, nnz = 3 * max(1, int(round(n / 3 * scale))), max(1, int(round(nnz * scale)))
    if kind == "stiffness3":
        return fe_stiffness_3d(n, nnz, 3, dtype, seed)
    return fe_mixed_dof(n, nnz, seed=seed, dtype=dtype, **spec)
