"""Partitions and partitioners used by the reference's constructors.

Mirrors the slice of ChainPartitioners.jl 1.1.6 (Manifest.toml:23-29; absent from the container)
that SparseMatrixVBCs.jl calls: `SplitPartition` (`.spl`), `pack_stripe(A, method)` (constructors_
1DVBC.jl:5), `pack_plaid(A, method)` (constructors_VBC.jl:11), the chunkers used by the tests and
bench (runtests.jl:19-25,56-59; test_table.jl:64-111) and the cost models of costs.jl:8-10.

The chunkers are the build's own restatements (native, libvbc vbcx_partition_*): PARTITION PARITY
IS UNPINNED.  Every numerical parity claim is made for a GIVEN partition, which both
the oracle and the GPU receive.
"""
import numpy as np

from . import _lib as _L


class SplitPartition:
    """1-based split points: part l covers [spl[l], spl[l+1]) (ChainPartitioners.SplitPartition)."""

    def __init__(self, spl):
        self.spl = np.ascontiguousarray(spl, dtype=np.int64)
        if self.spl.ndim != 1 or len(self.spl) < 1 or self.spl[0] != 1 or np.any(np.diff(self.spl) <= 0):
            raise _L.ArgumentError("spl must be strictly increasing and start at 1")

    def __len__(self):
        return len(self.spl) - 1

    def widths(self):
        return np.diff(self.spl)

    def __repr__(self):
        return f"SplitPartition({len(self)} parts)"

    def __eq__(self, other):
        return isinstance(other, SplitPartition) and np.array_equal(self.spl, other.spl)


class CSCFields:
    """A CSC matrix with its 1-based Int64 index arrays (the Julia SparseMatrixCSC fields), converted
    once and shared by the partitioner and the constructor (matrices.from_csc)."""

    def __init__(self, A):
        import scipy.sparse as sp
        A = sp.csc_matrix(A)
        if not A.has_canonical_format:
            A = A.copy()
            A.sum_duplicates()  # also sorts the indices
        self.A = A
        self.shape = A.shape
        self.colptr = np.add(A.indptr, 1, dtype=np.int64)
        self.rowval = np.add(A.indices, 1, dtype=np.int64)


def _csc(A):
    if isinstance(A, CSCFields):
        return A.A, A.colptr, A.rowval
    F = CSCFields(A)
    return F.A, F.colptr, F.rowval


# --- cost models (costs.jl:8-10) ------------------------------------------------------------
class AffineStripeModel:
    """cost(stripe) = c_stripe + c_col·w + c_pin·pins + c_row·rows + c_cell·w·rows."""

    def __init__(self, c_stripe=0.0, c_col=0.0, c_pin=0.0, c_row=0.0, c_cell=0.0):
        self.c = (float(c_stripe), float(c_col), float(c_pin), float(c_row), float(c_cell))

    def __repr__(self):
        return "AffineStripeModel(%g, %g, %g, %g, %g)" % self.c


def model_SparseMatrix1DVBC_blocks():
    """Number of stored row-blocks (costs.jl:8: AffineConnectivityModel(0, 0, 0, 1))."""
    return AffineStripeModel(c_row=1)


def model_SparseMatrix1DVBC_memory(Tv=np.float64, Ti=np.int64):
    """Storage bytes (costs.jl:10): 3·sizeof(Ti) per stripe + (sizeof(Ti) + w·sizeof(Tv)) per row."""
    ti, tv = np.dtype(Ti).itemsize, np.dtype(Tv).itemsize
    return AffineStripeModel(c_stripe=3 * ti, c_row=ti, c_cell=tv)


# --- chunkers ---------------------------------------------------------------------------------
class ColumnBlockCostModel:
    """ColumnBlockComponentCostModel (costs.jl:12): cost(stripe of width w, R rows) = alpha[w] + beta[w]·R.
    model_SparseMatrix1DVBC_TrSpMV_time (costs.py) fits alpha / beta to the GPU kernel."""

    def __init__(self, alpha, beta):
        self.alpha = np.ascontiguousarray(alpha, dtype=np.float64)
        self.beta = np.ascontiguousarray(beta, dtype=np.float64)
        if self.alpha.shape != self.beta.shape or self.alpha.ndim != 1:
            raise _L.ArgumentError("alpha and beta must be vectors of the same length W")

    def __repr__(self):
        return f"ColumnBlockCostModel(alpha={self.alpha.tolist()}, beta={self.beta.tolist()})"


class Line:
    """costs.jl:1-6: the affine functor x -> a + b·x."""

    def __init__(self, a, b):
        self.a, self.b = float(a), float(b)

    def __call__(self, x):
        return self.a + self.b * x

    def __repr__(self):
        return f"Line({self.a:g}, {self.b:g})"


def _eval_component(f, sizes):
    """A model component at the given part sizes: a number (constant), a callable (Line), or a table
    indexed by size (1-based: the fitted time model's per-size vectors, costs.jl:264-281)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    if callable(f):
        return np.asarray(f(sizes.astype(np.float64)), dtype=np.float64) * np.ones(len(sizes))
    a = np.asarray(f, dtype=np.float64)
    if a.ndim == 0:
        return np.full(len(sizes), float(a))
    if len(sizes) and (sizes.min() < 1 or sizes.max() > len(a)):
        raise _L.ArgumentError(f"part size outside the model's table 1..{len(a)}")
    return a[sizes - 1]


class BlockComponentCostModel:
    """ChainPartitioners' BlockComponentCostModel{Tv}(α_row, α_col, β_row, β_col) as costs.jl:138-142
    builds it for SparseMatrixVBC: a block row of height u costs α_row(u), a stripe of width w costs
    α_col(w), and every stored u x w block costs Σ_r β_row[r](u)·β_col[r](w).  Components are numbers,
    Lines or per-size tables.  As a column partitioner (DynamicTotalChunker) it sees the rows grouped
    by the current row partition; permutedims(model) swaps the roles for the row partition."""

    def __init__(self, alpha_row, alpha_col, beta_row, beta_col):
        self.alpha_row, self.alpha_col = alpha_row, alpha_col
        self.beta_row, self.beta_col = tuple(beta_row), tuple(beta_col)
        if len(self.beta_row) != len(self.beta_col) or not self.beta_row:
            raise _L.ArgumentError("β_row and β_col need the same number (>= 1) of components")

    def permutedims(self):
        return BlockComponentCostModel(self.alpha_col, self.alpha_row, self.beta_col, self.beta_row)

    def block_cost(self, u, w):
        u, w = np.atleast_1d(u), np.atleast_1d(w)
        return sum(_eval_component(br, u) * _eval_component(bc, w) for br, bc in zip(self.beta_row, self.beta_col))

    def __repr__(self):
        return f"BlockComponentCostModel({self.alpha_row!r}, {self.alpha_col!r}, {self.beta_row!r}, {self.beta_col!r})"


def permutedims(model):
    """permutedims(model) (bin/test_table.jl:96,102,109): the model for the other dimension."""
    if not isinstance(model, BlockComponentCostModel):
        raise _L.ArgumentError("permutedims applies to a BlockComponentCostModel")
    return model.permutedims()


def model_SparseMatrixVBC_blocks():
    """Number of stored blocks (costs.jl:138: BlockComponentCostModel{Int}(0, 0, (1,), (1,)))."""
    return BlockComponentCostModel(0, 0, (1,), (1,))


def model_SparseMatrixVBC_memory(Tv=np.float64, Ti=np.int64):
    """Storage bytes of a SparseMatrixVBC (costs.jl:140): Ti per block row (Π.spl), 3·Ti per stripe
    (Φ.spl, pos, ofs), and per u x w block Ti (its idx) + u·w·Tv (its tile)."""
    ti, tv = np.dtype(Ti).itemsize, np.dtype(Tv).itemsize
    return BlockComponentCostModel(ti, 3 * ti, (Line(1, 0), Line(0, 1)), (Line(ti, 0), Line(0, tv)))


def total_value_2d(B, model):
    """total_value(A, Π, Φ, mdl) + row_component_value(Π, mdl) (bin/test_table.jl:124) of a built
    SparseMatrixVBC: Σ_k α_row(u_k) + Σ_l α_col(w_l) + Σ over stored blocks of their block cost."""
    u = np.diff(B.Pi.spl)
    w = np.diff(B.Phi.spl)
    wq = np.repeat(w, np.diff(B.pos))
    uq = u[B.idx - 1]
    v = _eval_component(model.alpha_row, u).sum() + _eval_component(model.alpha_col, w).sum()
    if len(uq):
        v += model.block_cost(uq, wq).sum()
    return float(v)


class EquiChunker:
    def __init__(self, w=1):
        self.w = int(w)

    def partition(self, A):
        n = A.shape[1]
        spl = np.zeros(n + 1, np.int64)
        L = np.zeros(1, np.int64)
        _L.check(_L.lib().vbcx_partition_equi(n, self.w, spl.ctypes.data, L.ctypes.data), "EquiChunker")
        return SplitPartition(spl[:L[0] + 1])


class StrictChunker:
    """Consecutive columns with identical row patterns, width <= W."""

    def __init__(self, W):
        self.W = int(W)

    def partition(self, A):
        A, colptr, rowval = _csc(A)
        m, n = A.shape
        spl = np.zeros(n + 1, np.int64)
        L = np.zeros(1, np.int64)
        _L.check(_L.lib().vbcx_partition_strict(m, n, colptr.ctypes.data, rowval.ctypes.data, self.W,
                                                spl.ctypes.data, L.ctypes.data), "StrictChunker")
        return SplitPartition(spl[:L[0] + 1])


class OverlapChunker:
    """Greedy: column j joins the open stripe while |S(j) ∩ S(first)| >= ρ·max(|S(j)|, |S(first)|)."""

    def __init__(self, rho, W):
        self.rho, self.W = float(rho), int(W)

    def partition(self, A):
        A, colptr, rowval = _csc(A)
        m, n = A.shape
        spl = np.zeros(n + 1, np.int64)
        L = np.zeros(1, np.int64)
        _L.check(_L.lib().vbcx_partition_overlap(m, n, colptr.ctypes.data, rowval.ctypes.data, self.rho,
                                                 self.W, spl.ctypes.data, L.ctypes.data), "OverlapChunker")
        return SplitPartition(spl[:L[0] + 1])


class ConstrainedCost:
    """ConstrainedCost(model, VertexCount(), W): the model with a width cap (runtests.jl:22-23)."""

    def __init__(self, model, _count=None, W=None):
        self.model, self.W = model, W


class VertexCount:
    pass


class DynamicTotalChunker:
    """Optimal contiguous partition minimising the total model cost, width <= W (DP)."""

    def __init__(self, model, W=None):
        if isinstance(model, ConstrainedCost):
            W = model.W if W is None else W
            model = model.model
        if W is None:
            raise _L.ArgumentError("DynamicTotalChunker needs a width limit W")
        self.model, self.W = model, int(W)

    def partition(self, A, groups=None):
        """Column partition of A; `groups` (a SplitPartition of A's rows, the other dimension's
        partition in pack_plaid) groups the rows into block rows for a BlockComponentCostModel."""
        A, colptr, rowval = _csc(A)
        m, n = A.shape
        spl = np.zeros(n + 1, np.int64)
        L = np.zeros(1, np.int64)
        if isinstance(self.model, BlockComponentCostModel):
            md = self.model
            gspl = groups.spl if groups is not None else np.arange(1, m + 2, dtype=np.int64)
            u = np.diff(gspl)
            G = len(u)
            grp = np.repeat(np.arange(1, G + 1, dtype=np.int64), u)
            W = self.W
            ws = np.arange(1, W + 1)
            gw = np.ascontiguousarray(np.stack([_eval_component(br, u) for br in md.beta_row]) if G else
                                      np.zeros((len(md.beta_row), 1)))
            colw = np.ascontiguousarray(np.stack([_eval_component(bc, ws) for bc in md.beta_col]))
            alpha = np.ascontiguousarray(_eval_component(md.alpha_col, ws))
            _L.check(_L.lib().vbcx_partition_block(m, n, colptr.ctypes.data, rowval.ctypes.data, grp.ctypes.data,
                                                   max(G, 1) if m == 0 else G, len(md.beta_row), gw.ctypes.data, W,
                                                   alpha.ctypes.data, colw.ctypes.data, spl.ctypes.data,
                                                   L.ctypes.data), "DynamicTotalChunker")
            return SplitPartition(spl[:L[0] + 1])
        if isinstance(self.model, ColumnBlockCostModel):
            W = min(self.W, len(self.model.alpha))
            _L.check(_L.lib().vbcx_partition_dynamic_table(m, n, colptr.ctypes.data, rowval.ctypes.data, W,
                                                           self.model.alpha.ctypes.data, self.model.beta.ctypes.data,
                                                           spl.ctypes.data, L.ctypes.data), "DynamicTotalChunker")
        else:
            _L.check(_L.lib().vbcx_partition_dynamic(m, n, colptr.ctypes.data, rowval.ctypes.data, self.W,
                                                     *self.model.c, spl.ctypes.data, L.ctypes.data),
                     "DynamicTotalChunker")
        return SplitPartition(spl[:L[0] + 1])


def pack_stripe(A, method):
    """Column partition Φ of A (ChainPartitioners.pack_stripe)."""
    return method.partition(A)


class AlternatingPacker:
    """AlternatingPacker(method_1, method_2, ...) (runtests.jl:57-58, bin/test_table.jl:88-111) --
    and AlternatePacker, the spelling of the reference's default 5-phase packer (constructors_VBC.jl:
    2-8).  The phases alternate: odd phases partition the COLUMNS (Φ) of A with its rows grouped by the
    current row partition Π (singleton rows before the first row phase), even phases partition the
    ROWS (Π) -- the columns of Aᵀ -- with A's columns grouped by the current Φ.  The result is the
    last Π and the last Φ.  That order is the one the reference's own calls imply: its default packer
    and test_table.jl:98-111 put the width-W constraint on phases 1, 3, 5 and the height-U constraint
    (and the permuted 2D model) on phases 2, 4, and "1D 2D" (test_table.jl:89) pairs a 1D column
    partitioner with EquiChunker(1) rows.  (ChainPartitioners' source is absent: the phase semantics
    are restated from these call sites, partition parity unpinned.)"""

    def __init__(self, *methods):
        if len(methods) < 1:
            raise _L.ArgumentError("AlternatingPacker needs at least one method")
        self.methods = tuple(methods)

    @property
    def row_method(self):  # (round-3 attribute names); None: a one-phase packer has no row phase
        if len(self.methods) < 2:
            return None
        return self.methods[-1] if len(self.methods) % 2 == 0 else self.methods[-2]

    @property
    def col_method(self):
        return self.methods[-1] if len(self.methods) % 2 == 1 else self.methods[-2]


AlternatePacker = AlternatingPacker  # constructors_VBC.jl:2 spells it this way


def _merged_pattern(A, groups):
    """A's sparsity pattern with its rows merged into the block rows of `groups` (a block row is in
    column j's pattern when any of its rows is), as a CSC matrix of 1s."""
    import scipy.sparse as sp
    coo = A.tocoo()
    asg = np.repeat(np.arange(len(groups)), np.diff(groups.spl))
    Am = sp.csc_matrix((np.ones(coo.nnz), (asg[coo.row], coo.col)), shape=(len(groups), A.shape[1]))
    Am.sum_duplicates()
    Am.sort_indices()
    return Am


def _partition_given(C, method, groups):
    """One phase of the alternation: the columns of C with its rows grouped by `groups` (None or
    singletons: C as it is).  Block cost models see the groups' heights; the other chunkers see the
    merged (block-row) pattern."""
    if isinstance(method, DynamicTotalChunker) and isinstance(method.model, BlockComponentCostModel):
        return method.partition(C, groups)
    if groups is None or len(groups) == C.shape[0]:
        return method.partition(C)
    return method.partition(_merged_pattern(C, groups))


def pack_plaid(A, method):
    """(Π, Φ) for SparseMatrixVBC (ChainPartitioners.pack_plaid, constructors_VBC.jl:10-13)."""
    import scipy.sparse as sp
    if not isinstance(method, AlternatingPacker):
        raise _L.ArgumentError("pack_plaid takes an AlternatingPacker")
    A = sp.csc_matrix(A)
    if not A.has_canonical_format:
        A = A.copy()
        A.sum_duplicates()
    m, n = A.shape
    At = None
    Pi, Phi = SplitPartition(np.arange(1, m + 2, dtype=np.int64)), None
    for ph, mt in enumerate(method.methods):
        if ph % 2 == 0:
            Phi = _partition_given(A, mt, Pi)
        else:
            if At is None:
                At = A.T.tocsc()
                At.sort_indices()
            Pi = _partition_given(At, mt, Phi)
    assert Pi.spl[-1] == m + 1 and Phi.spl[-1] == n + 1
    return Pi, Phi
