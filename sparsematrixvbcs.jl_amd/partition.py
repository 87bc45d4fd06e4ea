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

    def partition(self, A):
        A, colptr, rowval = _csc(A)
        m, n = A.shape
        spl = np.zeros(n + 1, np.int64)
        L = np.zeros(1, np.int64)
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
    """2D packer for SparseMatrixVBC (runtests.jl:57-58).  Build's own scheme: the row partition Π
    is chosen by `row_method` on Aᵀ (rows of A as columns), then the column partition Φ by
    `col_method` on A with its rows merged into Π's block rows (so columns are compared at block-row
    granularity).  Extra chunkers (the reference's 3- and 5-argument forms) are accepted and the
    last row/column pair is used."""

    def __init__(self, *methods):
        if len(methods) < 2:
            raise _L.ArgumentError("AlternatingPacker needs at least a row and a column method")
        self.row_method, self.col_method = methods[-2], methods[-1]


AlternatePacker = AlternatingPacker  # constructors_VBC.jl:2 spells it this way


def pack_plaid(A, method):
    """(Π, Φ) for SparseMatrixVBC (ChainPartitioners.pack_plaid)."""
    import scipy.sparse as sp
    A = A.tocsc()
    Pi = method.row_method.partition(A.T.tocsc())
    # merge rows into block rows, then partition columns of the merged pattern
    m = A.shape[0]
    asg = np.repeat(np.arange(len(Pi)), np.diff(Pi.spl))
    coo = A.tocoo()
    Am = sp.csc_matrix((np.ones(coo.nnz), (asg[coo.row], coo.col)), shape=(len(Pi), A.shape[1]))
    Am.sum_duplicates()
    Phi = method.col_method.partition(Am)
    assert Pi.spl[-1] == m + 1
    return Pi, Phi
