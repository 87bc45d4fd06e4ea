"""Matrix Market / SuiteSparse inputs and an on-disk cache of built layouts.

The reference fetches matrices with MatrixDepot.mdopen (test/makematrices.jl, bin/test_table.jl:27),
a network download.  There is no network here or on the GPU box, so `mdopen(name)` only reads a
local copy: `$VBC_MATRIX_DIR/<group>/<name>/<name>.mtx` (the SuiteSparse tarball layout),
`$VBC_MATRIX_DIR/<group>/<name>.mtx` or `$VBC_MATRIX_DIR/<name>.mtx`, and raises FileNotFoundError
otherwise.  Symmetric files are expanded to the full pattern (runtests.jl:18 `SparseMatrixCSC(A)`),
pattern files get unit values.

`save_built` / `load_built` store the fields of a built SparseMatrix1DVBC / SparseMatrixVBC as a
plain .npz (loaded with allow_pickle=False), so the partition + layout of a large matrix is computed
once (setup is 6-14 products on ct20stif, ref.out:39-48).
"""
import os
from pathlib import Path

import numpy as np
import scipy.sparse as sp

from .matrices import SparseMatrix1DVBC, SparseMatrixVBC
from .partition import SplitPartition


def read_mtx(path, dtype=np.float64):
    """A Matrix Market file as a sorted scipy CSC matrix (full pattern, `dtype` values)."""
    import scipy.io
    A = scipy.io.mmread(str(path))
    A = sp.csc_matrix(A)
    if A.dtype == np.bool_ or A.dtype.kind not in "fc":
        A = A.astype(dtype)
    A = A.astype(dtype) if A.dtype != np.dtype(dtype) else A
    A.sum_duplicates()
    A.sort_indices()
    return A


class MatrixDesc:
    """What mdopen returns: `.A` (scipy CSC) and the resolved `.path`."""

    def __init__(self, name, path, A):
        self.name, self.path, self.A = name, path, A

    def __repr__(self):
        return f"MatrixDesc({self.name!r}, {self.A.shape}, nnz={self.A.nnz})"


def _candidates(name, root):
    group, _, base = name.rpartition("/")
    root = Path(root)
    c = []
    if group:
        c += [root / group / base / f"{base}.mtx", root / group / f"{base}.mtx"]
    c += [root / base / f"{base}.mtx", root / f"{base}.mtx"]
    return c


def mdopen(name, root=None, dtype=np.float64):
    """MatrixDepot.mdopen(name) on a local SuiteSparse copy (no download is ever attempted)."""
    root = root if root is not None else os.environ.get("VBC_MATRIX_DIR")
    if not root:
        raise FileNotFoundError(f"{name}: set VBC_MATRIX_DIR to a local SuiteSparse copy (no network access)")
    for p in _candidates(name, root):
        if p.exists():
            return MatrixDesc(name, p, read_mtx(p, dtype))
    raise FileNotFoundError(f"{name}: not found under {root} (tried {', '.join(map(str, _candidates(name, root)))})")


def save_built(B, path):
    """Write the fields of a built matrix (exactly the Julia struct's) to an .npz file."""
    f = dict(kind=np.array([2 if isinstance(B, SparseMatrixVBC) else 1]), m=np.array([B.m]), n=np.array([B.n]),
             W=np.array([B.W]), spl=B.Phi.spl, pos=B.pos, idx=B.idx, ofs=B.ofs, val=B.val)
    if isinstance(B, SparseMatrixVBC):
        f.update(U=np.array([B.U]), pspl=B.Pi.spl)
    np.savez(path, **f)


def load_built(path):
    """Inverse of save_built (no pickles: allow_pickle=False)."""
    with np.load(path, allow_pickle=False) as d:
        m, n, W = int(d["m"][0]), int(d["n"][0]), int(d["W"][0])
        if int(d["kind"][0]) == 2:
            return SparseMatrixVBC(int(d["U"][0]), W, m, n, SplitPartition(d["pspl"]), SplitPartition(d["spl"]),
                                   d["pos"], d["idx"], d["ofs"], d["val"])
        return SparseMatrix1DVBC(W, m, n, SplitPartition(d["spl"]), d["pos"], d["idx"], d["ofs"], d["val"])


def cached_build(builder, path):
    """load_built(path) if it exists, else builder() saved to path."""
    path = Path(path)
    if path.exists():
        return load_built(path)
    B = builder()
    path.parent.mkdir(parents=True, exist_ok=True)
    save_built(B, path)
    return B


def memory_bytes(B, ti=8):
    """The reference's `mem` column (bin/test_table.jl:78,120): sizeof(B.Φ) + [sizeof(B.Π)] + sizeof of
    pos, idx, ofs, val, index arrays of Ti (Int64 in the reference).  The partitions count their spl
    arrays (Ti·(L+1), Ti·(K+1)): that is what reproduces src/ref.out exactly -- thermal1's
    StrictChunker(8) row, 11,175,112 B = 24·(L+1) + 8·q + 8·|val| with L = n, q = nnz and the 8-value
    SIMD tail pad (ref.out:123; tests/test_io_costs.py pins it)."""
    n = ti * (len(B.Phi.spl) + len(B.pos) + len(B.idx) + len(B.ofs)) + B.val.nbytes
    if isinstance(B, SparseMatrixVBC):
        n += ti * len(B.Pi.spl)
    return n
