"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as the
checker / CPU baseline.  Every function restates a reference routine; see vbc_oracle.c for the
file:line of each.  Index arrays are 1-based int64 exactly like the Julia struct fields.
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"

_P = C.c_void_p
_I = C.c_int64
_D = C.c_double
_INT = C.c_int

_lib = None


def build(force=False):
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "vbc_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-s", "liboracle.so"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = C.CDLL(str(LIB_PATH))
        _lib.orc_max_threads.restype = _INT
    return _lib


def _p(a):
    return a.ctypes.data_as(_P) if a is not None else None


def _suf(dtype):
    dtype = np.dtype(dtype)
    if dtype == np.float64:
        return "f64"
    if dtype == np.float32:
        return "f32"
    raise TypeError(f"oracle supports float64/float32, got {dtype}")


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


class OracleError(RuntimeError):
    pass


def _check(st, what):
    if st == 1:
        raise OracleError(f"{what}: DimensionMismatch")
    if st == 6:
        raise OracleError(f"{what}: AssertionError")
    if st != 0:
        raise OracleError(f"{what}: status {st}")


class Ref1DVBC:
    """Plain container mirroring SparseMatrix1DVBC{W,Tv,Ti} fields (SparseMatrixVBCs.jl:36-53)."""

    def __init__(self, m, n, W, spl, pos, idx, ofs, val):
        self.m, self.n, self.W = int(m), int(n), int(W)
        self.spl, self.pos, self.idx, self.ofs, self.val = spl, pos, idx, ofs, val

    @property
    def L(self):
        return len(self.spl) - 1


class RefVBC(Ref1DVBC):
    """Mirror of SparseMatrixVBC{U,W,Tv,Ti} (SparseMatrixVBCs.jl:62-82); idx holds block-row ids."""

    def __init__(self, m, n, U, W, pspl, spl, pos, idx, ofs, val):
        super().__init__(m, n, W, spl, pos, idx, ofs, val)
        self.U = int(U)
        self.pspl = pspl

    @property
    def K(self):
        return len(self.pspl) - 1


def csc_arrays(A):
    """scipy CSC -> (colptr, rowval) 1-based int64 + nzval, like SparseMatrixCSC fields."""
    A = A.tocsc()
    A.sort_indices()
    return _i64(A.indptr) + 1, _i64(A.indices) + 1, np.ascontiguousarray(A.data)


def build_1dvbc(A, spl, W, pad=0, strict=False, dtype=np.float64):
    """SparseMatrix1DVBC{W}(A, Φ) (constructors_1DVBC.jl:9-92) or the StrictChunker fast path
    (:94-143) when strict=True.  `pad` = the reference's Δw*cld(W,Δw) tail (host-SIMD dependent)."""
    L_ = lib()
    m, n = A.shape
    colptr, rowval, nzval = csc_arrays(A)
    nzval = nzval.astype(dtype)
    spl = _i64(spl)
    L = len(spl) - 1
    pos = np.zeros(L + 1, np.int64)
    ofs = np.zeros(L + 1, np.int64)
    if strict:
        st = L_.orc_1dvbc_strict_count(_I(m), _I(n), _p(colptr), _I(L), _p(spl), _p(pos), _p(ofs))
    else:
        st = L_.orc_1dvbc_count(_I(m), _I(n), _p(colptr), _p(rowval), _I(L), _p(spl), _p(pos), _p(ofs))
    _check(st, "orc_1dvbc_count")
    idx = np.zeros(pos[-1] - 1, np.int64)
    val = np.zeros(ofs[-1] - 1 + pad, dtype)
    fn = getattr(L_, ("orc_1dvbc_strict_fill_" if strict else "orc_1dvbc_fill_") + _suf(dtype))
    st = fn(_I(m), _I(n), _I(W), _p(colptr), _p(rowval), _p(nzval), _I(L), _p(spl), _p(pos), _p(ofs),
            _p(idx), _p(val), _I(pad))
    _check(st, "orc_1dvbc_fill")
    return Ref1DVBC(m, n, W, spl, pos, idx, ofs, val)


def build_vbc(A, pspl, spl, U, W, pad=0, dtype=np.float64):
    """SparseMatrixVBC{U,W}(A, Π, Φ)  constructors_VBC.jl:15-133."""
    L_ = lib()
    m, n = A.shape
    colptr, rowval, nzval = csc_arrays(A)
    nzval = nzval.astype(dtype)
    pspl, spl = _i64(pspl), _i64(spl)
    K, L = len(pspl) - 1, len(spl) - 1
    pos = np.zeros(L + 1, np.int64)
    ofs = np.zeros(L + 1, np.int64)
    st = L_.orc_vbc_count(_I(m), _I(n), _p(colptr), _p(rowval), _I(K), _p(pspl), _I(L), _p(spl),
                          _p(pos), _p(ofs))
    _check(st, "orc_vbc_count")
    idx = np.zeros(pos[-1] - 1, np.int64)
    val = np.zeros(ofs[-1] - 1 + pad, dtype)
    fn = getattr(L_, "orc_vbc_fill_" + _suf(dtype))
    st = fn(_I(m), _I(n), _I(U), _I(W), _p(colptr), _p(rowval), _p(nzval), _I(K), _p(pspl), _I(L),
            _p(spl), _p(pos), _p(ofs), _p(idx), _p(val), _I(pad))
    _check(st, "orc_vbc_fill")
    return RefVBC(m, n, U, W, pspl, spl, pos, idx, ofs, val)


def mul(B, x, y, alpha=1.0, beta=0.0, trans=False, ref_semantics=True, nthreads=1):
    """mul!(y, B, x, α, β) / mul!(y, B', x, α, β) on a Ref1DVBC / RefVBC; y is updated in place."""
    L_ = lib()
    suf = _suf(B.val.dtype)
    assert x.dtype == B.val.dtype and y.dtype == B.val.dtype
    x = np.ascontiguousarray(x)
    assert y.flags.c_contiguous
    two_d = isinstance(B, RefVBC)
    if two_d:
        head = [_I(B.m), _I(B.n), _I(B.K), _p(B.pspl), _I(B.L)]
        name = ("orc_vbc_mul_t_" if trans else "orc_vbc_mul_") + suf
    else:
        head = [_I(B.m), _I(B.n), _I(B.L)]
        name = ("orc_1dvbc_mul_t_" if trans else "orc_1dvbc_mul_") + suf
    args = head + [_p(B.spl), _p(B.pos), _p(B.idx), _p(B.ofs), _p(B.val), _p(x), _I(len(x)), _p(y),
                   _I(len(y)), _D(alpha), _D(beta), _INT(int(ref_semantics))]
    if trans:
        args.append(_INT(nthreads))
    _check(getattr(L_, name)(*args), name)
    return y


def trspmv(A, x, y, nthreads=1):
    """TrSpMV!(y, A::SparseMatrixCSC, x)  TrSpMV.jl:1-20 (y = Aᵀx, overwrite)."""
    L_ = lib()
    colptr, rowval, nzval = csc_arrays(A)
    nzval = nzval.astype(y.dtype)
    m, n = A.shape
    fn = getattr(L_, "orc_trspmv_" + _suf(y.dtype))
    _check(fn(_I(m), _I(n), _p(colptr), _p(rowval), _p(nzval), _p(np.ascontiguousarray(x)), _I(len(x)),
              _p(y), _I(len(y)), _INT(nthreads)), "orc_trspmv")
    return y


def mulmat_t(B, X, Y, alpha=1.0, beta=0.0, nthreads=1):
    """Column-by-column Bᵀ·X for the multi-RHS parity anchor (no reference kernel exists)."""
    L_ = lib()
    suf = _suf(B.val.dtype)
    X = np.asfortranarray(X)
    assert Y.flags.f_contiguous
    k = X.shape[1]
    fn = getattr(L_, "orc_1dvbc_mulmat_t_" + suf)
    _check(fn(_I(B.m), _I(B.n), _I(B.L), _p(B.spl), _p(B.pos), _p(B.idx), _p(B.ofs), _p(B.val), _I(k),
              _p(X), _I(X.shape[0]), _p(Y), _I(Y.shape[0]), _D(alpha), _D(beta), _INT(nthreads)),
           "orc_mulmat_t")
    return Y


def vbc_to_dense(B):
    """Expand a Ref1DVBC/RefVBC to a dense array (structural round-trip check)."""
    D = np.zeros((B.m, B.n), dtype=B.val.dtype)
    two_d = isinstance(B, RefVBC)
    for l in range(B.L):
        j, w = B.spl[l] - 1, B.spl[l + 1] - B.spl[l]
        q = B.ofs[l] - 1
        for Q in range(B.pos[l] - 1, B.pos[l + 1] - 1):
            if two_d:
                k = B.idx[Q]
                i0, u = B.pspl[k - 1] - 1, B.pspl[k] - B.pspl[k - 1]
                for di in range(u):
                    D[i0 + di, j:j + w] += B.val[q + di * w:q + di * w + w]
                q += u * w
            else:
                D[B.idx[Q] - 1, j:j + w] += B.val[q:q + w]
                q += w
    return D


def max_threads():
    return lib().orc_max_threads()


if __name__ == "__main__":
    build(force=True)
    print("built", LIB_PATH, "threads", max_threads(), os.cpu_count())
