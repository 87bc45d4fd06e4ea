"""SparseMatrix1DVBC / SparseMatrixVBC / SparseMatrixCSC mirrors of the reference types.

Fields are the reference's, verbatim: 1-based int64 `spl`/`pos`/`idx`/`ofs` and a `val` vector with
the SIMD tail pad (SparseMatrixVBCs.jl:36-53, :62-82; constructors_1DVBC.jl:35-39).  The host arrays
are what a Julia caller owns; the GPU copy lives behind a libvbc handle created on first use per
(device, direction) and released with the object.
"""
import ctypes as C
import weakref

import numpy as np
import scipy.sparse as sp

from . import _lib as _L
from .partition import (AlternatingPacker, ConstrainedCost, DynamicTotalChunker, EquiChunker, SplitPartition,
                        VertexCount, model_SparseMatrix1DVBC_memory, model_SparseMatrixVBC_memory, pack_plaid,
                        pack_stripe, permutedims)

DEFAULT_SIMD_SIZE = 64  # CpuId.simdbytes() on the AVX-512 hosts the reference was run on


def _simd_pad(W, dtype, U=1):
    dw = max(1, DEFAULT_SIMD_SIZE // np.dtype(dtype).itemsize)
    return U * dw * (-(-W // dw))


def _value_dtype(A):
    """The reference's Tv as stored: Float64 / Float32 / Int64 / Int32 / Bool stay as they are (the
    products compute in eltype(y), multiply_1DVBC.jl:102); other integer widths widen to Int64."""
    if A.dtype in (np.float64, np.float32, np.int64, np.int32, np.bool_):
        return A.dtype
    if A.dtype.kind in "iu":
        return np.int64
    raise _L.UnsupportedDtype(f"eltype {A.dtype} has no GPU kernel")


def _csc_fields(A):
    from .partition import CSCFields
    F = A if isinstance(A, CSCFields) else CSCFields(A)
    nzval = np.ascontiguousarray(F.A.data, dtype=_value_dtype(F.A))
    return F.shape, F.colptr, F.rowval, nzval


class _Handles:
    """libvbc handles of one matrix, keyed by (device, create flags)."""

    def __init__(self):
        self.h = {}

    def get(self, key, create):
        if key not in self.h:
            hp = C.c_void_p()
            _L.check(create(C.byref(hp)), "create")
            self.h[key] = hp
        return self.h[key]

    def release(self):
        if _L._lib is not None:
            for hp in self.h.values():
                _L._lib.vbc_destroy(hp)
        self.h.clear()


class _DeviceMatrix:
    """Shared handle management for the three matrix mirrors."""

    def _init_handles(self):
        self._handles = _Handles()
        self._finalizer = weakref.finalize(self, _Handles.release, self._handles)

    def handle(self, device=0, trans=True, multi=False, compute=None):
        """libvbc handle for mul!(y, B', x) (trans), mul!(y, B, x), or -- multi=True -- the
        matrix-core multi-RHS product Y = B'X (trans) / Y = B·X (a separate panel layout of B / Bᵀ,
        built on first use).
        `compute` = the vbc_dtype the product runs in (eltype(y)); default: the value eltype's own
        (floats) or exact Int64 (integers, Bool).  One handle per (device, layout, compute).
        Setting `B.serial = True` before the first product builds layouts that keep the reference's
        serial per-stripe summation order whatever the size (vbc.h VBC_CREATE_SERIAL)."""
        if multi:  # matrix-core panels: of B for B'X, of Bᵀ for B·X
            flags = _L.VBC_CREATE_MULTI if trans else _L.VBC_CREATE_MULTI_FORWARD
        else:
            flags = _L.VBC_CREATE_TRANSPOSED if trans else _L.VBC_CREATE_FORWARD
        compute = _L.compute_code(self.val.dtype) if compute is None else int(compute)
        if compute == _L.VBC_I64 and self.val.dtype.kind == "f":
            raise _L.UnsupportedDtype("a floating-point matrix cannot run in an integer eltype (InexactError)")
        if multi and compute == _L.VBC_I64:  # integer eltypes: one SpMV per column
            flags = _L.VBC_CREATE_TRANSPOSED if trans else _L.VBC_CREATE_FORWARD
        if getattr(self, "serial", False) and not multi:
            flags |= _L.VBC_CREATE_SERIAL  # the reference's serial per-stripe order in every layout
        return self._handles.get((int(device), flags, compute),
                                 lambda out: self._create(out, int(device), flags, compute))

    def _types(self, compute):
        return _L.vbc_types(_L.dtype_code(self.val.dtype), 64, compute, 0)

    def info(self, device=0, trans=True, multi=False, compute=None):
        inf = _L.vbc_info()
        _L.check(_L.lib().vbc_get_info(self.handle(device, trans, multi, compute), C.byref(inf)), "info")
        return {f: getattr(inf, f) for f, _ in _L.vbc_info._fields_}

    def release(self):
        self._handles.release()

    @property
    def shape(self):
        return (self.m, self.n)

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim - 1]

    @property
    def dtype(self):
        return self.val.dtype

    # adjoint / transpose views (LinearAlgebra.Adjoint / Transpose)
    @property
    def T(self):
        return Transpose(self)

    def adjoint(self):
        return Adjoint(self)

    def __matmul__(self, x):
        from .multiply import matmul
        return matmul(self, x)


class SparseMatrix1DVBC(_DeviceMatrix):
    """SparseMatrix1DVBC{W,Tv,Ti} (SparseMatrixVBCs.jl:36-53).

    Construct like the reference:
        SparseMatrix1DVBC[W](A)                 default: min memory for its Tv (constructors_1DVBC.jl:1-7)
        SparseMatrix1DVBC[W](A, method)         pack_stripe(A, method)
        SparseMatrix1DVBC[W](A, Φ)              given SplitPartition (constructors_1DVBC.jl:9)
        SparseMatrix1DVBC(W, m, n, Φ, pos, idx, ofs, val)   inner constructor (:44)
    """

    def __class_getitem__(cls, W):
        return lambda *a, **k: cls.from_csc(W, *a, **k)

    def __init__(self, W, m, n, Phi, pos, idx, ofs, val):
        if m < 0:
            raise _L.ArgumentError(f"number of rows (m) must be ≥ 0, got {m}")
        if n < 0:
            raise _L.ArgumentError(f"number of columns (n) must be ≥ 0, got {n}")
        if not isinstance(W, (int, np.integer)):
            raise _L.ArgumentError("W must be an Int")
        if W <= 0:
            raise _L.ArgumentError("W must be > 0")
        self.W, self.m, self.n = int(W), int(m), int(n)
        self.Phi = Phi if isinstance(Phi, SplitPartition) else SplitPartition(Phi)
        self.pos = np.ascontiguousarray(pos, dtype=np.int64)
        self.idx = np.ascontiguousarray(idx, dtype=np.int64)
        self.ofs = np.ascontiguousarray(ofs, dtype=np.int64)
        self.val = np.ascontiguousarray(val)
        self._init_handles()

    @classmethod
    def from_csc(cls, W, A, method=None, dtype=None):
        from .partition import CSCFields
        A = CSCFields(A)  # one conversion for the partitioner and the builder
        if method is None:  # constructors_1DVBC.jl:1-2: the memory model of the matrix's own Tv (Ti = Int64)
            Tv = dtype if dtype is not None else _value_dtype(A.A)
            method = DynamicTotalChunker(model_SparseMatrix1DVBC_memory(Tv, np.int64), W)
        Phi = method if isinstance(method, SplitPartition) else pack_stripe(A, method)
        (m, n), colptr, rowval, nzval = _csc_fields(A)
        if dtype is not None:
            nzval = nzval.astype(dtype)
        lib = _L.lib()
        L = len(Phi)
        pos = np.zeros(L + 1, np.int64)
        ofs = np.zeros(L + 1, np.int64)
        _L.check(lib.vbcx_1dvbc_count(m, n, colptr.ctypes.data, rowval.ctypes.data, L, Phi.spl.ctypes.data,
                                      pos.ctypes.data, ofs.ctypes.data), "SparseMatrix1DVBC")
        pad = _simd_pad(W, nzval.dtype)
        idx = np.zeros(pos[-1] - 1, np.int64)
        val = np.zeros(ofs[-1] - 1 + pad, nzval.dtype)
        _L.check(lib.vbcx_1dvbc_fill(m, n, W, colptr.ctypes.data, rowval.ctypes.data, nzval.ctypes.data,
                                     _L.dtype_code(nzval.dtype), L, Phi.spl.ctypes.data, pos.ctypes.data,
                                     ofs.ctypes.data, idx.ctypes.data, val.ctypes.data, pad),
                 "SparseMatrix1DVBC")
        return cls(W, m, n, Phi, pos, idx, ofs, val)

    def _create(self, out, device, flags, compute):
        spl = self.Phi.spl
        t = self._types(compute)
        return _L.lib().vbc1d_create_ex(out, self.m, self.n, self.W, len(self.Phi), spl.ctypes.data,
                                        self.pos.ctypes.data, self.idx.ctypes.data, self.ofs.ctypes.data,
                                        self.val.ctypes.data, len(self.val), C.byref(t), device, flags)

    def __repr__(self):
        return (f"SparseMatrix1DVBC{{{self.W},{self.val.dtype},Int64}}({self.m}×{self.n}, "
                f"{len(self.Phi)} stripes, {len(self.idx)} row-blocks)")


def default_partitioner_vbc(U, W, Tv, Ti=np.int64):
    """default_partitioner(SparseMatrixVBC{U,W,Tv,Ti}) (constructors_VBC.jl:1-8): the 5-phase
    AlternatePacker -- unit columns, unit rows, then the 2D memory model (costs.jl:140) on the
    columns (width <= W), its permutation on the rows (height <= U) and again on the columns."""
    mdl = model_SparseMatrixVBC_memory(Tv, Ti)
    return AlternatingPacker(EquiChunker(1), EquiChunker(1),
                             DynamicTotalChunker(ConstrainedCost(mdl, VertexCount(), W)),
                             DynamicTotalChunker(ConstrainedCost(permutedims(mdl), VertexCount(), U)),
                             DynamicTotalChunker(ConstrainedCost(mdl, VertexCount(), W)))


class SparseMatrixVBC(_DeviceMatrix):
    """SparseMatrixVBC{U,W,Tv,Ti} (SparseMatrixVBCs.jl:62-82); idx holds block-row ids.

        SparseMatrixVBC[U, W](A)            default 5-phase packer, 2D memory model (constructors_VBC.jl:1-8)
        SparseMatrixVBC[U, W](A, method)    pack_plaid(A, method)
        SparseMatrixVBC[U, W](A, Π, Φ)      given partitions (constructors_VBC.jl:15)
    """

    def __class_getitem__(cls, UW):
        U, W = UW
        return lambda *a, **k: cls.from_csc(U, W, *a, **k)

    def __init__(self, U, W, m, n, Pi, Phi, pos, idx, ofs, val):
        if m < 0:
            raise _L.ArgumentError(f"number of rows (m) must be ≥ 0, got {m}")
        if n < 0:
            raise _L.ArgumentError(f"number of columns (n) must be ≥ 0, got {n}")
        for name, v in (("U", U), ("W", W)):
            if not isinstance(v, (int, np.integer)):
                raise _L.ArgumentError(f"{name} must be an Int")
            if v <= 0:
                raise _L.ArgumentError(f"{name} must be > 0")
        self.U, self.W, self.m, self.n = int(U), int(W), int(m), int(n)
        self.Pi = Pi if isinstance(Pi, SplitPartition) else SplitPartition(Pi)
        self.Phi = Phi if isinstance(Phi, SplitPartition) else SplitPartition(Phi)
        self.pos = np.ascontiguousarray(pos, dtype=np.int64)
        self.idx = np.ascontiguousarray(idx, dtype=np.int64)
        self.ofs = np.ascontiguousarray(ofs, dtype=np.int64)
        self.val = np.ascontiguousarray(val)
        self._init_handles()

    @classmethod
    def from_csc(cls, U, W, A, method=None, Phi=None, dtype=None):
        if isinstance(method, SplitPartition):
            Pi = method
            if Phi is None:
                raise _L.ArgumentError("SparseMatrixVBC(A, Π, Φ) needs both partitions")
        else:
            if method is None:
                method = default_partitioner_vbc(U, W, dtype if dtype is not None else _value_dtype(sp.csc_matrix(A)))
            Pi, Phi = pack_plaid(A, method)
        (m, n), colptr, rowval, nzval = _csc_fields(A)
        if dtype is not None:
            nzval = nzval.astype(dtype)
        lib = _L.lib()
        K, L = len(Pi), len(Phi)
        pos = np.zeros(L + 1, np.int64)
        ofs = np.zeros(L + 1, np.int64)
        _L.check(lib.vbcx_vbc_count(m, n, colptr.ctypes.data, rowval.ctypes.data, K, Pi.spl.ctypes.data, L,
                                    Phi.spl.ctypes.data, pos.ctypes.data, ofs.ctypes.data), "SparseMatrixVBC")
        pad = _simd_pad(W, nzval.dtype, U)
        idx = np.zeros(pos[-1] - 1, np.int64)
        val = np.zeros(ofs[-1] - 1 + pad, nzval.dtype)
        _L.check(lib.vbcx_vbc_fill(m, n, U, W, colptr.ctypes.data, rowval.ctypes.data, nzval.ctypes.data,
                                   _L.dtype_code(nzval.dtype), K, Pi.spl.ctypes.data, L, Phi.spl.ctypes.data,
                                   pos.ctypes.data, ofs.ctypes.data, idx.ctypes.data, val.ctypes.data, pad),
                 "SparseMatrixVBC")
        return cls(U, W, m, n, Pi, Phi, pos, idx, ofs, val)

    def _create(self, out, device, flags, compute):
        t = self._types(compute)
        return _L.lib().vbc2d_create_ex(out, self.m, self.n, self.U, self.W, len(self.Pi), self.Pi.spl.ctypes.data,
                                        len(self.Phi), self.Phi.spl.ctypes.data, self.pos.ctypes.data,
                                        self.idx.ctypes.data, self.ofs.ctypes.data, self.val.ctypes.data,
                                        len(self.val), C.byref(t), device, flags)

    def __repr__(self):
        return (f"SparseMatrixVBC{{{self.U},{self.W},{self.val.dtype},Int64}}({self.m}×{self.n}, "
                f"{len(self.Pi)}×{len(self.Phi)} partition, {len(self.idx)} blocks)")


class SparseMatrixCSC(_DeviceMatrix):
    """SparseMatrixCSC{Tv,Int64} fields (colptr, rowval, nzval), the operand of TrSpMV!."""

    def __init__(self, A):
        (self.m, self.n), self.colptr, self.rowval, self.nzval = _csc_fields(A)
        self.val = self.nzval
        self._init_handles()

    def _create(self, out, device, flags, compute):
        t = self._types(compute)
        return _L.lib().vbc_csc_create_ex(out, self.m, self.n, self.colptr.ctypes.data, self.rowval.ctypes.data,
                                          self.nzval.ctypes.data, C.byref(t), device, flags)


class Adjoint:
    """LinearAlgebra.Adjoint wrapper (real eltypes: identical to Transpose)."""

    def __init__(self, parent):
        self.parent = parent

    @property
    def shape(self):
        return (self.parent.n, self.parent.m)

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim - 1]

    def __matmul__(self, x):
        from .multiply import matmul
        return matmul(self, x)


class Transpose(Adjoint):
    """LinearAlgebra.Transpose wrapper."""


def adjoint(A):
    return Adjoint(A)


def transpose(A):
    return Transpose(A)
