"""mul! / * / TrSpMV! on the GPU through libvbc (the reference's operator surface).

    mul_(y, B, x[, α, β])      LinearAlgebra.mul!(y, B, x, α, β)     multiply_1DVBC.jl:9 / multiply_VBC.jl:3
    mul_(y, B.T, x[, α, β])    mul!(y, B', x, α, β)                   multiply_1DVBC.jl:85 / multiply_VBC.jl:89
    TrSpMV_(y, A, x)           TrSpMV!(y, A::SparseMatrixCSC, x)      TrSpMV.jl:1-20
    B @ x, B.T @ x             Base.:*                                multiply_1DVBC.jl:182-185

x / y are torch CUDA tensors (the product is enqueued on torch's current stream of that device, no
synchronisation) or numpy arrays (staged through HBM by libvbc; returns when y is final).  Like the
reference, the product computes in eltype(y) with the matrix values and x converted to it
(multiply_1DVBC.jl:27,34,102), and x / y may be any strided vectors.  Semantics are BLAS (y = α·op(B)·x + β·y); pass
`quirks=True` to reproduce the reference's α/β handling bit for bit (vbc.h VBC_MUL_REFERENCE_QUIRKS).
There is no CPU fallback: without libvbc or a GPU these raise.
"""
import numpy as np

from . import _lib as _L
from .matrices import Adjoint, SparseMatrixCSC, _DeviceMatrix


def _unwrap(A):
    if isinstance(A, Adjoint):
        return A.parent, True
    return A, False


def _is_torch(a):
    return type(a).__module__.startswith("torch")


def _mem_device_stream(x, y, stream):
    if _is_torch(x) or _is_torch(y):
        import torch
        if not (_is_torch(x) and _is_torch(y)):
            raise _L.ArgumentError("x and y must both be torch tensors or both numpy arrays")
        if not (x.is_cuda and y.is_cuda):
            raise _L.ArgumentError("torch tensors must live on a GPU (no CPU fallback)")
        if x.device != y.device:
            raise _L.ArgumentError("x and y must be on the same device")
        dev = x.device.index
        if stream is None:
            stream = torch.cuda.current_stream(x.device).cuda_stream
        elif hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        return _L.VBC_MEM_DEVICE, dev, stream
    return _L.VBC_MEM_HOST, 0, None


def _check_dtype(a, dtype, name):
    if _L.dtype_code(a.dtype) != _L.dtype_code(dtype):
        raise _L.UnsupportedDtype(f"{name} eltype {a.dtype} != {dtype}")


def _stride(a):
    """Element stride of a 1-D numpy array or torch tensor (StridedVector; may be negative in numpy)."""
    if isinstance(a, np.ndarray):
        if a.strides[0] % a.itemsize:
            raise _L.ArgumentError("stride is not a multiple of the element size")
        return a.strides[0] // a.itemsize if a.shape[0] > 1 else 1
    return a.stride(0) if a.shape[0] > 1 else 1


def _compute_for(y, B):
    """The eltype the product computes in: eltype(y) (multiply_1DVBC.jl:27,34,102)."""
    cy = _L.dtype_code(y.dtype)
    if cy in (_L.VBC_F64, _L.VBC_F32):
        return cy
    if cy in (_L.VBC_I64, _L.VBC_I32):
        if B.dtype.kind == "f":
            raise _L.UnsupportedDtype(f"integer y with a {B.dtype} matrix (InexactError in the reference)")
        return _L.VBC_I64
    raise _L.UnsupportedDtype(f"no GPU product into a {y.dtype} y")


def mul_(y, A, x, alpha=1.0, beta=0.0, *, stream=None, quirks=False, device=None, engine="auto"):
    """LinearAlgebra.mul!(y, A, x, α, β); returns y.  Any StridedVector x / y (strides, eltypes: the
    product computes in eltype(y) with x converted, as multiply_1DVBC.jl:102 does).  Matrix x / y go
    to mulmat_ (engine)."""
    B, trans = _unwrap(A)
    if hasattr(B, "_mul") and not isinstance(B, _DeviceMatrix):  # distributed.MultiGPUSparseMatrix1DVBC
        return B._mul(y, x, trans, alpha, beta, stream, quirks)
    if not isinstance(B, _DeviceMatrix):
        raise TypeError(f"mul_ expects SparseMatrix1DVBC / SparseMatrixVBC / SparseMatrixCSC, got {type(B)}")
    if len(y.shape) != 1 or len(x.shape) != 1:
        return mulmat_(y, A, x, alpha, beta, stream=stream, quirks=quirks, engine=engine)
    mem, dev, stream = _mem_device_stream(x, y, stream)
    if device is not None and mem == _L.VBC_MEM_HOST:
        dev = device
    # DimensionMismatch before any handle is built (multiply_1DVBC.jl:44-45, :139-140)
    nx, ny = x.shape[0], y.shape[0]
    if (nx, ny) != ((B.m, B.n) if trans else (B.n, B.m)):
        raise _L.DimensionMismatch(f"size(A)={A.shape}, length(x)={nx}, length(y)={ny}")
    cdt = _compute_for(y, B)
    xdt, ydt = _L.dtype_code(x.dtype), _L.dtype_code(y.dtype)
    incx, incy = _stride(x), _stride(y)
    h = B.handle(dev, trans, compute=cdt)
    flags = _L.VBC_MUL_REFERENCE_QUIRKS if quirks else 0
    if xdt == cdt and ydt == cdt and incx == 1 and incy == 1:
        _L.check(_L.lib().vbc_mul(h, int(trans), _L.ptr(x), nx, _L.ptr(y), ny, float(alpha), float(beta), mem,
                                  stream, flags), "mul!")
    else:
        _L.check(_L.lib().vbc_mul_ex(h, int(trans), _L.ptr(x), xdt, incx, nx, _L.ptr(y), ydt, incy, ny,
                                     float(alpha), float(beta), mem, stream, flags), "mul!")
    return y


def _layout(M):
    """'R' for row-major (C-contiguous, right-hand sides interleaved), 'C' for column-major."""
    if isinstance(M, np.ndarray):  # views with ld > extent are fine: only the extent is touched
        s0, s1 = M.strides[0] // M.itemsize, M.strides[1] // M.itemsize
        if M.strides[1] == M.itemsize and M.shape[1] > 1 and s0 >= M.shape[1]:
            return "R", s0
        if M.strides[0] == M.itemsize or M.shape[0] <= 1:
            if M.shape[1] <= 1:
                return "C", max(M.shape[0], 1)
            if s1 >= M.shape[0]:
                return "C", s1
    else:
        if M.stride(1) == 1 and M.shape[1] > 1:
            return "R", M.stride(0)
        if M.stride(0) == 1:
            return "C", M.stride(1) if M.shape[1] > 1 else max(M.shape[0], 1)
    raise _L.ArgumentError("matrix operands must be row-major or column-major with unit inner stride")


MFMA_MIN_RHS = 2


def mulmat_(Y, A, X, alpha=1.0, beta=0.0, *, stream=None, quirks=False, engine="auto"):
    """Multi-RHS Y = α·op(A)·X + β·Y (column-by-column semantics; the reference has no matrix
    mul!).  engine="mfma" (default with >= MFMA_MIN_RHS columns): the matrix-core panel product --
    of B for B'X, of Bᵀ for B·X -- row- or column-major operands, the matrix read once; engine="vector":
    the SpMV layout (fused vector kernel for row-major B'X, one SpMV per column otherwise)."""
    B, trans = _unwrap(A)
    mem, dev, stream = _mem_device_stream(X, Y, stream)
    cdt = _compute_for(Y, B)
    if X.shape[1] != Y.shape[1]:
        raise _L.DimensionMismatch("X and Y have different numbers of columns")
    if X.shape[1] <= 1 or cdt == _L.VBC_I64 or X.dtype != Y.dtype:
        # column by column as strided vectors (a single column, integer eltypes, mixed eltypes):
        # every column view keeps its own stride, so a column of a wider row-major array is read
        # and written exactly where it lives
        for c in range(X.shape[1]):
            mul_(Y[:, c], A, X[:, c], alpha, beta, stream=stream, quirks=quirks)
        return Y
    _check_dtype(X, Y.dtype, "X")  # eltype(X) == eltype(Y); the matrix runs in that eltype
    lx, ldx = _layout(X)
    ly, ldy = _layout(Y)
    if lx != ly:
        raise _L.ArgumentError("X and Y must have the same layout")
    nrhs = X.shape[1]
    if engine not in ("auto", "mfma", "vector"):
        raise _L.ArgumentError(f"engine must be 'auto', 'mfma' or 'vector', got {engine!r}")
    # matrix cores for B'X (panel layout of B) and B·X (panel layout of Bᵀ): the matrix is read once
    mfma = cdt != _L.VBC_I64 and (engine == "mfma" or (engine == "auto" and nrhs >= MFMA_MIN_RHS))
    h = B.handle(dev, trans, multi=mfma, compute=cdt)
    flags = (_L.VBC_MUL_REFERENCE_QUIRKS if quirks else 0) | (_L.VBC_MAT_ROWMAJOR if lx == "R" else 0)
    _L.check(_L.lib().vbc_mul_mat_ex(h, int(trans), nrhs, _L.ptr(X), _L.dtype_code(X.dtype), max(ldx, 1), X.shape[0],
                                     _L.ptr(Y), _L.dtype_code(Y.dtype), max(ldy, 1), Y.shape[0], float(alpha),
                                     float(beta), mem, stream, flags), "mul!")
    return Y


def promote_op_matprod(ta, tx):
    """Julia's promote_op(matprod, Ta, Tx) for the eltypes the kernels take (multiply_1DVBC.jl:182-183):
    matprod(a, b) = a*b + a*b, so a float on either side gives the wider float (Julia's
    promote_type(Float32, Int64) is Float32, unlike numpy's result_type), two integers the wider integer,
    and Bool*Bool + Bool*Bool is an Int64."""
    ta, tx = np.dtype(ta), np.dtype(tx)
    floats = [t for t in (ta, tx) if t.kind == "f"]
    if floats:
        return max(floats, key=lambda t: t.itemsize)
    ints = [t for t in (ta, tx) if t.kind in "iu"]
    if not ints:  # Bool * Bool: the sum of two Bools is an Int
        return np.dtype(np.int64)
    return max(ints, key=lambda t: t.itemsize)


def matmul(A, x):
    """Base.:*(A, x): y = similar(x, promote_op(matprod, eltype(A), eltype(x)), size(A, 1)), then
    mul!(y, A, x, true, false) (multiply_1DVBC.jl:182-183, multiply_VBC.jl:194-195)."""
    m = A.shape[0]
    B, _ = _unwrap(A)
    if _is_torch(x):
        import torch
        xt = np.dtype(str(x.dtype).replace("torch.", "").replace("bool", "bool_"))
        T = getattr(torch, promote_op_matprod(B.dtype, xt).name)
        y = torch.empty((m,) + tuple(x.shape[1:]), dtype=T, device=x.device)  # same layout as x
        if x.dim() == 2 and x.stride(0) == 1 and x.shape[1] > 1:
            y = torch.empty((x.shape[1], m), dtype=T, device=x.device).T
    else:
        order = "F" if (x.ndim == 2 and x.flags.f_contiguous and not x.flags.c_contiguous) else "C"
        y = np.empty((m,) + tuple(x.shape[1:]), dtype=promote_op_matprod(B.dtype, x.dtype), order=order)
    return mul_(y, A, x, True, False)


def TrSpMV_(y, A, x, *, stream=None):
    """TrSpMV!(y, A::SparseMatrixCSC, x): y = Aᵀx (overwrite), TrSpMV.jl:1-20."""
    if not isinstance(A, SparseMatrixCSC):
        cached = getattr(A, "_vbc_csc", None)
        if cached is None:
            cached = SparseMatrixCSC(A)
            try:
                A._vbc_csc = cached
            except AttributeError:
                pass
        A = cached
    return mul_(y, Adjoint(A), x, 1.0, 0.0, stream=stream)
