"""ctypes binding of libvbc (include/vbc.h, include/vbc_host.h).

The product path has no fallback: if libvbc.so is missing or cannot be loaded, every product call
raises.  Status codes map onto the reference's exception types (vbc.h `vbc_status`).
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("VBC_LIBRARY", PKG_DIR / "libvbc.so"))

VBC_OK, VBC_DIM_MISMATCH, VBC_INVALID_ARG, VBC_HIP_ERROR, VBC_RCCL_ERROR, VBC_UNSUPPORTED_DTYPE, \
    VBC_ASSERTION = range(7)
VBC_F64, VBC_F32, VBC_I64, VBC_I32, VBC_BOOL = range(5)
VBC_MEM_DEVICE, VBC_MEM_HOST = 0, 1
VBC_CREATE_TRANSPOSED, VBC_CREATE_FORWARD, VBC_CREATE_MULTI, VBC_CREATE_SERIAL = 0x1, 0x2, 0x4, 0x8
VBC_CREATE_MULTI_FORWARD = 0x10
VBC_VERSION_MAJOR = 3  # include/vbc.h VBC_VERSION / 10000: the vbc_info layout below is that version's
VBC_INFO_SIZE = 152
VBC_MUL_REFERENCE_QUIRKS = 0x1
VBC_MAT_ROWMAJOR = 0x2
VBC_SPLIT_STRIPES, VBC_SPLIT_ROWS, VBC_SPLIT_AUTO = 0, 1, 2

# Every symbol include/*.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "vbc1d_create", "vbc2d_create", "vbc_csc_create", "vbc_destroy", "vbc_mul", "vbc_mul_mat",
    "vbc1d_create_ex", "vbc2d_create_ex", "vbc_csc_create_ex", "vbc_mul_ex", "vbc_mul_mat_ex",
    "vbc_get_info", "vbc_last_error", "vbc_version",
    "vbc1d_create_sharded", "vbc2d_create_sharded", "vbc_sharded_mul", "vbc_sharded_mul_ex", "vbc_sharded_destroy",
    "vbc_sharded_count", "vbc_sharded_shard", "vbc_sharded_split", "vbc_sharded_xspan",
    "vbcx_partition_equi", "vbcx_partition_strict", "vbcx_partition_overlap",
    "vbcx_partition_dynamic", "vbcx_partition_dynamic_table", "vbcx_partition_block", "vbcx_1dvbc_count", "vbcx_1dvbc_fill", "vbcx_vbc_count",
    "vbcx_vbc_fill", "vbcx_transpose_pattern",
)


class DimensionMismatch(ValueError):
    """Julia's DimensionMismatch (multiply_1DVBC.jl:44-45,139-140)."""


class ArgumentError(ValueError):
    """Julia's ArgumentError (SparseMatrixVBCs.jl:45-50,72-79)."""


class HIPError(RuntimeError):
    pass


class UnsupportedDtype(TypeError):
    pass


class vbc_types(C.Structure):
    """include/vbc.h vbc_types: the reference's Tv / Ti type parameters and the compute eltype."""
    _fields_ = [("val_dtype", C.c_int32), ("index_bits", C.c_int32), ("compute_dtype", C.c_int32),
                ("reserved", C.c_int32)]


class vbc_info(C.Structure):
    _fields_ = [("m", C.c_int64), ("n", C.c_int64), ("L", C.c_int64), ("K", C.c_int64),
                ("nblocks", C.c_int64), ("nrows", C.c_int64), ("nval", C.c_int64),
                ("nnz_hint", C.c_int64), ("dtype", C.c_int32), ("device", C.c_int32),
                ("bins_t", C.c_int32), ("bins_f", C.c_int32), ("device_bytes", C.c_int64),
                ("bytes_t", C.c_int64), ("bytes_f", C.c_int64), ("bins_m", C.c_int32),
                ("slot_bins", C.c_int32), ("bytes_m", C.c_int64),
                ("sweep_bins", C.c_int32), ("planar_bins", C.c_int32),
                ("planar_run", C.c_int32), ("planar_split", C.c_int32),
                ("planar_pair", C.c_int32), ("fwd_run", C.c_int32),
                ("planar_mask", C.c_int32)]


_lib = None


def lib():
    """Load libvbc.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"libvbc.so not found at {LIB_PATH}; build it with `make -C {PKG_DIR}` "
                              "or __graft_entry__.build()")
        # PyTorch bundles its own HIP / HSA runtimes under the same sonames as /opt/rocm's
        # (libamdhip64.so.7, libhsa-runtime64.so.1) but links them by their unversioned names: if
        # libvbc were loaded first, torch would load a second pair of runtimes and whichever
        # initialised second would see no device.  Importing torch first makes libvbc bind to the
        # runtime already in the process (one runtime, shared streams and memory).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        ver = L.vbc_version()
        if ver // 10000 != VBC_VERSION_MAJOR or C.sizeof(vbc_info) != VBC_INFO_SIZE:
            raise ImportError(f"libvbc ABI {ver} does not match this binding (major {VBC_VERSION_MAJOR}, "
                              f"vbc_info {C.sizeof(vbc_info)} bytes); rebuild it")
        P, I64, INT, U, D = C.c_void_p, C.c_int64, C.c_int, C.c_uint, C.c_double
        L.vbc1d_create.argtypes = [C.POINTER(P), I64, I64, I64, I64, P, P, P, P, P, I64, INT, INT, U]
        L.vbc2d_create.argtypes = [C.POINTER(P), I64, I64, I64, I64, I64, P, I64, P, P, P, P, P, I64,
                                   INT, INT, U]
        L.vbc_csc_create.argtypes = [C.POINTER(P), I64, I64, P, P, P, INT, INT, U]
        T = C.POINTER(vbc_types)
        L.vbc1d_create_ex.argtypes = [C.POINTER(P), I64, I64, I64, I64, P, P, P, P, P, I64, T, INT, U]
        L.vbc2d_create_ex.argtypes = [C.POINTER(P), I64, I64, I64, I64, I64, P, I64, P, P, P, P, P, I64, T, INT, U]
        L.vbc_csc_create_ex.argtypes = [C.POINTER(P), I64, I64, P, P, P, T, INT, U]
        L.vbc_mul_ex.argtypes = [P, INT, P, INT, I64, I64, P, INT, I64, I64, D, D, INT, P, U]
        L.vbc_destroy.argtypes = [P]
        L.vbc1d_create_sharded.argtypes = [C.POINTER(P), I64, I64, I64, I64, P, P, P, P, P, I64, T, INT, P, INT, U]
        L.vbc2d_create_sharded.argtypes = [C.POINTER(P), I64, I64, I64, I64, I64, P, I64, P, P, P, P, P, I64, T, INT,
                                           P, INT, U]
        L.vbc_sharded_mul.argtypes = [P, INT, P, I64, P, I64, D, D, INT, P, U]
        L.vbc_sharded_mul_ex.argtypes = [P, INT, P, INT, I64, I64, P, INT, I64, I64, D, D, INT, P, U]
        L.vbc_sharded_destroy.argtypes = [P]
        L.vbc_sharded_count.argtypes = [P, C.POINTER(INT)]
        L.vbc_sharded_split.argtypes = [P, C.POINTER(INT)]
        L.vbc_sharded_shard.argtypes = [P, INT, C.POINTER(P), C.POINTER(I64), C.POINTER(I64), C.POINTER(INT)]
        L.vbc_sharded_xspan.argtypes = [P, INT, C.POINTER(I64), C.POINTER(I64)]
        L.vbc_mul.argtypes = [P, INT, P, I64, P, I64, D, D, INT, P, U]
        L.vbc_mul_mat.argtypes = [P, INT, I64, P, I64, I64, P, I64, I64, D, D, INT, P, U]
        L.vbc_mul_mat_ex.argtypes = [P, INT, I64, P, INT, I64, I64, P, INT, I64, I64, D, D, INT, P, U]
        L.vbc_get_info.argtypes = [P, C.POINTER(vbc_info)]
        L.vbc_last_error.argtypes = [C.c_char_p, C.c_size_t]
        L.vbcx_partition_equi.argtypes = [I64, I64, P, P]
        L.vbcx_partition_strict.argtypes = [I64, I64, P, P, I64, P, P]
        L.vbcx_partition_overlap.argtypes = [I64, I64, P, P, D, I64, P, P]
        L.vbcx_partition_dynamic.argtypes = [I64, I64, P, P, I64, D, D, D, D, D, P, P]
        L.vbcx_partition_dynamic_table.argtypes = [I64, I64, P, P, I64, P, P, P, P]
        L.vbcx_partition_block.argtypes = [I64, I64, P, P, P, I64, I64, P, I64, P, P, P, P]
        L.vbcx_1dvbc_count.argtypes = [I64, I64, P, P, I64, P, P, P]
        L.vbcx_1dvbc_fill.argtypes = [I64, I64, I64, P, P, P, INT, I64, P, P, P, P, P, I64]
        L.vbcx_vbc_count.argtypes = [I64, I64, P, P, I64, P, I64, P, P, P]
        L.vbcx_vbc_fill.argtypes = [I64, I64, I64, I64, P, P, P, INT, I64, P, I64, P, P, P, P, P, I64]
        L.vbcx_transpose_pattern.argtypes = [I64, I64, P, P, P, P]
        _lib = L
    return _lib


def last_error():
    buf = C.create_string_buffer(1024)
    lib().vbc_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(status, what=""):
    if status == VBC_OK:
        return
    msg = f"{what}: {last_error()}" if what else last_error()
    if status == VBC_DIM_MISMATCH:
        raise DimensionMismatch(msg)
    if status == VBC_INVALID_ARG:
        raise ArgumentError(msg)
    if status == VBC_ASSERTION:
        raise AssertionError(msg)
    if status == VBC_UNSUPPORTED_DTYPE:
        raise UnsupportedDtype(msg)
    raise HIPError(msg)


def ptr(a):
    """Address of a numpy array's data, a torch tensor's storage, or None."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


_CODES = {np.dtype(np.float64): VBC_F64, np.dtype(np.float32): VBC_F32, np.dtype(np.int64): VBC_I64,
          np.dtype(np.int32): VBC_I32, np.dtype(np.bool_): VBC_BOOL}


def dtype_code(dtype):
    """vbc_dtype of a numpy dtype, a torch dtype or its name."""
    name = str(dtype).replace("torch.", "")
    try:
        dtype = np.dtype("bool" if name == "bool" else name)
    except TypeError:
        raise UnsupportedDtype(f"no GPU eltype for {dtype}")
    if dtype not in _CODES:
        raise UnsupportedDtype(f"the GPU path supports Float64/Float32/Int64/Int32/Bool eltypes, got {dtype}")
    return _CODES[dtype]


def compute_code(val_dtype):
    """The compute eltype a matrix of this value eltype runs in by default: floats in themselves,
    integers and Bool in exact Int64 (vbc.h vbc_types)."""
    c = dtype_code(val_dtype)
    return c if c in (VBC_F64, VBC_F32) else VBC_I64
