"""The C-ABI library loads, exports every symbol include/*.h declares, and reports errors without a
GPU (no compute calls here)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from sparsematrixvbcs_amd import _lib as L
from tests.conftest import ROOT, has_gpu


def declared_symbols():
    syms = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        syms |= set(re.findall(r"^\s*(?:VBC_API\s+)?int\s+(vbcx?_?\w+)\s*\(", text, flags=re.M))
    return syms


def test_library_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 18
    assert syms == set(L.ABI_SYMBOLS)
    lib = C.CDLL(str(L.LIB_PATH))
    for s in sorted(syms):
        assert hasattr(lib, s), s
    # built with -fvisibility=hidden: the C ABI is the only dynamic interface
    out = subprocess.run(["nm", "-D", "--defined-only", str(L.LIB_PATH)], capture_output=True, text=True)
    if out.returncode == 0:
        exported = {ln.split()[-1] for ln in out.stdout.splitlines() if " T " in ln}
        assert exported == syms, exported ^ syms


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", str(L.LIB_PATH)],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-readelf unavailable")
    assert ".hip_fatbin" in out.stdout
    blob = L.LIB_PATH.read_bytes()
    assert b"gfx950" in blob


def test_error_paths_without_gpu():
    lib = L.lib()
    h = C.c_void_p()
    z = np.array([1, 1], dtype=np.int64)
    # W = 0 -> ArgumentError before any device call (SparseMatrixVBCs.jl:50)
    st = lib.vbc1d_create(C.byref(h), 2, 1, 0, 1, np.array([1, 2]).ctypes.data, z.ctypes.data, None,
                          z.ctypes.data, None, 0, L.VBC_F64, 0, 0)
    assert st == L.VBC_INVALID_ARG and "W must be > 0" in L.last_error()
    # w > W -> AssertionError
    spl = np.array([1, 4], dtype=np.int64)
    st = lib.vbc1d_create(C.byref(h), 2, 3, 2, 1, spl.ctypes.data, z.ctypes.data, None, z.ctypes.data,
                          None, 0, L.VBC_F64, 0, 0)
    assert st == L.VBC_ASSERTION
    assert lib.vbc_mul(None, 0, None, 0, None, 0, 1.0, 0.0, 0, None, 0) == L.VBC_INVALID_ARG
    assert lib.vbc_version() >= 100


@pytest.mark.skipif(has_gpu(), reason="checks the no-GPU failure mode")
def test_product_path_fails_loudly_without_gpu():
    import scipy.sparse as sp
    A = sp.random(8, 6, 0.5, random_state=0, format="csc")
    B = V.SparseMatrix1DVBC[2](A, V.EquiChunker(2))
    with pytest.raises(V.HIPError):
        V.mul_(np.zeros(8), B, np.zeros(6))
    with pytest.raises(V.DimensionMismatch):
        V.mul_(np.zeros(7), B, np.zeros(6))


def test_vbc2d_create_rejects_malformed_pos():
    """pos must be non-decreasing and stay inside idx (no out-of-bounds host reads)."""
    lib = L.lib()
    h = C.c_void_p()
    pspl = np.array([1, 3], dtype=np.int64)
    spl = np.array([1, 2, 3], dtype=np.int64)
    idx = np.array([1, 1], dtype=np.int64)
    val = np.zeros(8)
    for pos, ofs in (([1, 1000, 3], [1, 3, 5]), ([1, 3, 2], [1, 5, 3])):
        pos = np.array(pos, dtype=np.int64)
        ofs = np.array(ofs, dtype=np.int64)
        st = lib.vbc2d_create(C.byref(h), 2, 2, 2, 1, 1, pspl.ctypes.data, 2, spl.ctypes.data, pos.ctypes.data,
                              idx.ctypes.data, ofs.ctypes.data, val.ctypes.data, len(val), L.VBC_F64, 0, 0)
        assert st == L.VBC_INVALID_ARG, st
        assert "pos" in L.last_error()


def test_csc_create_rejects_null_arrays():
    lib = L.lib()
    h = C.c_void_p()
    colptr = np.array([1, 2], dtype=np.int64)
    st = lib.vbc_csc_create(C.byref(h), 1, 1, colptr.ctypes.data, None, None, L.VBC_F64, 0, 0)
    assert st == L.VBC_INVALID_ARG and "NULL" in L.last_error()


def test_typed_create_validation_without_gpu():
    """vbc*_create_ex checks the type description before any device call."""
    lib = L.lib()
    h = C.c_void_p()
    spl = np.array([1, 2], dtype=np.int32)
    z = np.array([1, 1], dtype=np.int32)
    bad = [L.vbc_types(L.VBC_F64, 16, L.VBC_F64, 0),      # index_bits
           L.vbc_types(L.VBC_F64, 32, L.VBC_I32, 0),      # compute eltype
           L.vbc_types(L.VBC_F32, 32, L.VBC_I64, 0),      # float values on an integer handle
           L.vbc_types(9, 32, L.VBC_F64, 0)]              # unknown val eltype
    for t in bad:
        st = lib.vbc1d_create_ex(C.byref(h), 1, 1, 1, 1, spl.ctypes.data, z.ctypes.data, None, z.ctypes.data,
                                 None, 0, C.byref(t), 0, 0)
        assert st in (L.VBC_INVALID_ARG, L.VBC_UNSUPPORTED_DTYPE), st
    # Int32 indices are widened and then validated like the Int64 path: W = 0 -> ArgumentError
    t = L.vbc_types(L.VBC_I32, 32, L.VBC_I64, 0)
    st = lib.vbc1d_create_ex(C.byref(h), 1, 1, 0, 1, spl.ctypes.data, z.ctypes.data, None, z.ctypes.data,
                             None, 0, C.byref(t), 0, 0)
    assert st == L.VBC_INVALID_ARG and "W must be > 0" in L.last_error()


def test_mirror_keeps_reference_eltypes():
    """Bool / Int32 / Int64 matrices keep their eltype (SparseMatrix1DVBC{W,Bool} etc.); their default
    compute eltype is exact Int64, Float32 / Float64 compute in themselves."""
    import scipy.sparse as sp
    for dt, comp in ((np.bool_, L.VBC_I64), (np.int32, L.VBC_I64), (np.int64, L.VBC_I64),
                     (np.float32, L.VBC_F32), (np.float64, L.VBC_F64)):
        A = sp.csc_matrix(np.array([[1, 0, 1], [0, 1, 1]], dtype=dt))
        B = V.SparseMatrix1DVBC[4](A, V.StrictChunker(4))
        assert B.val.dtype == np.dtype(dt)
        assert L.compute_code(B.val.dtype) == comp
        D = np.zeros((2, 3), dtype=np.int64)
        for l in range(len(B.Phi)):
            j, w = B.Phi.spl[l] - 1, B.Phi.spl[l + 1] - B.Phi.spl[l]
            q = B.ofs[l] - 1
            for Q in range(B.pos[l] - 1, B.pos[l + 1] - 1):
                D[B.idx[Q] - 1, j:j + w] += B.val[q:q + w].astype(np.int64)
                q += w
        assert np.array_equal(D, A.toarray().astype(np.int64))


def test_sharded_create_validation_without_gpu():
    """vbc1d_create_sharded / vbc_sharded_* reject bad arguments before touching a device."""
    lib = L.lib()
    h = C.c_void_p()
    spl = np.array([1, 3], np.int64)
    pos = np.array([1, 2], np.int64)
    idx = np.array([1], np.int64)
    ofs = np.array([1, 3], np.int64)
    val = np.ones(2)
    t = L.vbc_types(L.VBC_F64, 64, L.VBC_F64, 0)
    devs = (C.c_int * 2)(0, 0)
    args = (C.byref(h), 1, 2, 8, 1, spl.ctypes.data, pos.ctypes.data, idx.ctypes.data, ofs.ctypes.data,
            val.ctypes.data, 2, C.byref(t))
    assert lib.vbc1d_create_sharded(*args, 0, devs, L.VBC_SPLIT_STRIPES, 0) == L.VBC_INVALID_ARG  # no GPUs
    assert "ngpus" in L.last_error()
    assert lib.vbc1d_create_sharded(*args, 2, devs, 7, 0) == L.VBC_INVALID_ARG  # unknown split
    assert lib.vbc1d_create_sharded(*args[:-1], None, 2, devs, L.VBC_SPLIT_ROWS, 0) == L.VBC_INVALID_ARG
    assert lib.vbc_sharded_mul(None, 1, None, 0, None, 0, 1.0, 0.0, L.VBC_MEM_DEVICE, None, 0) == L.VBC_INVALID_ARG
    n = C.c_int()
    assert lib.vbc_sharded_count(None, C.byref(n)) == L.VBC_INVALID_ARG
    assert lib.vbc_sharded_shard(None, 0, None, None, None, None) == L.VBC_INVALID_ARG
    assert lib.vbc_sharded_xspan(None, 0, None, None) == L.VBC_INVALID_ARG
    assert lib.vbc_sharded_destroy(None) == L.VBC_OK


def test_sharded_ex_and_2d_validation_without_gpu():
    """vbc_sharded_mul_ex / vbc2d_create_sharded reject bad arguments before touching a device; the
    library reports the ABI version this binding was written for (vbc.h VBC_VERSION, vbc_info size)."""
    lib = L.lib()
    assert lib.vbc_version() // 10000 == L.VBC_VERSION_MAJOR
    assert C.sizeof(L.vbc_info) == L.VBC_INFO_SIZE
    assert lib.vbc_sharded_mul_ex(None, 1, None, L.VBC_F32, 1, 0, None, L.VBC_F32, 1, 0, 1.0, 0.0,
                                  L.VBC_MEM_HOST, None, 0) == L.VBC_INVALID_ARG
    h = C.c_void_p()
    pspl = np.array([1, 3], np.int64)
    spl = np.array([1, 3], np.int64)
    pos = np.array([1, 2], np.int64)
    idx = np.array([1], np.int64)
    ofs = np.array([1, 5], np.int64)
    val = np.ones(4)
    t = L.vbc_types(L.VBC_F64, 64, L.VBC_F64, 0)
    devs = (C.c_int * 2)(0, 0)
    args = (C.byref(h), 2, 2, 2, 2, 1, pspl.ctypes.data, 1, spl.ctypes.data, pos.ctypes.data, idx.ctypes.data,
            ofs.ctypes.data, val.ctypes.data, 4, C.byref(t))
    assert lib.vbc2d_create_sharded(*args, 0, devs, L.VBC_SPLIT_STRIPES, 0) == L.VBC_INVALID_ARG
    assert lib.vbc2d_create_sharded(*args, 2, devs, 9, 0) == L.VBC_INVALID_ARG
    assert lib.vbc2d_create_sharded(*args[:-1], None, 2, devs, L.VBC_SPLIT_ROWS, 0) == L.VBC_INVALID_ARG
    assert lib.vbc2d_create_sharded(C.byref(h), 2, 2, 2, 2, 1, None, *args[7:], 2, devs, 0, 0) == L.VBC_INVALID_ARG
    assert lib.vbc_mul_mat_ex(None, 1, 1, None, L.VBC_F64, 1, 0, None, L.VBC_F64, 1, 0, 1.0, 0.0,
                              L.VBC_MEM_HOST, None, 0) == L.VBC_INVALID_ARG
