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
