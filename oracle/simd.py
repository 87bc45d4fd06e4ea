"""ctypes wrapper of the CPU baseline port (oracle/libvbcsimd.so, vbc_simd.c).  BENCHMARK / TEST
INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/ use it to time the reference's own
SIMD CPU kernels (multiply_1DVBC.jl:90-180, TrSpMV.jl:1-20) on the host cores beside the GPU.
"""
import ctypes as C
import os
import platform
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "libvbcsimd.so"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "vbc_simd.c").stat().st_mtime:
            subprocess.run(["make", "-C", str(HERE), "-s", "libvbcsimd.so"], check=True)
        _lib = C.CDLL(str(LIB_PATH))
        P, I, INT = C.c_void_p, C.c_int64, C.c_int
        for suf in ("f64", "f32"):
            getattr(_lib, "simd_1dvbc_mul_t_" + suf).argtypes = [I, I, I, P, P, P, P, P, P, P, INT, I]
            getattr(_lib, "simd_1dvbc_mul_" + suf).argtypes = [I, I, I, P, P, P, P, P, P, P]
            getattr(_lib, "simd_trspmv_" + suf).argtypes = [I, I, P, P, P, P, P]
    return _lib


def _suf(dtype):
    return {np.dtype(np.float64): "f64", np.dtype(np.float32): "f32"}[np.dtype(dtype)]


def _p(a):
    return a.ctypes.data


def mul_t(B, x, y, nthreads=0, chunk=1):
    """mul!(y, B', x, true, false) for a SparseMatrix1DVBC mirror (val must carry the SIMD tail pad).
    chunk = stripes per atomic grab (1 = the reference's Atomic{Int} schedule, :169-177)."""
    assert x.dtype == B.val.dtype == y.dtype and len(B.val) >= B.ofs[-1] - 1 + 64 // B.val.dtype.itemsize
    st = getattr(lib(), "simd_1dvbc_mul_t_" + _suf(B.val.dtype))(
        B.m, B.n, len(B.Phi), _p(B.Phi.spl), _p(B.pos), _p(B.idx), _p(B.ofs), _p(B.val), _p(x), _p(y),
        int(nthreads), int(chunk))
    if st:
        raise RuntimeError(f"simd_1dvbc_mul_t: status {st}")
    return y


def mul(B, x, y):
    """mul!(y, B, x, true, false) (serial, multiply_1DVBC.jl:62-71)."""
    st = getattr(lib(), "simd_1dvbc_mul_" + _suf(B.val.dtype))(
        B.m, B.n, len(B.Phi), _p(B.Phi.spl), _p(B.pos), _p(B.idx), _p(B.ofs), _p(B.val), _p(x), _p(y))
    if st:
        raise RuntimeError(f"simd_1dvbc_mul: status {st}")
    return y


def trspmv(colptr, rowval, nzval, m, n, x, y):
    """TrSpMV!(y, A, x) on 1-based Int64 CSC fields (serial, TrSpMV.jl:1-20)."""
    st = getattr(lib(), "simd_trspmv_" + _suf(nzval.dtype))(m, n, _p(colptr), _p(rowval), _p(nzval), _p(x), _p(y))
    if st:
        raise RuntimeError(f"simd_trspmv: status {st}")
    return y


def isa():
    return {4: "avx512", 3: "avx2+fma", 0: "x86-64"}.get(lib().simd_isa(), "?")


def host_threads():
    """Cores this process may use: the affinity set, capped by OMP_NUM_THREADS when set (the GPU
    box sets it to the process's CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"
