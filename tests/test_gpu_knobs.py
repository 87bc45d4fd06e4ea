"""No environment variable turns the product library into an ablation variant (What's weak 1).

Every former ablation variable (and the tuning constants the product library no longer reads) is set to
every value it used to accept; the FE-2D, the ldoor stand-in and the NS (row-swept) matrices at small scale
and the structured C5 input (c5-mesh) are built afresh and multiplied in both directions.  The products
must be bit-identical to the same matrices built with a clean environment, and the clean products must
match the oracle: bitwise where the layout keeps the reference's serial order (B.serial, vbc.h
VBC_CREATE_SERIAL), else within the split layouts' stated rounding (fp64 normwise 1e-14); c5-mesh on
integer data is bitwise on all 16 columns.  The reference's results depend only on its type parameters
and the partition (multiply_1DVBC.jl:9-13, SparseMatrixVBCs.jl:17); so do these.
"""
import os

import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
DEV = "cuda:0"

FORMER = {  # variable -> the values it used to accept (round 5's libvbc.so)
    "VBC_DIAG": ["1", "2", "3", "4"],
    "VBC_SWEEP_DIAG": ["1", "2"],
    "VBC_TILE_DIAG": ["1", "2", "4", "8", "15"],
    "VBC_PANEL_DIAG": ["2", "4", "8", "16", "30"],
    "VBC_PANEL_VALU": ["1"],
    "VBC_NO_AFFINE": ["1"],
    "VBC_NO_FASTE": ["1"],
    # tuning constants the product keeps at their defaults (read by the VBC_ABLATION build only)
    "VBC_TARGET_RANGES": ["1", "7"],
    "VBC_TILE_SPR": ["1"],
    "VBC_TILE_K": ["4"],
    "VBC_TILE_NBT": ["4"],
    "VBC_TILE_DEPTH": ["3"],
    "VBC_PIPE": ["3"],
    "VBC_PAD": ["3:4"],
}


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    d = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (d if d else 1.0)


def build(name):
    import bench
    if name == "fe":
        B = bench.build_matrix("fe", np.float64, 0.002)
    elif name == "ldoor":
        B = bench.build_matrix("ldoor", np.float64, 0.01)
    elif name == "ns":
        B = V.synthetic.north_star(dtype=np.float64, scale=0.003)
    else:
        B = bench.build_matrix("c5-mesh", np.float32, 0.002)
        B.val[:] = np.random.default_rng(3).integers(-8, 9, B.val.shape)
    return B


def products(B, name):
    """y of B'x and B·x (vectors, or 16 row-major right-hand sides for c5-mesh), on fresh handles."""
    B.release()
    rng = np.random.default_rng(17)
    out = []
    for trans in (True, False):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        if name == "c5-mesh":
            X = rng.integers(-8, 9, (nx, 16)).astype(np.float32)
            Y = torch.full((ny, 16), float("nan"), dtype=torch.float32, device=DEV)
        else:
            X = rng.uniform(-1, 1, nx)
            Y = torch.full((ny,), float("nan"), dtype=torch.float64, device=DEV)
        V.mul_(Y, B.T if trans else B, torch.from_numpy(X).to(DEV))
        out.append((X, Y.cpu().numpy()))
    B.release()
    return out


@pytest.fixture(scope="module")
def clean():
    for k in FORMER:
        os.environ.pop(k, None)
    mats = {n: build(n) for n in ("fe", "ldoor", "ns", "c5-mesh")}
    return mats, {n: products(B, n) for n, B in mats.items()}


def test_clean_products_match_oracle(clean):
    mats, ys = clean
    for name, B in mats.items():
        for trans, (X, y) in zip((True, False), ys[name]):
            if name == "c5-mesh":
                Rd = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val.astype(np.float64))
                ny = B.n if trans else B.m
                want = np.stack([O.mul(Rd, np.ascontiguousarray(X[:, j], dtype=np.float64), np.zeros(ny), trans=trans)
                                 for j in range(16)], axis=1)
                assert np.array_equal(y, want.astype(np.float32)), (name, trans)
            else:
                R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
                ref = O.mul(R, X, np.zeros(len(y)), trans=trans)
                assert rel(y, ref) <= 1e-14, (name, trans)
    # the serial order: bitwise against the oracle, both directions (FE, ldoor)
    for name in ("fe", "ldoor"):
        B = mats[name]
        B.serial = True
        try:
            for trans, (X, _) in zip((True, False), ys[name]):
                ny = B.n if trans else B.m
                y = torch.full((ny,), float("nan"), dtype=torch.float64, device=DEV)
                V.mul_(y, B.T if trans else B, torch.from_numpy(X).to(DEV))
                R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
                assert np.array_equal(y.cpu().numpy(), O.mul(R, X, np.zeros(ny), trans=trans)), (name, trans)
        finally:
            B.serial = False
            B.release()


@pytest.mark.parametrize("var", sorted(FORMER))
def test_former_ablation_variable_changes_nothing(var, clean, monkeypatch):
    mats, ys = clean
    for val in FORMER[var]:
        monkeypatch.setenv(var, val)
        for name, B in mats.items():
            got = products(B, name)
            for (_, y0), (_, y1) in zip(ys[name], got):
                assert np.array_equal(y0, y1, equal_nan=True), (var, val, name)
        monkeypatch.delenv(var)
