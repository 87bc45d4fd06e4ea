"""The shipping libvbc.so cannot run an ablation variant, and every environment knob it reads is documented.

The reference's results depend only on its type parameters and the partition (multiply_1DVBC.jl:9-13,
SparseMatrixVBCs.jl:17).  libvbc's ablation variants (kernels with part of their work removed: x taken as 1,
gathers confined to a few lines, stores dropped) exist only in the -DVBC_ABLATION build (`make ablation`,
tools/exp/libs/libvbc_ablation.so); the product library neither reads their environment variables nor
instantiates their kernels.  The layout knobs it does read each select a layout the
-m gpu parity tests hold to the oracle (tests/test_gpu_knobs.py sets every former ablation variable too).
No GPU is needed here: the library's strings, its kernel symbols and the sources are inspected.
"""
import re
import shutil
import subprocess
import sys

import pytest

from sparsematrixvbcs_amd import _lib as L
from tests.conftest import ROOT

CSRC = ROOT / "sparsematrixvbcs.jl_amd" / "csrc"
ABLATION_KNOBS = ("VBC_DIAG", "VBC_SWEEP_DIAG", "VBC_TILE_DIAG", "VBC_PANEL_DIAG", "VBC_PANEL_VALU",
                  "VBC_NO_AFFINE", "VBC_NO_FASTE")
# kernel template -> 0-based position of its DIAG (ablation) template argument
DIAG_ARG = {"spmv_planar_lanes": 5, "spmv_planar_split": 5, "spmv_sweep": 3, "spmv_slots": 4, "spmv_ranges": 4}
REMOVED_KERNELS = ("spmm_quads", "spmm_tiles4", "spmm_tiles_x", "spmm_tiles_xp")


def lib_strings():
    blob = L.LIB_PATH.read_bytes()
    return set(s.decode() for s in re.findall(rb"[\x20-\x7e]{6,}", blob))


def test_no_ablation_knob_in_product_library():
    strs = lib_strings()
    found = {k for k in ABLATION_KNOBS if any(re.search(rf"\b{k}\b", s) for s in strs)}
    assert not found, found


def kernels():
    cxxfilt = shutil.which("c++filt")
    if cxxfilt is None:
        pytest.skip("c++filt unavailable")
    names = sorted(s for s in lib_strings() if s.startswith("_ZN3vbc"))
    out = subprocess.run([cxxfilt], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    ks = set()
    for d in out.splitlines():
        m = re.match(r"(?:void )?vbc::(sp\w+)<(.*)>\(", d)
        if m:
            ks.add((m.group(1), tuple(a.strip() for a in m.group(2).split(","))))
    return ks


def test_no_ablation_kernel_instantiated():
    ks = kernels()
    assert len(ks) > 500  # (every product kernel family is there)
    families = {k for k, _ in ks}
    assert {"spmv_slots", "spmv_planar", "spmv_planar_lanes", "spmv_sweep", "spmm_panel", "spmm_tiles"} <= families
    assert not families & set(REMOVED_KERNELS), families & set(REMOVED_KERNELS)
    bad = [(k, a) for k, a in ks if k in DIAG_ARG and len(a) > DIAG_ARG[k] and a[DIAG_ARG[k]] != "0"]
    assert not bad, bad[:5]


def knob_names(fn):
    names = set()
    for p in CSRC.iterdir():
        if p.suffix in (".hip", ".cpp", ".h", ".inc"):
            names |= set(re.findall(rf'{fn}\("(VBC_\w+)"\)', p.read_text()))
    return names


def test_every_knob_is_documented_and_no_raw_getenv():
    layout, ablation = knob_names("layout_knob"), knob_names("ablation_knob")
    assert set(ablation) <= set(ABLATION_KNOBS), ablation - set(ABLATION_KNOBS)
    assert not layout & ablation
    text = (ROOT / "INTEGRATION.md").read_text()
    sec = text[text.index("## 6."):]
    missing = sorted(k for k in layout | ablation if k not in sec)
    assert not missing, missing
    # the only raw getenv outside vbc_internal.h is the host builders' thread count
    raw = []
    for p in CSRC.iterdir():
        if p.name != "vbc_internal.h" and p.suffix in (".hip", ".cpp", ".h", ".inc"):
            raw += [f"{p.name}: {m}" for m in re.findall(r'getenv\("(\w+)"\)', p.read_text())]
    assert raw == ["vbc_host.cpp: VBC_HOST_THREADS"], raw
    assert len(layout) <= 60, len(layout)


def test_isa_check_sees_back_edge_hazards():
    """tools/isa_check.py (run by the Makefile on every build of the tile kernel): a VALU write of a DPP FMA's
    source reaches it through a loop back-edge -- flagged; with two wait states between -- clean."""
    sys.path.insert(0, str(ROOT / "tools"))
    import isa_check

    def prog(nops):
        return [
            "0000000000001000 <_ZN3vbc4testEv>:",
            "\tv_mov_b32 v3, v1 // 000000001000: 00000000",
            "\tv_fmac_f32_dpp v5, v2, v4 row_newbcast:1 row_mask:0xf bank_mask:0xf // 000000001004: 0",
            "\ts_nop 0 // 000000001008: 0",
            "\tv_mov_b32 v2, v7 // 00000000100C: 0",
        ] + ["\ts_nop 0 // 000000001010: 0"] * nops + [
            f"\ts_cbranch_scc1 {0x10000 - (4 + nops)} // 0000000010{(0x10 + 4 * nops):02X}: 0",
            "\ts_endpgm // 000000001100: 0",
        ]
    # the branch at 0x1010 + 4 nops jumps back to 0x1004 (the DPP FMA): v2 written just before the branch
    n, bad = isa_check.check_lines(prog(0))
    assert n == 1 and len(bad) == 1
    n, bad = isa_check.check_lines(prog(2))
    assert n == 1 and not bad


def test_isa_check_on_built_tile_kernel():
    obj = ROOT / "sparsematrixvbcs.jl_amd" / "build" / "vbc_tiles.o"
    if not obj.exists() or not shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("no in-tree build of vbc_tiles.o")
    sys.path.insert(0, str(ROOT / "tools"))
    import isa_check
    n, bad = isa_check.check(str(obj))
    assert n > 0 and not bad, bad[:5]
