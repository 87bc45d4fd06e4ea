"""Hazard check of the inline-asm DPP FMAs in the tile kernel (vbc_tiles.h fmac_bcast).

A VALU instruction that writes a VGPR followed within two wait states by a DPP instruction reading it is a
hazard the hardware does not interlock (the compiler inserts s_nop for its own DPP instructions, not for
inline asm).  The tile kernel's DPP sources are the values a vector-memory load wrote; this script reads
the gfx950 assembly of a build and fails if any `v_fmac_f32_dpp` reads a VGPR written by one of the two
preceding VALU instructions (s_nop N counts as N + 1 wait states).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Isparsematrixvbcs.jl_amd/csrc -c \\
        sparsematrixvbcs.jl_amd/csrc/vbc_tiles.hip -save-temps -o /tmp/t.o
    python tools/isa_check.py vbc_tiles-hip-amdgcn-amd-amdhsa-gfx950.s
"""
import re
import sys


def regs(op):
    """VGPR numbers named by one operand (v5, v[4:7])."""
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def check(path):
    bad, n = [], 0
    window = []  # recent (wait states, written VGPRs) of VALU instructions in this block
    for line in open(path):
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        if t.endswith(":"):  # a label: a new basic block (conservatively keep the window)
            continue
        op = t.split()[0]
        args = [a.strip() for a in t[len(op):].split(",")]
        if op == "s_nop":
            k = int(args[0], 0) + 1 if args and args[0] else 1
            window = [(w + k, r) for w, r in window]
            continue
        if op.startswith("v_fmac_f32_dpp"):
            n += 1
            src = regs(args[1].split()[0])
            for ws, wr in window:
                if ws < 2 and wr & src:
                    bad.append(t)
        if op.startswith("v_"):
            window = [(w + 1, r) for w, r in window if w + 1 < 2] + [(0, regs(args[0]) if args else set())]
        else:
            window = [(w + 1, r) for w, r in window if w + 1 < 2]
    return n, bad


if __name__ == "__main__":
    n, bad = check(sys.argv[1])
    print(f"{n} v_fmac_f32_dpp checked, {len(bad)} hazards")
    for b in bad[:20]:
        print("  HAZARD:", b)
    sys.exit(1 if bad or n == 0 else 0)
