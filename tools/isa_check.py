"""Hazard check of the inline-asm DPP FMAs in the tile kernel (vbc_tiles.h fmac_bcast).

A VALU instruction that writes a VGPR followed within two wait states by a DPP instruction reading it is a
hazard the hardware does not interlock (the compiler inserts s_nop for its own DPP instructions, not for
inline asm).  The tile kernel's DPP sources are the values a vector-memory load wrote; this script reads
the gfx950 code of a build and fails if any `v_fmac_f32_dpp` reads a VGPR written by one of the VALU
instructions within two wait states before it on ANY path: the linear predecessor and every branch that
jumps to it (a loop back-edge included; the branch itself is not counted as a wait state, s_nop N counts
N + 1).  It also fails when the code holds no such instruction (the check would be vacuous).

The Makefile runs it on every build of the tile kernel (`make` fails on a hazard):

    python tools/isa_check.py sparsematrixvbcs.jl_amd/build/vbc_tiles.o      # a hipcc -c object
    python tools/isa_check.py vbc_tiles-hip-amdgcn-amd-amdhsa-gfx950.s      # or -save-temps assembly
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def regs(op):
    """VGPR numbers named by one operand (v5, v[4:7])."""
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def disassemble(obj):
    """gfx950 disassembly of a hipcc -c object (its .hip_fatbin offload bundle)."""
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fatbin"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "junk.o")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={fb}",
                        f"--output={co}", "--unbundle"], check=True)
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                             text=True).stdout
    return out.splitlines()


def parse(lines):
    """(address or None, opcode, args) per instruction; None entries mark labels / function starts."""
    ins = []
    for line in lines:
        t = line.strip()
        addr = None
        if "//" in t:
            t, c = t.split("//", 1)
            t = t.strip()
            m = re.match(r"\s*([0-9A-Fa-f]+):", c)
            if m:
                addr = int(m.group(1), 16)
        if not t or t.startswith((";", ".")):
            continue
        if t.endswith(":"):  # a label or a function start: a new block (window restarts for functions)
            ins.append((None, t, []))
            continue
        op = t.split()[0]
        args = [a.strip() for a in t[len(op):].split(",")]
        ins.append((addr, op, args))
    return ins


def branch_target(addr, op, args):
    """Target address of an s_branch / s_cbranch_* with a numeric simm16 (objdump form)."""
    if addr is None or not (op == "s_branch" or op.startswith("s_cbranch_")) or not args or not args[0]:
        return None
    tok = args[0].split()[0]
    try:
        k = int(tok, 0)
    except ValueError:
        return None
    if k >= 0x8000:
        k -= 0x10000
    return addr + 4 + 4 * k


def check_lines(lines):
    ins = parse(lines)
    # pass 1: the window (written VGPRs of the VALU instructions < 2 wait states back) at every branch, by target
    incoming = {}

    def walk(record):
        bad, n = [], 0
        window = []  # (wait states since, written VGPRs)
        for addr, op, args in ins:
            if addr is None:
                if op.startswith("<") or re.match(r"[0-9A-Fa-f]+ <", op):
                    window = []  # function start
                continue
            if not record and addr in incoming:
                window = window + incoming[addr]
            tgt = branch_target(addr, op, args)
            if record and tgt is not None:
                incoming.setdefault(tgt, []).extend(window)
            if op == "s_nop":
                k = int(args[0].split()[0], 0) + 1 if args and args[0] else 1
                window = [(w + k, r) for w, r in window if w + k < 2]
                continue
            if op.startswith("v_fmac_f32_dpp"):
                n += 1
                src = regs(args[1].split()[0])
                if any(ws < 2 and wr & src for ws, wr in window):
                    bad.append(f"{addr:#x}: {op} {', '.join(args)}")
            if op.startswith("s_branch") or op.startswith("s_cbranch_"):
                continue  # (not counted as a wait state: conservative)
            if op.startswith("v_"):
                window = [(w + 1, r) for w, r in window if w + 1 < 2] + [(0, regs(args[0]) if args else set())]
            else:
                window = [(w + 1, r) for w, r in window if w + 1 < 2]
        return n, bad

    walk(True)
    return walk(False)


def check(path):
    if path.endswith(".o"):
        return check_lines(disassemble(path))
    with open(path) as f:
        return check_lines(f.read().splitlines())


if __name__ == "__main__":
    n, bad = check(sys.argv[1])
    print(f"isa_check: {n} v_fmac_f32_dpp checked, {len(bad)} hazards")
    for b in bad[:20]:
        print("  HAZARD:", b)
    sys.exit(1 if bad or n == 0 else 0)
