"""Which OverlapChunker(ρ, W) rule reproduces the reference's recorded `overlap` memory column?

ChainPartitioners.jl 1.1.6 (the reference's partitioner, not in /root/reference and not fetchable) decides
OverlapChunker's stripes; src/ref.out only records the memory of the partition it produced
(bin/test_table.jl:66, memory = sizeof of the built SparseMatrix1DVBC, :78).  This tool runs the plausible
greedy rules -- a column j joins the open stripe (at most W columns) when its row set S_j overlaps

    first   the stripe's first column's S_f,
    union   the union U of the stripe's columns so far,
    prev    the previous column's S_{j-1},

by at least ρ of the max / min of the two set sizes, or (jaccard) |S_j ∩ T| >= ρ |S_j ∪ T| -- on the
stand-ins pinned to ref.out (synthetic.STANDINS, A = permutedims(A) as test_table.jl:27) and prints the
memory each gives against the recorded one.

    python tools/overlap_rules.py [--rho 0.9] [--matrices ct20stif,thermal1,3dtube,chesapeake]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

NAMES = {"ct20stif": "Boeing/ct20stif", "thermal1": "Schmid/thermal1", "3dtube": "Rothberg/3dtube",
         "chesapeake": "DIMACS10/chesapeake"}
# src/ref.out OverlapChunker(0.9, 8) memory (ct20stif :42, chesapeake :73, thermal1 :125, 3dtube :174)
REF_OVERLAP = {"ct20stif": 28093088, "chesapeake": 6160, "thermal1": 13472080, "3dtube": 51962512}
RULES = [(t, n) for t in ("first", "union", "prev") for n in ("max", "min", "jaccard")]


def overlap_split(A, rho, W, target, norm):
    """Greedy left-to-right stripes of the CSC A under one rule; returns the 1-based spl."""
    A = A.tocsc()
    A.sort_indices()
    cp, rv = A.indptr, A.indices
    n = A.shape[1]
    spl = [1]
    col = lambda j: rv[cp[j]:cp[j + 1]]
    first = prev = union = None
    width = 0
    for j in range(n):
        s = col(j)
        if width == 0:
            first = prev = union = s
            width = 1
            continue
        t = {"first": first, "union": union, "prev": prev}[target]
        inter = np.intersect1d(s, t, assume_unique=True).size
        if norm == "max":
            ok = inter >= rho * max(s.size, t.size)
        elif norm == "min":
            ok = inter >= rho * min(s.size, t.size)
        else:
            ok = inter >= rho * (s.size + t.size - inter)
        if ok and width < W:
            width += 1
            union = np.union1d(union, s)
            prev = s
        else:
            spl.append(j + 1)
            first = prev = union = s
            width = 1
    spl.append(n + 1)
    return np.array(spl, np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rho", type=float, default=0.9)
    ap.add_argument("--W", type=int, default=8)
    ap.add_argument("--matrices", default="ct20stif,thermal1,3dtube,chesapeake")
    args = ap.parse_args()
    import sparsematrixvbcs_amd as V
    for key in args.matrices.split(","):
        A = V.synthetic.standin(NAMES[key]).T.tocsc()
        print(f"{key}: ref.out overlap memory {REF_OVERLAP[key]}", flush=True)
        for target, norm in RULES:
            spl = overlap_split(A, args.rho, args.W, target, norm)
            B = V.SparseMatrix1DVBC[args.W](A, V.SplitPartition(spl))
            mem = V.io.memory_bytes(B)
            print(f"  {target:6s} {norm:8s} stripes {len(spl) - 1:7d}  memory {mem:10d}  ratio {mem / REF_OVERLAP[key]:.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
