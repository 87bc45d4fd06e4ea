"""The reference's benchmark table (bin/test_table.jl) on the GPU: one row per construction method.

    python tools/test_table.py [--matrix Boeing/ct20stif] [--dtype f64] [--fit-time-model] [--json out.json]

For each matrix (mdopen from $VBC_MATRIX_DIR, else the synthetic stand-in with the same n and nnz,
synthetic.STANDINS) it builds A = permutedims(A) (test_table.jl:27) and reports, per method:
setup time (host partition + layout build), memory (the reference's `mem` formula, Int64 indices),
the GPU time of mul!(y, B', x, true, false) (one HIP-graph replay of --reps products, median of 5), the CPU
time of the same product (the reference's SIMD kernel restated, all host cores, as its @threads loop), and the
normwise error
against scipy's A'x.  Row 'reference' is TrSpMV!(y, A, x) on the CSC matrix (test_table.jl:29-41).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def gpu_time(B, x, y, reps):
    import torch
    import sparsematrixvbcs_amd as V
    op = V.adjoint(B)
    for _ in range(3):
        V.mul_(y, op, x, True, False)
    torch.cuda.synchronize()
    try:  # as bench.py: `reps` products captured in one HIP graph, the replay span / reps (a solver's
        # back-to-back products; per-launch event pairs add their own gaps to a few-µs kernel)
        g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                V.mul_(y, op, x, True, False)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / reps)
        return float(np.median(ts)) * 1e-3
    except RuntimeError:  # capture refused: per-launch event pairs
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        V.mul_(y, op, x, True, False)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e-3


def cpu_time(R, x, n, reps=5, trsp=None, B=None):
    """CPU time of the same product: the reference's SIMD kernel (oracle/vbc_simd.c) for 1DVBC B'x on
    all host threads with the reference's one-stripe grabs (multiply_1DVBC.jl:169-177) and on 1 core,
    its serial TrSpMV! for the CSC row; the scalar oracle for 2D VBC (no SIMD port).  Returns
    (seconds all threads, threads, seconds 1 core, kind, seconds all threads with 64-stripe grabs or None)."""
    from oracle import oracle as O
    from oracle import simd as S
    th = S.host_threads()
    y = np.zeros(n, dtype=x.dtype)

    def med(f):
        f()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))
    if trsp is not None:
        cp = np.add(trsp.indptr, 1, dtype=np.int64)
        rv = np.add(trsp.indices, 1, dtype=np.int64)
        t1 = med(lambda: S.trspmv(cp, rv, trsp.data, trsp.shape[0], trsp.shape[1], x, y))
        return t1, 1, t1, "simd (serial, TrSpMV.jl)", None
    if B is not None and not hasattr(B, "Pi"):
        # the reference's schedule (one stripe per atomic grab) and the same kernel with 64-stripe grabs (the
        # atomic counter is contended by the one-stripe grabs of these small matrices)
        return (med(lambda: S.mul_t(B, x, y, th, 1)), th, med(lambda: S.mul_t(B, x, y, 1, 1)),
                "simd (multiply_1DVBC.jl:90-180)", med(lambda: S.mul_t(B, x, y, th, 64)))
    t = med(lambda: O.mul(R, x, y, trans=True, nthreads=th))
    return t, th, med(lambda: O.mul(R, x, y, trans=True, nthreads=1)), "scalar oracle", None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrix", default="Boeing/ct20stif")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--W", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--fit-time-model", action="store_true", help="add the 'min time' row (fits the GPU model)")
    ap.add_argument("--no-2d", action="store_true")
    ap.add_argument("--localities", default="uniform,banded", help="generators of the 1D time-model fit")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import torch
    import sparsematrixvbcs_amd as V
    from oracle import oracle as O

    dtype = np.float64 if args.dtype == "f64" else np.float32
    try:
        A = V.io.mdopen(args.matrix).A
        source = "SuiteSparse file"
    except FileNotFoundError:
        A = V.synthetic.standin(args.matrix)
        source = "synthetic stand-in (synthetic.STANDINS / STANDIN_MODEL: same n, nnz; calibrated to src/ref.out)"
    A = A.T.tocsc().astype(dtype)  # permutedims(sparse(mdopen(mtx).A)), test_table.jl:27
    A.sort_indices()
    m, n = A.shape
    rng = np.random.default_rng(0xC0FFEE)
    xh = rng.random(m).astype(dtype)
    ref = (A.T @ xh.astype(np.float64))
    x = torch.from_numpy(xh).cuda()
    y = torch.empty(n, dtype=x.dtype, device="cuda")
    W = args.W
    lim = lambda mdl: V.ConstrainedCost(mdl, V.VertexCount(), W)
    rows = []

    def record(name, setup, mem, B=None, R=None, trsp=None, model_us=None):
        t_gpu = gpu_time(B, x, y, args.reps)
        err = float(np.linalg.norm(y.cpu().numpy().astype(np.float64) - ref) / np.linalg.norm(ref))
        t_cpu, th, t_cpu1, kind, t_cpu64 = cpu_time(R, xh, n, trsp=trsp, B=B)
        bytes_ = B.info()["bytes_t"] if hasattr(B, "info") else None
        row = dict(method=name, setup_s=round(setup, 4), memory=int(mem), gpu_us=round(t_gpu * 1e6, 2),
                   cpu_us=round(t_cpu * 1e6, 1), cpu_threads=th, cpu_1core_us=round(t_cpu1 * 1e6, 1), cpu_kind=kind,
                   cpu_chunk64_us=round(t_cpu64 * 1e6, 1) if t_cpu64 is not None else None,
                   speedup=round(t_cpu / t_gpu, 1),
                   gpu_GBs=round(bytes_ / t_gpu / 1e9, 1) if bytes_ else None, rel_err=err, model_us=model_us)
        if hasattr(B, "Phi"):
            wd = np.diff(B.Phi.spl)
            row["widths"] = {int(k): int(v) for k, v in zip(*np.unique(wd, return_counts=True))}
            if hasattr(B, "Pi"):
                ud = np.diff(B.Pi.spl)
                row["heights"] = {int(k): int(v) for k, v in zip(*np.unique(ud, return_counts=True))}
        rows.append(row)
        print(f"{name:22s} setup {setup:8.3f}s  mem {mem:12d}  gpu {t_gpu * 1e6:9.2f} us  cpu {t_cpu * 1e6:10.1f} us"
              f"  x{t_cpu / t_gpu:7.1f}  err {err:.1e}", flush=True)
        if hasattr(B, "release"):
            B.release()

    # reference row: TrSpMV!(y, A, x) on the CSC matrix
    C = V.SparseMatrixCSC(A)
    mem_csc = 8 * (len(A.indptr) + len(A.indices)) + A.data.nbytes
    record("reference (TrSpMV!)", 0.0, mem_csc, C, trsp=A)

    methods = [("strict", V.StrictChunker(W)), ("overlap", V.OverlapChunker(0.9, W)),
               ("min blocks", V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks()))),
               ("min memory", V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_memory(dtype, np.int64))))]
    if args.fit_time_model:  # the reference's generator (uniform rows) and the banded one (costs.py)
        for loc in args.localities.split(","):
            mdl = V.model_SparseMatrix1DVBC_TrSpMV_time(W, dtype, np.int64, dtype, locality=loc)
            methods.append((f"min time (GPU, {loc})", V.DynamicTotalChunker(lim(mdl))))
        # the candidates above and the two model partitions, timed on the GPU: the fastest wins
        methods.append(("min time (GPU, timed)", V.TimedChunker([mt for _, mt in methods], W, dtype)))
    for name, method in methods:
        t0 = time.perf_counter()
        B = V.SparseMatrix1DVBC[W](A, method)
        setup = time.perf_counter() - t0
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
        record(name, setup, V.io.memory_bytes(B), B, R)
    if not args.no_2d:
        b2, m2 = V.model_SparseMatrixVBC_blocks(), V.model_SparseMatrixVBC_memory(dtype, np.int64)
        methods2 = [
                ("1D 2D", V.AlternatingPacker(V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks())), V.EquiChunker(1))),
                ("strict 2D", V.AlternatingPacker(V.StrictChunker(W), V.StrictChunker(W))),
                ("overlap 2D 0.9", V.AlternatingPacker(V.OverlapChunker(0.9, W), V.OverlapChunker(0.9, W))),
                ("overlap 2D 0.8", V.AlternatingPacker(V.OverlapChunker(0.8, W), V.OverlapChunker(0.8, W))),
                ("overlap 2D 0.7", V.AlternatingPacker(V.OverlapChunker(0.7, W), V.OverlapChunker(0.7, W))),
                # test_table.jl:94-111: the 2D block cost models, alternated over columns and rows
                ("dynamic blocks 2D", V.AlternatingPacker(V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks())),
                                                          V.DynamicTotalChunker(lim(V.permutedims(b2))),
                                                          V.DynamicTotalChunker(lim(b2)))),
                ("dynamic memory 2D", V.AlternatingPacker(V.EquiChunker(1), V.EquiChunker(1),
                                                          V.DynamicTotalChunker(lim(m2)),
                                                          V.DynamicTotalChunker(lim(V.permutedims(m2))),
                                                          V.DynamicTotalChunker(lim(m2))))]
        t2 = None
        if args.fit_time_model:  # costs.jl:142 with R = 3 (test_table.jl:56), fitted on this GPU
            t2 = V.model_SparseMatrixVBC_TrSpMV_time(3, W, W, dtype, np.int64, dtype)
            methods2.append(("dynamic time 2D", V.AlternatingPacker(V.EquiChunker(1), V.EquiChunker(1),
                                                                    V.DynamicTotalChunker(lim(t2)),
                                                                    V.DynamicTotalChunker(lim(V.permutedims(t2))),
                                                                    V.DynamicTotalChunker(lim(t2)))))
        for name, method in methods2:
            t0 = time.perf_counter()
            B = V.SparseMatrixVBC[W, W](A, method)
            setup = time.perf_counter() - t0
            R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
            model = round(V.total_value_2d(B, t2) * 1e6, 2) if t2 is not None else None  # test_table.jl:124, us
            record(name, setup, V.io.memory_bytes(B), B, R, model_us=model)
    out = dict(matrix=args.matrix, source=source, m=m, n=n, nnz=int(A.nnz), dtype=args.dtype, W=W,
               device=torch.cuda.get_device_name(0), rows=rows)
    if args.json:
        Path(args.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
