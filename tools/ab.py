"""Interleaved in-process A/B timing of libvbc layout variants (env knobs read at handle creation).

    python tools/ab.py --workload fe --variants "VBC_TILE_K=4;VBC_TILE_K=8" [--rounds 5 --reps 20]
Each variant is a separate handle over the same matrix and vectors; rounds interleave the variants
(MI355X guide §5.4 rule 24) and the median / min per-launch time is reported with the GB/s figure
of bench.py's byte formula.  Also checks every variant's y against the first (bitwise/relative).
"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fe", help="fe | fe3d | ns | ns-mixed | c5 | ct20stif | ldoor | ldoor-csc")
    ap.add_argument("--variants", default="VBC_TILE_K=4;VBC_TILE_K=8")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--trans", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--nrhs", type=int, default=0, help=">0: time the multi-RHS product (row-major X / Y)")
    ap.add_argument("--shard", default="", help="R/N: time stripe shard R of the N-way split (distributed.stripe_split)")
    ap.add_argument("--method", default="", help="ct20stif / ldoor / 3dtube / thermal1: build the stand-in with this "
                    "bin/test_table.jl method instead of StrictChunker(8): overlap | blocks | memory | overlap2d07 | blocks2d")
    ap.add_argument("--graph", action="store_true",
                    help="time each variant as one HIP-graph replay of --reps products (span / reps), as bench.py "
                         "does: per-launch event brackets inflate small kernels")
    ap.add_argument("--copies", type=int, default=1,
                    help="build every variant this many times (A B .. A B ..): placement effects show as spread")
    ap.add_argument("--fresh", action="store_true",
                    help="run every variant as its own bench.py process (fresh allocation and placement), "
                         "--rounds rounds interleaved A B .. A B ..: the bench's own harness, required for a "
                         "default change under 3 %% (VERDICT r5)")
    args = ap.parse_args()
    if args.fresh:
        return fresh(args)
    import torch

    import bench
    import sparsematrixvbcs_amd as V
    from sparsematrixvbcs_amd import _lib as L

    dtype = np.float64 if args.dtype == "f64" else np.float32
    if args.workload == "ldoor-csc":
        B = V.SparseMatrixCSC(V.synthetic.standin("GHS_psdef/ldoor").T.tocsc().astype(dtype))
    elif args.method or args.workload in ("3dtube", "thermal1", "chesapeake"):
        names = {"ct20stif": "Boeing/ct20stif", "ldoor": "GHS_psdef/ldoor", "3dtube": "Rothberg/3dtube",
                 "thermal1": "Schmid/thermal1", "chesapeake": "DIMACS10/chesapeake"}
        A = V.synthetic.standin(names[args.workload], dtype=dtype).T.tocsc()
        lim = lambda mdl: V.ConstrainedCost(mdl, V.VertexCount(), 8)
        meth = {"": V.StrictChunker(8), "strict": V.StrictChunker(8), "overlap": V.OverlapChunker(0.9, 8),
                "blocks": V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks())),
                "memory": V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_memory(dtype, np.int64)))}
        if args.method == "blocks2d":  # bin/test_table.jl 'dynamic blocks 2D'
            b2 = V.model_SparseMatrixVBC_blocks()
            B = V.SparseMatrixVBC[8, 8](A, V.AlternatingPacker(V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks())),
                                                               V.DynamicTotalChunker(lim(V.permutedims(b2))),
                                                               V.DynamicTotalChunker(lim(b2))))
        elif args.method == "overlap2d07":
            B = V.SparseMatrixVBC[8, 8](A, V.AlternatingPacker(V.OverlapChunker(0.7, 8), V.OverlapChunker(0.7, 8)))
        else:
            B = V.SparseMatrix1DVBC[8](A, meth[args.method])
    else:  # fe | fe3d | ns | ns-mixed | c5 | ldoor | ct20stif: the bench's own matrices
        B = bench.build_matrix(args.workload, dtype, args.scale)
        if args.shard:
            r, n = (int(t) for t in args.shard.split("/"))
            cuts = V.distributed.stripe_split(B, n)
            B, _ = V.distributed.shard(B, int(cuts[r]), int(cuts[r + 1]))
    esz = np.dtype(dtype).itemsize
    trans = bool(args.trans)
    nx, ny = (B.m, B.n) if trans else (B.n, B.m)
    k = max(args.nrhs, 1)
    nbytes = (B.info(0, trans)["bytes_t" if trans else "bytes_f"] if args.workload == "ldoor-csc" else
              bench.algorithmic_bytes(B, esz) + (k - 1) * esz * (B.m + B.n)) if args.workload not in ("c5",) else \
        (len(B.val) * esz + 4 * len(B.idx) + (k * esz) * (B.m + B.n))
    x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, (nx, k) if args.nrhs else nx).astype(dtype)).cuda()
    variants = [v for v in args.variants.split(";")] * max(1, args.copies)
    handles, libs = [], []
    main_lib = L.lib()
    for v in variants:
        # "@lib=path": this variant runs another build of libvbc (compile-time variants, same process)
        lp = [t.split("=", 1)[1] for t in v.split(",") if t.strip().startswith("@lib=")]
        if lp:
            saved_path, saved_lib = L.LIB_PATH, L._lib
            L.LIB_PATH, L._lib = Path(lp[0]).resolve(), None
            vlib = L.lib()
            L.LIB_PATH = saved_path
        else:
            vlib, saved_lib = main_lib, main_lib
        L._lib = vlib
        libs.append(vlib)
        saved = dict(os.environ)
        for kv in v.split(","):
            if "=" in kv and not kv.strip().startswith("@"):
                ek, ev_ = kv.split("=", 1)
                os.environ[ek.strip()] = ev_.strip()
        hp = C.c_void_p()
        flags = L.VBC_CREATE_TRANSPOSED if trans else L.VBC_CREATE_FORWARD
        if "@multifwd" in v:  # multi-RHS forward product (panel / tile layout of B')
            flags = L.VBC_CREATE_MULTI_FORWARD
        elif "@multi" in v:  # matrix-core panel layout (multi-RHS transposed product)
            flags = L.VBC_CREATE_MULTI
        L.check(B._create(C.byref(hp), 0, flags, L.compute_code(B.val.dtype)), "create")
        os.environ.clear()
        os.environ.update(saved)
        handles.append(hp)
        L._lib = main_lib
    ys = [torch.empty((ny, k) if args.nrhs else ny, dtype=x.dtype, device="cuda") for _ in variants]
    stream = torch.cuda.current_stream()
    def run(i):
        lib = libs[i]
        if args.nrhs:
            L.check(lib.vbc_mul_mat(handles[i], int(trans), k, x.data_ptr(), k, nx, ys[i].data_ptr(), k, ny,
                                    1.0, 0.0, L.VBC_MEM_DEVICE, stream.cuda_stream, L.VBC_MAT_ROWMAJOR), "mul_mat")
        else:
            L.check(lib.vbc_mul(handles[i], int(trans), x.data_ptr(), nx, ys[i].data_ptr(), ny, 1.0, 0.0,
                                L.VBC_MEM_DEVICE, stream.cuda_stream, 0), "mul")

    for i in range(len(variants)):
        for _ in range(3):
            run(i)
    torch.cuda.synchronize()
    times = {i: [] for i in range(len(variants))}
    graphs = []
    if args.graph:
        gs = torch.cuda.Stream()
        for i in range(len(variants)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gs):
                stream = torch.cuda.current_stream()
                for _ in range(args.reps):
                    run(i)
            graphs.append(g)
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
    for _ in range(args.rounds):
        for i in range(len(variants)):
            if args.graph:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                graphs[i].replay()
                b.record(stream)
                torch.cuda.synchronize()
                times[i].append(a.elapsed_time(b) / args.reps)
                continue
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            for a, b in ev:
                a.record(stream)
                run(i)
                b.record(stream)
            torch.cuda.synchronize()
            times[i] += [a.elapsed_time(b) for a, b in ev]
    ref = ys[0].double()
    for i, v in enumerate(variants):
        t = np.array(times[i])
        d = (ys[i].double() - ref).norm().item() / max(ref.norm().item(), 1e-300)
        flops = 2.0 * len(B.val) * k / (np.median(t) * 1e-3) / 1e12
        print(f"{v:40s} {flops:6.2f} TFLOP/s median {np.median(t)*1e3:8.1f} us  min {t.min()*1e3:8.1f} us  "
              f"{nbytes / (np.median(t) * 1e-3) / 1e9:7.0f} GB/s  rel-diff-vs-first {d:.2e}", flush=True)
    for i, hp in enumerate(handles):
        libs[i].vbc_destroy(hp)


def fresh(args):
    """Each variant in a fresh `python bench.py --workload W` process (its env knobs set, "@lib=path" ->
    VBC_LIBRARY), rounds interleaved; reports the median and spread of the line's avg_launch_ms (events
    around the graph-replayed products) and ms_per_step (wall), and the line's parity."""
    import json
    import subprocess
    wl = args.workload + ("" if args.trans else "-fwd")
    variants = [v for v in args.variants.split(";")]
    res = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            env = dict(os.environ)
            for kv in v.split(","):
                kv = kv.strip()
                if kv.startswith("@lib="):
                    env["VBC_LIBRARY"] = str(Path(kv[5:]).resolve())
                elif "=" in kv and not kv.startswith("@"):
                    k, val = kv.split("=", 1)
                    env[k.strip()] = val.strip()
            cmd = [sys.executable, str(ROOT / "bench.py"), "--workload", wl, "--dtype", args.dtype, "--steps",
                   str(args.reps), "--no-cpu-baseline", "--no-secondary", "--scale", str(args.scale)]
            if args.nrhs:
                cmd += ["--nrhs", str(args.nrhs)]
            r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode or not line:
                print(f"{v}: failed ({r.returncode}): {r.stderr[-800:]}", flush=True)
                return 1
            d = json.loads(line[-1])
            res[v].append((d["roofline"]["avg_launch_ms"] * 1e3, d["ms_per_step"] * 1e3,
                           (d.get("parity") or {}).get("rel_err")))
            print(f"  {v:40s} {res[v][-1][0]:8.2f} us (events)  {res[v][-1][1]:8.2f} us (wall)  rel_err {res[v][-1][2]}",
                  flush=True)
    print("fresh-process A/B (bench.py per variant, rounds interleaved):")
    for v in variants:
        ev = np.array([t[0] for t in res[v]])
        wall = np.array([t[1] for t in res[v]])
        print(f"{v:40s} events median {np.median(ev):8.2f} us [{ev.min():.2f}, {ev.max():.2f}]  wall median "
              f"{np.median(wall):8.2f} us", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
