"""Benchmark: 1DVBC SpMV effective GB/s (and GFLOP/s) vs the MI355X HBM roofline (BASELINE.json).

A step is one mul!(y, B', x) -- the transposed 1D-VBR product the reference's paper and benchmark
time (bin/test_table.jl:80) -- fp64, inputs resident in HBM.  Primary workload (BASELINE.json
target: "10M x 10M, ~1e8-nnz SuiteSparse-like matrix"): `fe`, a 2D finite-element operator
(5-point stencil, 2 unknowns per node, 1.0e7 x 1.0e7, 1.0e8 stored values) in 1DVBC form.

N = 1 (plain `python bench.py`): the primary line carries `roofline` (HIP events on the launching
stream + the committed rocprofv3 / PMC summaries), `cpu_baseline` (the reference's SIMD CPU kernel,
oracle/vbc_simd.c, on the host cores) and `parity` (the GPU y of the timed region against the CPU
oracle, oracle/vbc_oracle.c, on the same full-size input).  Secondaries in the same line:
`fe3d` (irregular 3D stiffness stand-in, 1e7 rows / 1e8 nnz), `ns` (SURVEY §8d's uniform-random
NS-1DVBC from the reference's own generator, costs.jl:63-83) and `c5` (2D VBC, 16 RHS, matrix cores).

N > 1 (torchrun, one process per GPU): STRONG scaling of ONE matrix.  Every rank builds the same
matrix, keeps its byte-balanced stripe range (distributed.ShardedSparseMatrix1DVBC, the GPU grid
replacing the reference's threaded stripe loop multiply_1DVBC.jl:169-177) and times K products of
its shard; `value` = algorithmic bytes of the WHOLE matrix / the slowest rank's time.  B'x writes
disjoint y slices, so the primary needs no collective; `e2e` adds the all_gather that replicates y
(RCCL over xGMI), and the C3 secondary (ldoor stand-in) reports the same plus the forward product
with its RCCL all_reduce of y.

    python bench.py [--gpus N --steps K --warmup W --workload fe|fe3d|ns|ns-mixed|c5|ldoor|ct20stif
                     --dtype f64|f32]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
MALL_BYTES = 256 << 20  # MI355X Infinity Cache (MALL)
METRIC = "1DVBC SpMV effective GB/s (and GFLOP/s) vs HBM roofline, 1/2/4/8 GPU"
PARITY_TOL = {np.dtype(np.float64): 1e-10, np.dtype(np.float32): 1e-5}  # normwise rel-err (BASELINE)

WORKLOADS = {"ns": "NS-1DVBC-10Mx10M-1e8nnz-w4-uniform",
             "ns-mixed": "NS-1DVBC-mixed-w1..8-1e8nnz-uniform",
             "fe": "FE-2D-5pt-dof2-10Mx10M-1e8nnz-w2 (SuiteSparse-like mesh operator)",
             "fe3d": "FE-3D-stiffness-dof3-1e7x1e7-1e8nnz-w3 (irregular: random 18-neighbour subsets)",
             "c5": "C5-VBC2D-8x8-tiles-2Mx2M-1e8nnz-16RHS (costs.jl:200-220 generator)",
             "c5-fwd": "C5-VBC2D-8x8-tiles-2Mx2M-1e8nnz-16RHS forward Y = B*X (costs.jl:200-220 generator)",
             "c5-mesh": "C5-VBC2D-3x3-node-tiles-2Mx2M-1e8nnz-16RHS (structured: 3D stiffness stand-in, "
                        "AlternatingPacker(StrictChunker(8), StrictChunker(8)) tiles)",
             "c5-mesh-fwd": "C5-VBC2D-3x3-node-tiles-2Mx2M-1e8nnz-16RHS forward Y = B*X (structured 3D stiffness "
                            "stand-in)",
             "fe-fwd": "FE-2D-5pt-dof2-10Mx10M-1e8nnz-w2 (SuiteSparse-like mesh operator), forward y = B*x",
             "fe3d-fwd": "FE-3D-stiffness-dof3-1e7x1e7-1e8nnz-w3 (irregular: random 18-neighbour subsets), forward y = B*x",
             "ldoor": "C3/C4 GHS_psdef/ldoor stand-in 952203^2 42.5M nnz, StrictChunker(8) -> w=3",
             "ldoor-fwd": "C3 GHS_psdef/ldoor stand-in 952203^2 42.5M nnz, StrictChunker(8) -> w=3, forward y = B*x",
             "ct20stif": "C2 Boeing/ct20stif stand-in 52329^2 2.6M nnz, StrictChunker(8)",
             "ct20stif-fwd": "C2 Boeing/ct20stif stand-in 52329^2 2.6M nnz, StrictChunker(8), forward y = B*x",
             "ldoor-csc": "C4 TrSpMV!(y, A, x) on the GHS_psdef/ldoor stand-in (CSC, 952203^2, 42.5M nnz)"}


def algorithmic_bytes(B, esz, ti=4, nrhs=1):
    """SURVEY.md §8d, transposed: Tv·|val| + Ti·q + Ti·(3L+3) + Tx·m + Ty·n; 2D adds Ti·(K+1);
    k right-hand sides multiply the x and y terms by k.  CSC (TrSpMV!): Tv·nnz + Ti·nnz + Ti·(n+1)
    + Tx·m + Ty·n."""
    if not hasattr(B, "ofs"):  # SparseMatrixCSC
        A = B.A
        return (esz + ti) * int(A.nnz) + ti * (A.shape[1] + 1) + esz * (A.shape[0] + A.shape[1])
    nval = int(B.ofs[-1] - 1)
    q = int(B.pos[-1] - 1)
    L = len(B.Phi)
    extra = ti * (len(B.Pi) + 1) if hasattr(B, "Pi") else 0
    return esz * nval + ti * q + ti * (3 * L + 3) + extra + nrhs * esz * (B.m + B.n)


def load_traffic(workload, dtype):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (tools/pmc_traffic.py), if any."""
    p = ROOT / "profiles" / f"pmc_{workload}_{dtype}.json"
    if p.exists():
        try:
            d = json.loads(p.read_text())
            return d.get("hbm_bytes_per_launch"), str(p.relative_to(ROOT))
        except Exception:
            pass
    return None, None


def build_matrix(workload, dtype, scale=1.0, seed=0xDEADBEEF):
    import sparsematrixvbcs_amd as V
    if workload in ("fe-fwd", "fe3d-fwd", "ldoor-fwd", "ct20stif-fwd"):  # the same matrix, forward product
        workload = workload[:-4]
    if workload == "fe":
        return V.synthetic.fe_grid_2d(int(round(2236 * scale ** 0.5)), dof=2, dtype=dtype, seed=seed)
    if workload == "fe3d":
        n = 3 * int(round(3333333 * scale))
        return V.synthetic.fe_stiffness_3d_1dvbc(n, int(round(1e8 * scale)), 3, dtype=dtype, seed=seed)
    if workload in ("c5", "c5-fwd"):
        return V.synthetic.c5(dtype=dtype, scale=scale, seed=seed)
    if workload in ("c5-mesh", "c5-mesh-fwd"):
        return V.synthetic.c5_mesh(dtype=dtype, scale=scale, seed=seed)
    if workload in ("ldoor", "ct20stif", "ldoor-csc"):
        name = {"ldoor": "GHS_psdef/ldoor", "ct20stif": "Boeing/ct20stif", "ldoor-csc": "GHS_psdef/ldoor"}[workload]
        try:
            A = V.io.mdopen(name, dtype=dtype).A
        except FileNotFoundError:
            A = V.synthetic.standin(name, dtype=dtype, seed=seed, scale=scale)
        if workload == "ldoor-csc":  # TrSpMV!(y, A, x) = A'x on the CSC itself (TrSpMV.jl:1-20)
            C = V.SparseMatrixCSC(A.tocsc())
            C.A = A.tocsc()  # the scipy operand, for the byte count and the oracle
            return C
        # bin/test_table.jl:27 stores A = permutedims(A): B'x multiplies the original matrix
        return V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))
    return V.synthetic.north_star(dtype=dtype, scale=scale, seed=seed, mixed=(workload == "ns-mixed"))


def kernel_name(B, local, k, trans=True):
    if k > 1:
        if B.info(local, trans, multi=True)["planar_mask"] & 512:
            return ("vbc::spmm_tiles<T, UB, W, NBT, MASKU, BUF> (tile-granular: one key and one UB-row X block per "
                    "u x w tile, 4 streams of stripes per wave, csrc/vbc_tiles.h)")
        return "vbc::spmm_panel<T, NB, BUF, FAST> (v_mfma_*_16x16x4)"
    if not trans:
        inf = B.info(local, False)
        pm, R = inf["planar_mask"], inf["fwd_run"]
        if pm & 2048:
            return ("vbc::spmv_planar_pair<FASTE, NB, KC, MASK, DOT=true> (forward lane pairs: 3 x 3 node blocks "
                    "transposed into the B'x lane-pair layout, per-block dot products, csrc/vbc_planar.h)")
        if pm & 256:
            return ("the transposed kernels on C = B^T (forward of a mixed-width matrix: vbc::spmv_split_multi "
                    "fused split over C's row groups, csrc/vbc_planar.h)")
        if pm & 16:
            return (f"vbc::spmv_planar_lanes<T, W={R}, RUN, DEEP, RD> (forward lane streams: node blocks of "
                    f"{R} output rows transposed into the B'x lane-stream layout, csrc/vbc_planar.h)")
        if pm & 8:
            return f"vbc::spmv_planar_fwd_split<T, W, R={R}, P> (split forward chunks, csrc/vbc_planar.h)"
        if R > 1:
            return (f"vbc::spmv_planar_fwd<T, W, R={R}, FASTE, NB, KC> (forward row runs: one x-slice gather per "
                    f"block serves {R} output rows" + (", masked chunk-local order" if pm & 2 else "") +
                    ", csrc/vbc_planar.h)")
        if inf["sweep_bins"] > 0:
            return "vbc::spmv_sweep<T, TB> kind 1 (row-swept tiles, one accumulator per output row, csrc/vbc_sweep.hip)"
        if inf["slot_bins"] > 0:
            return "vbc::spmv_slots<T, 1, U, FASTE> (slotted output rows, csrc/vbc_slots.h)"
        return "vbc::spmv_ranges<T, 1, K, P> (merge layout, csrc/vbc_kernels.h)"
    inf = B.info(local, True)
    if inf["planar_mask"] & 32:
        return (f"vbc::spmv_split_multi<T, P={inf['planar_split']}, MODE> (fused small-matrix split: every width "
                "bucket in one launch, P waves per 64-stripe chunk, csrc/vbc_planar.h)")
    if inf["planar_bins"] > 0:
        if inf["planar_mask"] & 4:
            return (f"vbc::spmv_planar_lanes<T, W, RUN={inf['planar_run']}, DEEP, RD> (per-lane compacted streams: "
                    "tiles of stripes dealt to the lanes, csrc/vbc_planar.h)")
        if inf["planar_pair"]:
            return ("vbc::spmv_planar_pair<FASTE, NB, KC, MASK> (lane pairs, fp64 3-wide runs of 3"
                    + (", masked chunk-local order" if inf["planar_mask"] else "") + ", csrc/vbc_planar.h)")
        if inf["planar_split"] > 1:
            return (f"vbc::spmv_planar_split<T, W, KC, RUN={inf['planar_run']}, P={inf['planar_split']}> "
                    "(split planar chunks, csrc/vbc_planar.h)")
        if inf["planar_mask"]:
            return (f"vbc::spmv_planar<T, W, false, 0, KC, RUN={inf['planar_run']}, MASK=true> "
                    "(masked planar chunks, chunk-local length order, csrc/vbc_planar.h)")
        return (f"vbc::spmv_planar<T, W, FASTE, NB, KC, RUN={inf['planar_run']}> "
                "(planar slotted chunks, csrc/vbc_planar.h)")
    if inf["sweep_bins"] > 0:
        return "vbc::spmv_sweep<T, TB> (row-swept tiles, csrc/vbc_sweep.hip)"
    if inf["slot_bins"] > 0:
        return "vbc::spmv_slots<T, 0, U, FASTE> (slotted segments, csrc/vbc_slots.h)"
    return "vbc::spmv_ranges<T, 0, K, P> (+ vbc::fixup)"


def timed_products(step, steps, device, stream, world, graph=True):
    """Times EXACTLY `steps` calls of step() (barrier + synchronize on both sides).  With graph=True
    the K products are captured once into a HIP graph (torch.cuda.CUDAGraph) and the timed region is
    one replay; HIP events on the launching stream bracket it.  Returns (wall s, event ms / step)."""
    import torch
    import torch.distributed as dist
    g = None
    if graph:
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for _ in range(steps):
                    step()
            torch.cuda.synchronize(device)
        except Exception:  # capture unsupported for this call sequence: eager launches
            g = None
            torch.cuda.synchronize(device)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0.record(stream)
        if g is not None:
            g.replay()
        else:
            for _ in range(steps):
                step()
        ev1.record(stream)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    return elapsed, ev0.elapsed_time(ev1) / steps, g is not None


def parity(B, x_host, y_dev, k=1, cols=(0,), trans=True):
    """Normwise relative error of the GPU y against the CPU oracle on the same full-size input
    (oracle/vbc_oracle.c: multiply_1DVBC.jl:90-180 / multiply_VBC.jl:93-192 restated; trans=False:
    the forward products multiply_1DVBC.jl:13-83 / multiply_VBC.jl:7-87)."""
    from oracle import oracle as O
    from oracle import simd as S
    th = S.host_threads()
    if not hasattr(B, "ofs"):  # TrSpMV! on a CSC: orc_trspmv (TrSpMV.jl:1-20)
        t0 = time.perf_counter()
        ref = O.trspmv(B.A, x_host, np.zeros(B.n, B.A.dtype), nthreads=th)
        g = y_dev.cpu().numpy()
        err = float(np.linalg.norm(g.astype(np.float64) - ref) / max(np.linalg.norm(ref), 1e-300))
        tol = PARITY_TOL[np.dtype(B.A.dtype)]
        return {"rel_err": float(f"{err:.3e}"), "tol": tol, "pass": bool(err <= tol),
                "bitwise_equal": bool(np.array_equal(g, ref)), "oracle": "oracle/vbc_oracle.c orc_trspmv (TrSpMV.jl:1-20)",
                "columns": None, "oracle_s": round(time.perf_counter() - t0, 2)}
    if hasattr(B, "Pi"):
        R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    else:
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    yg = y_dev.cpu().numpy()
    nx, ny = (B.m, B.n) if trans else (B.n, B.m)
    X = x_host.reshape(nx, -1)
    Yg = yg.reshape(ny, -1)
    num = den = 0.0
    bitwise = True
    t0 = time.perf_counter()
    for c in (cols if k > 1 else (0,)):
        ref = O.mul(R, np.ascontiguousarray(X[:, c]), np.zeros(ny, B.val.dtype), trans=trans, nthreads=th)
        g = Yg[:, c]
        num += float(np.sum((g.astype(np.float64) - ref) ** 2))
        den += float(np.sum(ref.astype(np.float64) ** 2))
        bitwise = bitwise and bool(np.array_equal(g, ref))
    err = (num ** 0.5) / max(den ** 0.5, 1e-300)
    tol = PARITY_TOL[np.dtype(B.val.dtype)]
    return {"rel_err": float(f"{err:.3e}"), "tol": tol, "pass": bool(err <= tol), "bitwise_equal": bitwise,
            "oracle": ("oracle/vbc_oracle.c orc_*_mul_t (multiply_1DVBC.jl:90-180 / multiply_VBC.jl:93-192)" if trans
                       else "oracle/vbc_oracle.c orc_*_mul (multiply_1DVBC.jl:13-83 / multiply_VBC.jl:7-87)"),
            "columns": list(cols) if k > 1 else None, "oracle_s": round(time.perf_counter() - t0, 2)}


def cpu_baseline(B, x_host, esz, budget_s=4.0):
    """The reference's SIMD CPU kernel (oracle/vbc_simd.c: Vec{Δw} buckets, @fastmath, Int64
    indices; multiply_1DVBC.jl:90-180) on the full workload, on all host cores with the reference's
    one-stripe atomic self-scheduling (:169-177) and with 64-stripe grabs, and on 1 core.  `value` is
    the faster all-core figure (the honest, not understated, baseline)."""
    from oracle import simd as S
    th = S.host_threads()
    x = np.ascontiguousarray(x_host.reshape(B.m, -1)[:, 0])
    y = np.zeros(B.n, B.val.dtype)
    nbytes = algorithmic_bytes(B, esz)

    def run(nthreads, chunk):
        S.mul_t(B, x, y, nthreads, chunk)  # warm-up
        ts, t_start = [], time.perf_counter()
        while len(ts) < 30 and time.perf_counter() - t_start < budget_s:
            t0 = time.perf_counter()
            S.mul_t(B, x, y, nthreads, chunk)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), len(ts)

    t_ref, n_ref = run(th, 1)
    t_chk, n_chk = run(th, 64)
    t_one, n_one = run(1, 1)
    best = min(t_ref, t_chk)
    return dict(value=round(nbytes / best / 1e9, 3), unit="GB/s", cores=th, kind="port",
                sample=(f"full workload, mul!(y,B',x) with the reference's SIMD kernel (oracle/vbc_simd.c, "
                        f"{S.isa()}, -O3 -ffast-math, Int64 indices): {th} threads reference schedule "
                        f"(1 stripe per atomic grab) {t_ref * 1e3:.1f} ms (median of {n_ref}), 64-stripe grabs "
                        f"{t_chk * 1e3:.1f} ms ({n_chk}), 1 core {t_one * 1e3:.1f} ms ({n_one})"),
                ms_all_cores_ref_schedule=round(t_ref * 1e3, 3), ms_all_cores_chunk64=round(t_chk * 1e3, 3),
                ms_1core=round(t_one * 1e3, 3), value_1core=round(nbytes / t_one / 1e9, 3),
                nproc=os.cpu_count(), cpu_model=S.cpu_model(), isa=S.isa())


def box_info(device):
    """The GPU and its current clocks (rocm-smi --showclocks), recorded with every line: boxes of the
    pool differ by a few per cent on the same kernel (round 2: FE 176 us on the driver's box, 170 on
    others), and the clocks at measurement time are the first thing to compare."""
    import subprocess

    import torch
    p = torch.cuda.get_device_properties(device)
    out = {"name": p.name, "cus": p.multi_processor_count, "hbm_gib": round(p.total_memory / 2 ** 30, 1),
           "arch": getattr(p, "gcnArchName", None)}
    if any(k.startswith("ROCPROF") for k in os.environ):  # under rocprofv3 a child (rocm-smi, a python
        out["clocks"] = "not queried under rocprofv3"     # script) would re-exec an instrumented interpreter
        return out
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True, timeout=30)
        card = next(iter(json.loads(r.stdout).values()))
        out["clocks"] = {k: v for k, v in card.items() if "clock" in k.lower() or "level" in k.lower()}
    except Exception as e:  # no rocm-smi / no permission: the line still stands
        out["clocks"] = f"unavailable ({type(e).__name__})"
    return out


def measure(args, workload, dtype, device, local, with_cpu, with_parity, steps=None):
    """One single-GPU workload: build, warm up, time K products, optional CPU baseline + parity."""
    import torch

    import sparsematrixvbcs_amd as V

    steps = steps or args.steps
    esz = np.dtype(dtype).itemsize
    t_build = time.perf_counter()
    B = build_matrix(workload, dtype, args.scale)
    csc = not hasattr(B, "ofs")
    rng = np.random.default_rng(0xC0FFEE)
    k = args.nrhs if workload in ("c5", "c5-fwd", "c5-mesh", "c5-mesh-fwd") else 1
    trans = not workload.endswith("-fwd")
    nx, ny = (B.m, B.n) if trans else (B.n, B.m)
    x_host = rng.uniform(-1, 1, (nx, k) if k > 1 else nx).astype(dtype)
    x = torch.from_numpy(x_host).to(device)  # k > 1: row-major X (right-hand sides interleaved)
    y = torch.empty((ny, k) if k > 1 else ny, dtype=x.dtype, device=device)
    Bop = B.T if trans else B

    def step():
        if csc:
            V.TrSpMV_(y, B, x)
        else:
            V.mul_(y, Bop, x)
    stream = torch.cuda.Stream(device)
    with torch.cuda.stream(stream):
        B.handle(local, trans, multi=k > 1)  # build the HBM layout outside the timed region
        t_build = time.perf_counter() - t_build
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize(device)
    elapsed, kernel_ms, graphed = timed_products(step, steps, device, stream, 1, graph=not args.eager)
    bytes_launch = algorithmic_bytes(B, esz, nrhs=k)
    # TrSpMV! on a CSC: `value` keeps the CSC byte formula (what the reference's loop reads), but the
    # roofline prices the bytes the blocked layout must move (its index bytes are 1/3 of the CSC's), so
    # the fraction stays a fraction of what the kernel can reach
    bytes_roof = int(B.info(local, True)["bytes_t"]) if csc else bytes_launch
    nnz = int(B.A.nnz) if csc else int(np.count_nonzero(B.val))
    ms_per_step = elapsed / steps * 1e3
    achieved = bytes_roof / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(workload, "f64" if dtype == np.float64 else "f32")
    layout_bytes = int(B.info(local, trans, multi=k > 1)["device_bytes"])
    out = {
        # TrSpMV! on a CSC: priced on the bytes its blocked layout moves, so `value` is a bandwidth
        # (the CSC byte formula divided by the same time is reported apart as `csc_equivalent_GBs`)
        "value": round(bytes_roof * steps / elapsed / 1e9, 2),
        "unit": "GB/s",
        "ms_per_step": round(ms_per_step, 5),
        "gflops": round(2.0 * nnz * k * steps / elapsed / 1e9, 2),
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel_name(B, local, k, trans),
            "bytes_per_launch": bytes_roof, "avg_launch_ms": round(kernel_ms, 5), "traffic_source": traffic_src,
        },
        "config": {
            "workload": WORKLOADS[workload] + (f"-scale{args.scale}" if args.scale != 1.0 else ""),
            "op": ("TrSpMV!(y, A, x) -- CSC transposed product (TrSpMV.jl:1-20)" if csc else
                   ("mul!(y, B', x) -- transposed 1DVBC (multiply_1DVBC.jl:85-180)" if trans else
                    "mul!(y, B, x) -- forward 1DVBC (multiply_1DVBC.jl:9-83)") if k == 1 else
                   f"Y = B'X, {k} row-major right-hand sides -- 2D VBC (multiply_VBC.jl:89-192 per column), "
                   "multi-RHS kernel (roofline.kernel)" if trans else
                   f"Y = B*X, {k} row-major right-hand sides -- 2D VBC (multiply_VBC.jl:3-87 per column), "
                   "multi-RHS kernel on the layout of B' (the matrix read once; roofline.kernel)"),
            "m": B.m, "n": B.n, "stripes": B.n if csc else len(B.Phi),
            "row_blocks": nnz if csc else int(B.pos[-1] - 1), "nnz": nnz, "W": 1 if csc else B.W,
            "index_bytes": 4, "nrhs": k, "launch": "hipGraph of K products" if graphed else "eager",
            "build_s": round(t_build, 1), "layout_bytes": layout_bytes,
            "cache": ("warm, matrix < MALL: the layout fits the 256 MB Infinity Cache, so back-to-back "
                      "products may be served partly from it rather than HBM") if layout_bytes < MALL_BYTES
                     else "matrix > MALL: every product streams the layout from HBM",
        },
        "dtype": "f64" if dtype == np.float64 else "f32",
    }
    if traffic:  # the same launch time priced on the HBM bytes the PMC counters saw (the bytes moved)
        out["roofline"]["achieved_traffic"] = round(traffic / (kernel_ms * 1e-3) / 1e9, 1)
        out["roofline"]["frac_traffic"] = round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if csc:
        out["roofline"]["bytes_csc_formula"] = bytes_launch
        out["csc_equivalent_GBs"] = round(bytes_launch * steps / elapsed / 1e9, 2)
    if with_parity:
        out["parity"] = parity(B, x_host, y, k, cols=tuple(range(k)) if k > 1 else (0,), trans=trans)
    if with_cpu:
        out["cpu_baseline"] = cpu_baseline(B, x_host, esz)
    B.release()
    del x, y
    torch.cuda.empty_cache()
    return out


def measure_sharded(args, workload, dtype, world, rank, local, device, forward=False):
    """Strong scaling: ONE matrix split by stripes over the ranks; kernel-only and end-to-end."""
    import torch
    import torch.distributed as dist

    import sparsematrixvbcs_amd as V

    esz = np.dtype(dtype).itemsize
    B = build_matrix(workload, dtype, args.scale)  # same seed on every rank: one matrix
    S = V.distributed.ShardedSparseMatrix1DVBC(B, rank, world, split="stripes",
                                               comm="cpu" if args.backend == "gloo" else "device")
    bytes_total = algorithmic_bytes(B, esz)
    bytes_local = algorithmic_bytes(S.local, esz)
    nnz_total = int(np.count_nonzero(B.val[:B.ofs[-1] - 1]))
    rng = np.random.default_rng(0xC0FFEE)
    x_host = rng.uniform(-1, 1, B.m).astype(dtype)
    x = torch.from_numpy(x_host).to(device)
    y_local = torch.empty(S.n_local, dtype=x.dtype, device=device)
    stream = torch.cuda.Stream(device)
    with torch.cuda.stream(stream):
        S.local.handle(local, True)
        for _ in range(args.warmup):
            S.local_mul_t(y_local, x)
    torch.cuda.synchronize(device)
    elapsed, kernel_ms, graphed = timed_products(lambda: S.local_mul_t(y_local, x), args.steps, device, stream,
                                                 world, graph=not args.eager)

    # end-to-end: the product plus the all_gather that replicates y on every rank (RCCL over xGMI)
    y_full = torch.empty(B.n, dtype=x.dtype, device=device)

    def e2e():
        S.local_mul_t(y_local, x)
        S.gather(y_local, out=y_full)

    e2e_steps = max(5, args.steps // 5)
    with torch.cuda.stream(stream):
        e2e()
    torch.cuda.synchronize(device)
    dist.barrier()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(e2e_steps):
            e2e()
    torch.cuda.synchronize(device)
    e2e_elapsed = time.perf_counter() - t0
    dist.barrier()

    par = sharded_parity(args, B, S, x_host, x, y_full, y_local, world, rank, local, device, stream) \
        if not args.no_parity else None

    fwd = None
    if forward:  # mul!(y, B, x): partial y per rank + one RCCL all_reduce(sum)
        S.local.handle(local, False)
        xf = torch.from_numpy(rng.uniform(-1, 1, B.n).astype(dtype)).to(device)
        yf = torch.empty(B.m, dtype=x.dtype, device=device)
        with torch.cuda.stream(stream):
            S.mul(yf, xf)
        torch.cuda.synchronize(device)
        dist.barrier()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            for _ in range(e2e_steps):
                S.mul(yf, xf)
        torch.cuda.synchronize(device)
        fwd_elapsed = time.perf_counter() - t0
        dist.barrier()
        fwd = fwd_elapsed
        if not args.no_parity:  # the all_reduced y of the last timed product against the oracle's B·x
            xf_host = xf.cpu().numpy()
            fpar = parity(B, xf_host, yf, trans=False) if rank == 0 else None
            dist.barrier()

    stats = torch.tensor([elapsed, kernel_ms, e2e_elapsed, fwd or 0.0], dtype=torch.float64,
                         device=device if args.backend == "nccl" else "cpu")
    mx = stats.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    mn = stats.clone()
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    elapsed, kernel_ms, e2e_elapsed, fwd_elapsed = (v.item() for v in mx)
    out = {
        "value": round(bytes_total * args.steps / elapsed / 1e9, 2),
        "unit": "GB/s",
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "gflops": round(2.0 * nnz_total * args.steps / elapsed / 1e9, 2),
        "roofline": {
            "bound": "hbm", "achieved": round(bytes_local / (kernel_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(bytes_local / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": None, "kernel": kernel_name(S.local, local, 1), "bytes_per_launch": bytes_local,
            "avg_launch_ms": round(kernel_ms, 5), "scope": "rank 0 shard; avg_launch_ms is the max over ranks",
        },
        "e2e": {"value": round(bytes_total * e2e_steps / e2e_elapsed / 1e9, 2), "unit": "GB/s",
                "ms_per_step": round(e2e_elapsed / e2e_steps * 1e3, 4),
                "what": "mul!(y_local, B_r', x) + all_gather of y over RCCL (replicated y on every rank)"},
        "config": {
            "workload": WORKLOADS[workload] + (f"-scale{args.scale}" if args.scale != 1.0 else ""),
            "op": "mul!(y, B', x) -- transposed 1DVBC (multiply_1DVBC.jl:85-180), stripe-sharded",
            "m": B.m, "n": B.n, "stripes": len(B.Phi), "nnz": nnz_total, "W": B.W, "index_bytes": 4,
            "n_local_rank0": S.n_local, "stripe_cuts": S.cuts.tolist(),
            "parallelism": f"stripe split x{world}: disjoint y slices, no data-path collective",
            "launch": "hipGraph of K products" if graphed else "eager",
        },
        "dtype": "f64" if dtype == np.float64 else "f32",
    }
    if par is not None:
        out["parity"] = par
    if forward:
        out["forward_allreduce"] = {"value": round(bytes_total * e2e_steps / fwd_elapsed / 1e9, 2), "unit": "GB/s",
                                    "ms_per_step": round(fwd_elapsed / e2e_steps * 1e3, 4),
                                    "what": "mul!(y, B, x): partial y per rank + RCCL all_reduce(sum) of y"}
        if not args.no_parity:
            out["forward_allreduce"]["parity"] = fpar
    S.local.release()
    del x, y_local, y_full
    torch.cuda.empty_cache()
    return out


def sharded_parity(args, B, S, x_host, x, y_full, y_local, world, rank, local, device, stream):
    """Correctness of the N > 1 measurement (after its timed region):
    * the timed product's y -- every rank's disjoint B'x slice, gathered to rank 0 over the process
      group -- against the CPU oracle on the whole matrix (normwise rel-err, tolerance of BASELINE), and
      each rank's slice bit for bit;
    * the same shards rebuilt with VBC_CREATE_SERIAL (B.serial: the reference's serial per-stripe order
      in every layout, no split planar product): their gathered y must equal the oracle -- and so the
      single-GPU product, which matches it bit for bit -- exactly.
    Returns rank 0's dict (None on the other ranks)."""
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from oracle import simd as Sd
    y_ser = torch.empty_like(y_local)
    S.local.serial = True  # a second handle (layout flags are part of the handle key)
    with torch.cuda.stream(stream):
        S.local_mul_t(y_ser, x)
    torch.cuda.synchronize(device)
    y_ser_full = S.gather(y_ser, out=torch.empty_like(y_full))
    torch.cuda.synchronize(device)
    S.local.release()  # both handles; the caller's later products rebuild what they use
    S.local.serial = False
    res = None
    if rank == 0:
        t0 = time.perf_counter()
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
        ref = O.mul(R, x_host, np.zeros(B.n, B.val.dtype), trans=True, nthreads=Sd.host_threads())
        g, gs = y_full.cpu().numpy(), y_ser_full.cpu().numpy()
        err = float(np.linalg.norm(g.astype(np.float64) - ref) / max(np.linalg.norm(ref), 1e-300))
        tol = PARITY_TOL[np.dtype(B.val.dtype)]
        slices = [bool(np.array_equal(g[a:b], ref[a:b])) for a, b in zip(S.splits[:-1], S.splits[1:])]
        ser = bool(np.array_equal(gs, ref))
        res = {"rel_err": float(f"{err:.3e}"), "tol": tol, "bitwise_equal": bool(all(slices)),
               "slices_bitwise": slices, "serial_bitwise_equal": ser, "pass": bool(err <= tol and ser),
               "oracle": "oracle/vbc_oracle.c orc_1dvbc_mul_t (multiply_1DVBC.jl:90-180) on the whole matrix",
               "what": ("timed product: rank slices gathered to rank 0 vs the oracle; serial: shards built with "
                        "VBC_CREATE_SERIAL, gathered y must equal the oracle bit for bit"),
               "oracle_s": round(time.perf_counter() - t0, 2)}
    dist.barrier()
    return res


def abi_sharded_child(args):
    """One process driving devices 0..N-1 through the C ABI's sharded handle (vbc1d_create_sharded /
    vbc_sharded_mul_ex, distributed.MultiGPUSparseMatrix1DVBC) -- the configuration the Julia shim
    binds (julia/SparseMatrixVBCsHIP.jl): x broadcast over RCCL, the shards' products on their own
    devices, the disjoint y slices sent back to devices[0]; the forward product scatters x slices and
    ncclReduce(sum)s y.  Times K products of each direction (eager: the exchange spans devices) and
    checks both against the oracle.  Prints one JSON line."""
    import torch

    import sparsematrixvbcs_amd as V
    from sparsematrixvbcs_amd import distributed as D
    devices = [int(d) for d in args.abi_sharded_child.split(",")]
    dtype = np.float64 if args.dtype == "f64" else np.float32
    esz = np.dtype(dtype).itemsize
    B = build_matrix(args.workload, dtype, args.scale)
    t0 = time.perf_counter()
    S = D.MultiGPUSparseMatrix1DVBC(B, devices=devices, split="stripes")
    build_s = time.perf_counter() - t0
    dev0 = torch.device("cuda", devices[0])
    torch.cuda.set_device(dev0)
    rng = np.random.default_rng(0xC0FFEE)
    out = {"devices": devices, "split": "stripes", "build_s": round(build_s, 1),
           "rccl": len(set(devices)) > 1 or len(devices) == 1,
           "what": ("one process, C ABI vbc1d_create_sharded + vbc_sharded_mul_ex (the Julia drop-in's multi-GPU "
                    "configuration): x and y on devices[0]")}
    bytes_total = algorithmic_bytes(B, esz)
    for trans, key in ((True, "transposed"), (False, "forward")):
        nx, ny = (B.m, B.n) if trans else (B.n, B.m)
        xh = rng.uniform(-1, 1, nx).astype(dtype)
        x = torch.from_numpy(xh).to(dev0)
        y = torch.empty(ny, dtype=x.dtype, device=dev0)
        op = S.T if trans else S
        for _ in range(max(1, args.warmup)):
            V.mul_(y, op, x)
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(args.steps):
            V.mul_(y, op, x)
        ev1.record()
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)
        el = time.perf_counter() - t0
        out[key] = {"value": round(bytes_total * args.steps / el / 1e9, 2), "unit": "GB/s",
                    "ms_per_step": round(el / args.steps * 1e3, 5),
                    "event_ms_per_step": round(ev0.elapsed_time(ev1) / args.steps, 5),
                    "op": "mul!(y, B', x): x broadcast, y slices gathered" if trans else
                          "mul!(y, B, x): x slices, ncclReduce(sum) of y",
                    "parity": parity(B, xh, y, trans=trans) if not args.no_parity else None}
    S.release()
    out["pass"] = all(out[k]["parity"] is None or out[k]["parity"]["pass"] for k in ("transposed", "forward"))
    print(json.dumps(out), flush=True)


def run_abi_sharded(args, world):
    """Start abi_sharded_child in a fresh process once the rank processes are done with their GPUs
    (devices 0..N-1 when the box has them, else every shard on device 0), return its JSON."""
    import subprocess
    import torch
    nd = torch.cuda.device_count()
    devices = list(range(world)) if (nd >= world and not args.same_device) else [0] * world
    cmd = [sys.executable, str(Path(__file__).resolve()), "--abi-sharded-child", ",".join(map(str, devices)),
           "--workload", args.workload, "--dtype", args.dtype, "--steps", str(args.steps), "--warmup",
           str(args.warmup), "--scale", str(args.scale)] + (["--no-parity"] if args.no_parity else [])
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                                             "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)  # the line must not wait on a hang
    except subprocess.TimeoutExpired:
        return {"error": "timed out", "pass": False}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}: {r.stderr[-1500:]}", "pass": False}
    return json.loads(lines[-1])


def launch_ranks(n):
    """Run this script as ranks 0..n-1 (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, as
    torch.distributed.run sets them) in child processes; returns the first nonzero exit status."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    while True:  # a rank that fails would leave the others waiting in a collective: stop them
        codes = [p.poll() for p in procs]
        bad = next((c for c in codes if c not in (None, 0)), None)
        if bad is not None:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            return bad
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="fe", choices=list(WORKLOADS))
    ap.add_argument("--nrhs", type=int, default=16, help="right-hand sides of the c5 workload")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (debug only)")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of one graph replay")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 process group: nccl = RCCL over xGMI (the measurement); gloo = rehearsal of the "
                         "multi-rank code path with host-side collectives")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (a one-GPU box; needs --backend gloo)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary workloads")
    ap.add_argument("--no-abi-sharded", action="store_true",
                    help="N > 1: skip the one-process C-ABI sharded leg (secondary.abi_sharded)")
    ap.add_argument("--abi-sharded-child", default="", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.abi_sharded_child:
        abi_sharded_child(args)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: start the N ranks ourselves, one process per GPU (what
        # torchrun does), before this process touches a GPU; rank 0 prints the line, we exit with
        # the worst status
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.same_device:
        if args.backend != "gloo":
            raise SystemExit("--same-device needs --backend gloo (RCCL refuses two ranks on one GPU)")
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dtype = np.float64 if args.dtype == "f64" else np.float32
    head = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "higher_is_better": True, "vs_baseline": None,
            "data": "synthetic (matrix seed 0xDEADBEEF, x ~ U[-1,1) seed 0xC0FFEE); no SuiteSparse files offline"}

    if world == 1:
        p = measure(args, args.workload, dtype, device, local, with_cpu=not args.no_cpu_baseline,
                    with_parity=not args.no_parity)
        out = dict(head, value=p["value"], unit=p["unit"], ms_per_step=p["ms_per_step"], scaling="strong",
                   dtype=p["dtype"], config=dict(p["config"], parallelism="single GPU"), gflops=p["gflops"],
                   roofline=p["roofline"], cpu_baseline=p.get("cpu_baseline"), parity=p.get("parity"))
        if "parity" in p:
            out["rel_err"] = p["parity"]["rel_err"]
        out["device"] = box_info(device)
        if not args.no_secondary:
            sec = {}
            for wl, dt in (("fe-fwd", dtype), ("fe3d", dtype), ("fe3d-fwd", dtype), ("ns", dtype), ("c5", np.float32),
                           ("c5-fwd", np.float32), ("c5-mesh", np.float32), ("c5-mesh-fwd", np.float32),
                           ("ct20stif", np.float64),
                           ("ct20stif-fwd", np.float64), ("ldoor", np.float64), ("ldoor-fwd", np.float64),
                           ("ldoor-csc", np.float32)):
                if wl == args.workload:
                    continue
                s = measure(args, wl, dt, device, local, with_cpu=False, with_parity=not args.no_parity)
                sec[wl] = {"workload": s["config"]["workload"], "value": s["value"], "unit": s["unit"],
                           "ms_per_step": s["ms_per_step"], "gflops": s["gflops"], "dtype": s["dtype"],
                           "roofline_frac": s["roofline"]["frac"], "kernel": s["roofline"]["kernel"],
                           "kernel_us": round(s["roofline"]["avg_launch_ms"] * 1e3, 1),
                           "bytes_per_launch": s["roofline"]["bytes_per_launch"], "op": s["config"]["op"],
                           "cache": s["config"]["cache"]}
                if "csc_equivalent_GBs" in s:
                    sec[wl]["csc_equivalent_GBs"] = s["csc_equivalent_GBs"]
                if "parity" in s:
                    sec[wl]["rel_err"] = s["parity"]["rel_err"]
                    sec[wl]["parity_pass"] = s["parity"]["pass"]
            out["secondary"] = sec
    else:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        p = measure_sharded(args, args.workload, dtype, world, rank, local, device)
        out = dict(head, value=p["value"], unit=p["unit"], ms_per_step=p["ms_per_step"], scaling="strong",
                   dtype=p["dtype"], config=p["config"], gflops=p["gflops"], roofline=p["roofline"], e2e=p["e2e"],
                   cpu_baseline=None, parity=p.get("parity"))
        if p.get("parity"):
            out["rel_err"] = p["parity"]["rel_err"]
        out["secondary"] = {}
        if not args.no_secondary and args.workload != "ldoor":
            c3 = measure_sharded(args, "ldoor", dtype, world, rank, local, device, forward=True)
            out["secondary"]["c3_ldoor"] = {k: c3.get(k) for k in ("value", "unit", "ms_per_step", "e2e",
                                                                   "forward_allreduce", "parity")}
            out["secondary"]["c3_ldoor"]["workload"] = c3["config"]["workload"]
            out["secondary"]["c3_ldoor"]["roofline_frac_rank0"] = c3["roofline"]["frac"]
        dist.barrier()  # every rank is done with its GPU before the one-process leg starts
        dist.destroy_process_group()
        if rank == 0 and not args.no_abi_sharded:
            out["secondary"]["abi_sharded"] = run_abi_sharded(args, world)
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
