"""Benchmark: 1DVBC SpMV effective GB/s (and GFLOP/s) vs the MI355X HBM roofline (BASELINE.json).

A step is one mul!(y, B', x) -- the transposed 1D-VBR product the reference's paper and benchmark
time (bin/test_table.jl:80) -- fp64, inputs resident in HBM.  Primary workload (BASELINE.json
target: "10M x 10M, ~1e8-nnz SuiteSparse-like matrix"): `fe`, a 2D finite-element operator
(5-point stencil, 2 unknowns per node, 1.0e7 x 1.0e7, 1.0e8 stored values) in 1DVBC form.
Secondary (reported in the same line at N=1): `ns`, SURVEY.md §8d's NS-1DVBC, the reference's own
uniform-random VBR generator (costs.jl:63-83) at 1e7 x 1e7, 1e8 nonzeros, width-4 stripes.
N ranks = N GPUs, one process each (torchrun); every rank owns its own block-row shard of that size
(weak scaling, no data-path collective: the transposed product writes disjoint y ranges).
rank 0 prints one JSON line.

    python bench.py [--gpus N --steps K --warmup W --workload fe|ns|ns-mixed --dtype f64|f32]
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


def algorithmic_bytes(B, esz, ti=4, nrhs=1):
    """SURVEY.md §8d, transposed: Tv·|val| + Ti·q + Ti·(3L+3) + Tx·m + Ty·n; 2D adds Ti·(K+1);
    k right-hand sides multiply the x and y terms by k."""
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


def cpu_baseline(B, x, esz, budget_s=12.0, max_reps=20):
    """Oracle (C restatement of multiply_1DVBC.jl:85-180 / multiply_VBC.jl:89-192, OpenMP dynamic-1
    stripe scheduling) on the host cores, full-size product repeated until ~budget_s of CPU work;
    several right-hand sides run one oracle product per column (the reference has no matrix mul!)."""
    from oracle import oracle as O
    threads = max(1, min(16, os.cpu_count() or 1))
    if hasattr(B, "Pi"):
        R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    else:
        R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    X = x.reshape(B.m, -1)
    k = X.shape[1]
    cols = [np.ascontiguousarray(X[:, j]) for j in range(k)]
    y = np.zeros(B.n, dtype=B.val.dtype)

    def product():
        for c in cols:
            O.mul(R, c, y, trans=True, nthreads=threads)

    O.mul(R, cols[0], y, trans=True, nthreads=threads)  # warm-up (page faults)
    times = []
    t_start = time.perf_counter()
    while len(times) < max_reps and (time.perf_counter() - t_start) < budget_s:
        t0 = time.perf_counter()
        product()
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    what = "mul!(y,B',x)" if k == 1 else f"B'X ({k} columns, one mul!(y,B',x) each)"
    return dict(value=round(algorithmic_bytes(B, esz, nrhs=k) / t / 1e9, 3), unit="GB/s", cores=threads,
                kind="port", sample=f"full workload, median of {len(times)} oracle {what} "
                                    f"runs ({t * 1e3:.1f} ms each), {threads} OpenMP threads")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="fe", choices=["fe", "ns", "ns-mixed", "c5"])
    ap.add_argument("--nrhs", type=int, default=16, help="right-hand sides of the c5 workload")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--scale", type=float, default=1.0, help="shrink the workload (debug only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary (uniform) workload")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    dtype = np.float64 if args.dtype == "f64" else np.float32
    out = measure(args, args.workload, dtype, world, rank, local, device, with_cpu=not args.no_cpu_baseline)
    if world == 1 and not args.no_secondary:
        sec = "ns" if args.workload != "ns" else "fe"
        s = measure(args, sec, dtype, world, rank, local, device, with_cpu=False)
        out["secondary"] = {k: s[k] for k in ("value", "unit", "ms_per_step", "gflops")}
        out["secondary"]["workload"] = s["config"]["workload"]
        out["secondary"]["roofline_frac"] = s["roofline"]["frac"]
        out["secondary"]["kernel"] = s["roofline"]["kernel"]
        out["secondary"]["note"] = ("uniform-random rows (costs.jl:63-83 generator): no x locality; the row-swept "
                                    "layout keeps the grid's gathers in a moving window of x, bound by L2-miss "
                                    "throughput, see DESIGN.md §6")
        if args.workload != "c5":
            c = measure(args, "c5", np.float32, world, rank, local, device, with_cpu=False)
            out["secondary_c5"] = {k: c[k] for k in ("value", "unit", "ms_per_step", "gflops", "dtype")}
            out["secondary_c5"]["workload"] = c["config"]["workload"]
            out["secondary_c5"]["op"] = c["config"]["op"]
            out["secondary_c5"]["roofline_frac"] = c["roofline"]["frac"]
            out["secondary_c5"]["kernel_us"] = round(c["roofline"]["avg_launch_ms"] * 1e3, 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


WORKLOADS = {"ns": "NS-1DVBC-10Mx10M-1e8nnz-w4-uniform",
             "ns-mixed": "NS-1DVBC-mixed-w1..8-1e8nnz-uniform",
             "fe": "FE-2D-5pt-dof2-10Mx10M-1e8nnz-w2 (SuiteSparse-like mesh operator)",
             "c5": "C5-VBC2D-8x8-tiles-2Mx2M-1e8nnz-16RHS (costs.jl:200-220 generator)"}


def build_matrix(workload, dtype, scale, seed):
    import sparsematrixvbcs_amd as V
    if workload == "fe":
        return V.synthetic.fe_grid_2d(int(round(2236 * scale ** 0.5)), dof=2, dtype=dtype, seed=seed)
    if workload == "c5":
        return V.synthetic.c5(dtype=dtype, scale=scale, seed=seed)
    return V.synthetic.north_star(dtype=dtype, scale=scale, seed=seed, mixed=(workload == "ns-mixed"))


def measure(args, workload, dtype, world, rank, local, device, with_cpu):
    import torch
    import torch.distributed as dist

    import sparsematrixvbcs_amd as V

    esz = np.dtype(dtype).itemsize
    # each rank: its own block-row shard (different stripes' values), the same replicated x
    B = build_matrix(workload, dtype, args.scale, 0xDEADBEEF + rank)
    rng = np.random.default_rng(0xC0FFEE)
    k = args.nrhs if workload == "c5" else 1
    x_host = rng.uniform(-1, 1, (B.m, k) if k > 1 else B.m).astype(dtype)
    x = torch.from_numpy(x_host).to(device)  # k > 1: row-major X (right-hand sides interleaved)
    y = torch.empty((B.n, k) if k > 1 else B.n, dtype=x.dtype, device=device)
    Bt = B.T
    B.handle(local, True, multi=k > 1)  # build the HBM layout outside the timed region
    if k > 1:
        kernel_name = "vbc::spmm_panel<T, NB, BUF, FAST> (v_mfma_*_16x16x4)"
    elif B.info(local, True)["sweep_bins"] > 0:
        kernel_name = "vbc::spmv_sweep<T, TB> (row-swept tiles, csrc/vbc_sweep.hip)"
    elif B.info(local, True)["slot_bins"] > 0:
        kernel_name = "vbc::spmv_slots<T, 0, U, FASTE> (slotted segments, csrc/vbc_slots.h)"
    else:
        kernel_name = "vbc::spmv_ranges<T, 0, K, P> (+ vbc::fixup)"
    stream = torch.cuda.current_stream(device)

    for _ in range(args.warmup):
        V.mul_(y, Bt, x)
    torch.cuda.synchronize(device)

    # HIP events on the launching stream bracket the K back-to-back products of the timed region:
    # avg_launch_ms = event span / K (an event pair around every product would put two extra markers
    # between consecutive kernels of the timed region); rocprofv3's per-kernel average of the same
    # process agrees (profiles/r01_bench_kernel_stats.csv).
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        V.mul_(y, Bt, x)
    ev1.record(stream)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kernel_ms = ev0.elapsed_time(ev1) / args.steps

    bytes_rank = algorithmic_bytes(B, esz, nrhs=k)
    nnz = int(np.count_nonzero(B.val))
    stats = torch.tensor([elapsed, float(bytes_rank), float(nnz * k), kernel_ms], dtype=torch.float64, device=device)
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, kernel_ms = mx[0].item(), mx[3].item()
        total_bytes, total_nnz = sm[1].item(), sm[2].item()
    else:
        total_bytes, total_nnz = float(bytes_rank), float(nnz * k)

    ms_per_step = elapsed / args.steps * 1e3
    value = total_bytes * args.steps / elapsed / 1e9
    achieved = bytes_rank / (kernel_ms * 1e-3) / 1e9
    wname = WORKLOADS[workload] + (f"-scale{args.scale}" if args.scale != 1.0 else "")
    dname = "f64" if dtype == np.float64 else "f32"
    traffic, traffic_src = load_traffic(workload, dname)
    out = {
        "metric": "1DVBC SpMV effective GB/s (and GFLOP/s) vs HBM roofline, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dname,
        "data": "synthetic (seed 0xDEADBEEF+rank; x ~ U[-1,1), seed 0xC0FFEE); no SuiteSparse files offline",
        "config": {
            "workload": wname,
            "op": ("mul!(y, B', x) -- transposed 1DVBC (multiply_1DVBC.jl:85-180)" if k == 1 else
                   f"Y = B'X, {k} row-major right-hand sides -- 2D VBC (multiply_VBC.jl:89-192 per column), "
                   "matrix-core panel kernel"),
            "m": B.m, "n_per_rank": B.n, "stripes_per_rank": len(B.Phi), "row_blocks_per_rank": int(B.pos[-1] - 1),
            "nnz_per_rank": nnz, "W": B.W, "index_bytes": 4, "nrhs": k,
            "parallelism": f"stripe-shard x{world} (disjoint y, no collective)",
        },
        "gflops": round(2.0 * total_nnz * args.steps / elapsed / 1e9, 2),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": kernel_name,
            "bytes_per_launch": bytes_rank,
            "avg_launch_ms": round(kernel_ms, 5),
            "traffic_source": traffic_src,
        },
        "cpu_baseline": None,
    }
    if with_cpu and rank == 0 and world == 1:
        out["cpu_baseline"] = cpu_baseline(B, x_host, esz)
    B.release()
    del x, y
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
