"""Per-shard product times of the N-way stripe or row split, measured one shard at a time on ONE GPU.

The driver's 8-GPU scaling run is not ours to launch; this predicts it from the single-GPU box:
every shard of distributed.stripe_split(B, N) (or row_split with --split rows) gets its own handle and K
graph-replayed products (bench.timed_products), and the slowest shard bounds the strong-scaling step time
of bench.py --gpus N (the rank's kernel time).  Stripe split: B'x has disjoint y slices (no data-path
collective), --forward adds each shard's B x (a partial y -> one all-reduce).  Row split: B x has disjoint
y slices, B'x a partial y.  Every line also carries the cost model's end-to-end figure per direction
(distributed.predict_product_us: the MEASURED slowest shard plus the ASSUMED collective).

    python tools/shard_time.py --workload ldoor --worlds 1,2,4,8 [--split rows] [--forward] [--ranks 0]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fe")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--forward", action="store_true", help="also time the other direction of every shard")
    ap.add_argument("--split", default="stripes", choices=["stripes", "rows"])
    ap.add_argument("--ranks", default="", help="time only these shards (comma list; PMC runs of one shard)")
    args = ap.parse_args()
    import torch

    import bench
    import sparsematrixvbcs_amd as V

    dtype = np.float64 if args.dtype == "f64" else np.float32
    esz = np.dtype(dtype).itemsize
    device = torch.device("cuda", 0)
    B = bench.build_matrix(args.workload, dtype, args.scale)
    total = bench.algorithmic_bytes(B, esz)
    stream = torch.cuda.Stream(device)
    base = None
    fbase = [None]
    D = V.distributed
    rows = args.split == "rows"
    # the split's main product has disjoint y: B'x for stripes, B x for rows; --forward times the other one
    main_t = not rows
    for world in (int(w) for w in args.worlds.split(",")):
        cuts = D.row_split(B, world) if rows else D.stripe_split(B, world)
        per = []
        ranks = [int(r) for r in args.ranks.split(",")] if args.ranks else range(world)
        for r in ranks:
            # a rank's view of the split (distributed.ShardedSparseMatrix1DVBC: rows rebased / stripes trimmed to
            # what the shard touches); its products need no collective here -- the partial direction's
            # reduction is priced by the model below
            Sh = None if world == 1 else D.ShardedSparseMatrix1DVBC(B, r, world, split=args.split)
            S = B if world == 1 else Sh.local

            def time_dir(trans):
                nx, ny = (B.m, B.n) if trans else (B.n, B.m)
                xs = torch.from_numpy(np.random.default_rng(1 if trans else 2).uniform(-1, 1, nx).astype(dtype)).to(device)
                if Sh is None:
                    op = B.T if trans else B
                    ys = torch.empty(ny, dtype=xs.dtype, device=device)
                    step = lambda: V.mul_(ys, op, xs)  # noqa: E731
                else:  # the disjoint direction writes the rank's slice, the partial one a full-length y
                    disjoint = trans != rows
                    ys = torch.empty((Sh.n_local if trans else Sh.m_local) if disjoint else ny, dtype=xs.dtype,
                                     device=device)
                    step = (lambda: Sh.local_mul_t(ys, xs)) if trans else (lambda: Sh.local_mul(ys, xs))
                with torch.cuda.stream(stream):
                    S.handle(0, trans)
                    for _ in range(args.warmup):
                        step()
                torch.cuda.synchronize(device)
                wall, ev_ms, _ = bench.timed_products(step, args.steps, device, stream, 1)
                return round(ev_ms * 1e3, 2), round(wall / args.steps * 1e6, 2), bench.kernel_name(S, 0, 1, trans=trans)

            ev, wall, kern = time_dir(main_t)
            rec = {"rank": r, "range": [int(cuts[r]), int(cuts[r + 1])], "bytes": bench.algorithmic_bytes(S, esz),
                   "us_event": ev, "us_wall": wall, "kernel": kern}
            if Sh is not None:
                rec["local_rows"] = [Sh.row0, Sh.row0 + Sh.m_local]
                rec["local_cols"] = [Sh.col0, Sh.col0 + Sh.n_local]
            if args.forward:  # the other direction: a partial y (length m for stripes' B x, n for rows' B'x)
                fev, fwall, fkern = time_dir(not main_t)
                rec.update(fwd_us_event=fev, fwd_us_wall=fwall, fwd_kernel=fkern,
                           allreduce_bytes=int((B.n if rows else B.m) * esz) if world > 1 else 0)
            per.append(rec)
            if world > 1:
                S.release()
        slow = max(p["us_wall"] for p in per)
        if base is None:
            base = slow
        line = {"workload": args.workload, "dtype": args.dtype, "split": args.split, "world": world,
                "product": "B'x (disjoint y)" if main_t else "B x (disjoint y)",
                "max_us_wall": slow, "speedup_vs_first": round(base / slow, 3),
                "value_GBs": round(total / (slow * 1e-6) / 1e9, 1), "shards": per}
        # cost model end to end: measured slowest shard + assumed collective (y replicated)
        kind = "allgather"
        line["model_e2e_us"] = {"main": round(slow + D.collective_us(kind, esz * (B.n if main_t else B.m), world), 2),
                                "main_sharded_y": slow, "collective": kind + " of y (assumed rates)"}
        if args.forward:
            fslow = max(p["fwd_us_wall"] for p in per)
            if fbase[0] is None:
                fbase[0] = fslow
            other = esz * (B.m if main_t else B.n)
            line.update(other_product="B x (partial y)" if main_t else "B'x (partial y)",
                        fwd_max_us_wall=fslow, fwd_speedup_vs_first=round(fbase[0] / fslow, 3),
                        fwd_allreduce_bytes=per[0]["allreduce_bytes"],
                        fwd_model_e2e_us=round(fslow + D.collective_us("allreduce", other, world), 2),
                        fwd_note="kernel only, then one all_reduce(sum) of the partial y over RCCL (model: assumed "
                                 "rates, distributed.collective_us)")
        print(json.dumps(line), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
