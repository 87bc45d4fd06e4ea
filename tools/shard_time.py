"""Per-shard product times of the N-way stripe split, measured one shard at a time on ONE GPU.

The driver's 8-GPU scaling run is not ours to launch; this predicts it from the single-GPU box:
every shard of distributed.stripe_split(B, N) gets its own handle and K graph-replayed products
(bench.timed_products), and the slowest shard bounds the strong-scaling step time of bench.py
--gpus N (the rank's kernel time; B'x on the stripe split has no data-path collective).

    python tools/shard_time.py --workload fe --worlds 1,2,4,8 [--dtype f64 --steps 50]
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
    ap.add_argument("--forward", action="store_true", help="also time the forward product B_r x_r of every shard")
    args = ap.parse_args()
    import torch

    import bench
    import sparsematrixvbcs_amd as V

    dtype = np.float64 if args.dtype == "f64" else np.float32
    esz = np.dtype(dtype).itemsize
    device = torch.device("cuda", 0)
    B = bench.build_matrix(args.workload, dtype, args.scale)
    total = bench.algorithmic_bytes(B, esz)
    x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, B.m).astype(dtype)).to(device)
    stream = torch.cuda.Stream(device)
    base = None
    fbase = [None]
    for world in (int(w) for w in args.worlds.split(",")):
        cuts = V.distributed.stripe_split(B, world)
        per = []
        for r in range(world):
            S, _ = V.distributed.shard(B, int(cuts[r]), int(cuts[r + 1])) if world > 1 else (B, 0)
            y = torch.empty(S.n, dtype=x.dtype, device=device)
            St = S.T
            with torch.cuda.stream(stream):
                S.handle(0, True)
                for _ in range(args.warmup):
                    V.mul_(y, St, x)
            torch.cuda.synchronize(device)
            wall, ev_ms, _ = bench.timed_products(lambda: V.mul_(y, St, x), args.steps, device, stream, 1)
            rec = {"rank": r, "stripes": int(cuts[r + 1] - cuts[r]), "bytes": bench.algorithmic_bytes(S, esz),
                   "us_event": round(ev_ms * 1e3, 2), "us_wall": round(wall / args.steps * 1e6, 2),
                   "kernel": bench.kernel_name(S, 0, 1)}
            if args.forward:  # C3's forward leg: mul!(y, B_r, x_r) on the shard -> a partial y of length m
                xf = torch.from_numpy(np.random.default_rng(2).uniform(-1, 1, S.n).astype(dtype)).to(device)
                yf = torch.empty(S.m, dtype=x.dtype, device=device)
                with torch.cuda.stream(stream):
                    S.handle(0, False)
                    for _ in range(args.warmup):
                        V.mul_(yf, S, xf)
                torch.cuda.synchronize(device)
                fw, fev, _ = bench.timed_products(lambda: V.mul_(yf, S, xf), args.steps, device, stream, 1)
                rec.update(fwd_us_event=round(fev * 1e3, 2), fwd_us_wall=round(fw / args.steps * 1e6, 2),
                           fwd_kernel=bench.kernel_name(S, 0, 1, trans=False),
                           allreduce_bytes=int(S.m * esz) if world > 1 else 0)
                del xf, yf
            per.append(rec)
            if world > 1:
                S.release()
            del y
        slow = max(p["us_wall"] for p in per)
        if base is None:
            base = slow
        line = {"workload": args.workload, "dtype": args.dtype, "world": world,
                "max_us_wall": slow, "speedup_vs_first": round(base / slow, 3),
                "value_GBs": round(total / (slow * 1e-6) / 1e9, 1), "shards": per}
        if args.forward:
            fslow = max(p["fwd_us_wall"] for p in per)
            if fbase[0] is None:
                fbase[0] = fslow
            line.update(fwd_max_us_wall=fslow, fwd_speedup_vs_first=round(fbase[0] / fslow, 3),
                        fwd_allreduce_bytes=per[0]["allreduce_bytes"],
                        fwd_note="kernel only: each rank's partial y then goes through one all_reduce(sum) of "
                                 "allreduce_bytes over RCCL (not timed on one GPU)")
        print(json.dumps(line), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
