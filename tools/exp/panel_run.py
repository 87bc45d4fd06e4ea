"""Run the matrix-core multi-RHS product (panel layout) N times for profiling.

    python tools/exp/panel_run.py [--workload c5|fe|ns] [--dtype f32] [--nrhs 16] [--reps 20]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--nrhs", type=int, default=16)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--vector", action="store_true", help="the SpMV-layout vector kernel instead")
    args = ap.parse_args()
    import torch
    import sparsematrixvbcs_amd as V
    from sparsematrixvbcs_amd import _lib as L
    dtype = np.float64 if args.dtype == "f64" else np.float32
    if args.workload == "c5":
        B = V.synthetic.c5(dtype=dtype)
    elif args.workload == "fe":
        B = V.synthetic.fe_grid_2d(2236, dof=2, dtype=dtype)
    else:
        B = V.synthetic.north_star(dtype=dtype)
    k = args.nrhs
    X = torch.rand((B.m, k), dtype=torch.float32 if dtype == np.float32 else torch.float64, device="cuda")
    Y = torch.empty((B.n, k), dtype=X.dtype, device="cuda")
    h = B.handle(0, True, multi=not args.vector)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(args.reps):
        L.check(L.lib().vbc_mul_mat(h, 1, k, X.data_ptr(), k, B.m, Y.data_ptr(), k, B.n, 1.0, 0.0,
                                    L.VBC_MEM_DEVICE, s, L.VBC_MAT_ROWMAJOR), "mul_mat")
    torch.cuda.synchronize()
    print("done", B.m, B.n, float(Y.sum()))


if __name__ == "__main__":
    main()
