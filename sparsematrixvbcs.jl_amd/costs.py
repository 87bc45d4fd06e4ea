"""The TrSpMV time cost model, re-fitted to the gfx950 kernel (costs.jl:12-136).

The reference times mul!(y, B', x) on random VBR matrices of every width w = W..1 (its own
generator, costs.jl:45-83: d = 8 stored rows per stripe, sizes around a cache level) and fits, by
relative least squares, a per-stripe cost alpha[w] and a per-stored-row cost beta[w] (plus a per-row
term it then drops); the widths' costs are made monotone (costs.jl:124-128).  The partitioner then
minimises sum(alpha[w] + beta[w]·rows) (DynamicTotalChunker over ColumnBlockCostModel).

Here the same protocol times libvbc's kernel on the GPU.  Sizes follow costs.jl's "exceed" branch
scaled to this device's last-level cache (the 256 MiB MALL): the model describes the HBM-streaming
regime the kernel runs in.  Fitted parameters are cached as JSON (the reference's DiskCache): key =
(W, Tv, Ti, Tu, device name, libvbc version, locality).

locality: "uniform" draws rows over all of x, exactly the reference's generator (costs.jl:63-83).  On
the GPU those matrices run the row-swept kernel, whose cost is the x gathers (one per stored row,
whatever the width), so the fitted model prices rows, not values, and its partitions trade fill for
fewer rows ('min blocks'-like: the ct20stif stand-in 25.7 us against 5.4 us for 'strict',
profiles/archive/r03_table_ct20stif.log).  It is the default, so the model is the reference's protocol
unchanged.  "banded" (opt-in) draws each stripe's rows from a window around its own position -- the
x locality of the mesh operators the table is run on -- so the fit sees the streaming kernels the
partition will actually run (tools/test_table.py passes both).
"""
import json
import os
from pathlib import Path

import numpy as np

from . import _lib as _L
from .partition import ColumnBlockCostModel

CACHE_DIR = Path(os.environ.get("VBC_AUTOTUNE_DIR", Path.home() / ".cache" / "sparsematrixvbcs_amd" / "autotune"))
LLC_BYTES = 256 * 2 ** 20  # MI355X Infinity Cache (MI355X_MICROARCH.md)


def _key(W, Tv, Ti, Tu, device, locality="uniform"):
    import torch
    name = torch.cuda.get_device_name(device).replace(" ", "_").replace("/", "_")
    return (f"1DVBC_TrSpMV_W{W}_{np.dtype(Tv).name}_{np.dtype(Ti).name}_{np.dtype(Tu).name}_{name}"
            f"_v{_L.lib().vbc_version()}_{locality}")


def model_SparseMatrix1DVBC_TrSpMV_time_data(W, Tv=np.float64, Ti=np.int64, Tu=np.float64, device=0, reps=20,
                                            llc_bytes=LLC_BYTES, seed=0xDEADBEEF, locality="uniform", band=4096):
    """Time the transposed product on the reference's random VBR matrices (costs.jl:14-99); with
    locality="banded" each stripe's rows come from a `band`-row window around it.
    Returns (ms, ns, Ls, ws, qs, T) with T in seconds (median kernel time over `reps`)."""
    import torch
    from .synthetic import vbr_1dvbc, vbr_1dvbc_banded
    if locality not in ("uniform", "banded"):
        raise ValueError("locality must be 'uniform' or 'banded'")
    from .multiply import mul_
    ms, ns, Ls, ws, qs, T = [], [], [], [], [], []
    isz, vsz, usz = np.dtype(Ti).itemsize, np.dtype(Tv).itemsize, np.dtype(Tu).itemsize
    d = 8
    for w in range(W, 0, -1):
        C = 2 * llc_bytes
        L0 = int(np.ceil(C / ((3 + d) * isz + 2 * w * usz + d * w * vsz)))
        m0 = L0 * w
        q0 = L0 * d
        for (m, L, q) in ((m0, L0, q0), (m0, 2 * L0, q0), (2 * m0, L0, q0), (m0, L0, 2 * q0)):
            sd = seed + w * 131 + L + q
            B = (vbr_1dvbc(m, L, q, w, W=W, dtype=Tv, seed=sd) if locality == "uniform" else
                 vbr_1dvbc_banded(m, L, q, w, band, W=W, dtype=Tv, seed=sd))
            x = torch.ones(B.m, dtype=torch.float64 if np.dtype(Tu) == np.float64 else torch.float32, device=device)
            y = torch.ones(B.n, dtype=x.dtype, device=device)
            for _ in range(3):
                mul_(y, B.T, x)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record()
                mul_(y, B.T, x)
                b.record()
            torch.cuda.synchronize(device)
            t = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e-3
            ms.append(m); ns.append(B.n); Ls.append(L); ws.append(w); qs.append(int(B.pos[-1] - 1)); T.append(t)
            B.release()
            print(f"[costs] 1DVBC time data ({locality}): w {w} m {m} L {L} q {q} t {t * 1e6:.1f} us", flush=True)  # costs.jl:91
    return ms, ns, Ls, ws, qs, T


def fit_time_params(W, ms, Ls, ws, qs, T):
    """costs.jl:101-136: rows [m, onehot_w(L), onehot_w(q)], weights 1/T, least squares against 1;
    alpha_col = per-stripe, beta_col = per-stored-row cost of width w, both made monotone in w."""
    D = np.zeros((len(T), 1 + 2 * W))
    for i in range(len(T)):
        D[i, 0] = ms[i]
        D[i, ws[i]] = Ls[i]
        D[i, W + ws[i]] = qs[i]
    Tm = np.asarray(T, dtype=np.float64)
    P, *_ = np.linalg.lstsq(D / Tm[:, None], np.ones(len(T)), rcond=None)
    alpha = P[1:1 + W].copy()
    beta = P[1 + W:].copy()
    for w in range(1, W):  # monotonize (costs.jl:124-128)
        alpha[w] = max(alpha[w], alpha[w - 1])
        beta[w] = max(beta[w], beta[w - 1])
    return float(P[0]), alpha, beta


def model_SparseMatrix1DVBC_TrSpMV_time(W, Tv=np.float64, Ti=np.int64, Tu=np.float64, device=0, refit=False,
                                        locality="uniform", **kwargs):
    """ColumnBlockCostModel(alpha, beta) of this GPU's transposed product (cached; costs.jl:12)."""
    CACHE_DIR.mkdir(parents=True, exist_ok=True)
    path = CACHE_DIR / (_key(W, Tv, Ti, Tu, device, locality) + ".json")
    if path.exists() and not refit:
        d = json.loads(path.read_text())
        return ColumnBlockCostModel(d["alpha"], d["beta"])
    ms, ns, Ls, ws, qs, T = model_SparseMatrix1DVBC_TrSpMV_time_data(W, Tv, Ti, Tu, device, locality=locality, **kwargs)
    a_row, alpha, beta = fit_time_params(W, ms, Ls, ws, qs, T)
    path.write_text(json.dumps({"W": W, "locality": locality, "alpha": alpha.tolist(), "beta": beta.tolist(), "alpha_row": a_row,
                                "data": {"m": ms, "n": ns, "L": Ls, "w": ws, "q": qs, "t": T}}, indent=1))
    return ColumnBlockCostModel(alpha, beta)


class TimedChunker:
    """Column partition chosen by timing: every candidate chunker's partition is built and its
    mul!(y, B', x) timed on the GPU (one HIP-graph replay of `reps` products); the fastest wins.

    The linear model above prices a stripe by its width and rows, but on the GPU the cost of a
    partition is set by the layouts its width buckets get (a planar bucket streams at ~0.8 of HBM
    peak, a bucket with chunks too long to balance falls back to the merge kernel at ~1/3 of that) and
    by how many launches they need -- neither is a per-stripe term.  On the ct20stif stand-in the
    fitted model's partition runs 28-36 us against 5.5 us for StrictChunker (profiles/archive/r03_table_*).
    Measuring the candidates is the GPU counterpart of the reference's autotuned 'min time' row.
    `timings` keeps (candidate index, us) of the last call."""

    def __init__(self, candidates, W, dtype=np.float64, device=0, reps=20):
        if not candidates:
            raise _L.ArgumentError("TimedChunker needs at least one candidate")
        self.candidates, self.W, self.dtype, self.device, self.reps = list(candidates), int(W), dtype, device, reps
        self.timings = []

    def partition(self, A):
        import torch
        from .partition import CSCFields
        F = A if isinstance(A, CSCFields) else CSCFields(A)
        m, n = F.shape
        dev = torch.device("cuda", self.device)
        tdt = torch.float64 if np.dtype(self.dtype) == np.float64 else torch.float32
        x = torch.ones(m, dtype=tdt, device=dev)
        y = torch.empty(n, dtype=tdt, device=dev)
        best, self.timings = None, []
        with torch.cuda.device(dev):
            for i, cand in enumerate(self.candidates):
                Phi, t = self._time_one(cand, F, x, y, dev)
                self.timings.append((i, round(t, 2)))
                if best is None or t < best[0]:
                    best = (t, Phi)
        return best[1]

    def _time_one(self, cand, F, x, y, dev):
        """The candidate's partition and its product time (us): one HIP-graph replay of `reps`
        products, median of 3 replays."""
        import torch
        from .matrices import SparseMatrix1DVBC
        from .multiply import mul_
        from .partition import pack_stripe
        Phi = pack_stripe(F, cand)
        B = SparseMatrix1DVBC.from_csc(self.W, F.A, Phi, dtype=self.dtype)
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for _ in range(3):
                mul_(y, B.T, x)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(self.reps):
                mul_(y, B.T, x)
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize(dev)
            ts.append(a.elapsed_time(b) * 1e3 / self.reps)
        del g
        B.release()
        return Phi, float(np.median(ts))


# --- SparseMatrixVBC: the 2D time model (costs.jl:142-290) ---------------------------------------
def _key2d(U, W, Tv, Ti, Tu, device):
    import torch
    name = torch.cuda.get_device_name(device).replace(" ", "_").replace("/", "_")
    return (f"VBC_TrSpMV_U{U}_W{W}_{np.dtype(Tv).name}_{np.dtype(Ti).name}_{np.dtype(Tu).name}_{name}"
            f"_v{_L.lib().vbc_version()}")


def model_SparseMatrixVBC_TrSpMV_time_data(U, W, Tv=np.float64, Ti=np.int64, Tu=np.float64, device=0, reps=10,
                                           llc_bytes=LLC_BYTES, seed=0xDEADBEEF):
    """costs.jl:144-247 on the GPU: for every block shape u = U..1, w = W..1 the reference's random 2D
    VBR matrices (costs.jl:200-220: q distinct (k, l) blocks, dense u x w tiles) in its four sizes
    (K0, L0, q0), (K0, L0/2, q0), (K0/2, L0, q0), (K0, L0, q0/2) -- its non-exceed branch, d = 8
    blocks per stripe, sized so the product's bytes are half the cache: here half the 256 MiB MALL,
    the level the GPU kernel streams from -- and mul!(y, B', x) timed (one HIP-graph replay of `reps`
    products).  Returns (ms, ns, Ks, Ls, us, ws, qs, T), T in seconds."""
    import torch
    from .multiply import mul_
    from .synthetic import vbr_2d
    isz, vsz, usz = np.dtype(Ti).itemsize, np.dtype(Tv).itemsize, np.dtype(Tu).itemsize
    tdt = torch.float64 if np.dtype(Tu) == np.float64 else torch.float32
    out = ([], [], [], [], [], [], [], [])
    d = 8
    C = llc_bytes / 2
    dev = torch.device("cuda", device)
    s = torch.cuda.Stream(dev)
    for u in range(U, 0, -1):
        for w in range(W, 0, -1):
            L0 = int(C // ((3 + d + w / u) * isz + 2 * w * usz + d * u * w * vsz))
            K0 = (L0 * w) // u
            q0 = L0 * d
            if L0 < 4 or K0 < 4:
                raise ValueError("cache too small for the generator (costs.jl:197-198)")
            for (K, L, q) in ((K0, L0, q0), (K0, L0 // 2, q0), (K0 // 2, L0, q0), (K0, L0, q0 // 2)):
                B = vbr_2d(K, L, q, u, w, U=U, W=W, dtype=Tv, seed=seed + 131 * u + 17 * w + K + L + q)
                x = torch.ones(B.m, dtype=tdt, device=dev)
                y = torch.ones(B.n, dtype=tdt, device=dev)
                with torch.cuda.stream(s):
                    for _ in range(3):
                        mul_(y, B.T, x)
                torch.cuda.synchronize(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(reps):
                        mul_(y, B.T, x)
                ts = []
                for _ in range(3):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    g.replay()
                    b.record()
                    torch.cuda.synchronize(dev)
                    ts.append(a.elapsed_time(b) * 1e-3 / reps)
                del g
                for lst, v in zip(out, (B.m, B.n, K, L, u, w, int(B.pos[-1] - 1), float(np.median(ts)))):
                    lst.append(v)
                B.release()
                print(f"[costs] VBC time data: u {u} w {w} K {K} L {L} q {q} t {np.median(ts) * 1e6:.1f} us",
                      flush=True)  # costs.jl:241
    return out


def fit_time_params_2d(R, U, W, Ks, Ls, us, ws, qs, T):
    """costs.jl:249-290: one-hot rows [K at u | L at w | q at (u, w)], weights 1/T, least squares
    against 1; β made monotone in u and w (:268-277); rank-R SVD of β: β_row[r] = U[:, r],
    β_col[r] = S[r]·V[:, r].  Returns (α_row (U), α_col (W), β_row (R tables), β_col (R tables), β)."""
    D = np.zeros((len(T), U + W + U * W))
    for i in range(len(T)):
        D[i, us[i] - 1] = Ks[i]
        D[i, U + ws[i] - 1] = Ls[i]
        D[i, U + W + (ws[i] - 1) * U + (us[i] - 1)] = qs[i]  # column-major reshape(β, :), costs.jl:260
    Tm = np.asarray(T, dtype=np.float64)
    P, *_ = np.linalg.lstsq(D / Tm[:, None], np.ones(len(T)), rcond=None)
    a_row, a_col = P[:U].copy(), P[U:U + W].copy()
    beta = P[U + W:].reshape(W, U).T.copy()  # β[u, w]
    for w in range(1, W):
        beta[0, w] = max(beta[0, w], beta[0, w - 1])
    for u in range(1, U):
        beta[u, 0] = max(beta[u, 0], beta[u - 1, 0])
        for w in range(1, W):
            beta[u, w] = max(beta[u, w], beta[u - 1, w - 1], beta[u, w - 1])
    Uf, S, Vt = np.linalg.svd(beta)
    b_row = tuple(Uf[:, r].copy() for r in range(R))
    b_col = tuple(S[r] * Vt[r, :] for r in range(R))
    return a_row, a_col, b_row, b_col, beta


def model_SparseMatrixVBC_TrSpMV_time(R, U, W, Tv=np.float64, Ti=np.int64, Tu=np.float64, device=0, refit=False,
                                      **kwargs):
    """BlockComponentCostModel(α_row, α_col, β_row, β_col) of this GPU's 2D transposed product, rank R
    (costs.jl:142); fitted once per (U, W, Tv, Ti, Tu, device, library version) and cached as JSON."""
    from .partition import BlockComponentCostModel
    CACHE_DIR.mkdir(parents=True, exist_ok=True)
    path = CACHE_DIR / (_key2d(U, W, Tv, Ti, Tu, device) + ".json")
    if path.exists() and not refit:
        dd = json.loads(path.read_text())
    else:
        ms, ns, Ks, Ls, us, ws, qs, T = model_SparseMatrixVBC_TrSpMV_time_data(U, W, Tv, Ti, Tu, device, **kwargs)
        a_row, a_col, _, _, beta = fit_time_params_2d(1, U, W, Ks, Ls, us, ws, qs, T)
        dd = {"U": U, "W": W, "alpha_row": a_row.tolist(), "alpha_col": a_col.tolist(), "beta": beta.tolist(),
              "data": {"m": ms, "n": ns, "K": Ks, "L": Ls, "u": us, "w": ws, "q": qs, "t": T}}
        path.write_text(json.dumps(dd, indent=1))
    beta = np.asarray(dd["beta"])
    Uf, S, Vt = np.linalg.svd(beta)
    R = min(R, len(S))
    return BlockComponentCostModel(np.asarray(dd["alpha_row"]), np.asarray(dd["alpha_col"]),
                                   tuple(Uf[:, r].copy() for r in range(R)),
                                   tuple(S[r] * Vt[r, :] for r in range(R)))
