"""Host-side rows of SURVEY.md §8f: Matrix Market input + built-layout cache (row 3), the TrSpMV time
cost model and its partitioner (row 4), and the SuiteSparse stand-ins of configs C2-C4."""
import itertools

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

import sparsematrixvbcs_amd as V
from oracle import oracle as O


def test_mdopen_reads_local_matrix_market(tmp_path):
    A = sp.random(40, 30, 0.2, format="csc", random_state=3)
    (tmp_path / "HB").mkdir()
    scipy.io.mmwrite(str(tmp_path / "HB" / "tiny.mtx"), A)
    d = V.io.mdopen("HB/tiny", root=tmp_path)
    assert d.A.shape == (40, 30) and (abs(d.A - A) > 0).nnz == 0
    S = sp.random(25, 25, 0.2, format="csc", random_state=4)
    S = sp.tril(S).tocsc()
    scipy.io.mmwrite(str(tmp_path / "sym.mtx"), S + sp.tril(S, -1).T, symmetry="symmetric")
    full = V.io.mdopen("sym", root=tmp_path).A
    assert (abs(full - full.T) > 0).nnz == 0 and full.nnz == (S + sp.tril(S, -1).T).nnz
    with pytest.raises(FileNotFoundError):
        V.io.mdopen("Boeing/ct20stif", root=tmp_path)


def test_built_layout_cache_roundtrip(tmp_path, golden):
    A = golden["HB__west0132"]["A"] if "HB__west0132" in golden else next(iter(golden.values()))["A"]
    for B in (V.SparseMatrix1DVBC[4](A, V.StrictChunker(4)),
              V.SparseMatrixVBC[4, 4](A, V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)))):
        p = tmp_path / f"{type(B).__name__}.npz"
        calls = []
        B1 = V.io.cached_build(lambda: calls.append(1) or B, p)
        B2 = V.io.cached_build(lambda: calls.append(1) or B, p)
        assert calls == [1]
        for f in ("pos", "idx", "ofs", "val"):
            assert np.array_equal(getattr(B1, f), getattr(B2, f))
        assert np.array_equal(B1.Phi.spl, B2.Phi.spl) and (B1.m, B1.n, B1.W) == (B2.m, B2.n, B2.W)


def test_memory_column_matches_reference_formula():
    """mem = sizeof(Φ) + sizeof(pos) + sizeof(idx) + sizeof(ofs) + sizeof(val) (test_table.jl:78), the
    partition counting its spl array: 24·(L+1) + 8·q + 8·|val| with the tail pad -- the form that
    reproduces src/ref.out (test_standins_pin_reference_memory_column)."""
    B = V.synthetic.vbr_1dvbc(100, 20, 60, 3, W=8, seed=1)
    L, q = len(B.Phi), int(B.pos[-1] - 1)
    assert V.io.memory_bytes(B) == 24 * (L + 1) + 8 * q + 8 * len(B.val)


@pytest.mark.parametrize("name", sorted(V.synthetic.STANDINS))
def test_standins_match_suitesparse_shape(name):
    n, nnz = V.synthetic.STANDINS[name]
    if n > 100000:
        pytest.skip("large stand-in: exercised by tools/test_table.py on the GPU box")
    A = V.synthetic.standin(name)
    assert A.shape == (n, n) and A.nnz == nnz  # exact: the CSC memory column is 8(n+1) + 16 nnz
    assert (abs(A - A.T) > 1e-15).nnz == 0


# src/ref.out, the reference's recorded bin/test_table.jl run (W = 8, Float64, Int64 indices):
# CSC memory ("nothing" rows), StrictChunker(8), OverlapChunker(0.9, 8), min blocks, min memory
REF_OUT = {
    "Boeing/ct20stif": dict(csc=42023360, strict=29974176, overlap=28093088, blocks=30507264, memory=27115424),
    "DIMACS10/chesapeake": dict(csc=5760, strict=6464, overlap=6160, blocks=7768, memory=5704),
    "Schmid/thermal1": dict(csc=9852568, strict=11175112, overlap=13472080, blocks=17858760, memory=10981032),
    "Rothberg/3dtube": dict(csc=51780536, strict=34914640, overlap=51962512, blocks=40732624, memory=34817632),
}


@pytest.mark.parametrize("name", sorted(REF_OUT))
def test_standins_pin_reference_memory_column(name):
    """the stand-ins reproduce the reference's own structural numbers.  The memory column
    of src/ref.out (ct20stif :37-45, chesapeake :68-76, thermal1 :120-128, 3dtube :169-177) depends on
    the structure only for StrictChunker (identical-pattern runs) and for the optimal min-memory
    partition (a unique optimum value): the CSC figure must be exact, StrictChunker(8) within 1 %,
    min memory within 2 %.  OverlapChunker and min blocks depend on the partitioner (ChainPartitioners'
    overlap rule and tie-breaking, absent here) and are reported, not asserted."""
    ref = REF_OUT[name]
    A = V.synthetic.standin(name).T.tocsc()  # permutedims, bin/test_table.jl:27
    assert 8 * (A.shape[1] + 1) + 16 * A.nnz == ref["csc"]
    lim = V.ConstrainedCost(V.model_SparseMatrix1DVBC_memory(np.float64, np.int64), V.VertexCount(), 8)
    strict = V.io.memory_bytes(V.SparseMatrix1DVBC[8](A, V.StrictChunker(8)))
    memory = V.io.memory_bytes(V.SparseMatrix1DVBC[8](A, V.DynamicTotalChunker(lim)))
    assert abs(strict / ref["strict"] - 1) <= 0.01, (strict, ref["strict"])
    assert abs(memory / ref["memory"] - 1) <= 0.02, (memory, ref["memory"])
    assert memory <= strict  # the optimum never loses to a feasible partition


def test_overlap_chunker_rules_against_ref_out(capsys):
    """which greedy OverlapChunker(0.9, 8) rule reproduces src/ref.out's `overlap` memory
    column (ct20stif :42, thermal1 :125, chesapeake :73; 3dtube :174 runs in tools/overlap_rules.py) on the
    stand-ins pinned by their strict / min-memory columns?  Every rule (overlap against the stripe's first
    column, its running union or the previous column; max / min / Jaccard normalisation) is run and its
    ratio to the recorded memory reported.  Finding: all nine rules land within 0.3 % of each
    other and none reproduces ref.out (ct20stif 0.964, thermal1 0.83, 3dtube 0.67, chesapeake 1.05): the
    stand-ins' near-identical column pairs merge under every rule, while the reference's partition of the
    real matrices put 20-50 % more fill in its stripes -- a property of the real column patterns the
    stand-ins do not carry, so OverlapChunker's rule stays unpinned and the library keeps `first / max`."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from tools import overlap_rules as R
    ratios = {}
    for key in ("chesapeake", "thermal1", "ct20stif"):
        A = V.synthetic.standin(R.NAMES[key]).T.tocsc()
        for target, norm in R.RULES:
            spl = R.overlap_split(A, 0.9, 8, target, norm)
            mem = V.io.memory_bytes(V.SparseMatrix1DVBC[8](A, V.SplitPartition(spl)))
            ratios[(key, target, norm)] = mem / R.REF_OVERLAP[key]
        # the library's OverlapChunker is the `first / max` rule
        lib = V.io.memory_bytes(V.SparseMatrix1DVBC[8](A, V.OverlapChunker(0.9, 8)))
        assert lib == round(ratios[(key, "first", "max")] * R.REF_OVERLAP[key])
    with capsys.disabled():
        for (key, t, nrm), r in sorted(ratios.items()):
            print(f"overlap rule {key:10s} {t:6s} {nrm:8s} memory / ref.out {r:.3f}")
    for key in ("thermal1", "ct20stif"):  # no rule comes within 2 % of the recorded memory
        assert all(abs(r - 1) > 0.02 for (k, _, _), r in ratios.items() if k == key)


def _brute_force_best(A, W, alpha, beta):
    m, n = A.shape
    A = A.tocsc()
    best = (np.inf, None)
    for cuts in itertools.product([0, 1], repeat=n - 1):
        spl = [0] + [j + 1 for j, c in enumerate(cuts) if c] + [n]
        if max(np.diff(spl)) > W:
            continue
        cost = 0.0
        for a, b in zip(spl[:-1], spl[1:]):
            rows = np.unique(A[:, a:b].indices).size
            cost += alpha[b - a - 1] + beta[b - a - 1] * rows
        if cost < best[0] - 1e-12:
            best = (cost, spl)
    return best


def test_time_model_partitioner_is_optimal():
    rng = np.random.default_rng(7)
    for trial in range(6):
        A = sp.random(12, 9, 0.3, format="csc", random_state=trial)
        W = 4
        alpha = np.sort(rng.uniform(1, 3, W))
        beta = np.sort(rng.uniform(0.1, 1, W))
        P = V.DynamicTotalChunker(V.ConstrainedCost(V.ColumnBlockCostModel(alpha, beta), V.VertexCount(), W)).partition(A)
        spl = P.spl - 1
        cost = sum(alpha[b - a - 1] + beta[b - a - 1] * np.unique(A[:, a:b].indices).size
                   for a, b in zip(spl[:-1], spl[1:]))
        best, _ = _brute_force_best(A, W, alpha, beta)
        assert abs(cost - best) < 1e-9


def test_time_model_fit_recovers_parameters():
    """costs.jl:101-136 restated: exact synthetic timings t = a_row*m + alpha_w*L + beta_w*q are
    recovered by the weighted least squares, then monotonized."""
    W = 4
    a_row, alpha, beta = 1e-9, np.array([2e-9, 3e-9, 3.5e-9, 5e-9]), np.array([1e-9, 1.5e-9, 2.5e-9, 3e-9])
    ms, Ls, ws, qs, T = [], [], [], [], []
    for w in range(W, 0, -1):
        for (m, L, q) in ((1000, 100, 800), (1000, 200, 800), (2000, 100, 800), (1000, 100, 1600)):
            ms.append(m); Ls.append(L); ws.append(w); qs.append(q)
            T.append(a_row * m + alpha[w - 1] * L + beta[w - 1] * q)
    r, a, b = V.costs.fit_time_params(W, ms, Ls, ws, qs, T)
    assert np.allclose(a, alpha, rtol=1e-6) and np.allclose(b, beta, rtol=1e-6) and abs(r - a_row) < 1e-15


def test_banded_generator_keeps_rows_near_their_stripe():
    """The banded VBR generator of the GPU time-model fit (costs.py, locality="banded"): distinct
    ascending rows per stripe, every row within `band` of the stripe's scaled position, a valid
    1DVBC (the oracle's product equals scipy's on the same matrix)."""
    B = V.synthetic.vbr_1dvbc_banded(50000, 3000, 20000, np.arange(3000) % 4 + 1, 1000, W=4, seed=7)
    st = np.repeat(np.arange(3000), np.diff(B.pos))
    rows = B.idx - 1
    assert np.all(np.abs(rows - st * 50000 // 3000) <= 1000)
    for l in range(0, 3000, 97):
        r = rows[B.pos[l] - 1:B.pos[l + 1] - 1]
        assert np.all(np.diff(r) > 0)
    x = np.random.default_rng(2).uniform(-1, 1, B.m)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    y = O.mul(R, x, np.zeros(B.n), trans=True)
    import scipy.sparse as sp
    w = np.diff(B.Phi.spl)
    cnt = np.diff(B.pos)
    wr = np.repeat(w, cnt)  # width of each stored row
    I = np.repeat(rows, wr)
    col0 = np.repeat(B.Phi.spl[:-1] - 1, cnt)
    J = np.concatenate([c + np.arange(k) for c, k in zip(col0, wr)])
    A = sp.csc_matrix((B.val[:int(B.ofs[-1] - 1)], (I, J)), shape=(B.m, B.n))
    assert np.allclose(y, A.T @ x, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_gpu_time_model_fit(tmp_path, monkeypatch):
    """The model fitted to the GPU kernel (small sizes) is positive, monotone and cached; its
    partition builds a matrix whose product matches the oracle."""
    monkeypatch.setattr(V.costs, "CACHE_DIR", tmp_path)
    mdl = V.model_SparseMatrix1DVBC_TrSpMV_time(4, np.float64, np.int64, np.float64, llc_bytes=2 ** 22, reps=5)
    assert (mdl.alpha >= 0).all() and (np.diff(mdl.alpha) >= 0).all() and (np.diff(mdl.beta) >= 0).all()
    assert list(tmp_path.glob("*.json"))
    A = V.synthetic.standin("Boeing/ct20stif")
    B = V.SparseMatrix1DVBC[4](A, V.DynamicTotalChunker(V.ConstrainedCost(mdl, V.VertexCount(), 4)))
    import torch
    x = np.random.default_rng(1).random(B.m)
    y = torch.empty(B.n, dtype=torch.float64, device="cuda:0")
    V.mul_(y, B.T, torch.from_numpy(x).cuda())
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    yr = O.mul(R, x, np.zeros(B.n), trans=True, nthreads=8)
    assert np.linalg.norm(y.cpu().numpy() - yr) <= 1e-12 * np.linalg.norm(yr)


@pytest.mark.gpu
def test_library_loaded_before_torch_shares_its_runtime():
    """Host calls first (libvbc loaded before torch is imported), then GPU work through torch and
    libvbc in the same process: one HIP runtime (see _lib.lib)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, scipy.sparse as sp\n"
            "import sparsematrixvbcs_amd as V\n"
            "A = sp.random(50, 40, 0.1, format='csc', random_state=0)\n"
            "V.StrictChunker(4).partition(A)\n"
            "import torch\n"
            "B = V.SparseMatrix1DVBC[4](A, V.StrictChunker(4))\n"
            "x = torch.rand(50, dtype=torch.float64, device='cuda')\n"
            "y = V.mul_(torch.empty(40, dtype=torch.float64, device='cuda'), B.T, x)\n"
            "assert torch.allclose(y.cpu(), torch.from_numpy(A.T @ x.cpu().numpy()))\n"
            "print('ok')\n") % str(V._lib.PKG_DIR.parent)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


@pytest.mark.gpu
def test_timed_chunker_picks_the_fastest_candidate():
    """TimedChunker builds every candidate partition, times its product on the GPU and returns the
    fastest; the matrix built from it multiplies like the oracle.  On the ct20stif stand-in the
    'min blocks' partition (w = 6 stripes with fill, the merge kernel) is slower than 'strict'."""
    import torch
    A = V.synthetic.standin("Boeing/ct20stif").T.tocsc()
    lim = V.ConstrainedCost(V.model_SparseMatrix1DVBC_blocks(), V.VertexCount(), 8)
    tc = V.TimedChunker([V.DynamicTotalChunker(lim), V.StrictChunker(8)], 8)
    B = V.SparseMatrix1DVBC[8](A, tc)
    (i0, t0), (i1, t1) = tc.timings
    assert (i0, i1) == (0, 1) and t0 > 0 and t1 > 0
    S = V.SparseMatrix1DVBC[8](A, V.StrictChunker(8))
    assert np.array_equal(B.Phi.spl, S.Phi.spl) == (t1 < t0)
    x = np.random.default_rng(3).uniform(-1, 1, B.m)
    y = torch.empty(B.n, dtype=torch.float64, device="cuda:0")
    V.mul_(y, B.T, torch.from_numpy(x).cuda())
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    yr = O.mul(R, x, np.zeros(B.n), trans=True, nthreads=8)
    assert np.linalg.norm(y.cpu().numpy() - yr) <= 1e-12 * np.linalg.norm(yr)


def _model_cost_cols(A, groups_spl, col_spl, mdl):
    """Σ_l α_col(w_l) + Σ over the (block row, stripe) blocks A stores of β(u, w), by brute force."""
    u = np.diff(groups_spl)
    grp = np.repeat(np.arange(len(u)), u)
    A = A.tocsc()
    cost = 0.0
    for a, b in zip(col_spl[:-1] - 1, col_spl[1:] - 1):
        w = b - a
        cost += float(V.partition._eval_component(mdl.alpha_col, [w])[0])
        for g in np.unique(grp[A[:, a:b].indices]):
            cost += float(mdl.block_cost([u[g]], [w])[0])
    return cost


def _brute_best_cols(A, groups_spl, W, mdl):
    n = A.shape[1]
    best = np.inf
    for cuts in itertools.product([0, 1], repeat=n - 1):
        spl = np.array([0] + [j + 1 for j, c in enumerate(cuts) if c] + [n]) + 1
        if max(np.diff(spl)) > W:
            continue
        best = min(best, _model_cost_cols(A, groups_spl, spl, mdl))
    return best


@pytest.mark.parametrize("model", ["memory", "blocks", "random"])
def test_block_model_partitioner_is_optimal(model):
    """DynamicTotalChunker over the SparseMatrixVBC cost models (costs.jl:138-140) given a row
    partition Π is optimal: brute force over every column partition of width <= W on small matrices,
    for the model and -- on Aᵀ with the columns grouped by a Φ -- its permutedims."""
    rng = np.random.default_rng(17)
    for trial in range(5):
        A = sp.random(11, 9, 0.3, format="csc", random_state=40 + trial)
        W = 3
        if model == "memory":
            mdl = V.model_SparseMatrixVBC_memory(np.float64, np.int64)
        elif model == "blocks":
            mdl = V.model_SparseMatrixVBC_blocks()
        else:  # a rank-2 table model like the fitted time model (costs.jl:264-281)
            mdl = V.BlockComponentCostModel(rng.uniform(0, 2, 4), rng.uniform(0, 2, 4),
                                            (rng.uniform(0, 1, 4), rng.uniform(0, 1, 4)),
                                            (rng.uniform(0, 1, 4), rng.uniform(0, 1, 4)))
        Pi = np.concatenate([[1], 1 + np.cumsum(rng.integers(1, 4, 11))])
        Pi = V.SplitPartition(np.concatenate([Pi[Pi <= 11], [12]]))
        Phi = V.DynamicTotalChunker(V.ConstrainedCost(mdl, V.VertexCount(), W)).partition(A, Pi)
        assert np.diff(Phi.spl).max() <= W
        got = _model_cost_cols(A, Pi.spl, Phi.spl, mdl)
        assert abs(got - _brute_best_cols(A, Pi.spl, W, mdl)) < 1e-9
        # the row phase: permutedims(model) on Aᵀ with A's columns grouped by Φ
        At = A.T.tocsc()
        Pm = V.permutedims(mdl)
        Pi2 = V.DynamicTotalChunker(V.ConstrainedCost(Pm, V.VertexCount(), W)).partition(At, Phi)
        got = _model_cost_cols(At, Phi.spl, Pi2.spl, Pm)
        assert abs(got - _brute_best_cols(At, Phi.spl, W, Pm)) < 1e-9


def test_alternating_packer_phases():
    """Odd phases partition the columns given Π, even phases the rows given Φ (constructors_VBC.jl:1-8,
    bin/test_table.jl:88-111): "1D 2D" = the 1D min-blocks stripes with unit block rows; the 2D
    default packer's last Φ is optimal for the 2D memory model given its last Π; the memory column
    of a SparseMatrixVBC equals the model's total (costs.jl:140 counts exactly the stored arrays)."""
    A = sp.random(60, 50, 0.08, format="csc", random_state=3)
    lim = lambda mdl, W: V.ConstrainedCost(mdl, V.VertexCount(), W)
    Pi, Phi = V.pack_plaid(A, V.AlternatingPacker(V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks(), 4)),
                                                  V.EquiChunker(1)))
    assert len(Pi) == 60 and Phi == V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks(), 4)).partition(A)
    B = V.SparseMatrixVBC[4, 4](A)  # the default 5-phase packer
    mdl = V.model_SparseMatrixVBC_memory(np.float64, np.int64)
    assert np.diff(B.Pi.spl).max() <= 4 and np.diff(B.Phi.spl).max() <= 4
    # Φ (phase 5) is optimal for the model given Π (phase 4)
    again = V.DynamicTotalChunker(lim(mdl, 4)).partition(A, B.Pi)
    assert _model_cost_cols(A, B.Pi.spl, B.Phi.spl, mdl) <= _model_cost_cols(A, B.Pi.spl, again.spl, mdl) + 1e-9
    # memory bytes = the model's total + the value tail pad (the reference counts sizeof of every array)
    pad = len(B.val) - int(B.ofs[-1] - 1)
    assert V.io.memory_bytes(B) == V.total_value_2d(B, mdl) + 8 * pad + 8 * 4  # + Φ.spl, pos, ofs, Π.spl end entries
    S = V.SparseMatrixVBC[4, 4](A, V.AlternatingPacker(V.StrictChunker(4), V.StrictChunker(4)))
    assert V.io.memory_bytes(B) <= V.io.memory_bytes(S) + 8 * 64


def test_1dvbc_default_uses_matrix_eltype():
    """constructors_1DVBC.jl:1-2: the default partitioner is the memory model of the matrix's own Tv:
    a Float32 matrix trades fill at 4 bytes per value, not 8."""
    A = sp.random(300, 240, 0.04, format="csc", random_state=9)
    for dt in (np.float64, np.float32):
        B = V.SparseMatrix1DVBC[8](A.astype(dt))
        want = V.DynamicTotalChunker(V.model_SparseMatrix1DVBC_memory(dt, np.int64), 8).partition(A)
        assert B.Phi == want


def test_time_model_2d_fit_recovers_parameters():
    """costs.jl:249-290 restated: exact timings t = α_row[u]·K + α_col[w]·L + β[u,w]·q on the
    reference's four sizes per block shape are recovered by the weighted least squares; a rank-U SVD
    reconstructs β exactly, and the model's block cost is Σ_r β_row[r][u]·β_col[r][w]."""
    U = W = 3
    rng = np.random.default_rng(5)
    a_row, a_col = rng.uniform(1, 2, U) * 1e-9, rng.uniform(1, 2, W) * 1e-9
    beta = np.add.outer(np.arange(1, U + 1), np.arange(1, W + 1)) * 1e-9  # monotone in u and w
    Ks, Ls, us, ws, qs, T = [], [], [], [], [], []
    for u in range(U, 0, -1):
        for w in range(W, 0, -1):
            L0 = 1000 + 37 * w
            K0 = L0 * w // u
            q0 = 8 * L0
            for (K, L, q) in ((K0, L0, q0), (K0, L0 // 2, q0), (K0 // 2, L0, q0), (K0, L0, q0 // 2)):
                Ks.append(K); Ls.append(L); us.append(u); ws.append(w); qs.append(q)
                T.append(a_row[u - 1] * K + a_col[w - 1] * L + beta[u - 1, w - 1] * q)
    ar, ac, br, bc, b = V.costs.fit_time_params_2d(U, U, W, Ks, Ls, us, ws, qs, T)
    assert np.allclose(b, beta, rtol=1e-6)
    mdl = V.BlockComponentCostModel(ar, ac, br, bc)
    for u in range(1, U + 1):
        for w in range(1, W + 1):
            assert np.isclose(mdl.block_cost([u], [w])[0], beta[u - 1, w - 1], rtol=1e-6)


def test_mesh_vbc_generator_equals_strict_2d_packer():
    """synthetic.fe_stiffness_3d_vbc (the structured C5 input, bench workload c5-mesh) builds exactly
    the SparseMatrixVBC that AlternatingPacker(StrictChunker(8), StrictChunker(8)) makes of the same
    stiffness matrix (constructors_VBC.jl:15-133 via the oracle's builder): 3 x 3 node tiles."""
    n, nnz = 3000, 120000
    A = V.synthetic.fe_stiffness_3d(n, nnz, 3, np.float64, seed=7)
    Bd = V.synthetic.fe_stiffness_3d_vbc(n, nnz, 3, dtype=np.float64, seed=7)
    Bp = V.SparseMatrixVBC[8, 8](A, V.AlternatingPacker(V.StrictChunker(8), V.StrictChunker(8)))
    assert Bd.Pi == Bp.Pi and Bd.Phi == Bp.Phi
    for f in ("pos", "idx", "ofs"):
        assert np.array_equal(getattr(Bd, f), getattr(Bp, f)), f
    nv = int(Bd.ofs[-1] - 1)
    assert np.array_equal(Bd.val[:nv], Bp.val[:nv])
    R = O.RefVBC(Bd.m, Bd.n, Bd.U, Bd.W, Bd.Pi.spl, Bd.Phi.spl, Bd.pos, Bd.idx, Bd.ofs, Bd.val)
    x = np.random.default_rng(1).uniform(-1, 1, n)
    assert np.allclose(O.mul(R, x, np.zeros(n), trans=True), A.T @ x, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_gpu_products_from_2d_model_partitions(golden):
    """products built from the SparseMatrixVBC cost-model partitions -- the reference's
    default 5-phase memory packer (constructors_VBC.jl:1-8) and the "dynamic blocks 2D" / "dynamic
    memory 2D" rows of bin/test_table.jl:94-104 -- match the oracle on the GPU, both directions, on the
    reference corpus and the ct20stif stand-in."""
    import torch
    lim = lambda mdl, W: V.ConstrainedCost(mdl, V.VertexCount(), W)
    b2, m2 = V.model_SparseMatrixVBC_blocks(), V.model_SparseMatrixVBC_memory(np.float64, np.int64)
    packers = [None,
               V.AlternatingPacker(V.DynamicTotalChunker(lim(V.model_SparseMatrix1DVBC_blocks(), 4)),
                                   V.DynamicTotalChunker(lim(V.permutedims(b2), 4)), V.DynamicTotalChunker(lim(b2, 4))),
               V.AlternatingPacker(V.EquiChunker(1), V.EquiChunker(1), V.DynamicTotalChunker(lim(m2, 4)),
                                   V.DynamicTotalChunker(lim(V.permutedims(m2), 4)), V.DynamicTotalChunker(lim(m2, 4)))]
    mats = [g["A"] for g in golden.values()] + [V.synthetic.standin("Boeing/ct20stif").T.tocsc()]
    rng = np.random.default_rng(8)
    for A in mats:
        for pk in packers:
            B = V.SparseMatrixVBC[4, 4](A) if pk is None else V.SparseMatrixVBC[4, 4](A, pk)
            R = O.RefVBC(B.m, B.n, B.U, B.W, B.Pi.spl, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
            for trans in (True, False):
                nx, ny = (B.m, B.n) if trans else (B.n, B.m)
                x = rng.uniform(-1, 1, nx)
                y = torch.zeros(ny, dtype=torch.float64, device="cuda:0")
                V.mul_(y, B.T if trans else B, torch.from_numpy(x).cuda())
                ref = O.mul(R, x, np.zeros(ny), trans=trans)
                assert np.linalg.norm(y.cpu().numpy() - ref) <= 1e-12 * max(np.linalg.norm(ref), 1e-300)
            B.release()
