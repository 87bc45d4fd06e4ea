"""Multi-process (world_size 2, gloo, CPU) tests of the stripe-sharded products.

The per-rank product is the oracle here (the GPU path has no CPU fallback); what is under test is
the sharding, the byte balance and the collective assembly (all_gather for B'x, all_reduce for Bx).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sparsematrixvbcs_amd as V
from oracle import oracle as O


def oracle_mul(y, op, x, alpha, beta):
    trans = isinstance(op, V.Adjoint)
    B = op.parent if trans else op
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    yn = y.numpy()
    O.mul(R, np.ascontiguousarray(x.numpy()), yn, alpha, beta, trans=trans, ref_semantics=False)
    return y


def make_matrix(kind="random"):
    if kind == "mesh":  # a 3D stiffness operator: every shard touches its own rows / columns plus a halo
        return V.SparseMatrix1DVBC[8](V.synthetic.fe_stiffness_3d(3000, 60000), V.StrictChunker(8))
    w = np.arange(60) % 5 + 1
    return V.synthetic.vbr_1dvbc(500, 60, 700, w, W=8, seed=7)


def _worker(rank, world, port, q, split, kind="random"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        B = make_matrix(kind)
        S = V.distributed.ShardedSparseMatrix1DVBC(B, rank, world, local_mul=oracle_mul, split=split)
        rng = np.random.default_rng(3)
        xt = torch.from_numpy(rng.uniform(-1, 1, B.m))
        xf = torch.from_numpy(rng.uniform(-1, 1, B.n))
        y0 = torch.from_numpy(rng.uniform(-1, 1, B.m))
        y0t = torch.from_numpy(rng.uniform(-1, 1, B.n))
        yt = y0t.clone()
        S.mul_t(yt, xt, 1.5, 0.25)
        yf = y0.clone()
        S.mul(yf, xf, 2.0, 0.5)
        # the collective-free halves
        if split == "stripes":
            yl = torch.zeros(S.n_local, dtype=torch.float64)
            S.local_mul_t(yl, xt)
        else:
            yl = torch.zeros(S.m_local, dtype=torch.float64)
            S.local_mul(yl, xf)
        q.put((rank, yt.numpy(), yf.numpy(), yl.numpy(), S.cuts.tolist(), S.n_local, S.m_local, S.col0, S.row0))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put((rank, traceback.format_exc()))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("split", ["stripes", "rows"])
@pytest.mark.parametrize("kind", ["random", "mesh"])
def test_sharded_products_world2(split, kind):
    """Both splits, both directions, world 2 over gloo (the oracle as each rank's product).  On the mesh
    operator the local handles are rebased to the rows (stripe split) / trimmed to the columns (row split)
    their shard touches, and the partial-output products still sum to the oracle's."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, split, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 9, r
    B = make_matrix(kind)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(3)
    xt, xf, y0 = rng.uniform(-1, 1, B.m), rng.uniform(-1, 1, B.n), rng.uniform(-1, 1, B.m)
    y0t = rng.uniform(-1, 1, B.n)
    ref_t = O.mul(R, xt, y0t.copy(), 1.5, 0.25, trans=True, ref_semantics=False)
    ref_t1 = O.mul(R, xt, np.zeros(B.n), trans=True)
    ref_f = O.mul(R, xf, y0.copy(), 2.0, 0.5, ref_semantics=False)
    ref_f1 = O.mul(R, xf, np.zeros(B.m), ref_semantics=False)
    for rank, yt, yf, yl, cuts, nloc, mloc, col0, row0 in res:
        assert np.allclose(yt, ref_t, rtol=1e-13, atol=1e-13)
        assert np.allclose(yf, ref_f, rtol=1e-13, atol=1e-13)
        if split == "stripes":   # disjoint y columns: the same per-stripe arithmetic, bit for bit
            assert np.array_equal(yt, ref_t)
            assert np.array_equal(yl, ref_t1[col0:col0 + nloc])
        else:                    # disjoint y rows of the forward product
            assert np.allclose(yl, ref_f1[row0:row0 + mloc], rtol=1e-13, atol=1e-13)
    if split == "stripes":
        assert sum(r[5] for r in res) == B.n
    else:
        assert sum(r[6] for r in res) == B.m
    if kind == "mesh":  # the other dimension is rebased / trimmed to what each shard touches
        assert all((r[6] < B.m) if split == "stripes" else (r[5] < B.n) for r in res), [r[5:] for r in res]


def test_row_split_reassembly():
    """Row shards partition the stored rows: the shards' dense forms stack to B's."""
    B = make_matrix()
    D = O.vbc_to_dense(O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val))
    for parts in (1, 2, 3, 7):
        cuts = V.distributed.row_split(B, parts)
        assert cuts[0] == 0 and cuts[-1] == B.m and np.all(np.diff(cuts) >= 0)
        blocks = []
        for p in range(parts):
            S = V.distributed.row_shard(B, int(cuts[p]), int(cuts[p + 1]))
            blocks.append(O.vbc_to_dense(O.Ref1DVBC(S.m, S.n, S.W, S.Phi.spl, S.pos, S.idx, S.ofs, S.val)))
        assert np.array_equal(np.vstack(blocks), D)


def test_stripe_split_balance_and_reassembly():
    B = V.synthetic.north_star(scale=0.002)
    for parts in (1, 2, 3, 8):
        cuts = V.distributed.stripe_split(B, parts)
        assert cuts[0] == 0 and cuts[-1] == len(B.Phi) and np.all(np.diff(cuts) >= 0)
        esz = B.val.dtype.itemsize
        share = []
        vals, idxs = [], []
        for p in range(parts):
            S, col0 = V.distributed.shard(B, int(cuts[p]), int(cuts[p + 1]))
            share.append(len(S.val) * esz + len(S.idx) * 4)
            vals.append(S.val[:S.ofs[-1] - 1])
            idxs.append(S.idx)
            assert col0 == B.Phi.spl[cuts[p]] - 1
        assert np.array_equal(np.concatenate(vals), B.val[:B.ofs[-1] - 1])
        assert np.array_equal(np.concatenate(idxs), B.idx)
        assert max(share) <= 1.02 * sum(share) / parts + 64 * 40


def test_split_cost_model_and_auto_choice():
    """distributed.predict_product_us / choose_split: a disjoint output needs no collective
    (an all-gather when y is replicated), a partial output one all-reduce; the automatic split makes the
    requested direction disjoint (forward only -> rows, transposed only -> stripes), ties go to stripes."""
    D = V.distributed
    B = V.synthetic.standin("GHS_psdef/ldoor", scale=0.01).T.tocsc()
    B = V.SparseMatrix1DVBC[8](B, V.StrictChunker(8))
    for world in (2, 4, 8):
        t_s, k_s, c_s = D.predict_product_us(B, world, "stripes", trans=True, replicate=False)
        t_r, k_r, c_r = D.predict_product_us(B, world, "rows", trans=True, replicate=False)
        assert c_s == 0.0 and c_r > 0.0 and t_s < t_r
        f_s = D.predict_product_us(B, world, "stripes", trans=False)
        f_r = D.predict_product_us(B, world, "rows", trans=False)
        assert f_s[2] > f_r[2] > 0.0  # all-reduce vs all-gather of the replicated y
        assert D.choose_split(B, world, "f") == "rows"
        assert D.choose_split(B, world, "t") == "stripes"
        assert D.choose_split(B, world, "tf") == "stripes"
    assert D.predict_product_us(B, 1, "stripes", True)[2] == 0.0
    # the collective model: all-reduce of 7.6 MB over 8 GPUs, the assumption stated in the module
    ar = D.collective_us("allreduce", 7_617_624, 8)
    assert abs(ar - (2 * 7 / 8 * 7_617_624 / (D.COLL_GBS * 1e3) + 14 * D.COLL_STEP_US)) < 1e-9
    S = D.ShardedSparseMatrix1DVBC(B, 0, 4, split="auto", directions="f", local_mul=lambda *a: None)
    assert S.split == "rows"
    S = D.ShardedSparseMatrix1DVBC(B, 0, 4, split="auto", directions="t", local_mul=lambda *a: None)
    assert S.split == "stripes"
