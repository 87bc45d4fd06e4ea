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


def make_matrix():
    w = np.arange(60) % 5 + 1
    return V.synthetic.vbr_1dvbc(500, 60, 700, w, W=8, seed=7)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        B = make_matrix()
        S = V.distributed.ShardedSparseMatrix1DVBC(B, rank, world, local_mul=oracle_mul)
        rng = np.random.default_rng(3)
        xt = torch.from_numpy(rng.uniform(-1, 1, B.m))
        xf = torch.from_numpy(rng.uniform(-1, 1, B.n))
        y0 = torch.from_numpy(rng.uniform(-1, 1, B.m))
        yl = torch.zeros(S.n_local, dtype=torch.float64)
        S.mul_t(yl, xt)
        yt = S.gather(yl)
        yf = y0.clone()
        S.mul(yf, xf, 2.0, 0.5)
        q.put((rank, yt.numpy(), yf.numpy(), S.cuts.tolist(), S.n_local))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the parent
        q.put((rank, repr(e)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_products_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 5, r
    B = make_matrix()
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(3)
    xt, xf, y0 = rng.uniform(-1, 1, B.m), rng.uniform(-1, 1, B.n), rng.uniform(-1, 1, B.m)
    ref_t = O.mul(R, xt, np.zeros(B.n), trans=True)
    ref_f = O.mul(R, xf, y0.copy(), 2.0, 0.5, ref_semantics=False)
    for rank, yt, yf, cuts, nloc in res:
        assert np.array_equal(yt, ref_t)            # disjoint slices: same per-stripe arithmetic
        assert np.allclose(yf, ref_f, rtol=1e-13, atol=1e-13)
    assert sum(r[4] for r in res) == B.n


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
            vals.append(S.val)
            idxs.append(S.idx)
            assert col0 == B.Phi.spl[cuts[p]] - 1
        assert np.array_equal(np.concatenate(vals), B.val[:B.ofs[-1] - 1])
        assert np.array_equal(np.concatenate(idxs), B.idx)
        assert max(share) <= 1.02 * sum(share) / parts + 64 * 40
