"""The sharded products with libvbc doing every rank's product on the GPU (config C3's block-row
split): two ranks, one process each, both on cuda:0 (the box has one GPU), gloo process
group with the collectives on host copies (comm="cpu"); checked against the CPU oracle.

Stripe split: B'x (disjoint y slices, no collective; then all_gather) and Bx (all_reduce of partial y).
Row split: Bx (disjoint y rows; then all_gather) and B'x (all_reduce).  Matrices: a mixed-width
synthetic VBR and the GHS_psdef/ldoor stand-in (C3).
"""
import os
import socket

import numpy as np
import pytest

import sparsematrixvbcs_amd as V
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def make(kind):
    if kind == "vbr":
        return V.synthetic.vbr_1dvbc(20000, 3000, 60000, np.arange(3000) % 8 + 1, W=8, seed=11)
    A = V.synthetic.standin("GHS_psdef/ldoor")
    return V.SparseMatrix1DVBC[8](A.T.tocsc(), V.StrictChunker(8))


def _worker(rank, world, port, q, kind, split):
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        B = make(kind)
        S = V.distributed.ShardedSparseMatrix1DVBC(B, rank, world, split=split, comm="cpu")
        rng = np.random.default_rng(3)
        xt = torch.from_numpy(rng.uniform(-1, 1, B.m)).cuda()
        xf = torch.from_numpy(rng.uniform(-1, 1, B.n)).cuda()
        y0 = rng.uniform(-1, 1, B.m)
        yt = torch.zeros(B.n, dtype=torch.float64, device="cuda")
        S.mul_t(yt, xt)
        yf = torch.from_numpy(y0).cuda()
        S.mul(yf, xf, 2.0, 0.5)
        if split == "stripes":
            yl = torch.zeros(S.n_local, dtype=torch.float64, device="cuda")
            S.local_mul_t(yl, xt)
        else:
            yl = torch.zeros(S.m_local, dtype=torch.float64, device="cuda")
            S.local_mul(yl, xf)
        torch.cuda.synchronize()
        q.put((rank, yt.cpu().numpy(), yf.cpu().numpy(), yl.cpu().numpy(), S.col0, S.row0, S.n_local, S.m_local))
        S.local.release()
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("kind,split", [("vbr", "stripes"), ("vbr", "rows"), ("ldoor", "stripes")])
def test_sharded_gpu_products_world2(kind, split):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind, split)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in res:
        assert len(r) == 8, r[1]
    B = make(kind)
    R = O.Ref1DVBC(B.m, B.n, B.W, B.Phi.spl, B.pos, B.idx, B.ofs, B.val)
    rng = np.random.default_rng(3)
    xt, xf, y0 = rng.uniform(-1, 1, B.m), rng.uniform(-1, 1, B.n), rng.uniform(-1, 1, B.m)
    from oracle import simd
    th = simd.host_threads()
    ref_t = O.mul(R, xt, np.zeros(B.n), trans=True, nthreads=th)
    ref_f = O.mul(R, xf, y0.copy(), 2.0, 0.5, ref_semantics=False)
    ref_f1 = O.mul(R, xf, np.zeros(B.m), ref_semantics=False)

    def rel(a, b):
        return np.linalg.norm(a - b) / np.linalg.norm(b)

    for rank, yt, yf, yl, col0, row0, nloc, mloc in res:
        assert rel(yt, ref_t) <= 1e-12
        assert rel(yf, ref_f) <= 1e-12
        if split == "stripes":
            assert rel(yl, ref_t[col0:col0 + nloc]) <= 1e-12
        else:
            assert rel(yl, ref_f1[row0:row0 + mloc]) <= 1e-12
