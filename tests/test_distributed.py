"""CPU, world_size 2 over gloo: the multi-GPU path's host side.

* the all-reduce hook the engine calls through the C ABI (rsvd_allreduce_fn,
  rsvd_kamaneh_raganato_terrana_amd.make_allreduce_hook) sums workspace slices across ranks and
  rejects slices outside the workspace;
* the collective hook of the n-side sharding (rsvd_collective_fn, make_collective_hook):
  reduce-scatter and all-gather of workspace slices, in place and not, fp64 / fp32 / bf16;
* the row-sharded decomposition the wide engine implements: rank g holds rows
  rsvd_row_partition(m, P, g) of A (src/rSVD.cpp:20-23 split); the l x l Grams of the m-side
  CholeskyQR panels are all-reduced; the n side is either replicated (A^T Q all-reduced) or
  sharded (A^T Q reduce-scattered into n-row chunks of nc = ceil(n / P) rounded up to 32, each
  chunk orthonormalised with an all-reduced Gram, the next skinny operand and V all-gathered) --
  both restated here in numpy over gloo and checked against the single-process oracle.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)


def _hook_worker(rank, port, q):
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import rsvd_kamaneh_raganato_terrana_amd as R
        from rsvd_kamaneh_raganato_terrana_amd import _capi

        _init(rank, port)
        ws = torch.zeros(1024, dtype=torch.uint8)
        f64 = ws[256:256 + 8 * 10].view(torch.float64)
        f64.copy_(torch.arange(10, dtype=torch.float64) * (rank + 1))
        f32 = ws[512:512 + 4 * 6].view(torch.float32)
        f32.fill_(rank + 0.5)
        hook = R.make_allreduce_hook(lambda: ws)
        fn = ctypes.cast(hook, ctypes.c_void_p).value
        call = _capi.ALLREDUCE_FN(fn)  # call through the C function pointer the engine holds
        rc1 = call(ws.data_ptr() + 256, 10, _capi.F64, None, None)
        rc2 = call(ws.data_ptr() + 512, 6, _capi.F32, None, None)
        rc3 = call(ws.data_ptr() + 1000, 10, _capi.F64, None, None)  # runs past the workspace
        ok = (rc1 == 0 and rc2 == 0 and rc3 == 1
              and torch.equal(f64, torch.arange(10, dtype=torch.float64) * 3)
              and torch.all(f32 == 2.0).item())
        dist.destroy_process_group()
        q.put((rank, bool(ok), (rc1, rc2, rc3)))
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, False, repr(e)))


def _coll_worker(rank, port, q):
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import rsvd_kamaneh_raganato_terrana_amd as R
        from rsvd_kamaneh_raganato_terrana_amd import _capi

        _init(rank, port)
        ws = torch.zeros(4096, dtype=torch.uint8)
        hook = R.make_collective_hook(lambda: ws)
        call = _capi.COLLECTIVE_FN(ctypes.cast(hook, ctypes.c_void_p).value)  # through the C pointer
        base = ws.data_ptr()
        ok = []
        for dt, tdt, esz in ((_capi.F64, torch.float64, 8), (_capi.F32, torch.float32, 4),
                             (_capi.BF16, torch.bfloat16, 2)):
            cnt = 6
            full = ws[0:WORLD * cnt * esz].view(tdt)
            full.copy_((torch.arange(WORLD * cnt) + 10 * rank).to(tdt))
            # reduce-scatter in place: rank r keeps the sum of chunk r
            rc = call(_capi.COLL_REDUCE_SCATTER, base, base + rank * cnt * esz, cnt, dt, None, None)
            want = sum((torch.arange(WORLD * cnt) + 10 * g).to(tdt) for g in range(WORLD))[rank * cnt:(rank + 1) * cnt]
            ok.append(rc == 0 and torch.equal(full[rank * cnt:(rank + 1) * cnt], want))
            # reduce-scatter out of place
            full.copy_((torch.arange(WORLD * cnt) + 10 * rank).to(tdt))
            out = ws[2048:2048 + cnt * esz].view(tdt)
            rc = call(_capi.COLL_REDUCE_SCATTER, base, base + 2048, cnt, dt, None, None)
            ok.append(rc == 0 and torch.equal(out, want))
            # all-gather in place (stale values in the other chunks must not leak)
            full.fill_(-7)
            full[rank * cnt:(rank + 1) * cnt] = (torch.arange(cnt) + 100 * rank).to(tdt)
            rc = call(_capi.COLL_ALL_GATHER, base + rank * cnt * esz, base, cnt, dt, None, None)
            want = torch.cat([(torch.arange(cnt) + 100 * g).to(tdt) for g in range(WORLD)])
            ok.append(rc == 0 and torch.equal(full, want))
        ok.append(call(_capi.COLL_ALL_GATHER, base + 4000, base, 64, _capi.F64, None, None) == 1)  # outside
        ok.append(call(9, base, base, 1, _capi.F64, None, None) == 1)  # unknown op
        dist.destroy_process_group()
        q.put((rank, all(ok), ok))
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e)))


def _allreduce_np(x):
    t = torch.from_numpy(np.ascontiguousarray(x))
    dist.all_reduce(t)
    return t.numpy()


def _cholqr_sharded(Yg, passes=2):
    """CholeskyQR(2) of a row-sharded panel: Gram all-reduced, R identical on every rank."""
    Q = Yg
    for _ in range(passes):
        G = _allreduce_np(Q.T @ Q)
        Rt = np.linalg.cholesky(G)  # G = Rt Rt^T, R = Rt^T
        Q = np.linalg.solve(Rt, Q.T).T
    return Q


def _nshard_rows(n):
    nc = -(-(-(-n // WORLD)) // 32) * 32
    return nc


def _reduce_scatter_np(Z, nc, rank):
    full = np.zeros((WORLD * nc, Z.shape[1]))
    full[:Z.shape[0]] = Z
    t = torch.from_numpy(full)
    dist.all_reduce(t)
    return t.numpy()[rank * nc:(rank + 1) * nc]


def _all_gather_np(chunk, n):
    parts = [None] * WORLD
    dist.all_gather_object(parts, chunk)
    return np.vstack(parts)[:n]


def _rsvd_worker(rank, port, q, shard_n=False):
    try:
        import sys

        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.dirname(here))
        sys.path.insert(0, here)
        import oracle
        import rsvd_kamaneh_raganato_terrana_amd as R
        from conftest import gapped_matrix

        _init(rank, port)
        m, n, l, qq = 301, 180, 16, 2
        A = gapped_matrix(m, n, 40, decay=0.8, seed=21)
        Om = oracle.generate_omega(n, l, 5)
        rows, off = R.row_partition(m, WORLD, rank)
        Ag = A[off:off + rows]
        Qg = _cholqr_sharded(Ag @ Om)
        nc = _nshard_rows(n)
        for _ in range(qq):
            if shard_n:  # rows [rank nc, (rank + 1) nc) of A^T Q, orthonormalised by shard, gathered
                Zc = _reduce_scatter_np(Ag.T @ Qg, nc, rank)
                Qn = _all_gather_np(_cholqr_sharded(Zc, passes=1), n)
            else:
                Z = _allreduce_np(Ag.T @ Qg)
                Qn = np.linalg.qr(Z)[0]
            Qg = _cholqr_sharded(Ag @ Qn)
        if shard_n:
            Bc = _reduce_scatter_np(Ag.T @ Qg, nc, rank)
            QBc = _cholqr_sharded(Bc)
            Rb = _allreduce_np(QBc.T @ Bc)  # R = Q_B^T B^T summed over the n shards
            Uw, S, VwT = np.linalg.svd(Rb.T)
            Ug, V = Qg @ Uw, _all_gather_np(QBc @ VwT.T, n)
        else:
            Bt = _allreduce_np(Ag.T @ Qg)  # n x l, identical on all ranks
            QB, Rb = np.linalg.qr(Bt)
            Uw, S, VwT = np.linalg.svd(Rb.T)
            Ug, V = Qg @ Uw, QB @ VwT.T
        # gather U rows on every rank and compare with the single-process oracle
        parts = [None] * WORLD
        dist.all_gather_object(parts, (off, Ug))
        U = np.zeros((m, l))
        for o, u in parts:
            U[o:o + u.shape[0]] = u
        Uo, So, Vo = oracle.rsvd(A, l, q=qq, Omega=Om)
        s_u = np.sign(np.sum(U * Uo, axis=0))
        s_v = np.sign(np.sum(V * Vo, axis=0))
        k = l // 2
        err = (np.linalg.norm(S - So) / np.linalg.norm(So),
               np.linalg.norm(U[:, :k] * s_u[:k] - Uo[:, :k]) / np.linalg.norm(Uo[:, :k]),
               np.linalg.norm(V[:, :k] * s_v[:k] - Vo[:, :k]) / np.linalg.norm(Vo[:, :k]))
        dist.destroy_process_group()
        q.put((rank, max(err) < 1e-9, err))
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e)))


def _run(worker, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, port, q) + extra) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    return res


def test_allreduce_hook_gloo_world2():
    res = _run(_hook_worker)
    assert all(ok for _, ok, _ in res), res


def test_collective_hook_gloo_world2():
    res = _run(_coll_worker)
    assert all(ok for _, ok, _ in res), res


@pytest.mark.parametrize("shard_n", [False, True])
def test_row_sharded_rsvd_decomposition_gloo_world2(shard_n):
    res = _run(_rsvd_worker, shard_n)
    assert all(ok for _, ok, _ in res), res
