"""GPU: the RCCL transport of the row-sharded engine, on a one-GPU box.

RCCL refuses two ranks on one device, so the world-2 GPU tests (test_gpu_distributed.py) run the
hooks over gloo.  These tests put RCCL itself on the data path at world 1:

* the torch.distributed hooks (make_allreduce_hook / make_collective_hook) on an "nccl" group,
  called through the C function pointers the engine holds: all-reduce, in-place reduce-scatter
  and in-place all-gather of workspace slices, fp64 / fp32 / bf16 -- the exact calls
  (reduce_scatter_tensor / all_gather_into_tensor with recv = send + rank count) an N-GPU
  bench.py run makes;
* a full rSVD with RSVD_FLAG_FORCE_NSHARD (the n-side sharded code path: A^T Q reduce-scattered,
  the next skinny operand and V all-gathered) through those hooks, against the oracle;
* the library-owned communicator (rsvd_comm_unique_id / rsvd_comm_init, comm.cpp: ncclAllReduce /
  ncclReduceScatter / ncclAllGather on the handle's stream, no Python on the data path) -- what a
  C++ caller of include/rSVD.hpp uses -- on the same rSVD.

Reference: the collective rSVD of src/rSVD.cpp:15,20-23,49,52 (MPI ranks, root gather + Bcast).
Tolerances: fp64 1e-9 (S) / 1e-8 (leading half of U, V); bf16 1e-4 (north_star).
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, *args):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=target, args=(q,) + args)
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert res[0], res[1]
    return res[1]


def _init_nccl(port):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))


def _hooks_worker(q, port):
    try:
        sys.path.insert(0, REPO)
        import ctypes

        import torch
        import torch.distributed as dist

        import rsvd_kamaneh_raganato_terrana_amd as R
        from rsvd_kamaneh_raganato_terrana_amd import _capi

        _init_nccl(port)
        assert dist.get_backend() == "nccl"
        ws = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
        coll = _capi.COLLECTIVE_FN(ctypes.cast(R.make_collective_hook(lambda: ws), ctypes.c_void_p).value)
        allr = _capi.ALLREDUCE_FN(ctypes.cast(R.make_allreduce_hook(lambda: ws), ctypes.c_void_p).value)
        base = ws.data_ptr()
        out = []
        for dt, tdt, esz in ((_capi.F64, torch.float64, 8), (_capi.F32, torch.float32, 4),
                             (_capi.BF16, torch.bfloat16, 2)):
            cnt = 1000
            full = ws[4096:4096 + cnt * esz].view(tdt)
            ref = (torch.arange(cnt, device="cuda") * 0.25 - 7).to(tdt)
            full.copy_(ref)
            # in place (recv = send + rank count, rank 0): RCCL's in-place reduce-scatter
            rc1 = coll(_capi.COLL_REDUCE_SCATTER, base + 4096, base + 4096, cnt, dt, None, None)
            torch.cuda.synchronize()
            ok1 = rc1 == 0 and torch.equal(full, ref)
            # out of place
            dst = ws[32768:32768 + cnt * esz].view(tdt)
            dst.fill_(3)
            rc2 = coll(_capi.COLL_REDUCE_SCATTER, base + 4096, base + 32768, cnt, dt, None, None)
            torch.cuda.synchronize()
            ok2 = rc2 == 0 and torch.equal(dst, ref)
            # all-gather in place (send = recv + rank count)
            rc3 = coll(_capi.COLL_ALL_GATHER, base + 4096, base + 4096, cnt, dt, None, None)
            torch.cuda.synchronize()
            ok3 = rc3 == 0 and torch.equal(full, ref)
            rc4 = allr(base + 4096, cnt, dt, None, None) if dt != _capi.BF16 else 0
            torch.cuda.synchronize()
            ok4 = rc4 == 0 and torch.equal(full, ref)
            out.append((dt, ok1, ok2, ok3, ok4))
        bad = coll(_capi.COLL_ALL_GATHER, base + (1 << 16) - 8, base, 64, _capi.F64, None, None)  # outside
        dist.destroy_process_group()
        q.put((all(all(t[1:]) for t in out) and bad == 1, out))
    except Exception:
        import traceback

        q.put((False, traceback.format_exc()))


def test_torch_hooks_over_nccl_world1():
    """The collective / all-reduce hooks on an RCCL group, through their C pointers."""
    _spawn(_hooks_worker, _free_port())


def _case(dt):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from conftest import gapped_matrix

    if dt == "bf16":
        return 2048, 1000, 128, 2, gapped_matrix(2048, 1000, 256, decay=0.93, seed=8)
    return 600, 300, 96, 2, gapped_matrix(600, 300, 192, decay=0.93, seed=9)


def _rsvd_worker(q, port, dt, mode):
    """mode "hooks": torch.distributed (nccl) hooks; "library": rsvd_comm_init (no torch.distributed)."""
    try:
        sys.path.insert(0, REPO)
        import torch

        import rsvd_kamaneh_raganato_terrana_amd as R

        torch.cuda.set_device(0)
        m, n, l, qq, A = _case(dt)
        tdt = torch.bfloat16 if dt == "bf16" else torch.float64
        Ad = torch.from_numpy(np.ascontiguousarray(A.T)).cuda().to(tdt).t()
        eng = R.Engine(0)
        if mode == "hooks":
            _init_nccl(port)
            eng.set_comm(0, 1, shard_n=True)
        else:
            uid = R.Engine.comm_unique_id()
            eng.comm_init(uid, 0, 1, shard_n=True)
        U, S, V = eng.rsvd(Ad, l, q=qq, seed=77, force_nshard=True)
        info = eng.info()
        Om = eng.generate_omega(n, l, seed=77, dtype=tdt).cpu().double().numpy()
        res = (U.cpu().double().numpy(), S.cpu().double().numpy(), V.cpu().double().numpy(),
               Ad.double().cpu().numpy(), Om, info)
        if mode == "hooks":
            import torch.distributed as dist

            dist.destroy_process_group()
        else:
            eng.comm_destroy()
        eng.close()
        q.put((True, res))
    except Exception:
        import traceback

        q.put((False, traceback.format_exc()))


@pytest.mark.parametrize("mode", ["hooks", "library"])
@pytest.mark.parametrize("dt", ["f64", "bf16"])
def test_forced_nshard_rsvd_through_rccl_matches_oracle(dt, mode):
    """A whole rSVD on the n-side sharded path with RCCL moving the panels (world 1)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle
    from conftest import rel_fro, sign_align

    U, S, V, A, Om, info = _spawn(_rsvd_worker, _free_port(), dt, mode)
    n, l = A.shape[1], S.shape[0]
    assert info["n_shard_rows"] == -(-n // 32) * 32, info  # the sharded layout ran
    Uo, So, Vo = oracle.rsvd(A, l, q=2, Omega=Om)
    tol_s, tol_uv = (1e-9, 1e-8) if dt == "f64" else (1e-4, 1e-4)
    k = l // 2
    assert rel_fro(S, So) < tol_s
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < tol_uv
    assert rel_fro(sign_align(V[:, :k], Vo[:, :k]), Vo[:, :k]) < tol_uv
    assert np.linalg.norm(V.T @ V - np.eye(l)) < (1e-10 if dt == "f64" else 1e-3)
