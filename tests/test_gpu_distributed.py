"""GPU, world_size 2: the row-sharded engine path end to end on one MI355X.

Two processes share cuda:0 and exchange through the engine's all-reduce and collective hooks over
gloo (RCCL refuses two ranks on one device; the hooks and the engine code are the same that
bench.py drives over RCCL on N GPUs).  Every case runs with the n side sharded (reduce-scatter /
all-gather, the default) and replicated (all-reduce).  Rank g owns rows rsvd_row_partition(m, 2, g) of A (src/rSVD.cpp:20-23);
the gathered U rows, S and V must match the single-process oracle on the same A and Omega.
Tolerances: fp64 1e-9 (S) / 1e-8 (leading half of U, V) -- the sharded CholeskyQR factors the
all-reduced Gram (a different summation order than the single-GPU in-kernel reduction); fp32 /
bf16 1e-4 (north_star).
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _matrix(case):
    """The global A of a case: the gapped family, or the reference's own rank-2 input
    input/sparse_matrix.mtx (tests/golden/inputs.npz)."""
    m, n, l = case[:3]
    if len(case) > 5 and case[5] == "sparse_matrix":
        return np.load(os.path.join(REPO, "tests", "golden", "inputs.npz"))["sparse_matrix"].astype(np.float64)
    from conftest import gapped_matrix

    # the leading half of the spectrum stays above the noise floor (1e-3 N): l = 256 decays slower
    return gapped_matrix(m, n, min(2 * l, m, n), decay=0.93 if l < 256 else 0.985, seed=5).astype(np.float64)


def _worker(rank, port, case, q, shard_n, lowp=False, world=WORLD):
    try:
        sys.path.insert(0, REPO)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import torch
        import torch.distributed as dist

        import rsvd_kamaneh_raganato_terrana_amd as R
        from conftest import gapped_matrix

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        m, n, l, qq, dt = case[:5]
        A = _matrix(case)
        rows, off = R.row_partition(m, world, rank)
        tdt = {"f64": torch.float64, "f32": torch.float32, "bf16": torch.bfloat16,
               "e4m3": torch.float8_e4m3fn}[dt]
        # e4m3: one per-tensor scale of the GLOBAL A (every rank the same a_scale)
        scale = float(np.abs(A).max()) / 448.0 if dt == "e4m3" else 1.0
        Ag = torch.from_numpy(np.ascontiguousarray(A[off:off + rows].T / scale)).cuda().to(tdt).t()
        eng = R.Engine(0)
        eng.set_comm(rank, world, shard_n=shard_n)
        U, S, V = eng.rsvd(Ag, l, q=qq, seed=4242, a_scale=scale, lowp_intermediates=lowp)
        torch.cuda.synchronize()
        nsh = eng.info()["n_shard_rows"]
        assert (nsh == -(-(-(-n // world)) // 32) * 32) if shard_n else nsh == 0, nsh
        q.put((rank, off, U.cpu().double().numpy(), S.cpu().double().numpy(), V.cpu().double().numpy(),
               Ag.float().cpu().double().numpy() * scale))
        eng.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported through the queue
        import traceback

        q.put((rank, None, traceback.format_exc(), None, None, None))


def _run_world2(case, shard_n=True, lowp=False, world=WORLD):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, case, q, shard_n, lowp, world)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] is not None, r[2]
    res.sort(key=lambda t: t[1])
    return res


@pytest.mark.parametrize("shard_n", [True, False])
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_row_sharded_rank_deficient_is_orthonormal(dt, shard_n):
    """The reference's rank-2 input/sparse_matrix.mtx (A[i,j] = 100 i + j + 1) split over 2 ranks,
    l = 16: the breakdown columns of every output panel are completed (repair pass with disjoint
    Philox rows per rank), so U and V are orthonormal -- as the reference's Householder Q always is
    (src/rSVD.cpp:60-61) -- and sigma_1, sigma_2 are the known answers."""
    res = _run_world2((100, 100, 16, 2, dt, "sparse_matrix"), shard_n)
    U = np.vstack([r[2] for r in res])
    S, V = res[0][3], res[0][4]
    tol = 1e-10 if dt == "f64" else 1e-5
    assert np.linalg.norm(U.T @ U - np.eye(16)) < tol
    assert np.linalg.norm(V.T @ V - np.eye(16)) < tol
    rtol = 1e-12 if dt == "f64" else 1e-6
    assert abs(S[0] - 577391.767) < 1e-9 * 577391.767 + rtol * S[0]
    assert abs(S[1] - 1443.12761) < 1e-7 * 1443.12761 + rtol * S[0]
    assert np.all(S[2:] < (1e-9 if dt == "f64" else 1e-5) * S[0])


def _check_world2(case, shard_n, lowp=False, world=WORLD, tol_uv64=1e-8, frac=2):
    import oracle
    from conftest import rel_fro, sign_align

    m, n, l, qq, dt = case
    res = _run_world2(case, shard_n, lowp, world)
    U = np.vstack([r[2] for r in res])
    A = np.vstack([r[5] for r in res])  # the values the GPU saw (bf16 / fp32 rounded)
    assert A.shape[0] == m
    S0, V0 = res[0][3], res[0][4]
    # every rank holds the same S and V
    for r in res[1:]:
        assert np.array_equal(S0, r[3]) and np.array_equal(V0, r[4])
    # the same Omega the engine drew (Philox; rounded to bf16 for bf16 A)
    import torch

    import rsvd_kamaneh_raganato_terrana_amd as R

    eng = R.Engine(0)
    gdt = {"f64": torch.float64, "f32": torch.float32, "bf16": torch.bfloat16, "e4m3": torch.float8_e4m3fn}[dt]
    Om = eng.generate_omega(n, l, seed=4242, dtype=gdt).cpu().double().numpy()
    eng.close()
    Uo, So, Vo = oracle.rsvd(A, l, q=qq, Omega=Om)
    tol_s, tol_uv = (1e-9, tol_uv64) if dt == "f64" else (1e-4, 1e-4)
    k = l // frac
    assert rel_fro(S0, So) < tol_s
    assert rel_fro(sign_align(U[:, :k], Uo[:, :k]), Uo[:, :k]) < tol_uv
    assert rel_fro(sign_align(V0[:, :k], Vo[:, :k]), Vo[:, :k]) < tol_uv
    # orthonormality of the gathered U: Frobenius over l^2 entries (fp32 outputs: ~1e-6 per entry)
    assert np.linalg.norm(U.T @ U - np.eye(l)) < (1e-10 if dt == "f64" else 1e-3)


@pytest.mark.parametrize("case", [(600, 300, 32, 2, "f64"), (1024, 512, 64, 2, "f32"), (2048, 1024, 128, 1, "bf16"),
                                  (4096, 2048, 256, 2, "bf16")])
@pytest.mark.parametrize("shard_n", [True, False])
def test_row_sharded_world2_matches_oracle(case, shard_n):
    _check_world2(case, shard_n)


def test_row_sharded_world2_e4m3_l512_sharded_n():
    """C5's multi-GPU path (BASELINE configs[4]): e4m3 A with one global per-tensor scale, l = 512,
    q = 2, rows split over 2 ranks (4096 each: m and lda multiples of 16, so the sketch runs e4m3 x
    e4m3 on the fp8 MFMA, launch_wproj_s8) with the n side sharded (A^T Q reduce-scattered, the
    LP = 512 hi/lo panels all-gathered).  Oracle on the dequantised A and the engine's e4m3 Omega,
    the north-star 1e-4 bar."""
    _check_world2((8192, 2048, 512, 2, "e4m3"), True)


def test_row_sharded_world2_lowp_intermediates_sharded_n():
    """RSVD_FLAG_LOWP_INTERMEDIATES with the n side sharded: intermediate orthonormalisations write
    only the bf16 hi/lo panels (no fp32 Out), which are what the all-gather moves -- the combination
    the opt-in bench variant runs at N > 1.  0.985^i spectrum (decays across the sketch), 1e-4 bar."""
    _check_world2((4096, 2048, 256, 2, "bf16"), True, lowp=True)


@pytest.mark.parametrize("case", [(1501, 700, 96, 2, "f64"), (4099, 3000, 128, 2, "bf16"), (3002, 2000, 256, 2, "e4m3")])
def test_row_sharded_world3_uneven_matches_oracle(case):
    """Three ranks: m % 3 != 0, so rank 0 holds one row more than the others
    by the reference's remainder rule (src/rSVD.cpp:20-23, rsvd_row_partition); n is not a
    multiple of 3 x 32, so the last n shard carries zero padding rows; the e4m3 case's shards
    (1001, 1001, 1000 rows) are not multiples of 16, which takes the sketch off the fp8 x fp8
    kernel onto the widening one.  Against the oracle on the same A and Omega."""
    import rsvd_kamaneh_raganato_terrana_amd as R

    m = case[0]
    assert [R.row_partition(m, 3, r)[0] for r in range(3)] == [m // 3 + (r < m % 3) for r in range(3)]
    # fp64: the leading half of U / V to 1e-7 (three Gram partials per all-reduce; measured 3.3e-8
    # on the 0.93^i spectrum, whose 48th singular gap is 0.2 % of sigma_1)
    _check_world2(case, True, world=3, tol_uv64=1e-7)


@pytest.mark.parametrize("case", [(8191, 4000, 256, 2, "bf16"), (8192, 2000, 512, 2, "e4m3")])
def test_row_sharded_world8_matches_oracle(case):
    """Eight ranks, the partition C4 / C5 run at on one 8-GPU node (BASELINE configs[3] / [4];
    VERDICT r04 item 1), here as 8 gloo processes sharing the one GPU (the engine code and the hooks
    are the ones bench.py drives over RCCL).  C4-shaped: bf16, l = 256, q = 2, 8191 rows -- seven
    ranks of 1024 and one of 1023 by the reference's remainder rule (src/rSVD.cpp:20-23) -- and
    n = 4000, not a multiple of 8 x 32: n-shards of 512 rows, the last holding 416 rows of A^T Q and
    96 zero rows; eight Gram partials per all-reduce.  C5-shaped: e4m3 with one global scale, l = 512,
    1024 rows per rank (the fp8 x fp8 sketch), n = 2000 (last shard 208 valid rows).  Against the
    oracle on the same A and Omega at the north-star 1e-4 bar."""
    import rsvd_kamaneh_raganato_terrana_amd as R

    m = case[0]
    assert [R.row_partition(m, 8, r)[0] for r in range(8)] == [m // 8 + (r < m % 8) for r in range(8)]
    _check_world2(case, True, world=8)


@pytest.mark.parametrize("case", [(32768, 2048, 256, 2, "bf16"), (32768, 2048, 512, 2, "e4m3")])
def test_row_sharded_world8_larger_shards(case):
    """the world > 1 kernel choices (fp64 Grams of the sharded passes, the per-shard
    n-side passes, the deferred second pass's split Gram + G^-1/2 series) pinned at 4096 rows per rank --
    half of C4's 8-GPU shard and a quarter of C5's -- against the oracle on the same A and Omega, 1e-4."""
    _check_world2(case, True, world=8)


@pytest.mark.parametrize("case", [(8191, 4000, 256, 2, "bf16"), (8192, 2000, 512, 2, "e4m3")])
def test_row_sharded_world8_split_gram_sharded(case, monkeypatch):
    """RSVD_GRAM_SPLIT_SHARDED=1 (opt-in, round 6): the three-piece split Gram on sharded passes too --
    the rank's split Gram all-reduced and factored, the predicated fp64 fallback Gram summed whether
    or not it runs (DESIGN.md §5 prices it).  The world-8 cases above, against the oracle at 1e-4."""
    monkeypatch.setenv("RSVD_GRAM_SPLIT_SHARDED", "1")  # read once per process: the spawned ranks see it
    _check_world2(case, True, world=8)


@pytest.mark.parametrize("case", [(1600, 1000, 768, 1, "f32"), (2001, 1200, 640, 1, "bf16")])
def test_row_sharded_world2_l_past_512(case):
    """rSVD() past the wide engine's 512 sketch columns on two ranks: the
    dense_big.cpp path with its m-side panels row-sharded (Grams and block projections all-reduced,
    disjoint repair rows) and A^T Q all-reduced (the n side replicated); the reference has no cap on
    l (src/rSVD.cpp:72).  Uneven 2001-row split in the bf16 case: every rank must use the same global
    row count in the CholeskyQR shift (it is all-reduced; world * local rows made the ranks' R factors
    differ and moved U by 1.7e-4).  Against the oracle, 1e-4 (measured ~1e-5 on the leading half)."""
    _check_world2(case, False)


@pytest.mark.parametrize("case", [(1200, 1000, 768, 1, "f32"), (400, 600, 256, 1, "bf16")])
def test_row_sharded_world2_shard_smaller_than_l(case):
    """a row shard may hold fewer rows than l -- the reference partitions the GLOBAL m
    (src/rSVD.cpp:20-23) and only needs l <= min(m, n) globally.  600 rows per rank at l = 768 (the
    dense_big.cpp path: its m-side basis workspace is sized by l, not by the local rows) and 200 rows
    per rank at l = 256 (the wide engine, n side sharded).  Against the oracle, 1e-4."""
    _check_world2(case, case[2] <= 512)


def _worker_refused(rank, port, m_local, n, l, q):
    try:
        sys.path.insert(0, REPO)
        import torch
        import torch.distributed as dist

        import rsvd_kamaneh_raganato_terrana_amd as R

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        torch.cuda.set_device(0)
        g = torch.Generator().manual_seed(rank)
        Ag = torch.randn(n, m_local, generator=g).cuda().to(torch.bfloat16).t()
        eng = R.Engine(0)
        eng.set_comm(rank, 2, shard_n=True)
        msg = None
        try:
            eng.rsvd(Ag, l, q=1, seed=7)
        except Exception as e:  # the expected refusal (RSVD_ERR_UNSUPPORTED)
            msg = str(e)
        # the handle is usable afterwards: a legal request on the same ranks runs
        U, S, V = eng.rsvd(Ag, 32, q=1, seed=7)
        torch.cuda.synchronize()
        ok_after = bool(torch.isfinite(S).all())
        eng.close()
        dist.destroy_process_group()
        q.put((rank, msg, ok_after))
    except Exception:  # pragma: no cover - reported through the queue
        import traceback

        q.put((rank, "worker failed: " + traceback.format_exc(), False))


@pytest.mark.parametrize("l", [256, 600])
def test_row_sharded_world2_global_rows_below_l(l):
    """two shards of 100 (l = 256, the wide engine) or 250 rows (l = 600, dense_big.cpp)
    whose GLOBAL row count is below l.  The reference needs l <= min(m, n) of the global A
    (src/rSVD.cpp:20-23 partitions m); both ranks must refuse with RSVD_ERR_UNSUPPORTED, not run into
    a CholeskyQR breakdown.  The wide engine sums the count with its first m-side Gram all-reduce and
    reports it through rsvd_sync; the handle stays usable for the next (legal) request."""
    import torch.multiprocessing as mp

    m_local = 100 if l == 256 else 250
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_refused, args=(r, port, m_local, 700, l, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, msg, ok_after in res:
        assert msg is not None and "global row count" in msg, (rank, msg)
        assert ok_after, rank
