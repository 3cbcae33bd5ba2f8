#!/usr/bin/env python
"""bench.py -- BASELINE.json metric: "rSVD wall-clock + achieved TFLOP/s, dense m x n rank-k".

One step = one full rSVD() (src/rSVD.cpp:72-133: sketch, q power iterations with a QR after every
projection, B = Q^T A, its small SVD, U = Q Utilde) on a synthetic A already resident in HBM.
Synthetic A = X diag(0.9^t) Y^T / sqrt(n) + 1e-3 N, X, Y Gaussian.

Configurations (BASELINE.json "configs"; --config, default c4):
  c1  rank-10 rSVD of I_100 (the reference's input/sparse_matrix100.mtx, regenerated), fp64, q = 2,
      Jacobi -- the reference's own CPU-runnable case (configs[0]); a latency line: the GPU call
      next to the CPU oracle at -O3 (1 and all threads) and -O0 (the reference's build flag), with
      the known answers S = 1, |A - U S V^T|_F = sqrt(100 - l) checked (l = 10 and 16)
  c2  dense 4096 x 4096 fp32, l = 64, q = 2                       (configs[1])
  c3  tall-skinny 1048576 x 1024 bf16, l = 128, q = 1             (configs[2])
  c4  dense 65536 x 65536 bf16, l = 256, q = 2, rows sharded      (configs[3]: the north-star
      workload; 8.6 GB of A fits one MI355X, so N = 1 runs the whole matrix -- the default line)
  c5  131072 x 8192 e4m3 (per-tensor scale), l = 512, q = 2       (configs[4])
Scaling over N GPUs (torchrun, one process per GPU, RCCL): c2 / c3 are weak-scaled (each rank
owns m rows, the global matrix is N m x n); c4 / c5 are strong-scaled (the global m x n matrix is
row-partitioned, src/rSVD.cpp:20-23).  The n side is sharded as well (rsvd_set_collectives):
A^T Q is reduce-scattered, each rank orthonormalises its n/N rows (Gram all-reduced), the next
skinny operand and V are all-gathered; U stays row-sharded.  Only the l x l small SVD is
replicated.
value = whole-job algorithmic TFLOP/s (F_proj + F_qr + F_small of the global
problem) / max-over-ranks wall time; ms_per_step = rSVD wall-clock.

Extra fields: "roofline" (the dominant projection kernel, HIP-event timed on the engine's stream
in a second pass over the same K steps; bound = min(MFMA peak, AI x 8 TB/s) with AI = 2 l /
bytes per A element), "cpu_baseline" (the fp64 C oracle -- a restatement of the
reference, Eigen is absent -- on rank 0 at N = 1 on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# MI355X dense peaks (MI355X_MICROARCH.md): matrix fp32 157.3, fp64 78.6, bf16 2516.6 TF/s, fp8 5033.2
# (block-scaled f8f6f4 form; the non-scaled fp8 MFMA runs at the bf16 rate).  e4m3 A: the sketch
# A * Omega runs e4m3 x e4m3 on the fp8 MFMA; the hi/lo products widen A to bf16 (bf16 rate).
PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6, "bf16": 2516.6, "fp8": 2516.6}
PEAK_FP8_TFLOPS = 5033.2
ELEM_BYTES = {"f32": 4, "f64": 8, "bf16": 2, "fp8": 1}
PEAK_HBM_GBS = 8000.0

CONFIGS = {
    # name: (m, n, l, q, dtype, strong-scaled, cpu sample rows, label)
    "c1": (100, 100, 10, 2, "f64", False, None, "C1: rank-10 rSVD of I_100 (input/sparse_matrix100.mtx), fp64, q=2"),
    "c2": (4096, 4096, 64, 2, "f32", False, None, "C2: dense 4096x4096 fp32 rSVD, l=64, q=2"),
    "c3": (1048576, 1024, 128, 1, "bf16", False, 16384, "C3: tall-skinny 1048576x1024 bf16 rSVD, l=128, q=1"),
    "c4": (65536, 65536, 256, 2, "bf16", True, 2048, "C4: dense 65536x65536 bf16 rSVD, l=256, q=2"),
    "c5": (131072, 8192, 512, 2, "fp8", True, 8192, "C5: 131072x8192 e4m3 rSVD, l=512, q=2"),
}


def algorithmic_flops(m, n, l, q):
    """F_proj, F_qr, F_small of one rSVD."""
    f_proj = 2.0 * m * n * l * (2 * q + 2)
    f_qr = (q + 1) * (4.0 * m * l * l - 4.0 * l ** 3 / 3) + q * (4.0 * n * l * l - 4.0 * l ** 3 / 3)
    f_small = 4.0 * n * l * l - 4.0 * l ** 3 / 3 + 2.0 * n * l * l + 2.0 * m * l * l
    return f_proj, f_qr, f_small


def make_A(torch, m_local, n, row0, dtype, rank_cols=128, seed=0x5EED0002, amax_reduce=None):
    """Column-major rows [row0, row0 + m_local) of the synthetic A, built on the GPU in row
    chunks (A^T chunks, n x rows) so the fp32 temporaries stay small.  fp8: A / scale in e4m3 with
    scale = max|A| / 448 (per tensor: the max over every rank's rows via amax_reduce, so that all
    shards share one scale), returned with the scale."""
    dev = torch.device("cuda")
    gY = torch.Generator(device=dev).manual_seed(seed)
    sig = 0.9 ** torch.arange(rank_cols, device=dev, dtype=torch.float32)
    Ys = torch.randn(n, rank_cols, generator=gY, device=dev) * sig / (n ** 0.5)
    store = torch.float8_e4m3fn if dtype == "fp8" else {"f32": torch.float32, "f64": torch.float64,
                                                        "bf16": torch.bfloat16}[dtype]
    At = torch.empty(m_local, n, dtype=torch.float32 if dtype == "fp8" else store, device=dev)  # rows x n
    chunk = max(1, min(m_local, (1 << 28) // n))
    for c0 in range(0, m_local, chunk):
        c1 = min(m_local, c0 + chunk)
        g = torch.Generator(device=dev).manual_seed(seed + 1 + row0 + c0)
        X = torch.randn(c1 - c0, rank_cols, generator=g, device=dev)
        blk = X @ Ys.t() + 1e-3 * torch.randn(c1 - c0, n, generator=g, device=dev)
        At[c0:c1] = blk.to(At.dtype)
        del X, blk
    # column-major m x n: store A^T row-major
    if dtype == "fp8":
        amax = float(At.abs().max())
        if amax_reduce is not None:
            amax = amax_reduce(amax)
        scale = amax / 448.0
        Acm = (At / scale).t().contiguous().to(store).t()
        del At
        return Acm, scale
    Acm = At.t().contiguous().t()
    del At
    return Acm, 1.0


def lp_pad(l):
    """Panel width of the wide engine's LDS-DMA kernels (wide.cpp WideLayout: a power of two >= 128)."""
    lp = 128
    while lp < l:
        lp *= 2
    return lp


def pmc_traffic(key, kernel_prefix):
    """HBM bytes per launch of the kernel from the committed rocprofv3 PMC summary for this
    workload (profiles/*_traffic.json, written by tools/profile.sh + tools/traffic.py; FETCH_SIZE
    doubled per the gfx950 correction).  None when no summary for this workload exists."""
    import glob

    best = None
    import re

    def natural(f):  # r01_v7 < r01_v11: the newest pass for a workload wins
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))]

    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), key=natural):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") != key:
            continue
        for k, v in d.get("kernels", {}).items():
            if k.startswith(kernel_prefix):
                best = (v["hbm_bytes"], os.path.relpath(f, REPO))
    return best


def pmc_mfma_busy(key, kernel_prefix):
    """MFMA pipe occupancy of the kernel from the committed rocprofv3 pass for this workload
    (profiles/*_mfma_busy.json, tools/pmc_mfma.sh + tools/mfma_busy.py: SQ_VALU_MFMA_BUSY_CYCLES over
    the SIMD-cycles at the clock the kernel actually ran, GRBM_GUI_ACTIVE).  A clock estimate above
    the 2.4 GHz peak means GUI_ACTIVE also counted the dispatch overhead of a short kernel (C2's
    ~27-us projections): there the busy cycles are priced against the dispatch duration at 2.4 GHz
    instead -- a lower bound of the busy fraction, since the chip ran at most that clock -- and the
    entry says so.  None when absent."""
    import glob
    import re

    def natural(f):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))]

    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_mfma_busy.json")), key=natural):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") != key:
            continue
        for k, v in d.get("kernels", {}).items():
            if not k.startswith(kernel_prefix):
                continue
            clk = v.get("clock_GHz_est", 0.0)
            if 0 < clk <= 2.4:
                best = {"frac": v["mfma_busy_frac"], "clock_GHz": clk, "source": os.path.relpath(f, REPO)}
            elif clk > 2.4:  # busy / (1024 SIMDs x duration x 2.4 GHz), duration = GUI_ACTIVE / 8 / clk
                best = {"frac": v["mfma_busy_frac"] * clk / 2.4, "clock_GHz": None, "bound": "lower",
                        "note": "short dispatch: GUI_ACTIVE includes dispatch overhead (clock estimate "
                                f"{clk:.2f} GHz); busy cycles priced at the 2.4 GHz peak over the dispatch",
                        "source": os.path.relpath(f, REPO)}
    return best


def cpu_baseline(A_host, l, q, budget_s, threads, note):
    import oracle

    m, n = A_host.shape
    used = oracle.set_threads(threads)
    reps, t_all = 0, 0.0
    while reps < 10:
        t0 = time.perf_counter()
        oracle.rsvd(A_host, l, q=q, seed=1)
        t_all += time.perf_counter() - t0
        reps += 1
        if t_all >= budget_s:
            break
    per = t_all / reps
    fl = sum(algorithmic_flops(m, n, l, q))
    return {
        "value": fl / per / 1e12,
        "unit": "TFLOP/s",
        "cores": used,
        "kind": "port",
        "sample": f"{reps} full rSVD calls of a {m}x{n} A (l={l}, q={q}) {note} in the fp64 C oracle "
                  f"(oracle/rsvd_oracle.c, -O3 -fopenmp); {per * 1e3:.1f} ms per rSVD",
        "ms_per_rsvd": per * 1e3,
    }


def c1_extras(torch, R, eng, A, q, budget_s):
    """C1 (tests/rSVD_test.cpp:60-75 on input/sparse_matrix100.mtx = I_100): known answers on the GPU
    for l = 10 and 16, the synchronised single-call latency, and the CPU oracle at -O3 (1 thread and
    all threads) and -O0 (the reference Makefile's flag, 1 thread)."""
    import numpy as np

    import oracle

    out = {"known_answers": {}, "cpu_oracle_ms_per_rsvd": {}}
    m = A.shape[0]
    for l in (10, 16):
        U, S, V = eng.rsvd(A, l, q=q, seed=0x5EED0001)
        torch.cuda.synchronize()
        Uh, Sh, Vh = U.cpu().numpy(), S.cpu().numpy(), V.cpu().numpy()
        err = float(np.linalg.norm(np.eye(m) - (Uh * Sh) @ Vh.T))
        out["known_answers"][f"l{l}"] = {"max_abs_S_minus_1": float(np.abs(Sh - 1.0).max()),
                                         "residual_F": err, "expected_residual_F": float(np.sqrt(m - l))}
    lat = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.rsvd(A, 10, q=q, seed=0x5EED0001, check_errors=False)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    out["gpu_latency_ms_median"] = float(np.median(lat) * 1e3)
    Ah = np.eye(m)
    all_threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
    for opt, threads in (("O3", 1), ("O3", all_threads), ("O0", 1)):
        L = oracle.lib(opt)
        L.orc_set_threads(threads)
        Om = oracle.generate_omega(m, 10, 0x5EED0001)
        Uo, So, Vo = np.zeros((m, 10), order="F"), np.zeros(10), np.zeros((m, 10), order="F")
        ts = []
        t_all = 0.0
        while len(ts) < 200 and t_all < budget_s / 3:
            t0 = time.perf_counter()
            L.orc_rsvd(m, m, oracle._p(Ah), m, 10, q, oracle._p(Om), m, 0, oracle._p(Uo), oracle._p(So), oracle._p(Vo))
            ts.append(time.perf_counter() - t0)
            t_all += ts[-1]
        out["cpu_oracle_ms_per_rsvd"][f"-{opt} {threads} thread(s)"] = float(np.median(ts) * 1e3)
    oracle.set_threads(all_threads)
    return out


def self_check(torch, dist, A, a_scale, U, S, V, world, k_top=32):
    """Size-independent correctness of the run just timed (outside the timed region): the Ritz
    residuals |A v_i - s_i u_i| / s_i of the leading k_top triplets, summed over the row shards
    (this rank holds rows of A and U, every rank the same S and V), and the orthonormality of V.
    At N > 1 this is the end-to-end check of the RCCL exchange (reduce-scatter / all-gather)."""
    k = min(k_top, S.shape[0])
    Vk = V[:, :k].float()
    res = torch.zeros(k, dtype=torch.float64, device=A.device)
    step_rows = max(1, (1 << 30) // max(1, A.shape[1] * 4))
    for r0 in range(0, A.shape[0], step_rows):
        r1 = min(A.shape[0], r0 + step_rows)
        blk = A[r0:r1].float() * a_scale
        d = blk @ Vk - U[r0:r1, :k].float() * S[:k].float()
        res += (d.double() ** 2).sum(0)
        del blk, d
    if world > 1:
        dist.all_reduce(res)
    rel = (res.sqrt() / S[:k].double()).max().item()
    vo = torch.linalg.norm(V.double().t() @ V.double() - torch.eye(V.shape[1], dtype=torch.float64, device=V.device)).item()
    return {"top_k": k, "max_ritz_residual": rel, "V_orth_err": vo, "ok": bool(rel < 1e-2 and vo < 1e-2)}


def launch_ranks(n):
    """Run this script as N ranks under torch.distributed.run (a child process: nothing in this
    process has initialised the GPU, and it is never replaced by exec)."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    # the bench's own flags travel in the environment: torch.distributed.run's parser would take
    # abbreviations such as --m / --n placed after the script for its own options
    env = dict(os.environ, RSVD_BENCH_ARGV=json.dumps(sys.argv[1:]))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--m", type=int, default=None, help="override m (per GPU for weak-scaled configs)")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--l", type=int, default=None)
    ap.add_argument("--q", type=int, default=None)
    ap.add_argument("--dtype", default=None, choices=["f32", "f64", "bf16", "fp8"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-oracle work (0 = skip)")
    ap.add_argument("--comm", default="library", choices=["library", "torch"],
                    help="N > 1: the handle's own RCCL communicator (rsvd_comm_init) or torch.distributed hooks")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: torch.distributed backend (nccl = RCCL; gloo with --comm torch runs the whole "
                         "multi-rank path with every rank on one GPU, for the one-GPU test box)")
    ap.add_argument("--lda-pad", type=int, default=0,
                    help="diagnostics: store A column-major with leading dimension m + PAD (elements) instead of "
                         "m -- the caller's layout choice; the headline line keeps lda = m (Eigen's layout)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="diagnostics, one process: run rank 0 of an N-rank strong-scaled job alone (its rows of A, "
                         "its n shard, the sharded-panel kernels) with no-op collectives -- prices the per-rank "
                         "kernels of the N-GPU step on one GPU (outputs are not an SVD; no self-check, no CPU line)")
    argv = json.loads(os.environ["RSVD_BENCH_ARGV"]) if "RSVD_BENCH_ARGV" in os.environ and "WORLD_SIZE" in os.environ else None
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without torchrun: start the N ranks as child processes (one per
        # GPU, torch.distributed.run on 127.0.0.1) before this process touches the GPU, and exit
        # with their status; rank 0 prints the JSON line
        raise SystemExit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    import rsvd_kamaneh_raganato_terrana_amd as R

    cm, cn, cl, cq, cdt, strong, cpu_rows, label = CONFIGS[args.config]
    m_cfg = args.m or cm
    n = args.n or cn
    l = args.l or cl
    q = cq if args.q is None else args.q
    dt = args.dtype or cdt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; with --backend gloo several ranks may share the box's GPUs (test mode)
    ndev = max(1, torch.cuda.device_count())
    dev = local_rank % ndev
    if args.backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks over RCCL need {world} GPUs ({ndev} visible)")
    if args.backend == "gloo" and args.comm != "torch" and world > 1:
        raise SystemExit("--backend gloo needs --comm torch (the library communicator is RCCL)")
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group("gloo")

    emu = args.emulate_world if world == 1 and args.emulate_world > 1 else 0
    if strong:  # global m x n, rows partitioned (src/rSVD.cpp:20-23)
        m_global = m_cfg
        m_local, row0 = R.row_partition(m_global, emu or world, rank)
    else:
        m_local, row0 = m_cfg, m_cfg * rank
        m_global = m_cfg * world
    if args.config == "c1":  # I_100, exactly the reference's input/sparse_matrix100.mtx
        A, a_scale = torch.eye(m_local, n, dtype=torch.float64, device="cuda").t().contiguous().t(), 1.0
    else:
        def amax_all(x):  # one per-tensor e4m3 scale for the global A
            if world == 1:
                return x
            t = torch.tensor([x], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())

        A, a_scale = make_A(torch, m_local, n, row0, dt, amax_reduce=amax_all)
        if args.lda_pad > 0:  # the same A in a buffer whose column pitch is m + pad (BLAS lda > m)
            Ap = R.empty_colmajor(m_local, n, A.dtype, A.device, pad=args.lda_pad)
            Ap.copy_(A)
            del A
            A = Ap
    eng = R.Engine(dev)
    if world > 1:
        if args.comm == "library":  # rsvd_comm_init: RCCL owned by the C ABI, rank 0's id broadcast
            uid = [R.Engine.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            eng.comm_init(uid[0], rank, world, shard_n=True)
        else:
            eng.set_comm(rank, world)
    if emu:  # the rank's kernels alone; the workspace zeroed once so the never-exchanged rows are finite
        eng.emulate_world(0, emu)
        eng.reserve(eng.desc(A, l, q, seed=0x5EED0002, a_scale=a_scale))
        eng._ws.zero_()
    torch.cuda.synchronize()

    def step():
        return eng.rsvd(A, l, q=q, seed=0x5EED0002, a_scale=a_scale, check_errors=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    def timed(k):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        eng.sync()  # device-side failures of any of the K runs raise here (rsvd_sync)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt_s = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt_s], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt_s = float(t.item())
        return dt_s

    elapsed = timed(args.steps)
    # opt-in variant (not the headline): RSVD_FLAG_LOWP_INTERMEDIATES, power iterations before the last on
    # the bf16 operand alone (include/rsvd_c.h; its accuracy depends on the spectrum's decay)
    fast = None
    if dt in ("bf16", "fp8") and q >= 2:
        def step_fast():
            return eng.rsvd(A, l, q=q, seed=0x5EED0002, a_scale=a_scale, check_errors=False, lowp_intermediates=True)

        step_fast()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_fast()
        eng.sync()
        torch.cuda.synchronize()
        fast_s = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([fast_s], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            fast_s = float(t.item())
        fast = {"flag": "RSVD_FLAG_LOWP_INTERMEDIATES (opt-in, not the headline)",
                "ms_per_step": fast_s / args.steps * 1e3}
    # pass 2: same K steps with hipEvent pairs around every projection kernel (roofline)
    eng.set_timing(True)
    timed(args.steps)
    tm = eng.timing()
    eng.set_timing(False)
    info = eng.info()
    if emu:
        check = {"skipped": f"--emulate-world {emu}: no-op collectives, the outputs are not an SVD"}
    else:
        U_, S_, V_ = step()
        check = self_check(torch, dist, A, a_scale, U_, S_, V_, world)
        del U_, S_, V_

    f_proj, f_qr, f_small = algorithmic_flops(m_local if emu else m_global, n, l, q)
    f_total = f_proj + f_qr + f_small
    ms_per_step = elapsed / args.steps * 1e3
    value = f_total * args.steps / elapsed / 1e12
    if fast:
        fast["value_tflops"] = f_total / (fast["ms_per_step"] * 1e-3) / 1e12

    # dominant projection kernel (per launch: 2 m_local n l flops over m_local n A elements); the
    # sketch (its own kernel -- e4m3 x e4m3 on the fp8 MFMA for fp8 A -- and a single pass) is
    # reported apart in roofline.sketch, so it is taken out of the A*X (hi/lo) average here
    nn_ms = tm["nn_ms"] - tm.get("sketch_ms", 0.0)
    nn_n = tm["nn_launches"] - tm.get("sketch_launches", 0)
    kinds = [("proj_nn (Y = A X)", nn_ms, nn_n), ("proj_tn (Z = A^T Q)", tm["tn_ms"], tm["tn_launches"])]
    kname, kms, kn = max(kinds, key=lambda x: x[1])
    avg_ms = kms / max(kn, 1)
    flop_launch = 2.0 * m_local * n * l
    a_bytes = m_local * n * ELEM_BYTES[dt]
    ai = flop_launch / a_bytes
    t_s = avg_ms * 1e-3
    if ai * PEAK_HBM_GBS / 1e3 < PEAK_TFLOPS[dt]:  # HBM-bound: AI x 8 TB/s below the MFMA peak
        bound, achieved, peak, unit = "hbm", a_bytes / t_s / 1e9, PEAK_HBM_GBS, "GB/s"
    else:
        bound, achieved, peak, unit = "mfma", flop_launch / t_s / 1e12, PEAK_TFLOPS[dt], "TFLOP/s"
    key = f"{args.config}_{dt}_{m_local}x{n}_l{l}_q{q}"
    lowp = dt in ("bf16", "fp8")
    per_op = 1  # kernel dispatches per timed projection (the HIP events bracket the whole product)
    if lowp:  # the LDS-DMA kernels (hi/lo split skinny operand): wproj3 (bf16, LP 256 / 512; TN at
        # LP 256 with two-step A slots: wproj3tn2), wproj3tn4 (e4m3 TN, four-step A slots),
        # wproj2<FP8, NN, LP, SPLIT> otherwise
        nn = kname.startswith("proj_nn")
        LPk = lp_pad(l)
        if dt == "bf16" and LPk == 256 and not nn:
            kpref = "wproj3tn2_kernel<true"
        elif dt == "bf16" and LPk == 128 and not nn and os.environ.get("RSVD_TN128", "1") != "0":
            kpref = "wproj3tn128_kernel<true"  # C3's TN on separate A / S rings (K chunks of 64 rows)
        elif dt == "bf16" and LPk == 128 and nn and os.environ.get("RSVD_NN3_128", "1") != "0":
            kpref = "wproj3_kernel<true, 128, true"  # the hi / lo NN at LP = 128 on the v3 kernel
        elif dt == "fp8" and LPk == 512 and nn and os.environ.get("RSVD_NN8", "1") != "0":
            kpref = "wproj3nn8_kernel<true"  # e4m3 NN halves on the v3 addressing, one dispatch
        elif dt == "fp8" and LPk in (256, 512) and not nn:
            kpref = "wproj3tn4_kernel<true"  # e4m3 TN, 128-B A lines; LP = 512 as two column halves in one dispatch
        elif dt == "bf16" and LPk in (256, 512):
            kpref = f"wproj3_kernel<{'true' if nn else 'false'}, {LPk}, true"
        elif dt == "fp8" and LPk == 512:  # two 256-column halves per product (WProjPlan::half), one dispatch
            kpref = f"wproj2_kernel<true, {'true' if nn else 'false'}, 256, true"
        else:
            kpref = f"wproj2_kernel<{'true' if dt == 'fp8' else 'false'}, {'true' if nn else 'false'}, {LPk}, true"
    else:
        kpref = "proj_tn_kernel" if kname.startswith("proj_tn") else "proj_nn_kernel"
    tr = pmc_traffic(key, kpref)
    if tr:
        tr = (tr[0] * per_op, tr[1])
    mb = pmc_mfma_busy(key, kpref)
    roof = {
        "bound": bound,
        "kernel": kname,
        "achieved": achieved,
        "peak": peak,
        "unit": unit,
        "frac": achieved / peak,
        "traffic": tr[0] if tr else None,
        "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
        "kernel_dispatches_per_launch": per_op,
        "traffic_source": tr[1] if tr else None,
        "avg_launch_us": avg_ms * 1e3,
        "algorithmic_flop_per_launch": flop_launch,
        "algorithmic_bytes_per_launch": a_bytes,
        "achieved_TFLOPs": flop_launch / t_s / 1e12,
        "achieved_GBps": a_bytes / t_s / 1e9,
        "launches_timed": kn,
        "proj_share_of_step": (tm["nn_ms"] + tm["tn_ms"]) / (elapsed * 1e3) if elapsed > 0 else None,
        # MFMA pipe occupancy of the same kernel (hi/lo work included) from the committed PMC pass
        "mfma_busy_pmc": mb,
    }

    # the sketch Y = A Omega alone (single pass: Omega is exact in the storage type)
    sk_n = tm.get("sketch_launches", 0)
    if sk_n:
        sk_s = tm["sketch_ms"] / sk_n * 1e-3
        sk_tf = flop_launch / sk_s / 1e12
        sk_gbs = a_bytes / sk_s / 1e9
        sk_peak = PEAK_FP8_TFLOPS if dt == "fp8" else PEAK_TFLOPS[dt]
        if ai * PEAK_HBM_GBS / 1e3 < sk_peak:
            sk = {"bound": "hbm", "achieved": sk_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": sk_gbs / PEAK_HBM_GBS}
        else:
            sk = {"bound": "mfma", "achieved": sk_tf, "peak": sk_peak, "unit": "TFLOP/s", "frac": sk_tf / sk_peak}
        sk.update({"kernel": "sketch Y = A Omega" + (" (e4m3 x e4m3, block-scaled v_mfma_scale_f32_16x16x128_f8f6f4, unit scales)"
                                          if dt == "fp8" else ""),
                   "avg_launch_us": sk_s * 1e6, "achieved_TFLOPs": sk_tf, "achieved_GBps": sk_gbs, "launches_timed": sk_n})
        roof["sketch"] = sk

    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0 and not emu:
        rows = m_local if cpu_rows is None else min(cpu_rows, m_local)
        Ah = A[:rows]
        Ah = (Ah.float() * a_scale if dt == "fp8" else Ah).double().cpu().numpy()
        note = "(the full A)" if rows == m_local else f"(the first {rows} rows of the same A: bounded sample)"
        threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
        cpu = cpu_baseline(Ah, l, q, args.cpu_budget, threads, note)

    c1 = c1_extras(torch, R, eng, A, q, max(args.cpu_budget, 3.0)) if args.config == "c1" and rank == 0 else None

    if rank == 0:
        par = "single-gpu" if world == 1 else (f"row-partition x{world}" if strong else f"row-shard x{world}")
        if emu:
            par = (f"EMULATED rank 0 of {emu} on one GPU (no-op collectives; n shard {info.get('n_shard_rows')} "
                   f"rows): per-rank kernel time only, not an N-GPU measurement")
        if world > 1 and info.get("n_shard_rows"):
            par += f", n side sharded ({info['n_shard_rows']} rows/GPU)"
        if world > 1:
            par += (", gloo via torch.distributed hooks (test mode)" if args.backend == "gloo" else
                    ", RCCL " + ("owned by the C ABI (rsvd_comm_init)" if args.comm == "library" else "via torch.distributed hooks"))
        line = {
            "metric": "rSVD wall-clock + achieved TFLOP/s, dense m x n rank-k",
            "value": value,
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": dt,
            "data": "synthetic",
            "config": {
                "workload": label + (f"; {m_global}x{n} global, {m_local} rows/GPU" if world > 1 else ""),
                "m": m_global, "n": n, "l": l, "q": q, "m_per_gpu": m_local,
                "lda": int(A.stride(1)) if A.dim() == 2 else m_local,
                "parallelism": par,
                "algorithmic_tflop_per_step": f_total / 1e12,
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "engine_info": info,
            "check": check,
            "lowp_intermediates": fast,
        }
        if c1 is not None:
            line["c1"] = c1
        print(json.dumps(line), flush=True)
    eng.close()  # releases the handle's RCCL communicator (rsvd_destroy)
    if world > 1:
        dist.destroy_process_group()
    if os.environ.get("RSVD_MAPS_OUT"):  # diagnostics: the process's mappings, to symbolise an exit-time fault
        with open("/proc/self/maps") as f, open(os.environ["RSVD_MAPS_OUT"], "w") as g:
            g.write(f.read())


if __name__ == "__main__":
    main()
