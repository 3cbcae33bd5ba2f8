#!/usr/bin/env python
"""bench.py -- BASELINE.json metric: "rSVD wall-clock + achieved TFLOP/s, dense m x n rank-k".

Workload (BASELINE.json configs[1], "C2"): dense 4096 x 4096 fp32 A, l = 64, q = 2 power
iterations, SVDMethod::Jacobi small SVD -- one full rSVD() (src/rSVD.cpp:72-133) per step, A
resident in HBM before the timed region.  Synthetic A = X diag(0.9^t) Y^T / sqrt(n) + 1e-3 N
(SURVEY.md §8(d)), X, Y Gaussian with 128 columns.

N GPUs (torchrun, one process per GPU, RCCL): weak scaling by rows -- rank g owns
m_per_gpu = 4096 rows of a (4096 N) x 4096 matrix (src/rSVD.cpp:20-23 split); the n-side panels
are summed with all_reduce and orthonormalised redundantly, U stays row-sharded.
value = whole-job algorithmic TFLOP/s (F_proj + F_qr + F_small of the global
problem) / max-over-ranks wall time; ms_per_step = rSVD wall-clock.

Extra fields: "roofline" (the dominant projection kernel, HIP-event timed in a second pass over
the same K steps), "cpu_baseline" (the fp64 C oracle -- a restatement of the reference, Eigen is
absent -- on rank 0 at N = 1 on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# MI355X dense peaks (MI355X_MICROARCH.md): fp32 matrix 157.3 TF/s, fp64 matrix 78.6 TF/s, HBM 8 TB/s.
PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}
PEAK_HBM_GBS = 8000.0


def algorithmic_flops(m, n, l, q):
    """F_proj, F_qr, F_small of one rSVD."""
    f_proj = 2.0 * m * n * l * (2 * q + 2)
    f_qr = (q + 1) * (4.0 * m * l * l - 4.0 * l ** 3 / 3) + q * (4.0 * n * l * l - 4.0 * l ** 3 / 3)
    f_small = 4.0 * n * l * l - 4.0 * l ** 3 / 3 + 2.0 * n * l * l + 2.0 * m * l * l
    return f_proj, f_qr, f_small


def make_A(torch, m_local, n, rank, dtype, rank_cols=128, seed=0x5EED0002):
    """Column-major rows [rank*m_local, ...) of the synthetic A, built on the GPU."""
    dev = torch.device("cuda")
    gY = torch.Generator(device=dev).manual_seed(seed)
    gX = torch.Generator(device=dev).manual_seed(seed + 1 + rank)
    gN = torch.Generator(device=dev).manual_seed(seed + 7919 + rank)
    sig = 0.9 ** torch.arange(rank_cols, device=dev, dtype=torch.float32)
    Y = torch.randn(n, rank_cols, generator=gY, device=dev)
    X = torch.randn(m_local, rank_cols, generator=gX, device=dev)
    At = (Y * sig) @ X.t() / (n ** 0.5)                       # n x m_local row-major == A^T
    At += 1e-3 * torch.randn(n, m_local, generator=gN, device=dev)
    return At.to(dtype).t()                                    # m_local x n, column-major view


def pmc_traffic(key, kernel_prefix):
    """HBM bytes per launch of the kernel from the committed rocprofv3 PMC summary for this
    workload (profiles/*_traffic.json, written by tools/profile.sh + tools/traffic.py; FETCH_SIZE
    doubled per the gfx950 correction).  None when no summary for this workload exists."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json"))):
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


def cpu_baseline(A_host, l, q, flops_total, budget_s, threads):
    import oracle

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
    return {
        "value": flops_total / per / 1e12,
        "unit": "TFLOP/s",
        "cores": used,
        "kind": "port",
        "sample": f"{reps} full rSVD calls of the same {A_host.shape[0]}x{A_host.shape[1]} A (l={l}, q={q}) "
                  f"in the fp64 C oracle (oracle/rsvd_oracle.c, -O3 -fopenmp); {per * 1e3:.1f} ms per rSVD",
        "ms_per_rsvd": per * 1e3,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--m-per-gpu", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--l", type=int, default=64)
    ap.add_argument("--q", type=int, default=2)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-oracle work (0 = skip)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import rsvd_kamaneh_raganato_terrana_amd as R

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))

    tdt = torch.float32 if args.dtype == "f32" else torch.float64
    m_local, n, l, q = args.m_per_gpu, args.n, args.l, args.q
    m_global = m_local * world
    A = make_A(torch, m_local, n, rank, tdt)
    eng = R.Engine(local_rank)
    if world > 1:
        eng.set_comm(rank, world)
    torch.cuda.synchronize()

    def step():
        return eng.rsvd(A, l, q=q, seed=0x5EED0002)

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
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    elapsed = timed(args.steps)
    # pass 2: same K steps with hipEvent pairs around every projection kernel (roofline)
    eng.set_timing(True)
    timed(args.steps)
    tm = eng.timing()
    eng.set_timing(False)
    info = eng.info()

    f_proj, f_qr, f_small = algorithmic_flops(m_global, n, l, q)
    f_total = f_proj + f_qr + f_small
    ms_per_step = elapsed / args.steps * 1e3
    value = f_total * args.steps / elapsed / 1e12

    # dominant projection kernel (per launch: 2 m_local n l flops, m_local n A elements)
    kinds = [("proj_nn (Y = A X)", tm["nn_ms"], tm["nn_launches"]), ("proj_tn (Z = A^T Q)", tm["tn_ms"], tm["tn_launches"])]
    kname, kms, kn = max(kinds, key=lambda x: x[1])
    avg_ms = kms / max(kn, 1)
    flop_launch = 2.0 * m_local * n * l
    a_bytes = m_local * n * (4 if args.dtype == "f32" else 8)
    achieved = flop_launch / (avg_ms * 1e-3) / 1e12
    key = f"c2_{args.dtype}_{m_local}x{n}_l{l}_q{q}"
    tr = pmc_traffic(key, "proj_tn_kernel" if kname.startswith("proj_tn") else "proj_nn_kernel")
    roof = {
        "bound": "mfma",
        "kernel": kname,
        "achieved": achieved,
        "peak": PEAK_TFLOPS[args.dtype],
        "unit": "TFLOP/s",
        "frac": achieved / PEAK_TFLOPS[args.dtype],
        "traffic": tr[0] if tr else None,
        "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
        "traffic_source": tr[1] if tr else None,
        "avg_launch_us": avg_ms * 1e3,
        "algorithmic_flop_per_launch": flop_launch,
        "algorithmic_bytes_per_launch": a_bytes,
        "achieved_GBps": a_bytes / (avg_ms * 1e-3) / 1e9,
        "launches_timed": kn,
        "proj_share_of_step": (tm["nn_ms"] + tm["tn_ms"]) / (elapsed * 1e3) if elapsed > 0 else None,
    }

    cpu = None
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        A_host = A.detach().double().cpu().numpy()
        threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
        cpu = cpu_baseline(A_host, l, q, f_total, args.cpu_budget, threads)

    if rank == 0:
        line = {
            "metric": "rSVD wall-clock + achieved TFLOP/s, dense m x n rank-k",
            "value": value,
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic",
            "config": {
                "workload": f"C2: dense {m_global}x{n} {args.dtype} rSVD, l={l}, q={q}, Jacobi small SVD"
                            + (f", rows sharded {m_local}/GPU" if world > 1 else ""),
                "m": m_global, "n": n, "l": l, "q": q, "m_per_gpu": m_local,
                "parallelism": f"row-shard x{world}" if world > 1 else "single-gpu",
                "algorithmic_tflop_per_step": f_total / 1e12,
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "engine_info": info,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
