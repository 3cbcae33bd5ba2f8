"""The N-GPU step priced from kernels that really run.

Input: the rocprofv3 kernel stats of `bench.py --config <c> --emulate-world N` (rank 0 of an N-rank job on
one GPU: its rows of A, its n shard, the fp64 Grams of sharded panels; every collective a no-op) and the
config.  Output: per-rSVD kernel time by stage (tools/chain_stats.py's stages) plus the collectives the
engine issues at that world size, priced from their volumes -- RCCL over xGMI is not measurable on a
one-GPU box, so they carry stated assumptions: a reduce-scatter / all-gather of V bytes per rank moves
(N-1)/N V over the ring at RING_GBS per GPU, an all-reduce of V bytes costs 2 (N-1)/N V at that rate, and
every collective launch costs LAT_US.

usage: python tools/model8.py <kernel_stats.csv> <config c4|c5> [N] [extra all-reduces]
"""
import csv
import sys

RING_GBS = 300.0  # per-GPU ring bandwidth for 1-64 MB collectives over xGMI (2 of 7 ~153 GB/s links)
LAT_US = 40.0     # per collective (launch + ring latency for <= 2 MB)

STAGES = [
    ("projections", ("wproj", "proj_nn", "proj_tn", "sum_slabs")),
    ("factor chain (replicated)", ("chol_reg", "chol_wide", "rinv_wide", "gemmsq", "chol2_", "gram_chol")),
    ("small SVD (replicated)", ("tridiag", "cluster_orth", "wy_", "sqgemm", "block_jacobi", "small_svd", "convert_scale",
                                "finish_convert")),
    ("QR panel work (sharded)", ("gram_", "panel_", "split_mat", "repair", "robust_orth")),
    ("other", ("",)),
]
CFG = {"c4": (65536, 65536, 256, 2, 2), "c5": (131072, 8192, 512, 2, 1)}  # m, n, l, q, bytes of A


def main():
    path, cfg = sys.argv[1], sys.argv[2]
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    # extra LP^2 all-reduces per rSVD: RSVD_GRAM_SPLIT_SHARDED=1 sums each split pass's predicated fp64
    # fallback Gram whether or not it runs (8 per rSVD at q = 2)
    extra = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    m, n, l, q, _ = CFG[cfg]
    rows = list(csv.DictReader(open(path)))
    nr = max(int(r["Calls"]) for r in rows if "tridiag_bisect_kernel" in r["Name"] or "small_svd_kernel" in r["Name"])
    tot = {s: 0.0 for s, _ in STAGES}
    for r in rows:
        if "rsvd::" not in r["Name"]:
            continue
        t = float(r["TotalDurationNs"]) / nr / 1e3
        for s, keys in STAGES:
            if any(k in r["Name"] for k in keys):
                tot[s] += t
                break
    LP = 1 << (l - 1).bit_length()
    nc = -(-(-(-n // N)) // 32) * 32
    # collectives per rSVD (wide.cpp, n side sharded): Gram all-reduces -- m side q + 2 (the sketch, the
    # q - 1 intermediates, the output panel's two passes) and its repair pass, n side the same, the cross
    # Gram R -- 2 q + 7; reduce-scatters of A^T Q (q + 1); all-gathers of the hi / lo X panels (q, two
    # each) and of V
    ar_small = 2 * q + 7 + extra
    b_lp2 = LP * LP * 8
    rs = (q + 1) * N * nc * LP * 4
    ag = q * 2 * N * nc * LP * 2 + N * nc * LP * 4
    coll = {
        f"{ar_small} all-reduces of LP^2 fp64 ({b_lp2 / 2**20:.1f} MiB)":
            ar_small * (LAT_US + 2 * (N - 1) / N * b_lp2 / (RING_GBS * 1e3)),
        f"{q + 1} reduce-scatters of A^T Q ({N * nc * LP * 4 / 2**20:.0f} MiB)":
            (q + 1) * LAT_US + (N - 1) / N * rs / (RING_GBS * 1e3),
        f"{2 * q + 1} all-gathers (hi / lo X, V)": (2 * q + 1) * LAT_US + (N - 1) / N * ag / (RING_GBS * 1e3),
    }
    print(f"{path}: {nr} rSVDs; rank 0 of {N} ({cfg}: {m // N} rows of A, n shard {nc} rows)")
    for s, _ in STAGES:
        print(f"  {s:34s} {tot[s] / 1e3:7.3f} ms")
    kern = sum(tot.values()) / 1e3
    print(f"  {'kernels per rank':34s} {kern:7.3f} ms")
    for k, v in coll.items():
        print(f"  {k:34s} {v / 1e3:7.3f} ms (modelled)")
    total = kern + sum(coll.values()) / 1e3
    print(f"  {'N-GPU step (kernels + collectives)':34s} {total:7.3f} ms")


if __name__ == "__main__":
    main()
