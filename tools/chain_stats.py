"""Per-rSVD kernel time by stage from a rocprofv3 kernel-stats CSV (profiles/r05_*_kernel_stats.csv).

The rSVD count is the number of tridiag_bisect_kernel (eigensolver small SVD) or small_svd_kernel
launches: one per rSVD.  Stages: projections (wproj*, proj_*, sum_slabs), the QR panel work (Grams,
panel products, split, repair), the replicated l x l factor chain (leaf factors, R^-1, the two-level
GEMMs and glue, the predicated fallback launches), and the replicated small SVD (eigensolver stages
and the block-Jacobi check / finish).  usage: python tools/chain_stats.py <kernel_stats.csv>"""
import csv
import sys

STAGES = [
    ("projections", ("wproj", "proj_nn", "proj_tn", "sum_slabs")),
    ("factor chain (replicated)", ("chol_reg", "chol_wide", "rinv_wide", "gemmsq", "chol2_", "gram_chol")),
    ("small SVD (replicated)", ("tridiag", "cluster_orth", "wy_", "sqgemm", "block_jacobi", "small_svd", "convert_scale")),
    ("QR panel work (sharded)", ("gram_", "panel_", "split_mat", "repair", "robust_orth")),
    ("other", ("",)),
]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nr = None
    for r in rows:
        if "tridiag_bisect_kernel" in r["Name"] or "small_svd_kernel" in r["Name"]:
            nr = int(r["Calls"])
    tot = {s: 0.0 for s, _ in STAGES}
    for r in rows:
        n = r["Name"]
        if "rsvd::" not in n:
            continue  # bench.py's own torch kernels (A generation, the self-check)
        t = float(r["TotalDurationNs"]) / nr / 1e3
        for s, keys in STAGES:
            if any(k in n for k in keys):
                tot[s] += t
                break
    print(f"{sys.argv[1]}: {nr} rSVDs")
    for s, _ in STAGES:
        print(f"  {s:28s} {tot[s] / 1e3:7.3f} ms per rSVD")
    print(f"  {'total':28s} {sum(tot.values()) / 1e3:7.3f} ms")


if __name__ == "__main__":
    main()
