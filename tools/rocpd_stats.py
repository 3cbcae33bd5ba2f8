"""Per-kernel totals from a rocprofv3 rocpd database (the default output format on this image).

Usage: rocpd_stats.py <db> [marker]

`per_step` divides by the number of rSVDs the trace holds, counted from the launches of `marker`
(default: the small-SVD kernel every rSVD launches exactly once -- block_jacobi_kernel for the wide
engine, small_svd_kernel for the narrow one), not from the bench's --steps: a bench run also does
its warm-up steps, the opt-in lowp pass, the timing pass and the self-check, all inside the trace.
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = db.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels group by {name} "
                  "order by sum(end - start) desc").fetchall()
markers = [sys.argv[2]] if len(sys.argv) > 2 else ["block_jacobi_kernel", "small_svd_kernel"]
steps = 0
for mk in markers:
    steps = sum(c for n, c, _, _ in rows if mk in n and "finish" not in n and "scatter" not in n and "complete" not in n)
    if steps:
        break
steps = max(steps, 1)
tot = sum(r[2] for r in rows)
print(f"rSVDs in trace: {steps} (launches of {markers})")
for n, c, s, a in rows[:30]:
    print(f"{s / 1e6:9.3f} ms {100 * s / tot:6.2f}% n={c:>5} avg={a / 1e3:9.1f} us per_step={s / 1e6 / steps:8.3f} ms  {n[:100]}")
print(f"total {tot / 1e6:.3f} ms, per rSVD {tot / 1e6 / steps:.3f} ms of kernel time")
