"""Per-kernel totals from a rocprofv3 rocpd database (the default output format on this image)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = db.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels group by {name} "
                  "order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
for n, c, s, a in rows[:30]:
    print(f"{s / 1e6:9.3f} ms {100 * s / tot:6.2f}% n={c:>5} avg={a / 1e3:9.1f} us per_step={s / 1e6 / steps:8.3f} ms  {n[:100]}")
print(f"total {tot / 1e6:.3f} ms")
