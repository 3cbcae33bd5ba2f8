"""The kernel sequence of one rSVD from a rocprofv3 rocpd database: name, duration, gap to the previous
launch's end.  The rSVD is the one ending at the k-th launch of `marker` counted from the end
(default: the second-to-last tridiag_bisect_kernel, which sits inside the timed loop).

Usage: rocpd_seq.py <db> [marker] [k]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = db.execute(f"select {name}, start, end from kernels order by start").fetchall()
marker = sys.argv[2] if len(sys.argv) > 2 else "tridiag_bisect_kernel"
k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
idx = [i for i, r in enumerate(rows) if marker in r[0]]
hi, lo = idx[-k], idx[-k - 1]
# the rSVD: from just after the previous marker's rSVD (its last launch) to this one's; take the
# launches between the two markers, shifted so the sequence starts at this rSVD's first projection
seq = rows[lo + 1:hi + 1]
first = next((i for i, r in enumerate(seq) if "wproj" in r[0] or "proj_nn" in r[0]), 0)
seq_prev_tail = seq[:first]
seq = seq[first:] + []
tail = rows[hi + 1:hi + 1 + len(seq_prev_tail)]
seq = seq + tail


def short(n):
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"rsvd::\(anonymous namespace\)::", "", n)
    return re.sub(r"\(.*$", "", n)[:70]


tot = 0
prev_end = None
for n, s, e in seq:
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    tot += e - s
    print(f"{(e - s) / 1e3:9.1f} us  gap {gap:6.1f}  {short(n)}")
    prev_end = e
print(f"{len(seq)} launches, {tot / 1e3:.1f} us of kernel time, span {(seq[-1][2] - seq[0][1]) / 1e3:.1f} us")
