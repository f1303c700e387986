"""Per-kernel-name time of one steady-state step in two rocpd databases, side by side (ms)."""
import collections
import sqlite3
import sys


def step_totals(db, step=3):
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "k_noise" in r[0]]
    seg = rows[starts[step]:starts[step + 1]]
    t = collections.Counter()
    for r in seg:
        t[r[0].split("(")[0].replace("void ", "").replace("dn::", "")] += (r[2] - r[1]) / 1e6
    return t, (seg[-1][2] - seg[0][1]) / 1e6


a, wa = step_totals(sys.argv[1])
b, wb = step_totals(sys.argv[2])
print(f"wall {wa:.3f} -> {wb:.3f} ms")
for k in sorted(set(a) | set(b), key=lambda k: -max(a[k], b[k])):
    if abs(a[k] - b[k]) > 0.01:
        print(f"{a[k]:8.3f} {b[k]:8.3f} {b[k] - a[k]:+8.3f}  {k[:60]}")
