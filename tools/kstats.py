"""Summarise a rocprofv3 rocpd database (kernel-trace): per-kernel totals, or per-dispatch
shapes of the kernels matching a pattern.

    python tools/kstats.py gpurun_out/prof/run_results.db [--csv out.csv] [--shapes PATTERN]
"""
import argparse
import collections
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--shapes")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--seq", help="print the last --last dispatches matching this, in order")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, "
                     "accum_vgpr_count, lds_size from kernels").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0, 1e30, 0.0])
    for name, d, *_ in rows:
        s = agg[name]
        s[0] += 1; s[1] += d; s[2] = min(s[2], d); s[3] = max(s[3], d)
    tot = sum(v[1] for v in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for n, (k, t, mn, mx) in out:
                w.writerow([n, k, int(t), t / k, 100.0 * t / tot, int(mn), int(mx)])
    for n, (k, t, mn, mx) in out[:a.top]:
        print(f"{t/1e6:9.2f} ms {k:6d} {t/k/1e3:9.1f} us {100*t/tot:5.1f}% {n[:100]}")
    print(f"total {tot/1e6:.2f} ms")
    if a.seq:
        seq = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels "
                        "order by start").fetchall()
        seq = [r for r in seq if a.seq in r[0]][-a.last:]
        for name, d, gx, gy, gz, wx in seq:
            print(f"{d/1e3:9.1f} us  blocks {gx // max(wx, 1):6d} x {gy:3d} x {gz}  {name[:60]}")
    if a.shapes:
        shp = collections.defaultdict(lambda: [0, 0.0])
        for name, d, gx, gy, gz, wx, v, av, lds in rows:
            if a.shapes in name:
                key = (name[:60], gx // max(wx, 1), gy, gz, v, av, lds)
                shp[key][0] += 1; shp[key][1] += d
        for key, (k, t) in sorted(shp.items(), key=lambda kv: -kv[1][1]):
            print(f"{t/k/1e3:9.1f} us x{k:3d}  blocks {key[1]:7d} x {key[2]:3d} x {key[3]}  "
                  f"vgpr {key[4]}+{key[5]} lds {key[6]}  {key[0]}")


if __name__ == "__main__":
    main()
