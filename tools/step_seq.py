"""Kernel sequence of one steady-state training step from a rocprofv3 rocpd database (steps
delimited by k_noise): duration, name and grid per dispatch, and the step's busy/wall time.

    python tools/step_seq.py gpurun_out/prof_default/run_results.db [--step 3] [--grep PAT]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=3)
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute(
        "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "k_noise" in r[0]]
    seg = rows[starts[a.step]:starts[a.step + 1]]
    wall = (seg[-1][2] - seg[0][1]) / 1e6
    busy = sum(r[2] - r[1] for r in seg) / 1e6
    print(f"step {a.step}: {len(seg)} kernels, wall {wall:.3f} ms, busy {busy:.3f} ms")
    for r in seg:
        n = r[0].split("(")[0].replace("void ", "").replace("dn::", "")
        if a.grep and a.grep not in n:
            continue
        print(f"{(r[2] - r[1]) / 1e3:9.1f} us  {n[:44]:44s} grid={r[3] // r[6]}x{r[4]}x{r[5]}")


if __name__ == "__main__":
    main()
