"""Concurrency of the bench step's launches from a rocprofv3 --kernel-trace CSV
(tools/gpu_run.sh stats:TAG -> gpurun_out/prof/TAG/.../run_kernel_trace.csv):
    python tools/step_timeline.py TRACE.csv [short_us]
Steps are cut at each k_adam launch.  Per step: wall span, time with any kernel running, the sum of
kernel durations (> span when the two streams overlap), and the time during which only short
kernels (< short_us, the small-grid tail) are running -- the part of that tail on the critical
path."""
import csv
import sys


def main():
    path = sys.argv[1]
    short = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 60e3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
                for r in csv.DictReader(open(path)))
    ends = [i for i, e in enumerate(ev) if "k_adam" in e[2]]
    for si in range(1, len(ends)):
        seg = ev[ends[si - 1] + 1:ends[si] + 1]
        t0, t1 = min(e[0] for e in seg), max(e[1] for e in seg)
        iv = sorted((e[0], e[1]) for e in seg)
        busy, (cs, ce) = 0, iv[0]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        pts = sorted({e[0] for e in seg} | {e[1] for e in seg})
        small = 0
        for a, b in zip(pts, pts[1:]):
            act = [e for e in seg if e[0] < b and e[1] > a]
            if act and all(e[1] - e[0] < short for e in act):
                small += b - a
        print(f"step {si}: span {(t1 - t0) / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, kernel sum "
              f"{sum(e[1] - e[0] for e in seg) / 1e6:.2f} ms, {len(seg)} launches on "
              f"{len(set(e[3] for e in seg))} streams, only kernels < {short / 1e3:.0f} us running: "
              f"{small / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
