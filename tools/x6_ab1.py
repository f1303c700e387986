"""HIP-event timing of a few 96-output 3x3 shapes (A/B probes of the x6 / Winograd kernels):
python tools/x6_ab1.py -> one line per shape; SHAPES="fwd:48:48:256,dgrad:48:48:128" overrides."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.x6_shapes import dgrad, fwd  # noqa: E402

PEAK = 2500.0 / 6
N = int(os.environ.get("N", "64"))
SHAPES = [("fwd", 96, 96, 256), ("fwd", 96, 96, 128), ("dgrad", 96, 96, 128), ("fwd", 100, 96, 256),
          ("fwd", 144, 96, 128)]
if os.environ.get("SHAPES"):
    SHAPES = [(o, int(ci), int(co), int(h)) for o, ci, co, h in
              (t.split(":") for t in os.environ["SHAPES"].split(","))]
if __name__ == "__main__":
    for op, cin, cout, H in SHAPES:
        fl = 2.0 * N * H * H * cin * cout * 9
        ms = (fwd if op == "fwd" else dgrad)(cin, cout, H, True)
        print(f"{op:5s} {cin:3d}->{cout:3d} H{H:4d} {ms:7.3f} ms frac {fl / ms / 1e9 / PEAK:.3f}", flush=True)
