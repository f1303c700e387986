"""HIP-event timing of the split-bf16 3x3 kernels on the step's large shapes (N = 64):
python tools/x6_micro.py -> ms, fp32-equivalent TF/s and the fraction of the bf16/6 ceiling."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.x6_shapes import dgrad, fwd, wgrad  # noqa: E402

PEAK = 2500.0 / 6
N = int(os.environ.get("N", "64"))
SHAPES = [("fwd", 96, 96, 256), ("fwd", 100, 96, 256), ("fwd", 48, 48, 256), ("fwd", 144, 96, 128),
          ("fwd", 96, 96, 128), ("dgrad", 96, 96, 128), ("dgrad", 144, 96, 64), ("dgrad", 48, 48, 128),
          ("wgrad", 96, 96, 128), ("wgrad", 144, 96, 64), ("wgrad", 48, 48, 128)]

if __name__ == "__main__":
    for op, cin, cout, H in SHAPES:
        fl = 2.0 * N * H * H * cin * cout * 9
        f = {"fwd": fwd, "dgrad": dgrad, "wgrad": wgrad}[op]
        ms = f(cin, cout, H, True)
        tf = fl / ms / 1e9
        print(f"{op:5s} {cin:3d}->{cout:3d} H{H:4d}  x6 {ms:7.3f} ms {tf:6.1f} TF/s  frac {tf / PEAK:.3f}",
              flush=True)
