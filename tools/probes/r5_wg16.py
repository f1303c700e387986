"""48->48 / 96->96 weight gradients per level through the C ABI (kernel + reduction), ms"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.x6_shapes import wgrad  # noqa: E402

for cin, cout in ((48, 48), (96, 96)):
    for H in (128, 64, 32, 16, 8):
        print(f"wgrad {cin}->{cout} H{H}: {wgrad(cin, cout, H, True):.4f} ms", flush=True)
