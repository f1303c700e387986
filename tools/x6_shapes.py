"""fp32 vs bf16x6 3x3 kernels on the U-Net's layer shapes (N2N step sizes), HIP-event timed.
python tools/x6_shapes.py  -> one line per (op, Cin, Cout, H): fp32 ms, x6 ms, TF/s of each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import _lib  # noqa: E402
from tools.bench_ops import timeit  # noqa: E402

N = int(os.environ.get("N", "64"))


def fwd(cin, cout, H, x6):
    x = torch.randn(N, H, H, cin, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    b = torch.zeros(cout, device="cuda")
    y = torch.empty(N, H, H, cout, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    if x6:
        pk = _lib.scratch(_lib.lib().dn_conv2d_x6_pack_size(cin, cout, 0), "cuda")
        f = lambda: _lib.call("dn_conv2d_forward_x6", x.data_ptr(), cin, N, H, H, cin, w.data_ptr(),
                              b.data_ptr(), cout, 1, y.data_ptr(), cout, pk.data_ptr(), pk.numel(), st)
    else:
        pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(cin, cout, 3, 0), "cuda")
        f = lambda: _lib.call("dn_conv2d_forward", x.data_ptr(), cin, N, H, H, cin, w.data_ptr(),
                              b.data_ptr(), cout, 3, 1, y.data_ptr(), cout, pk.data_ptr(), pk.numel(), st)
    return timeit(f)


def dgrad(cin, cout, H, x6):  # dx [N,H,H,cin] from dz [N,H,H,cout]
    dz = torch.randn(N, H, H, cout, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    dx = torch.empty(N, H, H, cin, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    if x6:
        pk = _lib.scratch(_lib.lib().dn_conv2d_x6_pack_size(cin, cout, 1), "cuda")
        f = lambda: _lib.call("dn_conv2d_backward_data_x6", dz.data_ptr(), N, H, H, cout, w.data_ptr(),
                              cin, None, cin, 0, dx.data_ptr(), cin, pk.data_ptr(), pk.numel(), st)
    else:
        pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(cin, cout, 3, 1), "cuda")
        f = lambda: _lib.call("dn_conv2d_backward_data", dz.data_ptr(), N, H, H, cout, w.data_ptr(),
                              cin, 3, None, cin, 0, dx.data_ptr(), cin, pk.data_ptr(), pk.numel(), st)
    return timeit(f)


def wgrad(cin, cout, H, x6):  # dW, db from dz [N,H,H,cout] and x [N,H,H,cin] (+ the reduction)
    dz = torch.randn(N, H, H, cout, device="cuda")
    x = torch.randn(N, H, H, cin, device="cuda")
    dwb = torch.empty(cout * cin * 9 + cout, device="cuda")
    slab = _lib.scratch(_lib.lib().dn_conv2d_wgrad_slab_size(N, H, H, cin, cout, 3), "cuda")
    st = torch.cuda.current_stream().cuda_stream
    head = (dz.data_ptr(), x.data_ptr(), cin, N, H, H, cin, cout)
    if x6:
        f = lambda: _lib.call("dn_conv2d_backward_weight_x6", *head, dwb.data_ptr(), slab.data_ptr(), st)
    else:
        f = lambda: _lib.call("dn_conv2d_backward_weight", *head, 3, dwb.data_ptr(), slab.data_ptr(), st)
    return timeit(f)


if __name__ == "__main__":
    shapes = [("fwd", 48, 48, H) for H in (256, 128, 64, 32, 16, 8)] + \
             [("fwd", 96, 96, H) for H in (256, 128, 64, 32, 16)] + \
             [("fwd", 144, 96, H) for H in (128, 64, 32, 16)] + [("fwd", 100, 96, 256), ("fwd", 100, 96, 128)] + \
             [("dgrad", 48, 48, H) for H in (128, 64, 32, 16, 8, 4)] + \
             [("dgrad", 96, 96, H) for H in (128, 64, 32, 16, 8)] + \
             [("dgrad", 144, 96, H) for H in (64, 32, 16, 8)]
    for op, cin, cout, H in shapes:
        fl = 2.0 * N * H * H * cin * cout * 9
        f = fwd if op == "fwd" else dgrad
        a, b = f(cin, cout, H, False), f(cin, cout, H, True)
        print(f"{op:5s} {cin:3d}->{cout:3d} H{H:4d}  fp32 {a:7.3f} ms {fl/a/1e9:6.1f} TF/s   x6 {b:7.3f} ms "
              f"{fl/b/1e9:6.1f} TF/s   {'x6' if b < a else 'fp32'}", flush=True)
