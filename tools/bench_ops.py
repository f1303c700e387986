"""Micro-benchmarks of single C-ABI ops on the GPU (HIP events on the launch stream).
Used to tune layouts; not part of the product.  python tools/bench_ops.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import _lib  # noqa: E402


def timeit(fn, reps=10):
    s = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def deconv(N, h, w, C, y_stride):
    x = torch.randn(N, h, w, C, device="cuda")
    wt = torch.randn(C, C, 2, 2, device="cuda") * 0.05
    b = torch.zeros(C, device="cuda")
    y = torch.empty(N, 2 * h, 2 * w, y_stride, device="cuda")
    pk = _lib.scratch(_lib.lib().dn_deconv2x2_pack_size(C, C, 0), "cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.call("dn_deconv2x2_forward", x.data_ptr(), N, h, w, C, wt.data_ptr(),
                          b.data_ptr(), C, y.data_ptr(), y_stride, 0, pk.data_ptr(), pk.numel(), st)
    ms = timeit(f)
    gb = (x.numel() + N * 4 * h * w * C) * 4 / 1e9
    fl = 2.0 * N * h * w * 4 * C * C
    print(f"deconv N={N} {h}x{w} C={C} y_stride={y_stride}: {ms*1e3:8.1f} us  "
          f"{gb/ms:6.2f} TB/s(alg)  {fl/ms/1e9:6.1f} TF/s", flush=True)


def deconv_x6(N, h, w, y_stride, y_off=0):
    """the bf16x6 ConvTranspose2d(96, 96, 2, 2) of the training path (k_deconv_x6)"""
    x = torch.randn(N, h, w, 96, device="cuda")
    wt = torch.randn(96, 96, 2, 2, device="cuda") * 0.05
    b = torch.zeros(96, device="cuda")
    y = torch.empty(N, 2 * h, 2 * w, y_stride, device="cuda")
    pk = _lib.scratch(_lib.lib().dn_deconv2x2_x6_pack_size(), "cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.call("dn_deconv2x2_forward_x6", x.data_ptr(), N, h, w, wt.data_ptr(),
                          b.data_ptr(), y.data_ptr(), y_stride, y_off, pk.data_ptr(), pk.numel(), st)
    ms = timeit(f)
    gb = (x.numel() + N * 4 * h * w * 96) * 4 / 1e9
    print(f"deconv_x6 N={N} {h}x{w} y_stride={y_stride}: {ms*1e3:8.1f} us  "
          f"{gb/ms:6.2f} TB/s(alg)", flush=True)


def conv(N, H, W, Cin, Cout, k, x_stride, y_stride):
    x = torch.randn(N, H, W, x_stride, device="cuda")
    wt = torch.randn(Cout, Cin, k, k, device="cuda") * 0.05
    b = torch.zeros(Cout, device="cuda")
    y = torch.empty(N, H, W, y_stride, device="cuda")
    pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(Cin, Cout, k, 0), "cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.call("dn_conv2d_forward", x.data_ptr(), x_stride, N, H, W, Cin, wt.data_ptr(),
                          b.data_ptr(), Cout, k, 1, y.data_ptr(), y_stride, pk.data_ptr(),
                          pk.numel(), st)
    ms = timeit(f)
    fl = 2.0 * N * H * W * Cin * Cout * k * k
    print(f"conv{k}x{k} N={N} {H}x{W} {Cin}->{Cout} xs={x_stride} ys={y_stride}: {ms*1e3:8.1f} us "
          f"{fl/ms/1e9:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    if os.environ.get("OPS") == "deconv_x6":
        for (h, ys) in ((128, 100), (64, 144), (32, 144), (128, 96)):
            deconv_x6(64, h, h, ys)
        sys.exit(0)
    for ys in (96, 100, 128, 144):
        deconv(64, 128, 128, 96, ys)
    for ys in (96, 144):
        deconv(64, 64, 64, 96, ys)
    for xs, ys in ((96, 96), (100, 96), (128, 96), (96, 128)):
        conv(64, 256, 256, 96, 96, 1, xs, ys)
    conv(64, 256, 256, 96, 96, 3, 96, 96)
    conv(64, 256, 256, 97, 96, 3, 100, 96)
    conv(64, 256, 256, 97, 96, 3, 128, 96)
