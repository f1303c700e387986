"""Times the bf16x6 deconv (UP1 shape: 64 x 128^2 x 96 -> 64 x 256^2) into output buffers of
channel stride 96 / 100 / 104 / 128: whether partially written cache lines (stride 100: each
pixel leaves a 16-byte hole) cost write bandwidth."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import _lib  # noqa: E402

N, H, W = 64, 128, 128
x = torch.randn(N, H, W, 96, device="cuda")
w = torch.randn(96, 96, 2, 2, device="cuda") * 0.1
b = torch.zeros(96, device="cuda")
pk = _lib.scratch(_lib.lib().dn_deconv2x2_x6_pack_size(), "cuda")
s = torch.cuda.current_stream().cuda_stream
for stride in (96, 100, 104, 128):
    y = torch.zeros(N, 2 * H, 2 * W, stride, device="cuda")
    for _ in range(3):
        _lib.call("dn_deconv2x2_forward_x6", x.data_ptr(), N, H, W, w.data_ptr(), b.data_ptr(),
                  y.data_ptr(), stride, 0, pk.data_ptr(), pk.numel(), s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        _lib.call("dn_deconv2x2_forward_x6", x.data_ptr(), N, H, W, w.data_ptr(), b.data_ptr(),
                  y.data_ptr(), stride, 0, pk.data_ptr(), pk.numel(), s)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    gb = (x.numel() * 4 + N * 4 * H * W * 96 * 4) / 1e9
    print(f"stride {stride}: {ms * 1e3:7.1f} us  {gb / ms:6.2f} TB/s (algorithmic)")
    del y
