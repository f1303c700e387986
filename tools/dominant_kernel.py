"""Runs the bench's dominant kernel (dec_conv1b-shaped 3x3 conv 96->96, 64 x 256^2) a few times:
the workload profiled with rocprofv3 --pmc for the roofline 'traffic' field.  KERNEL=x6 runs the
split-bf16 fp32 kernel (--conv-precision fp32_x6) instead of the fp32 one; KERNEL=bf16 the bf16
kernel of the adapter-finetune frozen base (BASELINE configs[4]: 16 x 512^2); KERNEL=wgrad the
bf16x6 weight gradient (k_wgrad3s) of the same shape at 64 x 128^2."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import _lib  # noqa: E402

KIND = os.environ.get("KERNEL", "")
bs, H, W = {"bf16": (16, 512, 512), "wgrad": (64, 128, 128)}.get(KIND, (64, 256, 256))
dev = torch.device("cuda", 0)
x = torch.randn(bs, H, W, 96, device=dev)
w = torch.randn(96, 96, 3, 3, device=dev) * 0.05
b = torch.zeros(96, device=dev)
y = torch.empty_like(x)
s = torch.cuda.current_stream(dev).cuda_stream
x6 = KIND == "x6"
if KIND == "wgrad":  # the bf16x6 3x3 weight gradient of dec_conv1b's shape at the step's 128^2
    y.normal_()
    dwb = torch.empty(96 * 96 * 9 + 96, device=dev)
    pk = _lib.scratch(_lib.lib().dn_conv2d_wgrad_slab_size(bs, H, W, 96, 96, 3), dev)
elif x6:
    pk = _lib.scratch(_lib.lib().dn_conv2d_x6_pack_size(96, 96, 0), dev)
elif KIND == "bf16":
    pk = _lib.scratch(_lib.lib().dn_conv2d_bf16_pack_size(96, 96), dev)
else:
    pk = _lib.scratch(_lib.lib().dn_conv2d_pack_size(96, 96, 3, 0), dev)
for _ in range(int(os.environ.get("REPS", "4"))):
    if KIND == "wgrad":
        _lib.call("dn_conv2d_backward_weight_x6", y.data_ptr(), x.data_ptr(), 96, bs, H, W, 96, 96,
                  dwb.data_ptr(), pk.data_ptr(), s)
    elif x6:
        _lib.call("dn_conv2d_forward_x6", x.data_ptr(), 96, bs, H, W, 96, w.data_ptr(),
                  b.data_ptr(), 96, 1, y.data_ptr(), 96, pk.data_ptr(), pk.numel(), s)
    elif KIND == "bf16":
        _lib.call("dn_conv2d_forward_bf16", x.data_ptr(), 96, bs, H, W, 96, w.data_ptr(),
                  b.data_ptr(), 96, 1, y.data_ptr(), 96, pk.data_ptr(), pk.numel(), s)
    else:
        _lib.call("dn_conv2d_forward", x.data_ptr(), 96, bs, H, W, 96, w.data_ptr(), b.data_ptr(),
                  96, 3, 1, y.data_ptr(), 96, pk.data_ptr(), pk.numel(), s)
torch.cuda.synchronize()
print("done")
