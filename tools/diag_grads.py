"""Per-layer gradient error of the HIP UNet vs an fp64 oracle, next to the reference fp32 error."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import UNet  # noqa: E402
from oracle.unet_ref import forward, layer_table  # noqa: E402


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


g = dict(np.load("tests/golden/unet_c1.npz"))
torch.manual_seed(0)
net = UNet(1, 1, 48).cuda()
x = torch.from_numpy(g["x"])
for loss_kind in ("mean_y2", "sum_y"):
    y = net(x.cuda())
    for p in net.parameters():
        p.grad = None
    L = (y ** 2).mean() if loss_kind == "mean_y2" else y.sum()
    L.backward()
    gg = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).cpu().numpy()
    p64 = net.flat_params.detach().cpu().double().requires_grad_(True)
    y64 = forward(p64, x.double(), 1, 1)
    L64 = (y64 ** 2).mean() if loss_kind == "mean_y2" else y64.sum()
    L64.backward()
    g64 = p64.grad.numpy()
    p32 = net.flat_params.detach().cpu().clone().requires_grad_(True)
    y32 = forward(p32, x, 1, 1)
    ((y32 ** 2).mean() if loss_kind == "mean_y2" else y32.sum()).backward()
    g32 = p32.grad.numpy()
    print(f"== loss {loss_kind}")
    off = 0
    for name, ws, bl, _ in layer_table(1, 1):
        nw = int(np.prod(ws))
        sl = slice(off, off + nw)
        sb = slice(off + nw, off + nw + bl)
        print(f"{name:12s} W gpu {rel(gg[sl], g64[sl]):9.2e} cpu32 {rel(g32[sl], g64[sl]):9.2e} |g| {np.abs(g64[sl]).max():8.1e}"
              f"   b gpu {rel(gg[sb], g64[sb]):9.2e} cpu32 {rel(g32[sb], g64[sb]):9.2e}")
        off += nw + bl
