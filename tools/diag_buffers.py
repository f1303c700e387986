"""Compare every saved activation and gradient buffer of the HIP workspace with the oracle."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd import UNet, _lib  # noqa: E402
from image_denoising_amd.arch_unet import _UNetFunction  # noqa: E402
from oracle.unet_ref import forward  # noqa: E402

FWD = ["c1", "a0", "a1", "c2", "c3", "c4", "c5", "a2", "a3", "a4", "a5", "p5", "a6",
       "d2a", "d3a", "d4a", "d5a", "d2b", "d3b", "d4b", "d5b", "d1a", "d1b", "na", "nb"]
BWD = ["g_nb", "g_na", "g_d1b", "g_d1a", "g_c1", "g_c2", "g_c3", "g_c4", "g_c5",
       "g_d2a", "g_d3a", "g_d4a", "g_d5a", "g_d2b", "g_d3b", "g_d4b", "g_d5b",
       "g_a2", "g_a3", "g_a4", "g_a5", "g_a6", "g_p5", "g_a0", "g_a1"]


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def run(N, H, W, scale):
    torch.manual_seed(0)
    net = UNet(1, 1, 48).cuda()
    with torch.no_grad():
        for name, p in net.named_parameters():
            if name.endswith("weight"):
                p.mul_(scale)
    x = torch.rand(N, 1, H, W, generator=torch.Generator().manual_seed(1))
    r = torch.randn(N, 1, H, W, generator=torch.Generator().manual_seed(2))
    cfg = _lib.cfg(1, 1, 48)
    desc = (ctypes.c_int64 * 300)()
    n = ctypes.c_int()
    _lib.call("dn_unet_debug_buffers", ctypes.byref(cfg), N, H, W, 1, desc, 100, ctypes.byref(n))
    ws = net._workspace(N, H, W, True, fresh=True)
    y = torch.empty(N, 1, H, W, device="cuda")
    net._run_forward(x.cuda(), y, ws)
    dflat = torch.empty_like(net.flat_params)
    net._run_backward(r.cuda().contiguous(), dflat, ws, N, H, W)
    torch.cuda.synchronize()
    wsf = ws.view(torch.float32)
    rec = {}
    p64 = net.flat_params.detach().cpu().double().requires_grad_(True)
    y64 = forward(p64, x.double(), 1, 1, record=rec)
    (y64 * r.double()).sum().backward()
    names = FWD + BWD
    print(f"== N={N} {H}x{W} weight scale {scale}: y err {rel(y.cpu().numpy(), y64.detach().numpy()):.2e}")
    line = []
    for i, name in enumerate(names):
        off, stride, lvl = desc[3 * i], desc[3 * i + 1], desc[3 * i + 2]
        h, w = H >> lvl, W >> lvl
        buf = wsf[off:off + N * h * w * stride].view(N, h, w, stride).permute(0, 3, 1, 2).cpu().numpy()
        key = name[2:] if name.startswith("g_") else name
        if key not in rec:
            continue
        t = rec[key].grad if name.startswith("g_") else rec[key]
        if name.startswith("g_") and not (name.startswith("g_c") or name == "g_p5"):
            v = rec[key].detach()  # workspace holds the pre-activation gradient
            t = torch.where(v > 0, t, t * 0.2)
        t = t.detach().numpy()
        c = t.shape[1] if name != "g_c1" else 96
        e = rel(buf[:, :c], t[:, :c])
        line.append(f"{name}:{e:.1e}")
    print("  " + " ".join(line))


for args in [(1, 64, 64, 10.0), (1, 32, 32, 10.0), (1, 64, 32, 10.0), (1, 32, 64, 10.0)]:
    run(*args)
