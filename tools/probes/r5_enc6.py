"""Diagnostic: the enc_conv6 weight-gradient gap of the headline-size step (fp32 precision).
Device grad pass at 64 x 1 x 128^2 (reference init), fp64 backward with and without the device's
own LeakyReLU slopes / pool routing; per-layer errors for both precisions."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from tests.test_gpu_parity import _device_activations, _layer_errs, _net  # noqa: E402
from oracle.unet_ref import forward  # noqa: E402

N, H = int(os.environ.get("N", "64")), int(os.environ.get("H", "128"))
x = torch.rand(N, 1, H, H, generator=torch.Generator().manual_seed(1))
r = torch.randn(N, 1, H, H, generator=torch.Generator().manual_seed(2)) * 1e-3
for prec in ("fp32", "fp32_x6"):
    net = _net(1, prec)
    y, gg, acts = _device_activations(net, x, r)
    flat = net.flat_params.detach().cpu()
    out = {}
    for tag, m in (("masked", acts), ("free", None)):
        p64 = flat.double().requires_grad_(True)
        y64 = forward(p64, x.double(), 1, 1, masks=m)
        (y64 * r.double()).sum().backward()
        out[tag] = _layer_errs(gg.numpy(), p64.grad.numpy())
    p32 = flat.clone().requires_grad_(True)
    (forward(p32, x, 1, 1) * r).sum().backward()
    p64 = flat.double().requires_grad_(True)
    (forward(p64, x.double(), 1, 1) * r.double()).sum().backward()
    e32 = _layer_errs(p32.grad.numpy(), p64.grad.numpy())
    print(prec, "worst masked:", sorted(out["masked"].items(), key=lambda kv: -kv[1])[:3])
    print(prec, "worst free:  ", sorted(out["free"].items(), key=lambda kv: -kv[1])[:3])
    print(prec, "oracle fp32 free:", sorted(e32.items(), key=lambda kv: -kv[1])[:3])
    g = gg.numpy()
    print(prec, "enc_conv6 masked/free/fp32:", out["masked"]["enc_conv6"], out["free"]["enc_conv6"], e32["enc_conv6"])
