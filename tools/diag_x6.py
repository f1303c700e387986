"""bf16x6 vs fp32 kernel error statistics against fp64 (op level and whole-network gradients)."""
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_parity as tp  # noqa: E402
import test_gpu_x6 as tx  # noqa: E402

for cin, cout, N, H in [(96, 96, 2, 64), (144, 96, 2, 64), (48, 48, 4, 64), (96, 96, 8, 128)]:
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, cin, H, H, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * 0.1
    b = torch.zeros(cout)
    ref = F.conv2d(x.double(), w.double(), None, padding=1).numpy()
    for x6 in (False, True):
        y = tx._forward(x, w, b, 0, x6).numpy().astype(np.float64)
        d = y - ref
        sc = np.abs(ref).max()
        print(f"fwd {cin}->{cout} H{H} {'x6 ' if x6 else 'f32'} max {np.abs(d).max()/sc:.3e} "
              f"rms {np.sqrt((d**2).mean())/sc:.3e} mean {d.mean()/sc:+.3e} "
              f"corr(d,ref) {np.corrcoef(d.ravel(), ref.ravel())[0,1]:+.3f}", flush=True)

from oracle.unet_ref import forward, layer_table  # noqa: E402

C, N, H, W = 1, 2, 128, 128
x = torch.rand(N, C, H, W, generator=torch.Generator().manual_seed(1))
r = torch.randn(N, C, H, W, generator=torch.Generator().manual_seed(2))
res = {}
for prec in ("fp32", "fp32_x6"):
    net = tp._net(C, prec)
    tp._unit_gain(net)
    y, gg, acts = tp._device_activations(net, x, r)
    p64 = net.flat_params.detach().cpu().double().requires_grad_(True)
    y64 = forward(p64, x.double(), C, C, masks=acts)
    (y64 * r.double()).sum().backward()
    g64 = p64.grad.numpy()
    gg = gg.numpy()
    off = 0
    errs = []
    for name_, ws, bl, _ in layer_table(C, C):
        n = int(np.prod(ws)) + bl
        errs.append((name_, tp.rel_err(gg[off:off + n], g64[off:off + n])))
        off += n
    res[prec] = errs
    print(prec, "y err", tp.rel_err(y.numpy(), y64.detach().numpy()), flush=True)
for (n, a), (_, b) in zip(res["fp32"], res["fp32_x6"]):
    print(f"{n:12s} fp32 {a:.2e}  x6 {b:.2e}")
