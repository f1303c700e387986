"""ImprovedUNet backward diagnostic: device gradient buffers of each down level's ResBlock
(dr, dz2, dg1, dz1) and the up-block concat gradients vs torch autograd on the fp64 oracle."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from image_denoising_amd import _lib  # noqa: E402
from image_denoising_amd.improved_unet import ImprovedUNet  # noqa: E402
from oracle import iunet_ref  # noqa: E402

N, C, H, W = [int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (2, 1, 64, 96))]
torch.manual_seed(0)
net = ImprovedUNet(C, C, 48).cuda()
gen = torch.Generator().manual_seed(9)
x = torch.rand(N, C, H, W, generator=gen)
dy = torch.randn(N, C, H, W, generator=gen)
tr = iunet_ref.new_trace()
p = net.flat_params.cpu().double().requires_grad_(True)
for t in []:
    pass
y = iunet_ref.forward(p, x.double(), C, C, trace=tr)
keep = []
for k, d in tr.res.items():
    for v in d.values():
        v.retain_grad()
for name, t in tr:
    if name.endswith(":cc"):
        t.retain_grad()
y.backward(dy.double())
ws = net._workspace(N, H, W, True, fresh=True)
yd = torch.empty(N, C, H, W, device="cuda")
net._run_forward(x.cuda(), yd, ws)
g = torch.empty_like(net.flat_params)
net._run_backward(dy.cuda(), g, ws, N, H, W)
torch.cuda.synchronize()
desc = (ctypes.c_int64 * (3 * 128))()
n = ctypes.c_int()
_lib.call("dn_iunet_debug_buffers", ctypes.byref(net._cfg), N, H, W, 1, desc, 128, ctypes.byref(n))
fws = ws.view(torch.float32).cpu()


def buf(i, ch):
    off, stride, lvl = desc[3 * i], desc[3 * i + 1], desc[3 * i + 2]
    h, w = H >> lvl, W >> lvl
    return fws[off:off + N * h * w * stride].view(N, h, w, stride)[..., :ch].permute(0, 3, 1, 2).double()


def rel(a, b):
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


base = 2 + 5 * 4 + 5 + 6 * 4 + 2  # forward entries
for i in range(4):
    d = tr.res[f"downs.{i}.3"]
    ch = 48 << i
    a1 = d["a1"].detach()
    dg1_ref = d["a1"].grad * torch.where(a1 > 0, 1.0, 0.2)
    pairs = [("dr", d["r"].grad), ("dz2", d["z2"].grad), ("dg1", dg1_ref), ("dz1", d["z1"].grad)]
    for j, (nm, ref) in enumerate(pairs):
        got = buf(base + 4 * i + j, ch)
        print(f"level {i} {nm:4s} rel err {rel(got, ref):.2e}")
    print(f"level {i} dout(total d s_i) ref-norm {float(d['out'].grad.norm()):.3e}")
for k in range(4):
    cc = [t for nm, t in tr if nm == f"ups.{k}:cc"][0]
    got = buf(base + 16 + k, cc.shape[1])
    out = cc.shape[1] // 3
    print(f"up {k} dcc u-part rel {rel(got[:, :out], cc.grad[:, :out]):.2e}")
    # skip part on the device also holds the pool-backward contribution (= d s_i total)
    lvl = 3 - k
    s_tot = tr.res[f"downs.{lvl}.3"]["out"].grad
    print(f"up {k} dcc skip (after pool bwd) vs d s_{lvl} rel {rel(got[:, out:], s_tot):.2e}; "
          f"vs skip-only {rel(got[:, out:], cc.grad[:, out:]):.2e}")
print("--- decomposition of the level skip gradients (device total - oracle skip-only part)")
for k in range(4):
    cc = [t for nm, t in tr if nm == f"ups.{k}:cc"][0]
    out = cc.shape[1] // 3
    got = buf(base + 16 + k, cc.shape[1])[:, out:]
    s_tot = tr.res[f"downs.{3 - k}.3"]["out"].grad
    pool_part_ref = s_tot - cc.grad[:, out:]
    print(f"up {k}: pool-bwd part rel {rel(got - cc.grad[:, out:], pool_part_ref):.2e}")
    # where are the errors? per 2x2 window position / per channel block
    e = (got - s_tot).abs()
    print("   err by (y%2,x%2):", [float(e[:, :, a::2, b::2].max()) for a in (0, 1) for b in (0, 1)],
          " by 48-ch block:", [float(e[:, j:j + 48].max()) for j in range(0, e.shape[1], 48)])
