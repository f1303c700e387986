import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch, numpy as np
from test_gpu_parity import _net, _unit_gain, _rd_set, _pair_mask
DEV = "cuda"
for prec in ("fp32", "fp32_x6"):
    for (C, N, H, W) in ((1, 2, 64, 64), (1, 8, 128, 128)):
        net = _net(C, prec); _unit_gain(net)
        g = torch.Generator().manual_seed(3)
        x = torch.rand(N, C, H, W, generator=g).to(DEV)
        rd = _rd_set("mixed", N * (H // 2) * (W // 2), g).to(DEV)
        ws = net._workspace(N, H, W, with_backward=False, fresh=True)
        full = torch.empty(N, C, H, W, device=DEV); net._run_forward(x, full, ws)
        full2 = torch.empty(N, C, H, W, device=DEV); net._run_forward(x, full2, ws)
        den = torch.full((N, C, H, W), float("nan"), device=DEV); net._run_forward_n2n(x, den, ws, rd)
        sel = torch.from_numpy(_pair_mask(rd.cpu(), N, H, W)).to(DEV).expand(N, C, H, W)
        d = (den[sel] - full[sel]).abs()
        print(prec, (C, N, H, W), "full==full2", torch.equal(full, full2), "max|full|", full.abs().max().item(),
              "den-full max", d.max().item(), "n diff", int((d > 0).sum()), "of", d.numel(),
              "nan in sel", int(torch.isnan(den[sel]).sum()), flush=True)
