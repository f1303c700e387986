"""U-Net (fp32_x6) output determinism on the fixture input: no-grad pass repeated, grad pass,
max |diff| and the number of differing elements (DN_X6_DECONV=0 / DN_X6_HEAD=0 isolate a kernel)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_denoising_amd.arch_unet import UNet  # noqa: E402

g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "unet_c1.npz"))
torch.manual_seed(0)
net = UNet(in_nc=1, out_nc=1, n_feature=48).to("cuda").set_precision("fp32_x6")
x = torch.from_numpy(g["x"]).cuda()
with torch.no_grad():
    ys = [net(x) for _ in range(4)]
y = net(x).detach()


def rep(name, a, b):
    d = (a - b).abs()
    print(os.environ.get("TAG", ""), name, "max", float(d.max()), "ndiff", int((d > 0).sum()), "of",
          d.numel(), "rel_to_ref", float((a.cpu() - torch.from_numpy(g["y"])).abs().max()))


for i in range(1, 4):
    rep(f"nograd{i}", ys[i], ys[0])
rep("grad", y, ys[0])
