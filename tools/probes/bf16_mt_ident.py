"""Saves the bf16-base UNet forward of a fixed input (8 x 1 x 256^2: every encoder/decoder 3x3 on
the pipelined k_fwd_bf16p) to argv[1]; run under different DN_BF16_MT / DN_BF16_MT3 settings and
compare the files (the wave tile's row count must not change a single bit)."""
import sys

import torch

from image_denoising_amd import UNet

torch.manual_seed(0)
net = UNet(1, 1, 48).to("cuda").set_inference_precision("bf16")
x = torch.rand(8, 1, 256, 256, generator=torch.Generator().manual_seed(2))
with torch.no_grad():
    y = net(x.to("cuda")).cpu()
torch.save(y, sys.argv[1])
if len(sys.argv) > 2:
    y0 = torch.load(sys.argv[2], weights_only=True)
    print("bit-identical:", torch.equal(y, y0), "max diff", float((y - y0).abs().max()))
    sys.exit(0 if torch.equal(y, y0) else 1)
