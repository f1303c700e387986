"""per-op timing of one ImprovedUNet forward(256) + forward/backward(128) at bs 64 (DN_PROFILE_OPS)"""
import os
import sys

os.environ["DN_PROFILE_OPS"] = "1"
import torch  # noqa: E402

sys.path.insert(0, ".")
from image_denoising_amd.improved_unet import ImprovedUNet  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
net = ImprovedUNet(1, 1, 48).cuda()
x = torch.rand(bs, 1, 128, 128, device="cuda")
ws = net._workspace(bs, 128, 128, True, fresh=True)
y = torch.empty_like(x)
g = torch.empty_like(net.flat_params)
for _ in range(2):
    net._run_forward(x, y, ws)
    net._run_backward(y.clone(), g, ws, bs, 128, 128)
torch.cuda.synchronize()
