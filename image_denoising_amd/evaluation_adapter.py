"""evaluation_adapter.py on the HIP path: inference of a DenoiserWithAdapter checkpoint
(frozen base + OutputAdapter, adapter.py:29-67) over <data_dir>/noise/*, saving
<name>_denoised.png and, when <data_dir>/clean/ exists, printing each image's PSNR
(evaluation_adapter.py:63-166).

    python -m image_denoising_amd.evaluation_adapter --data_dir D --ckpt X.pth [--arch UNet]

The base runs on the HIP executors (UNet or ImprovedUNet), the adapter on dn_adapter_forward;
quantisation (clip(x*255 + 0.5) -> uint8) and PSNR on device (dn_quantize_u8, dn_psnr_u8).
"""
from __future__ import annotations

import argparse
import glob
import os

import numpy as np
import torch

from . import _lib
from .evaluation import _device, psnr_device


def parse_args(argv=None):
    """evaluation_adapter.py:17-43 (parse_known_args: unknown options are ignored there too)"""
    ap = argparse.ArgumentParser()
    ap.add_argument("--data_dir", type=str, required=True)
    ap.add_argument("--ckpt", type=str, required=True)
    ap.add_argument("--arch", type=str, default="UNetImproved", choices=["UNet", "RESNET", "UNetImproved"])
    ap.add_argument("--save_dir", type=str, default="./results_infer_adapter")
    ap.add_argument("--gpu_devices", default="0", type=str)
    ap.add_argument("--parallel", action="store_true")  # one GPU per process here: ignored
    ap.add_argument("--n_feature", type=int, default=48)
    ap.add_argument("--n_channel", type=int, default=1)
    ap.add_argument("--adapter_hidden", type=int, default=16)
    args, _ = ap.parse_known_args(argv)
    return args


def build_model(arch: str, n_channel: int, n_feature: int, hidden: int):
    """evaluation_adapter.py:46-55 + :114-121 (RESNET is out of scope on this path)"""
    from .adapter import DenoiserWithAdapter
    from .finetune import build_base_model

    if arch == "RESNET":
        raise SystemExit("RESNET is out of scope on this path (DESIGN.md §9)")
    base = build_base_model(arch, n_channel, n_feature)
    return DenoiserWithAdapter(base, in_channels=n_channel, hidden_channels=hidden,
                               freeze_base=True, use_no_grad_for_base=True)


def load_adapter_weights(model, ckpt_path: str):
    """evaluation_adapter.py:58-68: strip a DataParallel 'module.' prefix, load non-strict"""
    from .checkpoint import read_state_dict

    missing, unexpected = model.load_state_dict(read_state_dict(ckpt_path), strict=False)
    if missing:
        print(f"[Warning] Missing keys when loading adapter model: {missing}")
    if unexpected:
        print(f"[Warning] Unexpected keys when loading adapter model: {unexpected}")
    print(f"Loaded adapter+base weights from {ckpt_path}")


@torch.no_grad()
def denoise(model, noisy_u8: np.ndarray):
    """evaluation_adapter.py:133-145: [H,W(,C)] uint8 -> pred255 uint8 on device [C,H,W]"""
    dev = _device()
    x8 = torch.from_numpy(np.ascontiguousarray(noisy_u8)).to(dev)
    x8 = x8.unsqueeze(0) if x8.dim() == 2 else x8.permute(2, 0, 1).contiguous()
    C, H, W = x8.shape
    x = torch.empty((1, C, H, W), dtype=torch.float32, device=dev)
    _lib.call("dn_u8_to_unit", _lib.ptr(x8), x8.numel(), _lib.ptr(x), _lib.stream_of(x))
    pred = model(x).contiguous()
    p8 = torch.empty((C, H, W), dtype=torch.uint8, device=dev)
    _lib.call("dn_quantize_u8", _lib.ptr(pred), pred.numel(), 1, _lib.ptr(p8), _lib.stream_of(pred))
    return p8


def main(argv=None):
    from PIL import Image

    opt = parse_args(argv)
    noise_paths = sorted(glob.glob(os.path.join(opt.data_dir, "noise", "*")))
    if not noise_paths:
        raise RuntimeError(f"No files found in {os.path.join(opt.data_dir, 'noise')}")
    clean_dir = os.path.join(opt.data_dir, "clean")
    clean_paths = sorted(glob.glob(os.path.join(clean_dir, "*"))) if os.path.isdir(clean_dir) else []
    has_clean = len(clean_paths) > 0
    if has_clean and len(clean_paths) != len(noise_paths):
        print("[Warning] clean/ and noise/ have different counts; PSNR may be misaligned.")
    os.makedirs(opt.save_dir, exist_ok=True)
    print(f"Found {len(noise_paths)} noisy images for inference.")
    model = build_model(opt.arch, opt.n_channel, opt.n_feature, opt.adapter_hidden).to(_device())
    model.eval()
    load_adapter_weights(model, opt.ckpt)
    psnrs = []
    for idx, n_path in enumerate(noise_paths):
        name = os.path.basename(n_path)
        base_name = os.path.splitext(name)[0]
        noisy = np.array(Image.open(n_path), dtype=np.float32).astype(np.uint8)
        p8 = denoise(model, noisy)
        out = p8.cpu().numpy()
        img = Image.fromarray(out[0]).convert("L") if out.shape[0] == 1 else \
            Image.fromarray(np.transpose(out, (1, 2, 0))).convert("RGB")
        save_path = os.path.join(opt.save_dir, f"{base_name}_denoised.png")
        img.save(save_path)
        if has_clean and idx < len(clean_paths):
            clean = np.array(Image.open(clean_paths[idx]), dtype=np.float32).astype(np.uint8)
            c8 = torch.from_numpy(clean).to(p8.device)
            c8 = c8.unsqueeze(0) if c8.dim() == 2 else c8.permute(2, 0, 1).contiguous()
            # evaluation_adapter.py:75-83: mse == 0 -> 99.0
            ps = 99.0 if torch.equal(p8, c8) else float(psnr_device(p8, c8).cpu())
            psnrs.append(ps)
            print(f"[{idx + 1:03d}/{len(noise_paths):03d}] {name} → PSNR={ps:.2f} dB, saved to {save_path}")
        else:
            print(f"[{idx + 1:03d}/{len(noise_paths):03d}] {name} → saved to {save_path}")
    print("Inference with adapter model finished.")
    return dict(psnr=psnrs)


if __name__ == "__main__":
    main()
