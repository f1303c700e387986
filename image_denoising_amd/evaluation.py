"""Evaluation path on the HIP library.

Mirrors, with the same names and meanings:
  * `calculate_psnr(target, ref)`, `calculate_ssim(target, ref)`   utils_eval.py:19-53
  * `denoise_full`   = the per-image body of evaluation.py:58-93: x = noisy/255, one forward,
    L1(prediction, x), pred255 = uint8(clip(clamp(pred, 0, 1)*255 + 0.5, 0, 255)).
  * `denoise_tiled`  = evaluation_704.py:57-115: 352x352 tiles, 64 overlap (stride 288),
    numpy 'reflect' padding of edge tiles, tent weight mask, weighted blend, / contribution,
    pred255 = uint8(clip(blend*255, 0, 255)), L1 = mean over tiles of each tile's L1.
  * `evaluate` / `main` = evaluate() of evaluation.py / evaluation_704.py (same CLI flags,
    metrics.txt in the same format; images saved only with --save_images).

MI355X-first: all tiles of an image go through ONE batched dn_unet_forward; extraction, blend,
quantisation, PSNR (exact integer sum of squared errors), SSIM (fp64 window statistics) and L1
run as HIP kernels (csrc/eval.hip) with fixed-order reductions; the host reads back three
doubles per image.  Images are uint8 arrays/tensors [H,W] (grayscale, as the reference's
`validation_denoise` yields for single-channel data) or [C,H,W].
"""
from __future__ import annotations

import argparse
import glob
import os

import numpy as np
import torch

from . import _lib

PATCH, OVERLAP = 352, 64  # evaluation_704.py:57-59


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("the evaluation path runs on the GPU (HIP); no device visible")
    return torch.device("cuda", torch.cuda.current_device())


def _u8(img, device) -> torch.Tensor:
    if isinstance(img, torch.Tensor):
        t = img
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(img)))
    if t.dtype != torch.uint8:
        raise ValueError(f"expected uint8 image, got {t.dtype}")
    return t.to(device).contiguous()


def _parts(device) -> torch.Tensor:
    return _lib.scratch(_lib.lib().dn_eval_partials_size(), device)


def _chw(t: torch.Tensor) -> torch.Tensor:
    return t.unsqueeze(0) if t.dim() == 2 else t


def psnr_device(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """device double scalar; a, b uint8 tensors of equal shape"""
    if a.shape != b.shape:
        raise ValueError("Input images must have the same dimensions.")
    out = torch.empty(1, dtype=torch.float64, device=a.device)
    _lib.call("dn_psnr_u8", _lib.ptr(a), _lib.ptr(b), a.numel(), _lib.ptr(_parts(a.device)),
              _lib.ptr(out), _lib.stream_of(a))
    return out


def ssim_device(a: torch.Tensor, b: torch.Tensor, hwc: bool = False) -> torch.Tensor:
    if a.shape != b.shape:
        raise ValueError("Input images must have the same dimensions.")
    if a.dim() == 2:
        C, H, W = 1, a.shape[0], a.shape[1]
    elif a.dim() == 3 and hwc:
        H, W, C = a.shape
    elif a.dim() == 3:
        C, H, W = a.shape
    else:
        raise ValueError("Wrong input image dimensions.")
    out = torch.empty(1, dtype=torch.float64, device=a.device)
    _lib.call("dn_ssim_u8", _lib.ptr(a), _lib.ptr(b), C, H, W, int(hwc), _lib.ptr(_parts(a.device)),
              _lib.ptr(out), _lib.stream_of(a))
    return out


def calculate_psnr(target, ref) -> float:
    """utils_eval.py:49-53 (uint8 inputs; the sum of squared errors is exact)"""
    dev = _device()
    return float(psnr_device(_u8(target, dev), _u8(ref, dev)).item())


def calculate_ssim(target, ref) -> float:
    """utils_eval.py:36-46: 2-D image, or [H,W,3] / [H,W,1] (channel-last, as cv2/PIL)."""
    dev = _device()
    a, b = _u8(target, dev), _u8(ref, dev)
    if a.dim() == 3 and a.shape[2] not in (1, 3):
        raise ValueError("Wrong input image dimensions.")
    return float(ssim_device(a, b, hwc=a.dim() == 3).item())


def weight_mask(patch: int = PATCH) -> np.ndarray:
    """evaluation_704.py:62-68 (computed in float64, stored as float32)"""
    yy, xx = np.meshgrid(np.linspace(0, 1, patch), np.linspace(0, 1, patch), indexing="ij")
    return ((1 - np.abs(yy - 0.5) * 2) * (1 - np.abs(xx - 0.5) * 2)).astype(np.float32)


def _l1(a: torch.Tensor, b: torch.Tensor, parts: torch.Tensor, out: torch.Tensor) -> None:
    _lib.call("dn_l1_mean", _lib.ptr(a), _lib.ptr(b), a.numel(), _lib.ptr(parts), _lib.ptr(out),
              _lib.stream_of(a))


@torch.no_grad()
def denoise_full(net, noisy):
    """evaluation.py:66-82 -> (prediction [1,C,H,W] fp32 device, pred255 uint8 [C,H,W] device,
    l1 device double)"""
    dev = _device()
    x8 = _chw(_u8(noisy, dev))
    C, H, W = x8.shape
    x = torch.empty((1, C, H, W), dtype=torch.float32, device=dev)
    _lib.call("dn_u8_to_unit", _lib.ptr(x8), x8.numel(), _lib.ptr(x), _lib.stream_of(x))
    pred = net(x)
    l1 = torch.empty(1, dtype=torch.float64, device=dev)
    _l1(pred, x, _parts(dev), l1)
    p8 = torch.empty((C, H, W), dtype=torch.uint8, device=dev)
    _lib.call("dn_quantize_u8", _lib.ptr(pred), pred.numel(), 1, _lib.ptr(p8), _lib.stream_of(pred))
    return pred, p8, l1


@torch.no_grad()
def denoise_tiled(net, noisy, patch: int = PATCH, overlap: int = OVERLAP, max_batch: int = 64):
    """evaluation_704.py:70-115 -> (blended [C,H,W] fp32 device, pred255 uint8 [C,H,W] device,
    mean tile L1 as a device double).  All tiles go through the network in batches of up to
    max_batch (one dn_unet_forward per batch)."""
    dev = _device()
    x8 = _chw(_u8(noisy, dev))
    C, H, W = x8.shape
    stride = patch - overlap
    L = _lib.lib()
    nti, ntj = L.dn_tile_count(H, patch, stride), L.dn_tile_count(W, patch, stride)
    P = nti * ntj
    tiles = torch.empty((P, C, patch, patch), dtype=torch.float32, device=dev)
    st = _lib.stream_of(tiles)
    _lib.call("dn_tile_extract", _lib.ptr(x8), C, H, W, patch, stride, _lib.ptr(tiles), st)
    pred = torch.empty((P, net.out_nc, patch, patch), dtype=torch.float32, device=dev)
    for b0 in range(0, P, max_batch):
        pred[b0:b0 + max_batch] = net(tiles[b0:b0 + max_batch])
    # criterion(prediction_patch, noisy_input) of every tile (evaluation_704.py:98), one launch
    if net.out_nc != C:
        raise ValueError("tiled evaluation compares the prediction with its input: out_nc == C")
    l1s = torch.empty(P, dtype=torch.float64, device=dev)
    _lib.call("dn_l1_mean_batched", _lib.ptr(pred), _lib.ptr(tiles), P, C * patch * patch,
              _lib.ptr(l1s), st)
    wm = torch.from_numpy(weight_mask(patch)).to(dev)
    out = torch.empty((net.out_nc, H, W), dtype=torch.float32, device=dev)
    p8 = torch.empty((net.out_nc, H, W), dtype=torch.uint8, device=dev)
    _lib.call("dn_tile_blend", _lib.ptr(pred), net.out_nc, H, W, patch, stride, _lib.ptr(wm),
              _lib.ptr(out), _lib.ptr(p8), st)
    return out, p8, l1s.mean()


def evaluate(net, clean_imgs, noisy_imgs, tiled: bool = False, patch: int = PATCH,
             overlap: int = OVERLAP):
    """metrics of evaluation.py:95-108 (tiled=False) / evaluation_704.py:117-135 (tiled=True)
    for lists of uint8 images; returns dict(psnr=[..], ssim=[..], l1=[..], avg_*), plus the
    denoised uint8 images (host)."""
    dev = _device()
    psnr, ssim, l1, outs = [], [], [], []
    for clean, noisy in zip(clean_imgs, noisy_imgs):
        if tiled:
            _, p8, l1v = denoise_tiled(net, noisy, patch, overlap)
        else:
            _, p8, l1v = denoise_full(net, noisy)
        c8 = _chw(_u8(clean, dev))
        ps = psnr_device(p8, c8)
        ss = ssim_device(p8, c8)
        vals = torch.cat([ps, ss, l1v.reshape(1)]).cpu().numpy()  # one host sync per image
        psnr.append(float(vals[0]))
        ssim.append(float(vals[1]))
        l1.append(float(vals[2]))
        outs.append(p8.cpu().numpy().squeeze())
    return dict(psnr=psnr, ssim=ssim, l1=l1, avg_psnr=float(np.mean(psnr)),
                avg_ssim=float(np.mean(ssim)), avg_l1=float(np.mean(l1)), denoised=outs)


def validation_denoise(dataset_dir):
    """utils_eval.py:6-17 (PIL, sorted clean/* and noise/*), images as uint8"""
    from PIL import Image

    clean = sorted(glob.glob(os.path.join(dataset_dir, "clean", "*")))
    noise = sorted(glob.glob(os.path.join(dataset_dir, "noise", "*")))
    im1 = [np.array(Image.open(f), dtype=np.float32).astype(np.uint8) for f in clean]
    im2 = [np.array(Image.open(f), dtype=np.float32).astype(np.uint8) for f in noise]
    return im1, im2, clean, noise


def build_network(log_name: str, n_channel: int, n_feature: int):
    """evaluation.py:32-50's choice of network by --log_name, in the reference's branch order
    ('UNET' is matched case-sensitively, so 'UNetImproved' reaches the ImprovedUNet branch)"""
    from .arch_unet import UNet
    from .improved_unet import ImprovedUNet

    if "UNET" in log_name and "blindspot" in log_name:
        raise SystemExit("the blind-spot UNet is out of scope on this path (DESIGN.md §9)")
    if "UNET" in log_name:
        return UNet(in_nc=n_channel, out_nc=n_channel, n_feature=n_feature)
    if "RESNET" in log_name:
        raise SystemExit("RESNET is out of scope on this path (DESIGN.md §9)")
    if "UNetImproved" in log_name:
        return ImprovedUNet(in_nc=n_channel, out_nc=n_channel, n_feature=n_feature)
    raise SystemExit(f"--log_name {log_name!r} names no network (evaluation.py:32-50)")


def main(argv=None):
    from .checkpoint import load_checkpoint

    ap = argparse.ArgumentParser(description="evaluation.py / evaluation_704.py on the HIP path")
    ap.add_argument("--data_dir", type=str, default="./dataset/m1")
    ap.add_argument("--checkpoint", type=str, required=True)
    ap.add_argument("--save_dir", type=str, default="./eval_results")
    ap.add_argument("--n_feature", type=int, default=48)
    ap.add_argument("--n_channel", type=int, default=1)
    ap.add_argument("--log_name", type=str, default="UNetImproved")  # evaluation.py:19
    ap.add_argument("--gpu_devices", default="0", type=str)
    ap.add_argument("--tiled", action="store_true", help="evaluation_704.py tiling")
    ap.add_argument("--patch", type=int, default=PATCH)
    ap.add_argument("--overlap", type=int, default=OVERLAP)
    ap.add_argument("--save_images", action="store_true")
    opt = ap.parse_args(argv)
    net = build_network(opt.log_name, opt.n_channel, opt.n_feature)
    os.makedirs(opt.save_dir, exist_ok=True)
    clean, noisy, clean_paths, noisy_paths = validation_denoise(opt.data_dir)
    net = net.to(_device())
    load_checkpoint(net, opt.checkpoint)
    net.eval()
    print(f"Loaded checkpoint from {opt.checkpoint}")
    res = evaluate(net, clean, noisy, tiled=opt.tiled, patch=opt.patch, overlap=opt.overlap)
    for i, (p, s, l) in enumerate(zip(res["psnr"], res["ssim"], res["l1"])):
        name = os.path.basename(noisy_paths[i]).split(".")[0]
        print(f"[{i + 1}/{len(clean)}] {name} -> PSNR: {p:.2f}, SSIM: {s:.4f}, L1: {l:.6f}")
        if opt.save_images:
            from PIL import Image

            Image.fromarray(res["denoised"][i]).save(
                os.path.join(opt.save_dir, f"{name}_{i:03d}_denoised.png"))
    with open(os.path.join(opt.save_dir, "metrics.txt"), "w") as f:
        f.write(f"Average PSNR: {res['avg_psnr']:.2f}\n")
        f.write(f"Average SSIM: {res['avg_ssim']:.4f}\n")
        f.write(f"Average L1 Loss: {res['avg_l1']:.6f}\n")
    print(f"Average PSNR: {res['avg_psnr']:.2f}, Average SSIM: {res['avg_ssim']:.4f}, "
          f"Average L1 Loss: {res['avg_l1']:.6f}")
    return res


if __name__ == "__main__":
    main()
