"""Adapter finetune path of finetune.py (reference): a frozen base denoiser + a trainable
OutputAdapter, trained with L1 + lambda_grad * gradient_loss on random patches.

    base_out = base(noisy)           [no grad]   dn_unet_forward        (adapter.py:59-61)
    pred     = adapter(noisy, base_out)          dn_adapter_forward     (adapter.py:22-26)
    loss3, dpred = L1 + lambda*grad-L1           dn_finetune_loss       (finetune.py:153-162, :283-285)
    dA       = adapter backward(dpred)           dn_adapter_backward
    [data parallel: one RCCL all-reduce(sum) of the 449-float gradient]
    Adam(A, dA / world)                          dn_adam_step           (finetune.py:246-249, :288)

No host synchronisation inside the step.  The patch loader (`DenoisePatchDataset`,
finetune.py:100-150) is host code, as in the reference.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import dist as dp
from .adapter import DenoiserWithAdapter
from .arch_unet import UNet
from .checkpoint import strip_module_prefix
from .n2n import _partials_for
from .optim import FlatAdam


def gradient(x: torch.Tensor):
    """finetune.py:153-156 (views only)"""
    dx = x[:, :, :, 1:] - x[:, :, :, :-1]
    dy = x[:, :, 1:, :] - x[:, :, :-1, :]
    return dx, dy


def finetune_loss(pred: torch.Tensor, target: torch.Tensor, lambda_grad: float = 0.1):
    """loss_l1 + lambda_grad * gradient_loss (finetune.py:283-285) and its gradient in one HIP
    pass.  Returns (loss3 = [loss_l1, loss_grad, loss] device tensor, dloss/dpred)."""
    pred, target = pred.contiguous(), target.contiguous()
    if pred.shape != target.shape or pred.dim() != 4:
        raise ValueError("pred and target must share one [N,C,H,W] shape")
    N, C, H, W = pred.shape
    dpred = torch.empty_like(pred)
    loss3 = torch.empty(3, dtype=torch.float32, device=pred.device)
    _lib.call("dn_finetune_loss", _lib.ptr(pred), _lib.ptr(target), N, C, H, W,
              float(lambda_grad), _lib.ptr(dpred), _lib.ptr(loss3),
              _partials_for(pred.device).data_ptr(), _lib.stream_of(pred))
    return loss3, dpred


class _FinetuneLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, lam, which):
        loss3, dpred = finetune_loss(pred, target, lam)
        ctx.save_for_backward(dpred)
        return loss3[which]

    @staticmethod
    def backward(ctx, g):
        (dpred,) = ctx.saved_tensors
        return dpred * g, None, None, None


class FinetuneLoss(nn.Module):
    """l1_criterion(pred, clean) + lambda_grad * gradient_loss(pred, clean) as one module."""

    def __init__(self, lambda_grad: float = 0.1):
        super().__init__()
        self.lambda_grad = lambda_grad

    def forward(self, pred, target):
        return _FinetuneLossFn.apply(pred, target, self.lambda_grad, 2)


class DenoisePatchDataset(torch.utils.data.Dataset):
    """finetune.py:100-150: data_dir/{clean,noise}/* paired by sorted name (first 5 images),
    len = images x patches_per_image, one random ps x ps crop per item (np.random), /255."""

    def __init__(self, data_dir: str, patch_size: int, patches_per_image: int):
        super().__init__()
        self.data_dir = data_dir
        self.clean = sorted(glob.glob(os.path.join(data_dir, "clean", "*")))[:5]
        self.noise = sorted(glob.glob(os.path.join(data_dir, "noise", "*")))[:5]
        assert len(self.clean) == len(self.noise) and len(self.clean) > 0, \
            "clean and noise must have the same number of images and be non-empty."
        self.patch_size = patch_size
        self.patches_per_image = patches_per_image

    def __len__(self) -> int:
        return len(self.clean) * self.patches_per_image

    def _load_pair(self, i: int):
        from PIL import Image
        return (np.array(Image.open(self.clean[i]), dtype=np.float32),
                np.array(Image.open(self.noise[i]), dtype=np.float32))

    @staticmethod
    def _to_tensor(a: np.ndarray) -> torch.Tensor:
        # transforms.ToTensor on a float32 array: HW -> 1HW, HWC -> CHW, no rescaling
        if a.ndim == 2:
            a = a[:, :, None]
        return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))

    def __getitem__(self, index: int):
        clean, noise = self._load_pair(index // self.patches_per_image)
        h, w = clean.shape[:2]
        ps = self.patch_size
        assert h >= ps and w >= ps, f"Image size ({h},{w}) smaller than patch_size {ps}."
        top = np.random.randint(0, h - ps + 1)
        left = np.random.randint(0, w - ps + 1)
        c = clean[top:top + ps, left:left + ps]
        n = noise[top:top + ps, left:left + ps]
        return self._to_tensor(c) / 255.0, self._to_tensor(n) / 255.0


def build_base_model(arch: str, n_channel: int = 1, n_feature: int = 48) -> nn.Module:
    """finetune.py:180-196 (only the UNet base is built on the HIP path)."""
    if arch == "UNet":
        return UNet(in_nc=n_channel, out_nc=n_channel, n_feature=n_feature)
    if arch == "UNetImproved":
        from .improved_unet import ImprovedUNet
        return ImprovedUNet(in_nc=n_channel, out_nc=n_channel, n_feature=n_feature)
    raise ValueError(f"Unknown or unsupported arch: {arch}")


def load_base_weights(model: nn.Module, ckpt_path: str):
    """finetune.py:199-212: strip a DataParallel `module.` prefix, load non-strict."""
    state = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    state = strip_module_prefix(state)
    return model.load_state_dict(state, strict=False)


class FinetuneTrainer:
    """The finetune.py:269-289 step, fused; returns loss3 = [loss_l1, loss_grad, loss]."""

    def __init__(self, model: DenoiserWithAdapter, lr: float = 1e-4, lambda_grad: float = 0.1,
                 distributed: bool | None = None):
        if not isinstance(model, DenoiserWithAdapter):
            raise TypeError("FinetuneTrainer drives a DenoiserWithAdapter")
        self.model = model
        self.lambda_grad = lambda_grad
        self.distributed = dp.require_group(distributed)
        ad = model.adapter
        if self.distributed:  # identical replicas, as nn.DataParallel's per-forward broadcast
            base_flat = getattr(model.base, "flat_params", None)
            if base_flat is not None:  # the frozen base (loaded per rank from one checkpoint)
                dp.broadcast_params(base_flat.data)
            dp.broadcast_params(ad.flat_params)
        self.opt = FlatAdam(ad.flat_params, lr=lr)
        self.grad = torch.zeros_like(ad.flat_params)
        self._bufs = {}

    def _buffers(self, shape, device):
        key = (tuple(shape), device)
        if key not in self._bufs:
            f = dict(dtype=torch.float32, device=device)
            self._bufs = {key: dict(base=torch.empty(shape, **f), pred=torch.empty(shape, **f))}
        return self._bufs[key]

    def _base_forward(self, noisy, out):
        base = self.model.base
        if hasattr(base, "_run_forward"):  # HIP base: workspace reused across steps
            N, _, H, W = noisy.shape
            run = getattr(base, "_run_forward_inference", base._run_forward)  # bf16 if set
            run(noisy, out, base._workspace(N, H, W, with_backward=False))
        else:
            with torch.no_grad():
                out.copy_(base(noisy))

    def train_step(self, clean: torch.Tensor, noisy: torch.Tensor) -> torch.Tensor:
        clean, noisy = clean.contiguous(), noisy.contiguous()
        if clean.shape != noisy.shape:
            raise ValueError("clean and noisy must share one shape")
        ad = self.model.adapter
        b = self._buffers(noisy.shape, noisy.device)
        self._base_forward(noisy, b["base"])
        ad._run_forward(noisy, b["base"], b["pred"])
        loss3, dpred = finetune_loss(b["pred"], clean, self.lambda_grad)
        ad._run_backward(noisy, b["base"], dpred, self.grad)
        scale = dp.allreduce_grads(self.grad) if self.distributed else 1.0
        self.opt.step(self.grad, grad_scale=scale)
        return loss3
