"""ORACLE (test infrastructure only) — adapter finetune path of the reference as torch-CPU ops:
adapter.py:5-26 OutputAdapter, finetune.py:153-162 gradient / gradient_loss, and the
finetune.py:269-289 step (frozen base under no_grad, L1 + lambda_grad*gradient_loss, Adam).
Flat adapter parameters in state_dict order: net.0.weight, net.0.bias, net.2.weight, net.2.bias.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import unet_ref


def unflatten(flat: torch.Tensor, C: int, hidden: int = 16):
    shapes = [(hidden, 2 * C, 3, 3), (hidden,), (C, hidden, 3, 3), (C,)]
    out, off = [], 0
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        out.append(flat[off:off + n].view(s))
        off += n
    assert off == flat.numel(), (off, flat.numel())
    return out


def adapter_forward(flat: torch.Tensor, noisy: torch.Tensor, base_out: torch.Tensor,
                    hidden: int = 16) -> torch.Tensor:
    """adapter.py:22-26"""
    w1, b1, w2, b2 = unflatten(flat, noisy.shape[1], hidden)
    x = torch.cat([noisy, base_out], dim=1)
    delta = F.conv2d(F.relu(F.conv2d(x, w1, b1, padding=1)), w2, b2, padding=1)
    return base_out + delta


def gradient(x):
    """finetune.py:153-156"""
    return x[:, :, :, 1:] - x[:, :, :, :-1], x[:, :, 1:, :] - x[:, :, :-1, :]


def gradient_loss(pred, target):
    """finetune.py:159-162"""
    pdx, pdy = gradient(pred)
    tdx, tdy = gradient(target)
    return F.l1_loss(pdx, tdx) + F.l1_loss(pdy, tdy)


def finetune_loss(pred, target, lambda_grad: float = 0.1):
    """finetune.py:283-285 -> (loss_l1, loss_grad, loss)"""
    l1 = F.l1_loss(pred, target)
    lg = gradient_loss(pred, target)
    return l1, lg, l1 + lambda_grad * lg


def finetune_step(base_flat, adapter_flat, clean, noisy, C: int, lr: float = 1e-4,
                  lambda_grad: float = 0.1, nf: int = 48):
    """One finetune.py:269-289 step with a UNet base (arch='UNet').  Returns the loss terms, the
    adapter gradient and the adapter parameters after torch.optim.Adam (finetune.py:246-249)."""
    with torch.no_grad():
        base_out = unet_ref.forward(base_flat, noisy, C, C, nf)
    p = adapter_flat.clone().requires_grad_(True)
    opt = torch.optim.Adam([p], lr=lr)
    pred = adapter_forward(p, noisy, base_out)
    l1, lg, loss = finetune_loss(pred, clean, lambda_grad)
    opt.zero_grad()
    loss.backward()
    g = p.grad.detach().clone()
    opt.step()
    return dict(loss_l1=float(l1.detach()), loss_grad=float(lg.detach()), loss=float(loss.detach()),
                grad=g, params=p.detach().clone(), pred=pred.detach(), base_out=base_out)
