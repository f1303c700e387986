"""Structure_loss (util.py:41-70 of the reference), computed by one HIP reduction kernel.

L = alpha*L1(pred, target) + beta*(L1(pred2[:,:,1:],pred2[:,:,:-1]) + L1(pred2[...,1:],pred2[...,:-1]))/2
    + gamma*L1(pred2, target)      with pred = net(noisy), pred2 = net(clean) (train.py:361-363)
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .n2n import _partials_for


def structure_loss_into(pred, pred2, target, alpha, beta, gamma, dpred, dpred2, loss5):
    """dn_structure_loss into given contiguous buffers: loss5 = [pixel, tv1, tv2, cst, total],
    dpred = dL/dpred, dpred2 = dL/dpred2 (all on pred's device and stream)"""
    for t in (pred, pred2, target, dpred, dpred2, loss5):
        if not t.is_contiguous():
            raise ValueError("structure_loss_into needs contiguous tensors")
    if (pred.shape != pred2.shape or pred.shape != target.shape or pred.dim() != 4
            or dpred.shape != pred.shape or dpred2.shape != pred.shape or loss5.numel() != 5):
        raise ValueError("pred, pred2, target, dpred and dpred2 must share one [N,C,H,W] shape")
    N, C, H, W = pred.shape
    _lib.call("dn_structure_loss", _lib.ptr(pred), _lib.ptr(pred2), _lib.ptr(target), N, C, H, W,
              float(alpha), float(beta), float(gamma), _lib.ptr(dpred), _lib.ptr(dpred2),
              _lib.ptr(loss5), _partials_for(pred.device).data_ptr(), _lib.stream_of(pred))


def structure_loss(pred, pred2, target, alpha=1.0, beta=0.5, gamma=0.5):
    """returns (loss5 = [pixel, tv1, tv2, cst, total] device tensor, dpred, dpred2)"""
    pred, pred2, target = pred.contiguous(), pred2.contiguous(), target.contiguous()
    if pred.shape != pred2.shape or pred.shape != target.shape or pred.dim() != 4:
        raise ValueError("pred, pred2 and target must share one [N,C,H,W] shape")
    dpred = torch.empty_like(pred)
    dpred2 = torch.empty_like(pred2)
    loss5 = torch.empty(5, dtype=torch.float32, device=pred.device)
    structure_loss_into(pred, pred2, target, alpha, beta, gamma, dpred, dpred2, loss5)
    return loss5, dpred, dpred2


class _StructureFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, pred2, target, alpha, beta, gamma):
        loss5, dp, dp2 = structure_loss(pred, pred2, target, alpha, beta, gamma)
        ctx.save_for_backward(dp, dp2)
        return loss5[4]

    @staticmethod
    def backward(ctx, g):
        dp, dp2 = ctx.saved_tensors
        return dp * g, dp2 * g, None, None, None, None


class Structure_loss(nn.Module):  # noqa: N801  (reference name, util.py:41)
    def __init__(self, alpha: float = 1.0, beta: float = .5, gamma: float = .5,
                 reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("only reduction='mean' (the reference default) is supported")
        self.alpha, self.beta, self.gamma, self.reduction = alpha, beta, gamma, reduction

    def forward(self, pred, pred2, target):
        return _StructureFn.apply(pred, pred2, target, self.alpha, self.beta, self.gamma)
