"""Adam over the flat parameter buffer + the reference's MultiStepLR schedule.

train.py:332-340: optim.Adam(network.parameters(), lr=opt.lr) and
MultiStepLR(milestones=[int(20r)-1, int(40r)-1, int(60r)-1, int(80r)-1], gamma=opt.gamma),
r = n_epoch/100, stepped once per epoch (train.py:375).
"""
from __future__ import annotations

import torch

from . import _lib


class FlatAdam:
    """torch.optim.Adam (amsgrad=False, weight_decay=0) as ONE fused HIP kernel over a flat
    fp32 buffer; state tensors are flat too.  `grad_scale` folds the 1/world_size of a
    data-parallel all-reduce(sum) into the same pass."""

    def __init__(self, params: torch.Tensor, lr: float = 3e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8):
        if params.dtype != torch.float32 or not params.is_contiguous():
            raise ValueError("FlatAdam needs a contiguous fp32 buffer")
        self.params = params
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.exp_avg = torch.zeros_like(params)
        self.exp_avg_sq = torch.zeros_like(params)
        self.step_count = 0

    def step(self, grad: torch.Tensor, grad_scale: float = 1.0) -> None:
        if grad.shape != self.params.shape:
            raise ValueError("grad and params differ in shape")
        self.step_count += 1
        adam_launch(self, grad.contiguous(), float(grad_scale))

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "lr": self.lr, "betas": self.betas, "eps": self.eps}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.lr, self.betas, self.eps = sd["lr"], tuple(sd["betas"]), sd["eps"]


def adam_launch(opt: FlatAdam, grad: torch.Tensor, grad_scale: float) -> None:
    """one dn_adam_step over the flat buffers (step count already incremented)"""
    b1, b2 = opt.betas
    _lib.call("dn_adam_step", _lib.ptr(opt.params), _lib.ptr(grad), _lib.ptr(opt.exp_avg),
              _lib.ptr(opt.exp_avg_sq), opt.params.numel(), float(opt.lr), float(b1), float(b2),
              float(opt.eps), opt.step_count, float(grad_scale), _lib.stream_of(opt.params))


def reference_milestones(n_epoch: int):
    ratio = n_epoch / 100
    return [int(20 * ratio) - 1, int(40 * ratio) - 1, int(60 * ratio) - 1, int(80 * ratio) - 1]


def lr_at_epoch(epoch: int, base_lr: float, n_epoch: int, gamma: float = 0.5) -> float:
    """lr in effect during 1-based `epoch` (MultiStepLR.last_epoch == epoch-1).

    MultiStepLR multiplies by gamma**count(m) when last_epoch reaches milestone m (the
    construction step sets last_epoch = 0, so a milestone 0 fires at once; repeated milestones
    count with multiplicity).  last_epoch never equals a negative milestone, which
    reference_milestones() yields for n_epoch < 5 (int(20r) = 0): those never fire."""
    last = epoch - 1
    k = sum(1 for m in reference_milestones(n_epoch) if 0 <= m <= last)
    return base_lr * gamma ** k
