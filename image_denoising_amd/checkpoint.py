"""Checkpoint interop with the reference's `.pth` files.

* `save_checkpoint` writes `net.state_dict()` exactly like `train.py:47-53` (`torch.save` of
  the plain state dict; the reference's file naming `epoch_{name}_{epoch:03d}.pth`), optionally
  with the `module.` key prefix an `nn.DataParallel` run produces (`train.py:324-326`), so the
  reference's evaluation scripts (`evaluation.py:52-53`, strict load) read our weights.
* `load_checkpoint` reads a reference checkpoint with or without that prefix, stripping it the
  way `finetune.py:207-218` does, through `torch.load(weights_only=True)` (no unpickling of code).

The keys and shapes are those of `arch_unet.UNet` (`arch_unet.py:115-192`); our `UNet` keeps
its parameters as views of one flat buffer, so loading is one copy per tensor.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

PREFIX = "module."


def strip_module_prefix(state: dict) -> dict:
    """finetune.py:210-212: drop one leading 'module.' from every key if any key has it"""
    if any(k.startswith(PREFIX) for k in state):
        return OrderedDict((k[len(PREFIX):] if k.startswith(PREFIX) else k, v) for k, v in state.items())
    return state


def read_state_dict(path: str) -> dict:
    state = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(state, dict):
        raise ValueError(f"{path}: expected a state_dict, got {type(state).__name__}")
    return strip_module_prefix(state)


def load_checkpoint(net: torch.nn.Module, path: str, strict: bool = True):
    """load a reference (or our) checkpoint into `net`; returns torch's (missing, unexpected)"""
    return net.load_state_dict(read_state_dict(path), strict=strict)


def checkpoint_name(epoch: int, name: str) -> str:
    """train.py:49 file name"""
    return "epoch_{}_{:03d}.pth".format(name, epoch)


def save_checkpoint(net: torch.nn.Module, path: str, data_parallel: bool = False) -> str:
    """torch.save(net.state_dict()) (train.py:52); data_parallel=True adds the 'module.' prefix
    of a DataParallel-wrapped network.  Tensors are saved on the CPU."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    state = OrderedDict((PREFIX + k if data_parallel else k, v.detach().cpu().clone())
                        for k, v in net.state_dict().items())
    torch.save(state, path)
    return path
