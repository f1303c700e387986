"""Drop-in `OutputAdapter` / `DenoiserWithAdapter` (adapter.py:5-67 of the reference),
computed by libdenoise_hip.so on gfx950.

Same constructors, same `state_dict` keys (`adapter.net.0.weight`, ..., `base.*`), same
forward.  The adapter's four tensors are views into ONE flat fp32 buffer (the layout
dn_adapter_forward / dn_adapter_backward consume); the frozen base runs its own HIP forward
under no_grad (adapter.py:59-63).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib


def adapter_reference_init(in_channels: int, hidden_channels: int = 16) -> torch.Tensor:
    """Flat CPU params drawn like adapter.py:13-20 (nn.Conv2d default init, construction order
    conv1 then conv2), so `torch.manual_seed(s); OutputAdapter(...)` matches the reference."""
    with torch.no_grad():
        c1 = nn.Conv2d(2 * in_channels, hidden_channels, kernel_size=3, padding=1, bias=True)
        c2 = nn.Conv2d(hidden_channels, in_channels, kernel_size=3, padding=1, bias=True)
        return torch.cat([c1.weight.reshape(-1), c1.bias, c2.weight.reshape(-1), c2.bias]).float()


class _Holder(nn.Module):
    pass


class _AdapterFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, noisy, base_out, mod, *params):
        out = torch.empty_like(base_out)
        mod._run_forward(noisy, base_out, out)
        ctx.mod = mod
        ctx.save_for_backward(noisy, base_out)
        return out

    @staticmethod
    def backward(ctx, dout):
        noisy, base_out = ctx.saved_tensors
        mod = ctx.mod
        dflat = torch.empty_like(mod._flat)
        mod._run_backward(noisy, base_out, dout.contiguous(), dflat)
        grads = [dflat[o:o + n].view(shape) for (o, n, shape) in mod._views]
        return (None, None, None, *grads)


class OutputAdapter(nn.Module):
    """adapter.py:5 OutputAdapter(in_channels=1, hidden_channels=16):
    out = base_out + net(cat[noisy, base_out]), net = Conv3x3(2C,16) -> ReLU -> Conv3x3(16,C)."""

    def __init__(self, in_channels: int = 1, hidden_channels: int = 16):
        super().__init__()
        n = ctypes.c_size_t()
        _lib.check(_lib.lib().dn_adapter_param_count(in_channels, hidden_channels, ctypes.byref(n)),
                   "dn_adapter_param_count")
        self.in_channels, self.hidden_channels = in_channels, hidden_channels
        flat = adapter_reference_init(in_channels, hidden_channels)
        assert flat.numel() == n.value
        self._flat = flat
        C, Hd = in_channels, hidden_channels
        self.net = _Holder()
        shapes = [("0", "weight", (Hd, 2 * C, 3, 3)), ("0", "bias", (Hd,)),
                  ("2", "weight", (C, Hd, 3, 3)), ("2", "bias", (C,))]
        self._views, self._layout = [], []
        off = 0
        for mod, attr, shape in shapes:
            if not hasattr(self.net, mod):
                self.net.add_module(mod, _Holder())
            cnt = int(torch.Size(shape).numel())
            setattr(getattr(self.net, mod), attr, nn.Parameter(flat[off:off + cnt].view(shape)))
            self._views.append((off, cnt, shape))
            self._layout.append((getattr(self.net, mod), attr, off, cnt, shape))
            off += cnt
        self.net.add_module("1", nn.ReLU(inplace=True))  # adapter.py:17 (no parameters)
        self._slab = None

    @property
    def flat_params(self) -> torch.Tensor:
        return self._flat

    def _apply(self, fn, recurse=True):  # keep the parameters views of ONE flat buffer
        new = fn(self._flat)
        if not isinstance(new, torch.Tensor) or new.dtype != torch.float32:
            raise ValueError("adapter parameters are fp32")
        self._flat = new.contiguous()
        for (h, a, off, cnt, shape) in self._layout:
            p = getattr(h, a)
            p.data = self._flat[off:off + cnt].view(shape)
            p.grad = None
        self._slab = None
        return self

    def _params(self):
        return [getattr(h, a) for (h, a, *_ ) in self._layout]

    def _check(self, noisy, base_out):
        if noisy.device.type != "cuda":
            raise RuntimeError("the HIP adapter runs on a GPU: move the module and inputs to cuda")
        if noisy.shape != base_out.shape or noisy.dim() != 4 or noisy.shape[1] != self.in_channels:
            raise ValueError(f"expected noisy and base_out of one [N,{self.in_channels},H,W] shape")
        if noisy.dtype != torch.float32 or base_out.dtype != torch.float32:
            raise ValueError("adapter inputs must be float32")

    def _run_forward(self, noisy, base_out, out):
        N, C, H, W = noisy.shape
        _lib.call("dn_adapter_forward", _lib.ptr(self._flat), _lib.ptr(noisy), _lib.ptr(base_out),
                  _lib.ptr(out), N, C, H, W, self.hidden_channels, _lib.stream_of(noisy))

    def _run_backward(self, noisy, base_out, dout, dflat):
        N, C, H, W = noisy.shape
        need = _lib.lib().dn_adapter_slab_size(N, C, H, W, self.hidden_channels)
        if self._slab is None or self._slab.numel() < need or self._slab.device != noisy.device:
            self._slab = _lib.scratch(need, noisy.device)
        _lib.call("dn_adapter_backward", _lib.ptr(self._flat), _lib.ptr(noisy), _lib.ptr(base_out),
                  _lib.ptr(dout), _lib.ptr(dflat), N, C, H, W, self.hidden_channels,
                  self._slab.data_ptr(), self._slab.numel(), _lib.stream_of(noisy))

    def forward(self, noisy: torch.Tensor, base_out: torch.Tensor) -> torch.Tensor:
        noisy, base_out = noisy.contiguous(), base_out.contiguous()
        self._check(noisy, base_out)
        if noisy.requires_grad or base_out.requires_grad:
            raise NotImplementedError("gradients w.r.t. the adapter inputs are not computed "
                                      "(the reference runs the base under no_grad)")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self._params()):
            return _AdapterFunction.apply(noisy, base_out, self, *self._params())
        out = torch.empty_like(base_out)
        self._run_forward(noisy, base_out, out)
        return out


class DenoiserWithAdapter(nn.Module):
    """adapter.py:29 DenoiserWithAdapter(base_model, in_channels=1, hidden_channels=16,
    freeze_base=True, use_no_grad_for_base=True)."""

    def __init__(self, base_model: nn.Module, in_channels: int = 1, hidden_channels: int = 16,
                 freeze_base: bool = True, use_no_grad_for_base: bool = True):
        super().__init__()
        self.base = base_model
        self.in_channels = in_channels
        self.freeze_base = freeze_base
        self.use_no_grad_for_base = use_no_grad_for_base
        if freeze_base:
            for p in self.base.parameters():
                p.requires_grad = False
        self.adapter = OutputAdapter(in_channels=in_channels, hidden_channels=hidden_channels)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.use_no_grad_for_base:
            with torch.no_grad():
                base_out = self.base(x)
        else:
            if any(p.requires_grad for p in self.base.parameters()):
                raise NotImplementedError("training the base through the adapter is out of scope "
                                          "(finetune.py freezes it)")
            base_out = self.base(x)
        return self.adapter(x, base_out)
