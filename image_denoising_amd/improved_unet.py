"""Drop-in `ImprovedUNet` for arch_unet.py:421-531 (the model train.sh and evaluation.py
default to), computed by libdenoise_hip.so on gfx950 (dn_iunet_forward / dn_iunet_backward).

Same constructor, same `state_dict` keys and shapes (reference checkpoints load with
`load_state_dict`), same forward.  The module tree below only carries the parameters (drawn in
the reference's construction order, so `torch.manual_seed(s); ImprovedUNet(...)` matches the
reference bit for bit); every parameter is then re-pointed into ONE flat fp32 buffer, the layout
the C-ABI consumes.  Only the reference's defaults depth=4, noise=True and n_feature=48 are built.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib

GROWTH = 32


def _gn(ch: int) -> nn.GroupNorm:  # norm2d('gn', ch, groups=32), arch_unet.py:7-15
    g = min(32, ch)
    while ch % g != 0 and g > 1:
        g -= 1
    return nn.GroupNorm(g, ch, affine=True)


class _RDB(nn.Module):  # parameter holder of arch_unet.py:436-444
    def __init__(self, ch):
        super().__init__()
        self.convs = nn.ModuleList()
        c = ch
        for _ in range(4):
            self.convs.append(nn.Conv2d(c, GROWTH, 3, 1, 1, bias=True))
            c += GROWTH
        self.lff = nn.Conv2d(c, ch, 1, 1, 0, bias=True)
        self.act = nn.LeakyReLU(0.2, True)


class _ResBlock(nn.Module):  # arch_unet.py:422-431
    def __init__(self, ch):
        super().__init__()
        self.block = nn.Sequential(nn.Conv2d(ch, ch, 3, 1, 1, bias=False), _gn(ch),
                                   nn.LeakyReLU(0.2, True), nn.Conv2d(ch, ch, 3, 1, 1, bias=False),
                                   _gn(ch))


class _UpBlock(nn.Module):  # arch_unet.py:454-461
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv_ps = nn.Conv2d(in_ch, out_ch * 4, 3, 1, 1, bias=True)
        self.ps = nn.PixelShuffle(2)
        self.fuse = nn.Conv2d(out_ch * 3, out_ch, 3, 1, 1, bias=True)
        self.rdb = _RDB(out_ch)
        self.res = _ResBlock(out_ch)


class _IUNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, *params):
        N, _, H, W = x.shape
        y = torch.empty((N, net.out_nc, H, W), dtype=torch.float32, device=x.device)
        ws = net._workspace(N, H, W, with_backward=True, fresh=True)
        net._run_forward(x, y, ws)
        ctx.net, ctx.ws, ctx.shape = net, ws, (N, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        net = ctx.net
        N, H, W = ctx.shape
        dflat = torch.empty_like(net._flat)
        net._run_backward(dy.contiguous(), dflat, ctx.ws, N, H, W)
        ctx.ws = None
        grads = [dflat[o:o + p.numel()].view_as(p) for (o, p) in net._param_views()]
        return (None, None, *grads)


class ImprovedUNet(nn.Module):
    """arch_unet.py:475 ImprovedUNet(in_nc=3, out_nc=3, n_feature=48, depth=4, noise=True)."""

    def __init__(self, in_nc=3, out_nc=3, n_feature=48, depth=4, noise=True):
        super().__init__()
        if depth != 4 or not noise or n_feature != 48:
            raise NotImplementedError("the HIP ImprovedUNet is built for depth=4, noise=True, "
                                      "n_feature=48 (the reference's defaults)")
        self.in_nc, self.out_nc, self.n_feature, self.noise = in_nc, out_nc, n_feature, noise
        self._cfg = _lib.cfg(in_nc, out_nc, n_feature)
        n = ctypes.c_size_t()
        _lib.check(_lib.lib().dn_iunet_param_count(ctypes.byref(self._cfg), ctypes.byref(n)),
                   "dn_iunet_param_count")
        # construction order of arch_unet.py:476-516 (every Conv2d draws from the global RNG)
        nf = n_feature
        self.noise_estimator = nn.Sequential(nn.Conv2d(in_nc, nf, 3, 1, 1, bias=True),
                                             nn.LeakyReLU(0.2, True),
                                             nn.Conv2d(nf, 1, 3, 1, 1, bias=True), nn.Sigmoid())
        self.downs, self.pools = nn.ModuleList(), nn.ModuleList()
        for i in range(depth):
            inc = in_nc + 1 if i == 0 else nf // 2
            self.downs.append(nn.Sequential(nn.Conv2d(inc, nf, 3, 1, 1, bias=True),
                                            nn.LeakyReLU(0.2, True), _RDB(nf), _ResBlock(nf)))
            self.pools.append(nn.MaxPool2d(2))
            nf *= 2
        self.bottle = nn.Sequential(_RDB(nf // 2), _ResBlock(nf // 2))
        nf //= 2
        self.ups = nn.ModuleList()
        for _ in range(depth):
            self.ups.append(_UpBlock(nf, nf // 2))
            nf //= 2
        self.final = nn.Conv2d(n_feature // 2 + in_nc, out_nc, 3, 1, 1, bias=True)
        self.sigmoid = nn.Sigmoid()
        # one flat buffer in state_dict order; parameters become views of it
        named = list(self.named_parameters())
        flat = torch.cat([p.detach().reshape(-1) for _, p in named]).float().contiguous()
        assert flat.numel() == n.value, (flat.numel(), n.value)
        self._flat = flat
        self._layout = []
        off = 0
        for name, p in named:
            mod = self.get_submodule(name.rsplit(".", 1)[0])
            attr = name.rsplit(".", 1)[1]
            cnt = p.numel()
            setattr(mod, attr, nn.Parameter(flat[off:off + cnt].view(p.shape)))
            self._layout.append((mod, attr, off, tuple(p.shape)))
            off += cnt
        self._ws_cache = {}

    @property
    def flat_params(self) -> torch.Tensor:
        return self._flat

    def _param_views(self):
        return [(off, getattr(m, a)) for (m, a, off, _) in self._layout]

    def _apply(self, fn, recurse=True):  # keep the parameters views of ONE flat buffer
        new = fn(self._flat)
        if not isinstance(new, torch.Tensor) or new.dtype != torch.float32:
            raise ValueError("ImprovedUNet parameters are fp32 (the HIP path computes in fp32)")
        self._flat = new.contiguous()
        for (m, a, off, shape) in self._layout:
            p = getattr(m, a)
            p.data = self._flat[off:off + int(torch.Size(shape).numel())].view(shape)
            p.grad = None
        self._ws_cache = {}
        return self

    def _workspace(self, N, H, W, with_backward, fresh=False):
        key = (N, H, W, bool(with_backward), self._flat.device)
        if not fresh and key in self._ws_cache:
            return self._ws_cache[key]
        nbytes = ctypes.c_size_t()
        _lib.check(_lib.lib().dn_iunet_workspace_size(ctypes.byref(self._cfg), N, H, W,
                                                      int(with_backward), ctypes.byref(nbytes)),
                   "dn_iunet_workspace_size")
        ws = torch.empty(nbytes.value, dtype=torch.uint8, device=self._flat.device)
        if not fresh:
            self._ws_cache = {key: ws}
        return ws

    # arithmetic of the 3x3 convolutions (include/denoise_hip.h DN_PREC_*)
    _PRECISIONS = {"fp32": 0, "fp32_x6": 2}

    def set_precision(self, mode: str) -> "ImprovedUNet":
        """Arithmetic of the 3x3 convolutions' forward and data gradient: 'fp32' (fp32 matrix
        cores) or 'fp32_x6' (exact three-piece bf16 split, six products, fp32 accumulation;
        DESIGN.md §12).  Weight gradients and the 1x1 / noise-estimator convs stay fp32."""
        if mode not in self._PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(self._PRECISIONS)}")
        self.precision = mode
        return self

    def _prec(self) -> int:
        return self._PRECISIONS[getattr(self, "precision", "fp32")]

    def _run_forward(self, x, y, ws):
        N, _, H, W = x.shape
        _lib.call("dn_iunet_forward_prec", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(x), _lib.ptr(y), N, H, W, ws.data_ptr(), ws.numel(), self._prec(),
                  _lib.stream_of(x))

    def _run_forward_n2n(self, x, den, ws, rd_idx):
        """the N2N no-grad pass (N2NTrainer): the whole image, a superset of the rd pair pixels
        the loss reads (the pair-pixel fast path is built for the UNet's dec_conv1b / head)"""
        self._run_forward(x, den, ws)

    def _run_backward(self, dy, dflat, ws, N, H, W):
        _lib.call("dn_iunet_backward_prec", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(dy), _lib.ptr(dflat), N, H, W, ws.data_ptr(), ws.numel(), self._prec(),
                  _lib.stream_of(dy))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        if x.device.type != "cuda":
            raise RuntimeError("the HIP ImprovedUNet runs on a GPU: move the module and input to cuda")
        if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != self.in_nc:
            raise ValueError(f"expected float32 [N,{self.in_nc},H,W], got {x.dtype} {tuple(x.shape)}")
        N, _, H, W = x.shape
        if H % 16 or W % 16:
            raise ValueError("H and W must be multiples of 16 (ImprovedUNet: 4 pooling levels)")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            if x.requires_grad:
                raise NotImplementedError("gradient w.r.t. the network input is not computed")
            return _IUNetFunction.apply(x, self, *[p for _, p in self._param_views()])
        y = torch.empty((N, self.out_nc, H, W), dtype=torch.float32, device=x.device)
        self._run_forward(x, y, self._workspace(N, H, W, with_backward=False))
        return y
