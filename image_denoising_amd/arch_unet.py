"""Drop-in `UNet` for arch_unet.py:100-260, computed by libdenoise_hip.so on gfx950.

Same constructor signature, same `state_dict` keys/shapes (so reference checkpoints load with
`load_state_dict`), same `forward(x[N,C,H,W]) -> [N,out_nc,H,W]`.  Internally all parameters are
views into ONE flat fp32 buffer in state_dict order (the layout the C-ABI consumes), and the
forward/backward run through dn_unet_forward / dn_unet_backward (parameter gradients and, when the
input requires grad, dL/dx).  The blind-spot variant
(arch_unet.py:65-97) is out of scope and raises.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
import torch.nn.init as init

from . import _lib

# state_dict order of arch_unet.py:115-192
LAYER_NAMES = [
    "enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5", "enc_conv6",
    "up5.deconv", "dec_conv5a", "dec_conv5b", "up4.deconv", "dec_conv4a", "dec_conv4b",
    "up3.deconv", "dec_conv3a", "dec_conv3b", "up2.deconv", "dec_conv2a", "dec_conv2b",
    "up1.deconv", "dec_conv1a", "dec_conv1b", "nin_a", "nin_b", "nin_c",
]


def layer_shapes(in_nc: int, out_nc: int, nf: int):
    """[(name, weight_shape, bias_len, is_deconv)] in state_dict order (arch_unet.py:115-192)."""
    C, OC = in_nc, out_nc
    s = []
    conv = lambda name, co, ci, k: s.append((name, (co, ci, k, k), co, False))
    dec = lambda name, ci, co: s.append((name, (ci, co, 2, 2), co, True))
    conv("enc_conv0", nf, C, 3)
    for i in range(1, 7):
        conv(f"enc_conv{i}", nf, nf, 3)
    dec("up5.deconv", nf, nf)
    conv("dec_conv5a", 2 * nf, 2 * nf, 3)
    conv("dec_conv5b", 2 * nf, 2 * nf, 3)
    for lvl in (4, 3, 2):
        dec(f"up{lvl}.deconv", 2 * nf, 2 * nf)
        conv(f"dec_conv{lvl}a", 2 * nf, 3 * nf, 3)
        conv(f"dec_conv{lvl}b", 2 * nf, 2 * nf, 3)
    dec("up1.deconv", 2 * nf, 2 * nf)
    conv("dec_conv1a", 96, 2 * nf + C, 3)
    conv("dec_conv1b", 96, 96, 3)
    conv("nin_a", 96, 96, 1)
    conv("nin_b", 96, 96, 1)
    conv("nin_c", OC, 96, 1)
    return s


def param_count(in_nc: int, out_nc: int, nf: int) -> int:
    return sum(int(torch.Size(w).numel()) + b for _, w, b, _ in layer_shapes(in_nc, out_nc, nf))


def _kaiming01(m: nn.Module) -> None:
    # arch_unet.py:24-48 initialize_weights(m, 0.1) for Conv2d / ConvTranspose2d
    init.kaiming_normal_(m.weight, a=0, mode="fan_in")
    m.weight.data *= 0.1
    if m.bias is not None:
        m.bias.data.zero_()


def reference_init(in_nc: int, out_nc: int, nf: int = 48, zero_last: bool = False) -> torch.Tensor:
    """Flat CPU fp32 parameters drawn exactly like arch_unet.UNet.__init__ does.

    The reference constructs torch modules (each consuming the global CPU RNG in its
    reset_parameters) and re-initialises them with kaiming_normal_; the construction /
    initialisation ORDER of arch_unet.py:115-192 is replayed here, so that
    `torch.manual_seed(s); UNet(...)` yields bit-identical weights to the reference.
    """
    C, OC = in_nc, out_nc
    mods = {}

    def conv(name, ci, co, k):
        mods[name] = nn.Conv2d(ci, co, k, 1, (k - 1) // 2)

    def up(name, ci, co):  # UpsampleCat.__init__ (arch_unet.py:52-58)
        mods[name] = nn.ConvTranspose2d(ci, co, 2, 2, 0, 0)
        _kaiming01(mods[name])

    with torch.no_grad():
        conv("enc_conv0", C, nf, 3)
        conv("enc_conv1", nf, nf, 3)
        _kaiming01(mods["enc_conv0"])
        _kaiming01(mods["enc_conv1"])
        for i in range(2, 7):
            conv(f"enc_conv{i}", nf, nf, 3)
            _kaiming01(mods[f"enc_conv{i}"])
        up("up5.deconv", nf, nf)
        conv("dec_conv5a", 2 * nf, 2 * nf, 3)
        conv("dec_conv5b", 2 * nf, 2 * nf, 3)
        _kaiming01(mods["dec_conv5a"])
        _kaiming01(mods["dec_conv5b"])
        for lvl in (4, 3, 2):
            up(f"up{lvl}.deconv", 2 * nf, 2 * nf)
            conv(f"dec_conv{lvl}a", 3 * nf, 2 * nf, 3)
            conv(f"dec_conv{lvl}b", 2 * nf, 2 * nf, 3)
            _kaiming01(mods[f"dec_conv{lvl}a"])
            _kaiming01(mods[f"dec_conv{lvl}b"])
        up("up1.deconv", 2 * nf, 2 * nf)
        conv("dec_conv1a", 2 * nf + C, 96, 3)
        _kaiming01(mods["dec_conv1a"])
        conv("dec_conv1b", 96, 96, 3)
        _kaiming01(mods["dec_conv1b"])
        conv("nin_a", 96, 96, 1)
        conv("nin_b", 96, 96, 1)
        _kaiming01(mods["nin_a"])
        _kaiming01(mods["nin_b"])
        conv("nin_c", 96, OC, 1)
        if not zero_last:
            _kaiming01(mods["nin_c"])
        parts = []
        for name in LAYER_NAMES:
            parts += [mods[name].weight.reshape(-1), mods[name].bias.reshape(-1)]
        return torch.cat(parts).float().contiguous()


class _Holder(nn.Module):
    """Parameter container so that state_dict keys read e.g. 'enc_conv0.weight'."""


class _UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, *params):
        N, C, H, W = x.shape
        y = torch.empty((N, net.out_nc, H, W), dtype=torch.float32, device=x.device)
        ws = net._workspace(N, H, W, with_backward=True, fresh=True)
        net._run_forward(x, y, ws)
        ctx.net = net
        ctx.ws = ws
        ctx.shape = (N, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        net = ctx.net
        N, H, W = ctx.shape
        dy = dy.contiguous()
        dflat = torch.empty_like(net._flat)
        dx = None
        if ctx.needs_input_grad[0]:  # dL/dx from the same backward pass (dn_unet_backward dx)
            dx = torch.empty((N, net.in_nc, H, W), dtype=torch.float32, device=dy.device)
        net._run_backward(dy, dflat, ctx.ws, N, H, W, dx=dx)
        ctx.ws = None
        grads = [dflat[o:o + p.numel()].view_as(p) if need else None
                 for (o, p), need in zip(net._param_views(), ctx.needs_input_grad[2:])]
        return (dx, None, *grads)


class UNet(nn.Module):
    """arch_unet.py:100 UNet(in_nc=3, out_nc=3, n_feature=48, blindspot=False, zero_last=False)."""

    def __init__(self, in_nc=3, out_nc=3, n_feature=48, blindspot=False, zero_last=False):
        super().__init__()
        if blindspot:
            raise NotImplementedError("blind-spot UNet (arch_unet.py:65-97) is out of scope")
        self.in_nc, self.out_nc, self.n_feature = in_nc, out_nc, n_feature
        self.blindspot, self.zero_last = blindspot, zero_last
        self._cfg = _lib.cfg(in_nc, out_nc, n_feature)
        n = ctypes.c_size_t()
        _lib.check(_lib.lib().dn_unet_param_count(ctypes.byref(self._cfg), ctypes.byref(n)),
                   "dn_unet_param_count")
        flat = reference_init(in_nc, out_nc, n_feature, zero_last)
        assert flat.numel() == n.value, (flat.numel(), n.value)
        self._flat = flat
        self._layout = []  # (holder, attr, offset, shape)
        off = 0
        for name, wshape, blen, _ in layer_shapes(in_nc, out_nc, n_feature):
            holder = self
            parts = name.split(".")
            for p in parts:
                if not hasattr(holder, p) or not isinstance(getattr(holder, p), nn.Module):
                    setattr(holder, p, _Holder())
                holder = getattr(holder, p)
            wn = int(torch.Size(wshape).numel())
            holder.weight = nn.Parameter(flat[off:off + wn].view(wshape))
            self._layout.append((holder, "weight", off, wshape))
            off += wn
            holder.bias = nn.Parameter(flat[off:off + blen])
            self._layout.append((holder, "bias", off, (blen,)))
            off += blen
        self._ws_cache = {}

    # ---- flat-buffer plumbing -------------------------------------------------------
    @property
    def flat_params(self) -> torch.Tensor:
        """the flat fp32 parameter buffer every parameter is a view of"""
        return self._flat

    def _param_views(self):
        return [(off, getattr(h, a)) for (h, a, off, _) in self._layout]

    def _apply(self, fn, recurse=True):  # keep the parameters views of ONE flat buffer
        new = fn(self._flat)
        if not isinstance(new, torch.Tensor) or new.dtype != torch.float32:
            raise ValueError("UNet parameters are fp32 (the HIP path computes in fp32)")
        self._flat = new.contiguous()
        for (h, a, off, shape) in self._layout:
            p = getattr(h, a)
            n = int(torch.Size(shape).numel())
            p.data = self._flat[off:off + n].view(shape)
            p.grad = None
        self._ws_cache = {}
        return self

    def _workspace(self, N, H, W, with_backward, fresh=False):
        key = (N, H, W, bool(with_backward), self._flat.device)
        if not fresh and key in self._ws_cache:
            return self._ws_cache[key]
        nbytes = ctypes.c_size_t()
        _lib.check(_lib.lib().dn_unet_workspace_size(ctypes.byref(self._cfg), N, H, W,
                                                     int(with_backward), ctypes.byref(nbytes)),
                   "dn_unet_workspace_size")
        ws = torch.empty(nbytes.value, dtype=torch.uint8, device=self._flat.device)
        if not fresh:
            self._ws_cache = {key: ws}
        return ws

    def _check_input(self, x):
        if x.device.type != "cuda":
            raise RuntimeError("the HIP UNet runs on a GPU: move the module and input to cuda")
        if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != self.in_nc:
            raise ValueError(f"expected float32 [N,{self.in_nc},H,W], got {x.dtype} {tuple(x.shape)}")
        if self._flat.device != x.device:
            raise RuntimeError("module parameters and input are on different devices")

    # arithmetic of the 3x3 convolutions (include/denoise_hip.h DN_PREC_*)
    _PRECISIONS = {"fp32": 0, "fp32_x6": 2}

    def set_precision(self, mode: str) -> "UNet":
        """Arithmetic of the 3x3 convolutions in training and fp32 inference:
        'fp32'    fp32 operands on the fp32 matrix cores (v_mfma_f32_16x16x4_f32);
        'fp32_x6' fp32 operands split exactly into three bf16 pieces, the six piece products
                  of order <= 2 on the bf16 matrix cores, fp32 accumulation -- the rounding
                  error of an fp32 dot product at 2.67x the matrix-core peak."""
        if mode not in self._PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(self._PRECISIONS)}")
        self.precision = mode
        return self

    def _prec(self) -> int:
        return self._PRECISIONS[getattr(self, "precision", "fp32")]

    def _run_forward(self, x, y, ws):
        N, _, H, W = x.shape
        _lib.call("dn_unet_forward_prec", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(x), _lib.ptr(y), N, H, W, ws.data_ptr(), ws.numel(), self._prec(),
                  _lib.stream_of(x))

    def _infer_prec(self) -> int:
        """the precision code of a no-grad forward (bf16 for the configs[4] frozen base)"""
        return 1 if getattr(self, "inference_precision", "fp32") == "bf16" else self._prec()

    def _pack_weights(self, ws, N, H, W):
        """dn_unet_pack_weights: the forward's weight images for (N, H, W) into ws, once, for
        _run_forward_prepacked calls with these parameters (SURVEY §8b persistent packing)"""
        _lib.call("dn_unet_pack_weights", ctypes.byref(self._cfg), _lib.ptr(self._flat), N, H, W,
                  ws.data_ptr(), ws.numel(), self._infer_prec(), _lib.stream_of(self._flat))

    def _run_forward_prepacked(self, x, y, ws):
        """the no-grad forward on the images _pack_weights left in ws (no re-pack): bit-identical
        to _run_forward_inference while the parameters are unchanged"""
        N, _, H, W = x.shape
        _lib.call("dn_unet_forward_prepacked", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(x), _lib.ptr(y), N, H, W, ws.data_ptr(), ws.numel(), self._infer_prec(),
                  _lib.stream_of(x))

    def _run_forward_n2n(self, x, den, ws, rd_idx):
        """the N2N no-grad pass: den = UNet(x) at the pair pixels of rd_idx only
        (dn_unet_forward_n2n; training_script.md:141-144 reads nothing else)"""
        N, _, H, W = x.shape
        _lib.call("dn_unet_forward_n2n", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(x), _lib.ptr(den), _lib.ptr(rd_idx), N, H, W, ws.data_ptr(), ws.numel(),
                  self._prec(), _lib.stream_of(x))

    def set_inference_precision(self, dtype: str) -> "UNet":
        """'fp32' (default, the parity path) or 'bf16': no-grad forwards then multiply
        bf16-rounded operands on the bf16 matrix cores (fp32 accumulation and storage) —
        the mixed-precision frozen base of BASELINE configs[4].  Training is always fp32."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError("inference precision must be 'fp32' or 'bf16'")
        self.inference_precision = dtype
        return self

    def _run_forward_inference(self, x, y, ws):
        if getattr(self, "inference_precision", "fp32") != "bf16":
            return self._run_forward(x, y, ws)
        N, _, H, W = x.shape
        _lib.call("dn_unet_forward_bf16", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(x), _lib.ptr(y), N, H, W, ws.data_ptr(), ws.numel(), _lib.stream_of(x))

    def _run_backward(self, dy, dflat, ws, N, H, W, dx=None):
        """dflat = dL/dparams (and dx = dL/dx when given) for dy = dL/dy"""
        _lib.call("dn_unet_backward_prec", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(dy), _lib.ptr(dflat), _lib.ptr(dx), N, H, W, ws.data_ptr(), ws.numel(),
                  self._prec(), _lib.stream_of(dy))

    def _run_backward_split(self, dy, dflat, ws, N, H, W, tail_ready):
        """_run_backward that records tail_ready (a torch.cuda.Event) once dflat[tail_begin():]
        is final, while the encoder's gradients are still being computed
        (dn_unet_backward_split: the data-parallel step all-reduces that range early)"""
        _lib.call("dn_unet_backward_split", ctypes.byref(self._cfg), _lib.ptr(self._flat),
                  _lib.ptr(dy), _lib.ptr(dflat), None, N, H, W, ws.data_ptr(), ws.numel(),
                  self._prec(), _lib.stream_of(dy), ctypes.c_void_p(tail_ready.cuda_event), None)

    def tail_begin(self) -> int:
        """first flat-parameter index of the range (dec_conv5a .. nin_c, state_dict order) whose
        gradient the backward finishes before the encoder's"""
        t = ctypes.c_int64()
        _lib.call("dn_unet_backward_split", ctypes.byref(self._cfg), None, None, None, None, 1, 32,
                  32, None, 0, self._prec(), None, None, ctypes.byref(t))
        return int(t.value)

    # ---- nn.Module API ----------------------------------------------------------------
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        self._check_input(x)
        N, _, H, W = x.shape
        if H % 32 or W % 32:
            raise ValueError("H and W must be multiples of 32 (arch_unet.py: 5 pooling levels)")
        if torch.is_grad_enabled() and (x.requires_grad or
                                        any(p.requires_grad for p in self.parameters())):
            # autograd: parameter gradients and/or dL/dx, as the reference module gives
            return _UNetFunction.apply(x, self, *[p for _, p in self._param_views()])
        y = torch.empty((N, self.out_nc, H, W), dtype=torch.float32, device=x.device)
        self._run_forward_inference(x, y, self._workspace(N, H, W, with_backward=False))
        return y
