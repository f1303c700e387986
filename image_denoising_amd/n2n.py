"""Neighbor2Neighbor sampler, noise and loss (train.py:64-190, training_script.md:126-155).

Drop-in functions keep the reference names and argument meaning:
  generate_mask_pair(img)            -> (mask1, mask2) bool[N*H/2*W/2*4]     train.py:141-172
  generate_subimages(img, mask)      -> [N,C,H/2,W/2]                         train.py:175-190
  AugmentNoise(style).add_train_noise(x)                                     train.py:64-101
and the fused fast path used by the trainer:
  n2n_subsample(img, rd_idx=None, seed, offset, cell_base) -> (sub1, sub2, rd_idx)
  n2n_loss(out, sub2, den, rd_idx, lam)                     -> (loss3, dout)

Random choices come from an in-kernel counter-based Philox stream keyed on (seed, offset,
global index) instead of train.py:56-61's torch generator (whose counter global is never
initialised in the reference, train.py:43).  Passing an explicit `rd_idx` reproduces any
reference mask pair bit-exactly.
"""
from __future__ import annotations

import itertools

import torch

from . import _lib

# train.py:151-154, within-cell index k = 2*dy + dx (unfold order, train.py:134-138)
PAIR_TABLE = ((0, 1), (0, 2), (1, 3), (2, 3), (1, 0), (2, 0), (3, 1), (3, 2))

_seed_counter = itertools.count(1)  # train.py:56-61: counter += 1 per generator


def _check_img(img: torch.Tensor):
    if img.dim() != 4 or img.dtype != torch.float32:
        raise ValueError(f"expected float32 [N,C,H,W], got {img.dtype} {tuple(img.shape)}")
    if img.shape[2] % 2 or img.shape[3] % 2:
        raise ValueError("H and W must be even")
    return img.contiguous()


def n2n_subsample(img: torch.Tensor, rd_idx: torch.Tensor | None = None, seed: int = 0,
                  offset: int = 0, cell_base: int = 0):
    """Both N2N sub-images in one HIP pass.  rd_idx: uint8 [N*H/2*W/2] (values 0..7)."""
    img = _check_img(img)
    N, C, H, W = img.shape
    cells = N * (H // 2) * (W // 2)
    sub1 = torch.empty((N, C, H // 2, W // 2), dtype=img.dtype, device=img.device)
    sub2 = torch.empty_like(sub1)
    if rd_idx is not None:
        rd_idx = rd_idx.to(device=img.device, dtype=torch.uint8).contiguous().view(-1)
        if rd_idx.numel() != cells:
            raise ValueError(f"rd_idx must have {cells} entries")
        rd_out = None
        rd_in = rd_idx
    else:
        rd_out = torch.empty(cells, dtype=torch.uint8, device=img.device)
        rd_in = None
    _lib.call("dn_n2n_subsample", _lib.ptr(img), N, C, H, W, _lib.ptr(rd_in), seed, offset,
              cell_base, _lib.ptr(sub1), _lib.ptr(sub2), _lib.ptr(rd_out), _lib.stream_of(img))
    return sub1, sub2, (rd_in if rd_in is not None else rd_out)


def rd_to_masks(rd_idx: torch.Tensor):
    """rd_idx -> (mask1, mask2) in generate_mask_pair's format (bool[4*cells])."""
    rd = rd_idx.to(torch.uint8).contiguous().view(-1)
    m1 = torch.empty(rd.numel() * 4, dtype=torch.bool, device=rd.device)
    m2 = torch.empty_like(m1)
    _lib.call("dn_n2n_masks", _lib.ptr(rd), rd.numel(), _lib.ptr(m1), _lib.ptr(m2),
              _lib.stream_of(rd))
    return m1, m2


def generate_mask_pair(img: torch.Tensor, rd_idx: torch.Tensor | None = None, seed: int | None = None):
    """train.py:141-172.  Returns (mask1, mask2) bool[N*H/2*W/2*4] with exactly one True per
    2x2 cell each, never at the same position.  `rd_idx` (0..7 per cell) pins the choice."""
    img = _check_img(img)
    N, _, H, W = img.shape
    cells = N * (H // 2) * (W // 2)
    if rd_idx is None:
        s = next(_seed_counter) if seed is None else seed
        rd_idx = torch.empty(cells, dtype=torch.uint8, device=img.device)
        # a zero-channel call of the sub-sampler only draws the per-cell choices
        dummy = img[:, :1]
        d1 = torch.empty((N, 1, H // 2, W // 2), dtype=img.dtype, device=img.device)
        d2 = torch.empty_like(d1)
        _lib.call("dn_n2n_subsample", _lib.ptr(dummy.contiguous()), N, 1, H, W, None, s, 0, 0,
                  _lib.ptr(d1), _lib.ptr(d2), _lib.ptr(rd_idx), _lib.stream_of(img))
    return rd_to_masks(rd_idx)


def generate_subimages(img: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """train.py:175-190: sub[n,c,i,j] = img[n,c,2i+(k>>1),2j+(k&1)], k = the cell's True slot."""
    img = _check_img(img)
    N, C, H, W = img.shape
    mask = mask.to(device=img.device, dtype=torch.uint8).contiguous().view(-1)
    if mask.numel() != N * (H // 2) * (W // 2) * 4:
        raise ValueError("mask size does not match img")
    sub = torch.empty((N, C, H // 2, W // 2), dtype=img.dtype, device=img.device)
    _lib.call("dn_n2n_subimage_from_mask", _lib.ptr(img), N, C, H, W, _lib.ptr(mask),
              _lib.ptr(sub), _lib.stream_of(img))
    return sub


class AugmentNoise:
    """train.py:64-111.  'gauss25' -> sigma = 25/255; 'gauss5_50' -> per-image sigma ~ U[5/255,
    50/255]; 'poisson30' -> Poisson(30 x) / 30; 'poisson5_50' -> per-image lam ~ U[5, 50].  The
    random streams are Philox on the GPU (global element index, seed, offset), not torch's
    generator."""

    def __init__(self, style: str, seed: int = 0):
        if style.startswith("gauss"):
            self.params = [float(p) / 255.0 for p in style.replace("gauss", "").split("_")]
            self.style = "gauss_fix" if len(self.params) == 1 else "gauss_range"
        elif style.startswith("poisson"):
            self.params = [float(p) for p in style.replace("poisson", "").split("_")]
            self.style = "poisson_fix" if len(self.params) == 1 else "poisson_range"
            if not all(0.0 < p <= 500.0 for p in self.params):
                raise ValueError("poisson lam must be in (0, 500]")
        else:
            raise ValueError(f"unknown noise style {style!r}")
        if len(self.params) not in (1, 2):
            raise ValueError(f"noise style {style!r}: one value or a min_max range")
        self.seed = seed
        self.calls = 0

    def add_train_noise(self, x: torch.Tensor, offset: int | None = None, elem_base: int = 0):
        x = x.contiguous()
        N = x.shape[0]
        per = x.numel() // max(N, 1)
        out = torch.empty_like(x)
        per_img = None
        if self.style.endswith("_range"):  # train.py:95-96 / :108-109: one value per image
            lo, hi = self.params
            g = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + self.calls)
            per_img = (torch.rand(N, generator=g) * (hi - lo) + lo).to(x.device)
        off = self.calls if offset is None else offset
        self.calls += 1
        fn = "dn_add_gauss_noise" if self.style.startswith("gauss") else "dn_add_poisson_noise"
        _lib.call(fn, _lib.ptr(x), N, per, float(self.params[0]), _lib.ptr(per_img), self.seed, off,
                  elem_base, _lib.ptr(out), _lib.stream_of(x))
        return out


_partials = {}


def _partials_for(device) -> torch.Tensor:
    t = _partials.get(device)
    if t is None:
        t = torch.empty(_lib.lib().dn_loss_partials_size(), dtype=torch.uint8, device=device)
        _partials[device] = t
    return t


def n2n_loss(out: torch.Tensor, sub2: torch.Tensor, den: torch.Tensor, rd_idx: torch.Tensor,
             lam: float):
    """training_script.md:141-153 with den1/den2 = generate_subimages(den, mask1/2).
    Returns (loss3 = [loss1, loss2, loss_all] device tensor, dout = dloss_all/dout)."""
    out, sub2, den = out.contiguous(), sub2.contiguous(), den.contiguous()
    N, C, h, w = out.shape
    if tuple(sub2.shape) != (N, C, h, w) or tuple(den.shape) != (N, C, 2 * h, 2 * w):
        raise ValueError("shape mismatch between out, sub2 and den")
    rd = rd_idx.to(device=out.device, dtype=torch.uint8).contiguous()
    dout = torch.empty_like(out)
    loss3 = torch.empty(3, dtype=torch.float32, device=out.device)
    _lib.call("dn_n2n_loss", _lib.ptr(out), _lib.ptr(sub2), _lib.ptr(den), _lib.ptr(rd), N, C, h,
              w, float(lam), _lib.ptr(dout), _lib.ptr(loss3), _partials_for(out.device).data_ptr(),
              _lib.stream_of(out))
    return loss3, dout
