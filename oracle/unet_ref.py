"""arch_unet.py:100-260 UNet (non-blind-spot) as torch-CPU functional ops on the flat
parameter buffer (test oracle; see oracle/__init__.py).  Backward = torch autograd."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def layer_table(in_nc: int, out_nc: int, nf: int = 48):
    """[(name, weight_shape, bias_len, kind)] in state_dict order (arch_unet.py:115-192)"""
    t = [("enc_conv0", (nf, in_nc, 3, 3), nf, "conv")]
    t += [(f"enc_conv{i}", (nf, nf, 3, 3), nf, "conv") for i in range(1, 7)]
    t += [("up5.deconv", (nf, nf, 2, 2), nf, "deconv"),
          ("dec_conv5a", (2 * nf, 2 * nf, 3, 3), 2 * nf, "conv"),
          ("dec_conv5b", (2 * nf, 2 * nf, 3, 3), 2 * nf, "conv")]
    for lvl in (4, 3, 2):
        t += [(f"up{lvl}.deconv", (2 * nf, 2 * nf, 2, 2), 2 * nf, "deconv"),
              (f"dec_conv{lvl}a", (2 * nf, 3 * nf, 3, 3), 2 * nf, "conv"),
              (f"dec_conv{lvl}b", (2 * nf, 2 * nf, 3, 3), 2 * nf, "conv")]
    t += [("up1.deconv", (2 * nf, 2 * nf, 2, 2), 2 * nf, "deconv"),
          ("dec_conv1a", (96, 2 * nf + in_nc, 3, 3), 96, "conv"),
          ("dec_conv1b", (96, 96, 3, 3), 96, "conv"),
          ("nin_a", (96, 96, 1, 1), 96, "conv"),
          ("nin_b", (96, 96, 1, 1), 96, "conv"),
          ("nin_c", (out_nc, 96, 1, 1), out_nc, "conv")]
    return t


def unflatten(flat: torch.Tensor, in_nc: int, out_nc: int, nf: int = 48):
    """flat -> {name: (weight view, bias view)}"""
    out, off = {}, 0
    for name, ws, bl, _ in layer_table(in_nc, out_nc, nf):
        n = 1
        for d in ws:
            n *= d
        w = flat[off:off + n].view(ws)
        off += n
        b = flat[off:off + bl]
        off += bl
        out[name] = (w, b)
    assert off == flat.numel(), (off, flat.numel())
    return out


class _LeakyWithMask(torch.autograd.Function):
    """LeakyReLU(0.2) whose backward slope is taken from a given (e.g. fp32 device) activation"""

    @staticmethod
    def forward(ctx, z, ref):
        ctx.save_for_backward(ref)
        return F.leaky_relu(z, 0.2)

    @staticmethod
    def backward(ctx, g):
        (ref,) = ctx.saved_tensors
        return torch.where(ref > 0, g, g * 0.2), None


class _PoolWithArgmax(torch.autograd.Function):
    """MaxPool2d(2) whose backward routes to the argmax (first max, row-major) of `ref`"""

    @staticmethod
    def forward(ctx, a, ref):
        _, idx = F.max_pool2d(ref, 2, return_indices=True)
        ctx.save_for_backward(idx)
        ctx.shape = a.shape
        return F.max_pool2d(a, 2)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return F.max_unpool2d(g, idx, 2, output_size=ctx.shape[-2:]), None


def _bf16(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype)


def forward(flat: torch.Tensor, x: torch.Tensor, in_nc: int, out_nc: int, nf: int = 48,
            record: dict | None = None, masks: dict | None = None, bf16_3x3: bool = False):
    """arch_unet.py:194-260 with the same op order (conv -> LeakyReLU(0.2) -> pool ...).
    `record` (optional) receives the intermediate tensors under the workspace names
    (c1 a0 a1 c2..c5 a2..a5 p5 a6 d2a..d5b d1a d1b na nb) with retain_grad() set.
    `bf16_3x3` rounds the operands of the 3x3 layers (not enc_conv0), the deconvs and nin_a /
    nin_b to bf16 (the mixed-precision inference path).
    `masks` (optional) maps the post-activation names to tensors (e.g. the device's fp32
    activations) that decide LeakyReLU slopes and max-pool routing in the backward, so a
    high-precision backward can be compared with a low-precision one without the slope flips
    that tiny forward rounding differences cause at pre-activations near zero."""
    P = unflatten(flat, in_nc, out_nc, nf)

    def conv(t, n, pad=1):
        # bf16_3x3 emulates dn_unet_forward_bf16: the 3x3 layers after enc_conv0, nin_a / nin_b
        # and the deconvs multiply bf16-rounded activations and weights (exact products),
        # accumulated in t's precision
        w = P[n][0]
        if bf16_3x3 and n not in ("enc_conv0", "nin_c"):
            return F.conv2d(_bf16(t), _bf16(w), P[n][1], 1, pad)
        return F.conv2d(t, w, P[n][1], 1, pad)
    def up(t, skip, n):
        w = _bf16(P[n][0]) if bf16_3x3 else P[n][0]
        t = _bf16(t) if bf16_3x3 else t
        return torch.cat([F.conv_transpose2d(t, w, P[n][1], 2), skip], 1)

    def act(t, name):
        if masks is not None:
            return _LeakyWithMask.apply(t, masks[name].to(t.dtype))
        return F.leaky_relu(t, 0.2)

    def pool(t, name):
        if masks is not None:
            return _PoolWithArgmax.apply(t, masks[name].to(t.dtype))
        return F.max_pool2d(t, 2)

    def rec(name, t):
        if record is not None and t.requires_grad:
            t.retain_grad()
            record[name] = t
        return t

    pool0 = x
    h = rec("a0", act(conv(x, "enc_conv0"), "a0"))
    h = rec("a1", act(conv(h, "enc_conv1"), "a1"))
    h = pool(h, "a1")
    pool1 = h
    h = pool(rec("a2", act(conv(h, "enc_conv2"), "a2")), "a2")
    pool2 = h
    h = pool(rec("a3", act(conv(h, "enc_conv3"), "a3")), "a3")
    pool3 = h
    h = pool(rec("a4", act(conv(h, "enc_conv4"), "a4")), "a4")
    pool4 = h
    h = rec("p5", pool(rec("a5", act(conv(h, "enc_conv5"), "a5")), "a5"))
    h = rec("a6", act(conv(h, "enc_conv6"), "a6"))
    h = rec("c5", up(h, pool4, "up5.deconv"))
    h = rec("d5a", act(conv(h, "dec_conv5a"), "d5a"))
    h = rec("d5b", act(conv(h, "dec_conv5b"), "d5b"))
    h = rec("c4", up(h, pool3, "up4.deconv"))
    h = rec("d4a", act(conv(h, "dec_conv4a"), "d4a"))
    h = rec("d4b", act(conv(h, "dec_conv4b"), "d4b"))
    h = rec("c3", up(h, pool2, "up3.deconv"))
    h = rec("d3a", act(conv(h, "dec_conv3a"), "d3a"))
    h = rec("d3b", act(conv(h, "dec_conv3b"), "d3b"))
    h = rec("c2", up(h, pool1, "up2.deconv"))
    h = rec("d2a", act(conv(h, "dec_conv2a"), "d2a"))
    h = rec("d2b", act(conv(h, "dec_conv2b"), "d2b"))
    h = rec("c1", up(h, pool0, "up1.deconv"))
    h = rec("d1a", act(conv(h, "dec_conv1a"), "d1a"))
    h = rec("d1b", act(conv(h, "dec_conv1b"), "d1b"))
    h = rec("na", act(conv(h, "nin_a", 0), "na"))
    h = rec("nb", act(conv(h, "nin_b", 0), "nb"))
    return conv(h, "nin_c", 0)


def forward_backward(flat: torch.Tensor, x: torch.Tensor, dy: torch.Tensor, in_nc: int,
                     out_nc: int, nf: int = 48):
    """(y, dflat) for the cotangent dy."""
    p = flat.detach().clone().requires_grad_(True)
    y = forward(p, x, in_nc, out_nc, nf)
    y.backward(dy)
    return y.detach(), p.grad.detach()


def n2n_step(flat: torch.Tensor, noisy: torch.Tensor, rd_idx, lam: float, lr: float = 3e-4,
             in_nc: int = 1, out_nc: int = 1, nf: int = 48, adam_state=None):
    """training_script.md:137-155 for one step with torch.optim.Adam (train.py:332).
    Returns dict(loss1, loss2, loss, dout, grad, params, adam_state)."""
    import numpy as np

    from . import n2n_ref

    noisy_np = noisy.numpy()
    m1, m2 = n2n_ref.masks_from_rd(rd_idx)
    sub1 = torch.from_numpy(n2n_ref.generate_subimages(noisy_np, m1))
    sub2 = torch.from_numpy(n2n_ref.generate_subimages(noisy_np, m2))
    with torch.no_grad():
        den = forward(flat, noisy, in_nc, out_nc, nf)
    p = torch.nn.Parameter(flat.detach().clone())
    opt = torch.optim.Adam([p], lr=lr)
    if adam_state is not None:
        opt.load_state_dict(adam_state)
    out = forward(p, sub1, in_nc, out_nc, nf)
    out.retain_grad()
    d1 = torch.from_numpy(n2n_ref.generate_subimages(den.numpy(), m1))
    d2 = torch.from_numpy(n2n_ref.generate_subimages(den.numpy(), m2))
    diff = out - sub2
    exp_diff = d1 - d2
    loss1 = torch.mean(diff ** 2)
    loss2 = lam * torch.mean((diff - exp_diff) ** 2)
    loss = loss1 + loss2
    opt.zero_grad()
    loss.backward()
    grad = p.grad.detach().clone()
    opt.step()
    return dict(loss1=float(loss1), loss2=float(loss2), loss=float(loss),
                dout=out.grad.detach().numpy(), grad=grad, params=p.detach().clone(),
                den=den, sub1=sub1, sub2=sub2, adam_state=opt.state_dict(),
                rd_idx=np.asarray(rd_idx))
