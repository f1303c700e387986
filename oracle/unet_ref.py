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


def forward(flat: torch.Tensor, x: torch.Tensor, in_nc: int, out_nc: int, nf: int = 48):
    """arch_unet.py:194-260 with the same op order (conv -> LeakyReLU(0.2) -> pool ...)."""
    P = unflatten(flat, in_nc, out_nc, nf)
    act = lambda t: F.leaky_relu(t, 0.2)
    conv = lambda t, n, pad=1: F.conv2d(t, P[n][0], P[n][1], 1, pad)
    up = lambda t, skip, n: torch.cat([F.conv_transpose2d(t, P[n][0], P[n][1], 2), skip], 1)
    pool0 = x
    h = act(conv(x, "enc_conv0"))
    h = act(conv(h, "enc_conv1"))
    h = F.max_pool2d(h, 2)
    pool1 = h
    h = F.max_pool2d(act(conv(h, "enc_conv2")), 2)
    pool2 = h
    h = F.max_pool2d(act(conv(h, "enc_conv3")), 2)
    pool3 = h
    h = F.max_pool2d(act(conv(h, "enc_conv4")), 2)
    pool4 = h
    h = F.max_pool2d(act(conv(h, "enc_conv5")), 2)
    h = act(conv(h, "enc_conv6"))
    h = up(h, pool4, "up5.deconv")
    h = act(conv(h, "dec_conv5a"))
    h = act(conv(h, "dec_conv5b"))
    h = up(h, pool3, "up4.deconv")
    h = act(conv(h, "dec_conv4a"))
    h = act(conv(h, "dec_conv4b"))
    h = up(h, pool2, "up3.deconv")
    h = act(conv(h, "dec_conv3a"))
    h = act(conv(h, "dec_conv3b"))
    h = up(h, pool1, "up2.deconv")
    h = act(conv(h, "dec_conv2a"))
    h = act(conv(h, "dec_conv2b"))
    h = up(h, pool0, "up1.deconv")
    h = act(conv(h, "dec_conv1a"))
    h = act(conv(h, "dec_conv1b"))
    h = act(conv(h, "nin_a", 0))
    h = act(conv(h, "nin_b", 0))
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
