"""ORACLE (test infrastructure only) — arch_unet.py:421-531 ImprovedUNet(in_nc, out_nc, 48,
depth=4, noise=True) as torch-CPU functional ops on the flat parameter buffer (state_dict order).
Backward = torch autograd."""
from __future__ import annotations

import torch
import torch.nn.functional as F

GROWTH = 32


def gn_groups(ch: int, groups: int = 32) -> int:
    """arch_unet.py:12-15"""
    g = min(groups, ch)
    while ch % g != 0 and g > 1:
        g -= 1
    return g


def layer_table(in_nc: int, out_nc: int, nf: int = 48):
    """[(key, shape)] in state_dict order"""
    t = []
    conv = lambda k, co, ci, ks, bias=True: t.extend(
        [(f"{k}.weight", (co, ci, ks, ks))] + ([(f"{k}.bias", (co,))] if bias else []))
    gn = lambda k, ch: t.extend([(f"{k}.weight", (ch,)), (f"{k}.bias", (ch,))])

    def rdb(k, ch):
        for j in range(4):
            conv(f"{k}.convs.{j}", GROWTH, ch + GROWTH * j, 3)
        conv(f"{k}.lff", ch, ch + 4 * GROWTH, 1)

    def res(k, ch):
        conv(f"{k}.block.0", ch, ch, 3, False)
        gn(f"{k}.block.1", ch)
        conv(f"{k}.block.3", ch, ch, 3, False)
        gn(f"{k}.block.4", ch)

    conv("noise_estimator.0", nf, in_nc, 3)
    conv("noise_estimator.2", 1, nf, 3)
    c = nf
    for i in range(4):
        conv(f"downs.{i}.0", c, in_nc + 1 if i == 0 else c // 2, 3)
        rdb(f"downs.{i}.2", c)
        res(f"downs.{i}.3", c)
        c *= 2
    c //= 2
    rdb("bottle.0", c)
    res("bottle.1", c)
    for k in range(4):
        o = c // 2
        conv(f"ups.{k}.conv_ps", 4 * o, c, 3)
        conv(f"ups.{k}.fuse", o, 3 * o, 3)
        rdb(f"ups.{k}.rdb", o)
        res(f"ups.{k}.res", o)
        c = o
    conv("final", out_nc, nf // 2 + in_nc, 3)
    return t


def unflatten(flat: torch.Tensor, in_nc: int, out_nc: int, nf: int = 48) -> dict:
    out, off = {}, 0
    for k, shape in layer_table(in_nc, out_nc, nf):
        n = 1
        for d in shape:
            n *= d
        out[k] = flat[off:off + n].view(shape)
        off += n
    assert off == flat.numel(), (off, flat.numel())
    return out


def _conv(P, k, x, pad=1):
    return F.conv2d(x, P[f"{k}.weight"], P.get(f"{k}.bias"), padding=pad)


def _rdb(P, k, x, tr=None):  # arch_unet.py:446-451
    feats = [x]
    for j in range(4):
        feats.append(F.leaky_relu(_conv(P, f"{k}.convs.{j}", torch.cat(feats, 1)), 0.2))
    cat = torch.cat(feats, 1)
    r = x + _conv(P, f"{k}.lff", cat, pad=0)
    if tr is not None:
        tr += [(f"{k}:F", cat), (f"{k}:r", r)]
    return r


def _res(P, k, x, tr=None):  # arch_unet.py:432-433
    ch = x.shape[1]
    g = gn_groups(ch)
    z1 = _conv(P, f"{k}.block.0", x)
    a1 = F.leaky_relu(F.group_norm(z1, g, P[f"{k}.block.1.weight"], P[f"{k}.block.1.bias"]), 0.2)
    z2 = _conv(P, f"{k}.block.3", a1)
    if tr is not None:
        tr += [(f"{k}:z1", z1), (f"{k}:a1", a1), (f"{k}:z2", z2)]
    out = x + F.group_norm(z2, g, P[f"{k}.block.4.weight"], P[f"{k}.block.4.bias"])
    if tr is not None and tr.__class__ is _Trace:
        tr.res[k] = dict(r=x, z1=z1, a1=a1, z2=z2, out=out)
    return out


class _Trace(list):
    """trace list that also keeps each ResBlock's tensors (for gradient diagnostics)"""

    def __init__(self):
        super().__init__()
        self.res = {}
        self.lvl_in = {}


def new_trace():
    return _Trace()


def forward(flat: torch.Tensor, x: torch.Tensor, in_nc: int, out_nc: int, nf: int = 48,
            trace: list | None = None):
    """arch_unet.py:518-531.  `trace` (optional list) receives (name, NCHW tensor) of the
    intermediate activations in the order of dn_iunet_debug_buffers (x0 h | down levels: F r z1
    a1 z2 | bottle | up blocks: cc F r z1 a1 z2 | xb cf)."""
    P = unflatten(flat, in_nc, out_nc, nf)
    tr = trace
    hid = F.leaky_relu(_conv(P, "noise_estimator.0", x), 0.2)
    sigma = torch.sigmoid(_conv(P, "noise_estimator.2", hid))
    h = torch.cat([x, sigma], 1)
    if tr is not None:
        tr += [("x0", h), ("h", hid)]
    orig = h[:, :in_nc]
    skips = []
    for i in range(4):
        if tr is not None and tr.__class__ is _Trace:
            tr.lvl_in[i] = h
        h = F.leaky_relu(_conv(P, f"downs.{i}.0", h), 0.2)
        h = _res(P, f"downs.{i}.3", _rdb(P, f"downs.{i}.2", h, tr), tr)
        skips.append(h)
        h = F.max_pool2d(h, 2)
    h = _res(P, "bottle.1", _rdb(P, "bottle.0", h, tr), tr)
    xb = h
    for k, skip in zip(range(4), reversed(skips)):
        u = F.pixel_shuffle(_conv(P, f"ups.{k}.conv_ps", h), 2)
        cc = torch.cat([u, skip], 1)
        if tr is not None:
            tr.append((f"ups.{k}:cc", cc))
        h = F.leaky_relu(_conv(P, f"ups.{k}.fuse", cc), 0.2)
        h = _res(P, f"ups.{k}.res", _rdb(P, f"ups.{k}.rdb", h, tr), tr)
    cf = torch.cat([h, orig], 1)
    if tr is not None:
        tr += [("xb", xb), ("cf", cf)]
    return torch.sigmoid(_conv(P, "final", cf))
