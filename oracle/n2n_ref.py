"""N2N sampler / losses restated on the CPU (test oracle; see oracle/__init__.py)."""
from __future__ import annotations

import numpy as np
import torch

# train.py:151-154
PAIRS = np.array([[0, 1], [0, 2], [1, 3], [2, 3], [1, 0], [2, 0], [3, 1], [3, 2]], dtype=np.int64)


def space_to_depth(x: np.ndarray, block: int = 2) -> np.ndarray:
    """train.py:134-138: unfold(k=b, s=b).view(n, c*b*b, h/b, w/b); channel = c*b*b + dy*b + dx"""
    n, c, h, w = x.shape
    y = x.reshape(n, c, h // block, block, w // block, block)
    y = y.transpose(0, 1, 3, 5, 2, 4)  # n, c, dy, dx, i, j
    return y.reshape(n, c * block * block, h // block, w // block)


def masks_from_rd(rd_idx: np.ndarray):
    """train.py:163-171: mask[4*cell + pair[rd][0|1]] = True"""
    rd = np.asarray(rd_idx, dtype=np.int64).reshape(-1)
    cells = rd.size
    pair = PAIRS[rd] + (np.arange(cells, dtype=np.int64) * 4)[:, None]
    m1 = np.zeros(cells * 4, dtype=bool)
    m2 = np.zeros(cells * 4, dtype=bool)
    m1[pair[:, 0]] = True
    m2[pair[:, 1]] = True
    return m1, m2


def generate_subimages(img: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """train.py:175-190, literal: per channel space_to_depth -> permute(0,2,3,1) -> [mask]"""
    n, c, h, w = img.shape
    sub = np.zeros((n, c, h // 2, w // 2), dtype=img.dtype)
    for i in range(c):
        s2d = space_to_depth(img[:, i:i + 1], 2).transpose(0, 2, 3, 1).reshape(-1)
        sub[:, i:i + 1] = s2d[mask].reshape(n, h // 2, w // 2, 1).transpose(0, 3, 1, 2)
    return sub


def subimages_closed_form(img: np.ndarray, rd_idx: np.ndarray):
    """sub[n,c,i,j] = img[n,c,2i+(k>>1),2j+(k&1)], k = pair[rd][0] (sub1) / [1] (sub2)"""
    n, c, h, w = img.shape
    rd = np.asarray(rd_idx, dtype=np.int64).reshape(n, h // 2, w // 2)
    out = []
    for col in (0, 1):
        k = PAIRS[rd][..., col]
        ii = 2 * np.arange(h // 2)[None, :, None] + (k >> 1)
        jj = 2 * np.arange(w // 2)[None, None, :] + (k & 1)
        nn_ = np.arange(n)[:, None, None]
        out.append(np.stack([img[nn_, ch, ii, jj] for ch in range(c)], axis=1))
    return out[0], out[1]


def n2n_loss(out, sub2, den, rd_idx, lam):
    """training_script.md:141-153 in torch fp32 on the CPU; returns (loss1, loss2, loss, dout)."""
    out = torch.as_tensor(out).float().clone().requires_grad_(True)
    sub2 = torch.as_tensor(sub2).float()
    den = np.asarray(den, dtype=np.float32)
    m1, m2 = masks_from_rd(rd_idx)
    d1 = torch.from_numpy(generate_subimages(den, m1))
    d2 = torch.from_numpy(generate_subimages(den, m2))
    diff = out - sub2
    exp_diff = d1 - d2
    loss1 = torch.mean(diff ** 2)
    loss2 = lam * torch.mean((diff - exp_diff) ** 2)
    loss = loss1 + loss2
    loss.backward()
    return float(loss1), float(loss2), float(loss), out.grad.numpy()


def structure_loss(pred, pred2, target, alpha=1.0, beta=0.5, gamma=0.5):
    """util.py:56-70 in torch fp32 on the CPU; returns (loss, dpred, dpred2, parts)."""
    l1 = torch.nn.L1Loss()
    p = torch.as_tensor(pred).float().clone().requires_grad_(True)
    p2 = torch.as_tensor(pred2).float().clone().requires_grad_(True)
    t = torch.as_tensor(target).float()
    pixel = l1(p, t)
    tv1 = l1(p2[:, :, 1:, :], p2[:, :, :-1, :])
    tv2 = l1(p2[:, :, :, 1:], p2[:, :, :, :-1])
    tv = (tv1 + tv2) / 2
    cst = l1(p2, t)
    loss = alpha * pixel + beta * tv + gamma * cst
    loss.backward()
    parts = [float(pixel), float(tv1), float(tv2), float(cst), float(loss)]
    return float(loss), p.grad.numpy(), p2.grad.numpy(), parts
