"""Philox4x32-10 in numpy — restatement of image_denoising_amd/csrc/philox.h (test oracle)."""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32) for v in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def _blocks(seed, offset, q):
    q = np.asarray(q, dtype=np.uint64)
    blk = q >> np.uint64(2)
    return philox4x32_10((blk & _MASK).astype(np.uint32), (blk >> np.uint64(32)).astype(np.uint32),
                         np.full(q.shape, offset & 0xFFFFFFFF, np.uint32),
                         np.full(q.shape, (offset >> 32) & 0xFFFFFFFF, np.uint32),
                         seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def cell_u32(seed: int, offset: int, q) -> np.ndarray:
    """word q&3 of Philox block q>>2 (philox_cell_u32)"""
    q = np.asarray(q, dtype=np.uint64)
    o = np.stack(_blocks(seed, offset, q))
    return o[(q & np.uint64(3)).astype(np.int64), np.arange(q.size).reshape(q.shape)]


def rd_idx(seed: int, offset: int, ncells: int, cell_base: int = 0) -> np.ndarray:
    q = np.arange(cell_base, cell_base + ncells, dtype=np.uint64)
    return (cell_u32(seed, offset, q) & np.uint32(7)).astype(np.uint8)


def normal(seed: int, offset: int, q) -> np.ndarray:
    """Box-Muller normals (philox_normal), evaluated in float64"""
    q = np.asarray(q, dtype=np.uint64)
    o = np.stack(_blocks(seed, offset, q))
    p = ((q >> np.uint64(1)) & np.uint64(1)).astype(np.int64)
    idx = np.arange(q.size).reshape(q.shape)
    a, b = o[2 * p, idx], o[2 * p + 1, idx]
    u1 = ((a >> np.uint32(8)).astype(np.float64) + 1.0) / 16777216.0
    u2 = (b >> np.uint32(8)).astype(np.float64) / 16777216.0
    r = np.sqrt(-2.0 * np.log(u1))
    th = 2.0 * np.pi * u2
    return np.where((q & np.uint64(1)) == 1, r * np.sin(th), r * np.cos(th))


def uniform53(seed: int, offset: int, q) -> np.ndarray:
    """53-bit uniform in (0, 1) for element q (philox_uniform53): words (2p, 2p+1), p = q & 1,
    of Philox block q >> 1"""
    q = np.asarray(q, dtype=np.uint64)
    shape = q.shape
    q = q.reshape(-1)
    blk = q >> np.uint64(1)
    o = np.stack(philox4x32_10((blk & _MASK).astype(np.uint32),
                               (blk >> np.uint64(32)).astype(np.uint32),
                               np.full(q.shape, offset & 0xFFFFFFFF, np.uint32),
                               np.full(q.shape, (offset >> 32) & 0xFFFFFFFF, np.uint32),
                               seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    p = (q & np.uint64(1)).astype(np.int64)
    idx = np.arange(q.size).reshape(q.shape)
    a = (o[2 * p, idx] >> np.uint32(5)).astype(np.float64)
    b = (o[2 * p + 1, idx] >> np.uint32(6)).astype(np.float64)
    return ((a * 67108864.0 + b + 0.5) / 9007199254740992.0).reshape(shape)


def poisson_counts(mu: np.ndarray, u: np.ndarray) -> np.ndarray:
    """k = min{k : u <= F(k)} for Poisson(mu), F accumulated in fp64 from exp(-mu) as k_poisson
    does (the loop bound mu + 20 sqrt(mu) + 40 included): the sampler behind train.py:102-111's
    torch.poisson, restated for the Philox stream"""
    mu = np.maximum(np.asarray(mu, dtype=np.float64), 0.0)
    u = np.asarray(u, dtype=np.float64)
    p = np.exp(-mu)
    F = p.copy()
    k = np.zeros(mu.shape, dtype=np.int64)
    kmax = (mu + 20.0 * np.sqrt(mu)).astype(np.int64) + 40
    live = (u > F) & (k < kmax)
    while live.any():
        k = np.where(live, k + 1, k)
        p = np.where(live, p * (mu / np.maximum(k, 1)), p)
        F = np.where(live, F + p, F)
        live = live & (u > F) & (k < kmax)
    return k


def poisson_noise(clean: np.ndarray, lam, seed: int, offset: int, elem_base: int = 0) -> np.ndarray:
    """dn_add_poisson_noise: Poisson(lam * clean) / lam in fp32 (lam scalar or per image)"""
    clean = np.asarray(clean, dtype=np.float32)
    lam_e = np.broadcast_to(np.asarray(lam, dtype=np.float32).reshape(-1, *([1] * (clean.ndim - 1))),
                            clean.shape) if np.ndim(lam) else np.float32(lam)
    mu = (lam_e * clean).astype(np.float32)
    q = np.arange(elem_base, elem_base + clean.size, dtype=np.uint64).reshape(clean.shape)
    k = poisson_counts(mu.astype(np.float64), uniform53(seed, offset, q))
    return (k.astype(np.float32) / lam_e).astype(np.float32)
