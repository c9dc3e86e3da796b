"""CPU oracle of the multiresolution hash-grid encoding (config C5) — TEST INFRASTRUCTURE ONLY.

Restates `INGPTable` / `INGPEncoding` of the reference's 3d-ingp/model.py:14-121 (hash 44-56,
trilinear interpolation 58-90, levels and the x/8 + 0.5 normalisation 92-121) from SURVEY.md
§8(a) row a9; the builder's read of that file was refused in round 1, so this
restatement follows the survey's description.  The arithmetic the reference's 2-D copy of the
same module shares with it (2d-ingp/model.py:13-115: the fp32 resolution schedule, bijective
indexing, the int64 product-xor hash with primes 1 and 2654435761 and torch.remainder, multilinear
weights on the unclipped corners) is pinned by tests/golden/hashgrid2d.npz, generated from that
file; the 3-D specifics (third prime 805459861, x/8 + 0.5, the clip of bijective corners) remain
as the survey states them, unpinned.  numpy int64 for the integer index arithmetic (the reference hashes in int64
with Python-style `remainder`), fp32 for the interpolation, corners summed in a fixed order
(k = dx + 2 dy + 4 dz) with separate multiplies and adds.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
from __future__ import annotations

import math

import numpy as np

PRIMES = (1, 2654435761, 805459861)


def resolutions(levels: int = 16, n_min: int = 16, n_max: int = 1600) -> list[int]:
    """r_l = floor(n_min * b^l), b = exp((ln n_max - ln n_min) / (levels - 1)) (model.py:92-110)."""
    if levels == 1:
        return [n_min]
    b = math.exp((math.log(n_max) - math.log(n_min)) / (levels - 1))
    return [int(math.floor(n_min * b ** l)) for l in range(levels)]


def corner_index(c: np.ndarray, r: int, table_size: int) -> np.ndarray:
    """Table row of integer corners c [..., 3] (int64) at resolution r (model.py:44-56):
    bijective (r + 1)^3 <= T: clip to [0, r], x + (r+1) y + (r+1)^2 z; otherwise the product-xor
    hash with primes (1, 2654435761, 805459861) in int64, Python-style (non-negative) remainder."""
    c = c.astype(np.int64)
    if (r + 1) ** 3 <= table_size:
        cc = np.clip(c, 0, r)
        return cc[..., 0] + (r + 1) * cc[..., 1] + (r + 1) * (r + 1) * cc[..., 2]
    h = (c[..., 0] * PRIMES[0]) ^ (c[..., 1] * PRIMES[1]) ^ (c[..., 2] * PRIMES[2])
    return np.mod(h, table_size)


def corner_index_2d(c: np.ndarray, r: int, table_size: int) -> np.ndarray:
    """The reference's 2-D statement of the same indexing (2d-ingp/model.py:22,33-50): bijective
    when (r + 1)^2 <= T, x + (r+1) y (no clip there: the 2-D inputs stay in [0, r]); otherwise
    (x * 1) ^ (y * 2654435761) in int64 with torch.remainder (non-negative)."""
    c = c.astype(np.int64)
    if (r + 1) ** 2 <= table_size:
        return c[..., 0] + (r + 1) * c[..., 1]
    return np.mod((c[..., 0] * PRIMES[0]) ^ (c[..., 1] * PRIMES[1]), table_size)


def level_corners_2d(u: np.ndarray, r: int, table_size: int):
    """(indices [N, 4], weights [N, 4]) of 2d-ingp/model.py:52-81 for points u [N, 2] in [0, 1):
    x_hat = u * r, corners (x_i, y_j) in the order (0,0), (0,1), (1,0), (1,1), weights
    prod_d (1 - |x_hat_d - corner_d|)."""
    xh = u.astype(np.float32) * np.float32(r)
    base = np.floor(xh).astype(np.int64)
    idx = np.empty((u.shape[0], 4), dtype=np.int64)
    w = np.empty((u.shape[0], 4), dtype=np.float32)
    for k, (i, j) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        c = base + np.array([i, j], dtype=np.int64)
        idx[:, k] = corner_index_2d(c, r, table_size)
        d = np.float32(1.0) - np.abs(xh - c.astype(np.float32))
        w[:, k] = d[:, 0] * d[:, 1]
    return idx, w


def encode_2d(u: np.ndarray, tables: list[np.ndarray], res: list[int], table_size: int) -> np.ndarray:
    """2d-ingp INGPEncoding.forward (model.py:109-115): per level sum_k w_k * table[idx_k] in the
    corner order above, levels concatenated."""
    outs = []
    for t, r in zip(tables, res):
        idx, w = level_corners_2d(u, r, table_size)
        acc = np.zeros((u.shape[0], t.shape[1]), dtype=np.float32)
        for k in range(4):
            acc = acc + t[idx[:, k]] * w[:, k:k + 1]
        outs.append(acc)
    return np.concatenate(outs, axis=1)


def scaled(x: np.ndarray, r: int) -> np.ndarray:
    """x_hat = (x / 8 + 0.5) * r in fp32 (model.py:111-121)."""
    x = x.astype(np.float32)
    return (x / np.float32(8.0) + np.float32(0.5)) * np.float32(r)


def level_corners(x: np.ndarray, r: int, table_size: int):
    """(indices [N, 8] int64, weights [N, 8] fp32) of the 8 corners k = dx + 2 dy + 4 dz; weights
    prod_d (1 - |x_hat_d - corner_d|) on the unclipped corner (model.py:58-90)."""
    xh = scaled(x, r)
    base = np.floor(xh).astype(np.int64)
    idx = np.empty((x.shape[0], 8), dtype=np.int64)
    w = np.empty((x.shape[0], 8), dtype=np.float32)
    for k in range(8):
        off = np.array([k & 1, (k >> 1) & 1, (k >> 2) & 1], dtype=np.int64)
        c = base + off
        idx[:, k] = corner_index(c, r, table_size)
        d = np.float32(1.0) - np.abs(xh - c.astype(np.float32))
        w[:, k] = (d[:, 0] * d[:, 1]) * d[:, 2]
    return idx, w


def encode(x: np.ndarray, table: np.ndarray, res: list[int]) -> np.ndarray:
    """Hash-grid features [N, L * F] (level-major) of positions x [N, 3] with table [L, T, F]."""
    L, T, F = table.shape
    out = np.zeros((x.shape[0], L * F), dtype=np.float32)
    for l in range(L):
        idx, w = level_corners(x, res[l], T)
        acc = np.zeros((x.shape[0], F), dtype=np.float32)
        for k in range(8):
            acc = acc + w[:, k:k + 1] * table[l][idx[:, k]]
        out[:, l * F:(l + 1) * F] = acc
    return out


def encode_backward(x: np.ndarray, grad_out: np.ndarray, table_shape, res: list[int]) -> np.ndarray:
    """Gradient of sum(encode(x) * grad_out) w.r.t. the table [L, T, F], accumulated in fp64."""
    L, T, F = table_shape
    g = np.zeros((L, T, F), dtype=np.float64)
    for l in range(L):
        idx, w = level_corners(x, res[l], T)
        for k in range(8):
            np.add.at(g[l], idx[:, k], w[:, k:k + 1].astype(np.float64) * grad_out[:, l * F:(l + 1) * F])
    return g
