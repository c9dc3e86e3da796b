"""CPU oracle of the multiresolution hash-grid encoding (config C5) — TEST INFRASTRUCTURE ONLY.

Restates `INGPTable` / `INGPEncoding` of the reference's 3d-ingp/model.py:14-121 (hash 44-56,
interpolation 58-90, levels and the x/8 + 0.5 normalisation 92-121).  The builder's read of that
file was refused in round 1 and is not attempted again; this restatement follows
SURVEY.md §8(a) row a9, the interface VERDICT r2 states (per-level tables of (r+1)^3 rows when
bijective and T rows otherwise, primes pi1..pi3, corners stacked (0,0,0), (0,0,1), (0,1,0), ... —
z fastest — and summed with th.sum over that axis) and the reference's readable 2-D statement of
the same module, 2d-ingp/model.py:13-115, whose arithmetic tests/golden/hashgrid2d.npz pins (the
fp32 resolution schedule, bijective indexing, the int64 product-xor hash with torch.remainder,
multilinear weights on the unclipped corners, the corner stacking order and the sequential sum
over it).  3-D specifics that stay unpinned: the third prime's role, x/8 + 0.5, the clip of
bijective corners.

numpy int64 for the integer index arithmetic (the reference hashes in int64 with Python-style
`remainder`), fp32 for the interpolation: each corner's weight prod_d (1 - |x_hat_d - c_d|) as
((w_x * w_y) * w_z), its product with the table row rounded, then the corners added in stacking
order.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
from __future__ import annotations

import math

import numpy as np

PRIMES = (1, 2654435761, 805459861)

# the reference's stacking order (3d-ingp/model.py:70-76 as VERDICT r2 states it; 2-D:
# 2d-ingp/model.py:65): (i, j, k) over x, y, z with z fastest
CORNERS_3D = tuple((i, j, k) for i in (0, 1) for j in (0, 1) for k in (0, 1))
CORNERS_2D = ((0, 0), (0, 1), (1, 0), (1, 1))


def resolutions(levels: int = 16, n_min: int = 16, n_max: int = 1600) -> list[int]:
    """r_l = floor(n_min * b^l), b = exp((ln n_max - ln n_min) / (levels - 1)) — the reference forms
    it as th.floor(resolution_min * b ** th.arange(n_levels)) in fp32 (2d-ingp/model.py:101-103);
    both agree on every schedule the tests use (tests/test_hashgrid.py)."""
    if levels == 1:
        return [n_min]
    b = math.exp((math.log(n_max) - math.log(n_min)) / (levels - 1))
    return [int(math.floor(n_min * b ** l)) for l in range(levels)]


def level_rows(r: int, table_size: int) -> int:
    """Rows of one level's table: (r + 1)^3 when bijective, else table_size."""
    return (r + 1) ** 3 if (r + 1) ** 3 <= table_size else table_size


def init_tables(res: list[int], table_size: int, n_features: int, seed: int = 0) -> list[np.ndarray]:
    """Random per-level tables of the reference's shapes (values in [-1e-4, 1e-4) by default scale)."""
    rng = np.random.default_rng(seed)
    return [((rng.random((level_rows(r, table_size), n_features)) * 2 - 1) * 1e-4).astype(np.float32)
            for r in res]


def hash3(c: np.ndarray, table_size: int, primes=PRIMES) -> np.ndarray:
    """(x*pi1) ^ (y*pi2) ^ (z*pi3) in int64 with wrapping products, non-negative remainder."""
    c = c.astype(np.int64)
    with np.errstate(over="ignore"):
        h = (c[..., 0] * np.int64(primes[0])) ^ (c[..., 1] * np.int64(primes[1])) ^ (c[..., 2] * np.int64(primes[2]))
    return np.mod(h, table_size)


def corner_index(c: np.ndarray, r: int, table_size: int, primes=PRIMES) -> np.ndarray:
    """Table row of integer corners c [..., 3] (int64) at resolution r: bijective (r + 1)^3 <= T:
    clip to [0, r], x + (r+1) y + (r+1)^2 z; otherwise the product-xor hash."""
    c = c.astype(np.int64)
    if (r + 1) ** 3 <= table_size:
        cc = np.clip(c, 0, r)
        return cc[..., 0] + (r + 1) * cc[..., 1] + (r + 1) * (r + 1) * cc[..., 2]
    return hash3(c, table_size, primes)


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
    for k, (i, j) in enumerate(CORNERS_2D):
        c = base + np.array([i, j], dtype=np.int64)
        idx[:, k] = corner_index_2d(c, r, table_size)
        d = np.float32(1.0) - np.abs(xh - c.astype(np.float32))
        w[:, k] = d[:, 0] * d[:, 1]
    return idx, w


def encode_2d(u: np.ndarray, tables: list[np.ndarray], res: list[int], table_size: int) -> np.ndarray:
    """2d-ingp INGPEncoding.forward (model.py:109-115): per level sum_k w_k * table[idx_k] in the
    corner order above (products rounded, then added in order), levels concatenated."""
    outs = []
    for t, r in zip(tables, res):
        idx, w = level_corners_2d(u, r, table_size)
        acc = np.zeros((u.shape[0], t.shape[1]), dtype=np.float32)
        for k in range(4):
            acc = acc + t[idx[:, k]] * w[:, k:k + 1]
        outs.append(acc)
    return np.concatenate(outs, axis=1)


def normalised(x: np.ndarray) -> np.ndarray:
    """INGPEncoding.forward's x / 8 + 0.5 in fp32."""
    x = x.astype(np.float32)
    return x / np.float32(8.0) + np.float32(0.5)


def level_corners(x: np.ndarray, r: int, table_size: int, primes=PRIMES, normalize: bool = True):
    """(indices [N, 8] int64, weights [N, 8] fp32) of the 8 corners in stacking order (z fastest);
    weights prod_d (1 - |x_hat_d - corner_d|) on the unclipped corner."""
    u = normalised(x) if normalize else x.astype(np.float32)
    xh = u * np.float32(r)
    base = np.floor(xh).astype(np.int64)
    idx = np.empty((x.shape[0], 8), dtype=np.int64)
    w = np.empty((x.shape[0], 8), dtype=np.float32)
    for k, off in enumerate(CORNERS_3D):
        c = base + np.array(off, dtype=np.int64)
        idx[:, k] = corner_index(c, r, table_size, primes)
        d = np.float32(1.0) - np.abs(xh - c.astype(np.float32))
        w[:, k] = (d[:, 0] * d[:, 1]) * d[:, 2]
    return idx, w


def encode(x: np.ndarray, tables: list[np.ndarray], res: list[int], table_size: int, primes=PRIMES,
           normalize: bool = True) -> np.ndarray:
    """Hash-grid features [N, L * F] (level-major) of positions x [N, 3] with per-level tables."""
    F = tables[0].shape[1]
    out = np.zeros((x.shape[0], len(res) * F), dtype=np.float32)
    for l, (t, r) in enumerate(zip(tables, res)):
        idx, w = level_corners(x, r, table_size, primes, normalize)
        acc = np.zeros((x.shape[0], F), dtype=np.float32)
        for k in range(8):
            acc = acc + t[idx[:, k]] * w[:, k:k + 1]
        out[:, l * F:(l + 1) * F] = acc
    return out


def encode_backward(x: np.ndarray, grad_out: np.ndarray, res: list[int], table_size: int, n_features: int,
                    primes=PRIMES, normalize: bool = True) -> list[np.ndarray]:
    """Gradient of sum(encode(x) * grad_out) w.r.t. each level's table, accumulated in fp64."""
    F = n_features
    grads = []
    for l, r in enumerate(res):
        g = np.zeros((level_rows(r, table_size), F), dtype=np.float64)
        idx, w = level_corners(x, r, table_size, primes, normalize)
        for k in range(8):
            np.add.at(g, idx[:, k], w[:, k:k + 1].astype(np.float64) * grad_out[:, l * F:(l + 1) * F])
        grads.append(g)
    return grads


def encode_position_grad(x: np.ndarray, tables: list[np.ndarray], res: list[int], table_size: int,
                         grad_out: np.ndarray, primes=PRIMES, normalize: bool = True) -> np.ndarray:
    """d sum(encode(x) * grad_out) / dx [N, 3] in float64: per level, torch autograd w.r.t. x_hat at
    the fp32 x_hat the forward evaluates ((x / 8 + 0.5) r, or x r), through weights
    prod_d (1 - |x_hat_d - c_d|) on the unclipped corner (corners floor(x_hat) + offsets and the
    rows of level_corners are constants; abs backward sign(0) = 0), then dx_hat/dx = r / 8 (or r).
    The reference computes this gradient with autograd through its fp32 ops (3d-ingp/model.py:58-121
    as SURVEY §8(a) a9 restates it) — parity unpinned, as the 3-D hash grid itself."""
    import torch
    F = tables[0].shape[1]
    gx = np.zeros((x.shape[0], 3), dtype=np.float64)
    for l, (t, r) in enumerate(zip(tables, res)):
        idx, _ = level_corners(x, r, table_size, primes, normalize)
        u32 = normalised(x) if normalize else x.astype(np.float32)
        xh32 = u32 * np.float32(r)
        xh = torch.tensor(xh32.astype(np.float64), requires_grad=True)
        base = torch.floor(torch.tensor(xh32.astype(np.float64)))
        g = torch.tensor(grad_out[:, l * F:(l + 1) * F].astype(np.float64))
        tt = torch.tensor(t.astype(np.float64))
        total = torch.zeros((), dtype=torch.float64)
        for k, off in enumerate(CORNERS_3D):
            c = base + torch.tensor(off, dtype=torch.float64)
            d = 1.0 - torch.abs(xh - c)
            w = (d[:, 0] * d[:, 1]) * d[:, 2]
            total = total + (w.unsqueeze(1) * tt[torch.from_numpy(idx[:, k])] * g).sum()
        total.backward()
        gx += xh.grad.numpy() * (r / 8.0 if normalize else float(r))
    return gx


def pack(tables: list[np.ndarray]) -> np.ndarray:
    """The kernels' packed layout: the levels' tables back to back, [sum rows, F]."""
    return np.concatenate(tables, axis=0)
