"""Execution plan + autograd for NeRF field MLPs on the fp32 MFMA linear kernels.

A field MLP (NerfModel, NerfModelINGP, ...) is lowered once into a list of
``LayerPlan``s.  Each layer reads a column-concatenation of *sources* —
the padded position encoding ("pos"), the (per-sample or per-ray) direction
encoding ("dir") or an earlier layer's output ("act", j) — so the reference's
``th.cat`` copies (model_interpolation_architecture.py:111-125) never exist.
Weights are repacked into the kernels' K-padded layout (forward) and its transpose
(input-gradient GEMMs) on every call that uses them: one small gather launch per layer, never
keyed on the parameter's version counter (``p.data`` updates and fused optimizers do not bump
it, and a stale pack would silently train on old weights).

``MLPFunction`` is one autograd node for the whole network:
  forward : one ``nerf_linear_fwd`` launch per layer (bias + ReLU fused), all
            layer outputs kept for backward;
  backward: per layer (in reverse) one ``nerf_linear_wgrad`` + reduce for
            (dW, db) and one ``nerf_linear_fwd`` per consumed source for dX,
            with the ReLU mask of the producing layer fused into its epilogue (read
            as the bit mask the forward epilogue wrote, 1 bit per activation).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn

from . import kernels as K
from . import mlp_fused
from ._lib import (NERF_EPI_ACCUM, NERF_EPI_BIAS, NERF_EPI_MASK, NERF_EPI_MASKBITS, NERF_EPI_MASKOUT,
                   NERF_EPI_RELU, NERF_EPI_TANH, NERF_EPI_TANH_BWD)


def matmul_precision() -> str:
    """"fp32" (exact fp32 MFMA), "x3" (3 x bf16 split MFMA, ~2^-17 per product) or "x1" (one bf16
    pass, bf16(w) * bf16(x) with fp32 accumulation, 2^-8 per product).

    Follows torch.get_float32_matmul_precision(), the knob the reference itself sets
    (barf/run_barf.py:101 "high", naive-to-vanilla/main.py:53 "medium"): "highest" -> exact fp32;
    "high" -> split precision, ~64x more accurate than the TF32 it selects on the reference's
    hardware; "medium" -> single-pass bf16, the class of the single-pass bf16 / fp16 products the
    reference's C2 run computes (main.py:53,58: "medium" under precision="16-mixed").  The fused
    field-MLP kernels and the weight gradients run "x1" in one pass; the layer-by-layer GEMMs
    (Gaussian / tanh layers, fields the fused kernel does not take) keep the 3-pass split there."""
    if PRECISION_OVERRIDE is not None:
        return PRECISION_OVERRIDE
    p = torch.get_float32_matmul_precision()
    return "fp32" if p == "highest" else ("x1" if p == "medium" else "x3")


def is_split(prec: str) -> bool:
    """The bf16 split-precision kernels (either pass count) rather than the fp32 MFMA ones."""
    return prec in ("x3", "x1")


def passes(prec: str) -> int:
    return 1 if prec == "x1" else 3


PRECISION_OVERRIDE: str | None = None

# the 257-row (density + feature) layer's split-precision weight gradient as one 256 x 256 tile + a
# vector-ALU row (NERF_WGRAD_257=0: the 128-tile kernel over the row count padded to 260)
WGRAD_ROW257 = os.environ.get("NERF_WGRAD_257", "1") != "0"

# With a direct gradient sink, the split-precision weight gradient of a field used twice per step
# (coarse and fine passes of one NerfModel) runs once over both passes' rows: the first backward
# stashes each layer's (dY, X) in the sink, the second sums both blocks in one launch and one
# reduce (nerf_linear_wgrad_x3_rows; NERF_MERGE_PASSES=0: one launch per pass and an accumulating
# reduce).  The result differs from the per-pass sum only in fp32 summation order.
MERGE_PASSES = os.environ.get("NERF_MERGE_PASSES", "1") != "0"

# Alpha compositing fused into the field MLP's launches (nerf_mlp_fused_render): the forward
# composites each tile's rays at the tile end and the input-gradient chain takes the compositing's
# gradient from per-sample coefficients (NERF_FUSE_COMPOSITE=0: nerf_composite_fwd/bwd launches).
FUSE_COMPOSITE = os.environ.get("NERF_FUSE_COMPOSITE", "1") != "0"


class CompositeSpec:
    """The renderer's compositing of one field pass (barf/model_interpolation.py:316-353 with the
    NerfModel head activations), run inside the field MLP's launches: interval lengths [M], samples
    per ray, density factor and shift.  The forward stores its per-sample backward coefficients in
    ``coef`` ([M, 8], include/nerf_amd.h nerf_fused_composite)."""

    __slots__ = ("dist", "S", "sa", "sb", "shift", "coef")

    def __init__(self, dist: torch.Tensor, S: int, sa: float, sb: float, shift: float = 0.0):
        self.dist, self.S, self.sa, self.sb, self.shift = dist, int(S), float(sa), float(sb), float(shift)
        self.coef = None


def composite_sigma_layer(plan) -> int:
    """The layer whose column output is the raw density, or -1 (row 3 of the head layer)."""
    return plan.column_outputs[0][0] if plan.column_outputs else -1


def composite_eligible(plan, M: int, S: int) -> bool:
    """The fused forward runs this plan and its last layer can hand its heads to the compositing."""
    if not FUSE_COMPOSITE or not is_split(matmul_precision()) or not mlp_fused.eligible(plan, M):
        return False
    # whole rays per 128-sample tile, or rays of 256 samples over two tiles run back to back
    if not ((16 <= S <= 128 and 128 % S == 0) or S == 256) or M % S or M * 32 >= (1 << 31):
        return False
    L = len(plan.layers)
    if len(plan.column_outputs) > 1 or (plan.column_outputs and plan.column_outputs[0][0] == L - 1):
        return False
    kbr, _ = mlp_fused._layer_shape(plan, L - 1)
    N = plan.layers[L - 1].module.out_features
    return kbr > 0 and (4 if composite_sigma_layer(plan) < 0 else 3) <= N <= 16


def composite_grads_torch(comp: CompositeSpec, g_rgb: torch.Tensor, sigma_col: bool):
    """The compositing's gradient rows from its coefficients where the fused chain cannot take them:
    d head [M, 3] (+ d sigma-raw [M]) = coef * grad_rgb of the sample's ray."""
    gr = g_rgb.repeat_interleave(comp.S, dim=0)
    gh = comp.coef[:, 0:3] * gr
    gs = (comp.coef[:, 4:7] * gr).sum(dim=1)
    return gh, gs


def _wgrad_workspace(ws: torch.Tensor, M: int, N4: int, Kp: int) -> torch.Tensor:
    need = K.linear_wgrad_workspace_bytes(M, N4, Kp)
    if ws.numel() * ws.element_size() >= need:
        return ws
    return torch.empty((need + 3) // 4, device=ws.device, dtype=torch.float32)


# The weight gradient of a layer whose last input is per ray (NerfModel's colour layer reads the
# direction encoding once per ray: row divisor S) as the streamed single-tile kernel over its other
# inputs, which also sums dY over each ray's samples, then the per-ray input's part over the B rays:
# sum_m dY[m] x[ray(m)] = sum_ray (sum_{m in ray} dY[m]) x[ray] (nerf_linear_wgrad_x3_rays;
# NERF_WGRAD_RAYS=0: the 128-tile kernel over every sample's row, as before)
WGRAD_RAYS = os.environ.get("NERF_WGRAD_RAYS", "1") != "0"


def _ray_split(blocks, N4: int):
    """(main segments per block, ray segment per block) when the layer's weight gradient can take
    its last, per-ray input from per-ray dY sums; None otherwise."""
    if not WGRAD_RAYS or N4 > 256:
        return None
    mains, rays = [], []
    for dZ, segs, M in blocks:
        if len(segs) < 2 or M == 0:
            return None
        t, k, S = segs[-1]
        # rays of S | 128 samples, or of a multiple of 128 (nerf_linear_wgrad_x3_rays: no split cuts a ray)
        if not (16 <= S <= 4096 and (128 % S == 0 or S % 128 == 0) and M % S == 0) \
                or any(rd != 1 for _, _, rd in segs[:-1]):
            return None
        mains.append(segs[:-1])
        rays.append((t, k, S))
    kmain = sum(K.pad32(k) for _, k, _ in mains[0])
    if kmain > 256 or not (N4 > 128 or kmain > 128) or blocks[0][2] % 128:
        return None
    if len(blocks) > 1 and blocks[0][2] % math.lcm(128, *(S for _, _, S in rays)):
        return None                                     # block 1 would start inside a split's ray
    return mains, rays


def _wgrad_rays(blocks, N4: int, lp, workspace, gW, gb, acc, split, npass: int = 3) -> None:
    """The weight gradient of `blocks` (one or two passes' rows) through the per-ray route (_ray_split)."""
    mains, rays = split
    Mt = sum(M for _, _, M in blocks)
    kmain = sum(K.pad32(k) for _, k, _ in mains[0])
    dev = blocks[0][0].device
    Bs = [M // r[2] for (_, _, M), r in zip(blocks, rays)]
    raysum = torch.empty(sum(Bs), N4, device=dev, dtype=torch.float32)
    b0 = (blocks[0][0], mains[0], blocks[0][2])
    b1 = (blocks[1][0], mains[1], blocks[1][2]) if len(blocks) > 1 else (blocks[0][0], mains[0], 0)
    ws = _wgrad_workspace(workspace, Mt, N4, kmain)
    K.linear_wgrad_x3_rays([b0, b1], N4, ws, raysum, rays[0][2], rays[1][2] if len(blocks) > 1 else 0, passes=npass)
    K.linear_wgrad_reduce(Mt, N4, kmain, lp.N, ws, lp.col_map[:kmain], gW, gb, accumulate=acc)
    kray = K.pad32(rays[0][1])
    Bt = sum(Bs)
    ws2 = _wgrad_workspace(workspace, Bt, N4, kray)
    r0 = (raysum[:Bs[0]], [(rays[0][0], rays[0][1], 1)], Bs[0])
    if len(blocks) > 1:
        K.linear_wgrad_x3_rows([r0, (raysum[Bs[0]:], [(rays[1][0], rays[1][1], 1)], Bs[1])], N4, ws2, passes=npass)
    else:
        K.linear_wgrad_x3(r0[0], N4, r0[1], Bs[0], ws2, passes=npass)
    K.linear_wgrad_reduce(Bt, N4, kray, lp.N, ws2, lp.col_map[kmain:kmain + kray], gW, None, accumulate=acc)


# The weight gradient of a layer larger than the single-tile kernel's 256 (257) rows x 256 padded
# columns — mip-NeRF's skip layer [trunk activation 256 | encoding 96] (barf/model_mip.py:85-130
# through NerfModel's skip connections), GARF's Linear(1024, 256), Linear(512, 256) and
# Linear(131, 512) (garf/model_radiance.py, model_proposal.py) — as single-tile launches over row
# blocks of <= 256 output rows (views of dY and of the gradient) and column groups of <= 256 padded
# input columns (whole segments, or 256-column slices of a wider one), one reduce per tile into its
# rows and columns, instead of the 128 x 128-tile kernel that re-reads dY per 128-column block
# (profiles/r06k; NERF_WGRAD_TILESPLIT=0: the 128-tile kernel, as before).  Only when every tile
# can take the single-tile kernel (more than 128 rows or columns).
WGRAD_TILESPLIT = os.environ.get("NERF_WGRAD_TILESPLIT", "1") != "0"


def _tile_split(segs, nrow: int):
    """(row blocks [(n0, nb)], column groups [[(segment, c0, c1)]]) of the layer's weight gradient
    as single-tile launches (nrow: the row count the kernels take, 257 or the padded N), or None.
    The pieces of a group are consecutive in the packed layout: one col_map range per group."""
    if not WGRAD_TILESPLIT:
        return None
    kp = [K.pad32(k) for _, k, _ in segs]
    if nrow <= 257 and sum(kp) <= 256:
        return None                                        # one tile already
    rows = [(0, nrow)] if nrow <= 257 else [(n0, min(256, nrow - n0)) for n0 in range(0, nrow, 256)]
    groups, cur, used = [], [], 0
    for j, (_, k, rd) in enumerate(segs):
        if kp[j] > 256 and rd != 1:
            return None
        for c0 in range(0, k, 256):                        # 256-column slices of a wider segment
            c1 = min(c0 + 256, k)
            w = K.pad32(c1 - c0)
            if used + w > 256:
                groups.append(cur)
                cur, used = [], 0
            cur.append((j, c0, c1))
            used += w
    groups.append(cur)
    gk = [sum(K.pad32(c1 - c0) for _, c0, c1 in g) for g in groups]
    if len(rows) > 1 and min(gk) <= 128:
        # row blocks of a narrow input (GARF's Linear(3, 1024)): the 128-tile kernel streams dY
        # faster than single-tile launches whose X side is nearly empty (profiles/r06k)
        return None
    if any(not (nb > 128 or k > 128) for _, nb in rows for k in gk):
        return None                                        # a tile the single-tile kernel does not take
    return rows, groups


def _wgrad_tiles(blocks, nrow: int, N4: int, lp, workspace, gW, gb, acc, split, npass: int) -> None:
    """The weight gradient of `blocks` (one or two passes' rows) tile by tile (_tile_split)."""
    rows, groups = split
    Mt = sum(M for _, _, M in blocks)
    poff = [0]                                             # packed column offset of each segment
    for _, k, _ in blocks[0][1]:
        poff.append(poff[-1] + K.pad32(k))

    def piece(segs, j, c0, c1):
        t, k, rd = segs[j]
        return (t, k, rd) if (c0, c1) == (0, k) else (t[:, c0:c1], c1 - c0, rd)

    whole = len(rows) == 1
    for n0, nb in rows:
        nr = nrow if whole else nb                         # 257: the 256 x 256 tile + its 257th row
        n4 = N4 if whole else nb
        nvalid = lp.N if whole else min(nb, lp.N - n0)
        for gi, g in enumerate(groups):
            pb = [(dZ if whole else dZ[:, n0:n0 + nb], [piece(segs, j, c0, c1) for j, c0, c1 in g], M)
                  for dZ, segs, M in blocks]
            p0 = poff[g[0][0]] + g[0][1]
            kp = sum(K.pad32(c1 - c0) for _, c0, c1 in g)
            ws = _wgrad_workspace(workspace, Mt, n4, kp)
            if len(pb) > 1:
                K.linear_wgrad_x3_rows(pb, nr, ws, passes=npass)
            else:
                K.linear_wgrad_x3(pb[0][0], nr, pb[0][1], pb[0][2], ws, passes=npass)
            K.linear_wgrad_reduce(Mt, n4, kp, nvalid, ws, lp.col_map[p0:p0 + kp], gW[n0:n0 + nvalid],
                                  gb[n0:n0 + nvalid] if gi == 0 else None, accumulate=acc)


def _flush_wgrad(entry, sink) -> None:
    """A stashed pass whose partner never ran its backward (BucketedGradAllReduce.finish()): its
    weight gradient alone, landed as the sink expects."""
    dZ, segs, M, nrow, N4, lp, npass = entry
    w, b = lp.module.weight, lp.module.bias
    gW, acc = sink.target(w)
    gb, _ = sink.target(b)
    ws = torch.empty((K.linear_wgrad_workspace_bytes(M, N4, lp.Kp) + 3) // 4, device=dZ.device, dtype=torch.float32)
    rsplit = _ray_split([(dZ, segs, M)], N4) if nrow == N4 else None
    tsplit = _tile_split(segs, nrow) if rsplit is None else None
    if rsplit is not None:          # the route the unmerged backward takes: the same result, bitwise
        _wgrad_rays([(dZ, segs, M)], N4, lp, ws, gW, gb, acc, rsplit, npass)
    elif tsplit is not None:
        _wgrad_tiles([(dZ, segs, M)], nrow, N4, lp, ws, gW, gb, acc, tsplit, npass)
    else:
        K.linear_wgrad_x3(dZ, nrow, segs, M, ws, passes=npass)
        K.linear_wgrad_reduce(M, N4, lp.Kp, lp.N, ws, lp.col_map, gW, gb, accumulate=acc)
    sink.landed(w)
    sink.landed(b)


# Gaussian activation fused into the split-precision GEMM epilogues (nerf_linear_gauss_x3); False
# runs the separate nerf_gauss_act_fwd / _bwd passes (tests compare the two)
GAUSS_EPILOGUE = True

# test hook: when a list, every MLPFunction.forward appends (layer outputs, ReLU mask bits)
CAPTURE: list | None = None

# Direct weight-gradient sink (nerf_amd.ddp.BucketedGradAllReduce(direct=True) installs itself):
# a forward recorded for autograd claims its layers' weight and bias parameters (one expected
# contribution each), and the backward writes each layer's gradient straight into the sink's
# target — the parameter's gradient-bucket view, or .grad — accumulating in the slab reduce's
# epilogue when an earlier pass of the same step already landed there, instead of returning it
# to autograd (no separate add per parameter for a field used twice per step).  The sink learns
# of every landing at once, so a complete gradient bucket can start its all-reduce while the
# remaining layers' weight gradients are still being computed.
GRAD_SINK = None


@dataclass
class Source:
    kind: str          # "pos" | "dir" | "act"
    k_valid: int       # columns of the source consumed (reference layout width)
    k_pad: int         # columns the source occupies in the packed weight layout (multiple of 32)
    layer: int = -1    # producing layer for "act"
    # optional: Linear input column of each buffer column (-1 = unused, zero weight); len = k_valid.
    # Default: buffer column j feeds input column j.  (Nerf2d's [cos xy | cos 0 | sin xy | sin 0]
    # encoding of 2-D points padded to 3-D feeds its 40 inputs from one buffer.)
    cols: list[int] | None = None

    @property
    def n_inputs(self) -> int:
        return self.k_valid if self.cols is None else sum(1 for c in self.cols if c >= 0)

    @property
    def k_seg(self) -> int:
        """Columns the kernel reads from the buffer (multiple of 4; the rest of the
        32-wide chunk is zero-filled)."""
        return (self.k_valid + 3) // 4 * 4

    def __post_init__(self):
        if self.kind == "act" and self.k_valid % 4:
            raise NotImplementedError("nerf_amd needs hidden widths that are multiples of 4")


@dataclass
class LayerPlan:
    """One nn.Linear of a field MLP.  Activation: ReLU (fused in the GEMM epilogue), or the
    GARF Gaussian activation with learnable inverse std ``gauss`` (garf/gaussian.py:34-63;
    the pre-activation is kept for the backward), or none.  ``residual`` = index of an earlier
    layer whose output's first ``residual_cols`` columns are added to this layer's output
    (RadianceNetwork's ``z1[:, :128] + z2[:, :128]``, garf/model_radiance.py:92)."""
    module: nn.Linear
    sources: list[Source]
    relu: bool
    gauss: nn.Parameter | None = None
    residual: int = -1
    residual_cols: int = 0
    tanh: bool = False     # tanh in the epilogue (2d-reconstruction/model.py:48-56); backward reads the output
    N: int = 0
    out_ld: int = 0
    Kp: int = 0
    ldwt: int = 0
    koffs: list[int] = field(default_factory=list)
    col_map: torch.Tensor | None = None
    Wp: torch.Tensor | None = None
    Wt: torch.Tensor | None = None
    Wpx: torch.Tensor | None = None
    Wtx: torch.Tensor | None = None

    def finalize(self, device):
        self.N = self.module.out_features
        # outputs are stored with 16-byte rows (N rounded up to 4); the kernels zero-fill
        # the remaining columns of a 32-wide K chunk when such a buffer is an operand
        self.out_ld = (self.N + 3) // 4 * 4
        self.ldwt = K.pad32(self.N)
        cm = []
        orig = 0
        self.koffs = []
        kp = 0
        for s in self.sources:
            self.koffs.append(kp)
            for j in range(s.k_pad):
                if s.cols is None:
                    cm.append(orig + j if j < s.k_valid else -1)
                else:
                    cm.append(orig + s.cols[j] if j < len(s.cols) and s.cols[j] >= 0 else -1)
            orig += s.n_inputs
            kp += s.k_pad
        if orig != self.module.in_features:
            raise ValueError(f"layer input width mismatch: sources give {orig}, Linear expects "
                             f"{self.module.in_features}")
        self.Kp = kp
        self.col_map = torch.tensor(cm, dtype=torch.int32, device=device)
        self.Wp = torch.empty(K.pad128(self.N), self.Kp, device=device, dtype=torch.float32)
        self.Wt = torch.empty(K.pad128(self.Kp) + 128, self.ldwt, device=device, dtype=torch.float32)
        self.Wpx = self.Wtx = None

    def pack(self, precision: str = "fp32", forward: bool = True):
        """Pack the current weights: the forward layouts (Wp / Wpx) when forward=True, the transposed
        ones the input-gradient GEMMs use (Wt / Wtx) when forward=False.  Every call packs (no
        version-keyed cache: see the module docstring)."""
        w = self.module.weight.detach().contiguous()
        x3 = is_split(precision)
        # in split precision the fp32 packs only serve GEMMs with <= 32 output columns: this
        # layer's forward (N <= 32) and the input gradients of sources <= 32 columns wide
        p = forward and (not x3 or self.N <= 32)
        t = (not forward) and (not x3 or any(s.k_pad <= 32 for s in self.sources))
        if p or t:
            K.pack_weight(w, self.col_map, self.Kp, self.Wp if p else None, self.Wt if t else None, self.ldwt)
        if x3:
            if self.Wpx is None:
                dev = self.Wp.device
                self.Wpx = torch.empty(self.Wp.shape[0], 2 * self.Wp.shape[1], device=dev, dtype=torch.bfloat16)
                self.Wtx = torch.empty(self.Wt.shape[0], 2 * self.Wt.shape[1], device=dev, dtype=torch.bfloat16)
            K.pack_weight_x3(w, self.col_map, self.Kp, self.Wpx if forward else None,
                             None if forward else self.Wtx, self.ldwt)

    def gemm(self, precision: str, segs, M: int, transpose: bool, N: int, bias, out, epi, aux=None,
             row_offset: int = 0):
        """Forward (W) or input-gradient (W^T) GEMM in the requested precision; outputs of at
        most 32 columns always use the fp32 kernel's 128 x 32 tile (measured: the 4-wide head at
        M = 262144 takes 42 us there against 55 us on the split-precision 256 x 128 tile)."""
        if is_split(precision) and N > 32:
            K.linear_fwd_x3(segs, M, self.Wtx if transpose else self.Wpx, self.ldwt if transpose else self.Kp, N, bias,
                            out, epi, aux=aux, w_row_offset=row_offset)
        else:
            K.linear_fwd(segs, M, self.Wt if transpose else self.Wp, self.ldwt if transpose else self.Kp, N, bias,
                         out, epi, aux=aux, w_row_offset=row_offset)


class MLPPlan:
    """Layers in execution order; ``outputs`` are layer indices exposed to autograd;
    ``column_outputs`` are (layer, column) pairs additionally exposed as contiguous [M] tensors
    (NerfModel's density column inside the 257-wide last segment output: the compositor reads
    and differentiates a 1 MB vector instead of the 268 MB layer output)."""

    def __init__(self, layers: list[LayerPlan], outputs: list[int], column_outputs: list[tuple[int, int]] = ()):
        self.layers = layers
        self.outputs = outputs
        self.column_outputs = list(column_outputs)
        self.device = None
        self.fused = {}            # device -> mlp_fused.FusedForward
        self.fused_dgrad = {}      # device -> mlp_fused.FusedInputGrad
        self.infer = False         # set per call by MLPFunction.apply: no autograd graph is recorded
        self.consumed = [False] * len(layers)
        # terms of each layer's output gradient (consumer GEMMs, residual adds, autograd outputs):
        # a Gaussian layer with exactly one consumer GEMM gets its activation backward in that
        # GEMM's epilogue
        self.contributors = [0] * len(layers)
        for lp in layers:
            for s in lp.sources:
                if s.kind == "act":
                    self.consumed[s.layer] = True
                    self.contributors[s.layer] += 1
            if lp.residual >= 0:
                self.consumed[lp.residual] = True
                self.contributors[lp.residual] += 1
        for i in outputs:
            self.contributors[i] += 1
        for li, _ in self.column_outputs:
            self.contributors[li] += 1

    def to_device(self, device):
        if self.device != device:
            for lp in self.layers:
                lp.finalize(device)
            self.device = device

    def linear_params(self):
        """The layers' weight and bias parameters (what a direct gradient sink takes over)."""
        return [t for lp in self.layers for t in (lp.module.weight, lp.module.bias)]

    def params(self):
        """Autograd inputs in a fixed order: per layer weight, bias (+ Gaussian inverse std)."""
        ps = []
        for lp in self.layers:
            ps += [lp.module.weight, lp.module.bias]
            if lp.gauss is not None:
                ps.append(lp.gauss)
        return ps


def _src_tensor(src: Source, pos, dirs, acts, dir_rd):
    if src.kind == "pos":
        return pos, 1
    if src.kind == "dir":
        return dirs, dir_rd
    return acts[src.layer], 1


class MLPFunction(torch.autograd.Function):
    @classmethod
    def apply(cls, plan: MLPPlan, *args, composite: CompositeSpec | None = None):
        # grad mode is off inside forward (and needs_input_grad ignores it): note it for forward.
        # composite: the renderer's compositing run inside the fused launches (composite_eligible);
        # the outputs then end with (rgb [B, 3], weights [B, S]) (weights non-differentiable)
        plan.infer = not torch.is_grad_enabled()
        plan.composite = composite
        return super().apply(plan, *args)

    @staticmethod
    def forward(ctx, plan: MLPPlan, M: int, pos: torch.Tensor, dirs: torch.Tensor | None, dir_rd: int, *params):
        plan.to_device(pos.device)
        # outputs the caller never uses get None gradients instead of materialised zeros
        # (NerfModel with delayed density never reads z_last: a 268 MB memset + clone per step)
        ctx.set_materialize_grads(False)
        ctx.fused_forward = False
        comp = getattr(plan, "composite", None)
        plan.composite = None
        ctx.comp = None
        rgb = w = None
        prec = matmul_precision()
        if comp is not None and not composite_eligible(plan, M, comp.S):
            raise RuntimeError("MLPFunction: fused compositing requested for a plan / size it does not fit")
        acts: list[torch.Tensor] = []
        masks: list[torch.Tensor | None] = []
        pre: list[torch.Tensor] = []
        cols = None
        if is_split(prec) and mlp_fused.eligible(plan, M):
            # the whole network in one launch (csrc/mlp_fused.hip); same outputs as the loop below
            fused = plan.fused.get(pos.device)
            if fused is None:
                fused = plan.fused[pos.device] = mlp_fused.FusedForward(plan, pos.device)
            # without autograd (rendering) only the exposed outputs are stored: the kernel drops
            # the other layers' stores and the ReLU bits (11 x 268 MB less HBM traffic at M = 2^18)
            keep_all = not getattr(plan, "infer", False)
            for idx, lp in enumerate(plan.layers):
                # no packing here: the backward packs the input-gradient layouts (Wt / Wtx) only
                # if it runs the layer-by-layer GEMMs instead of the fused chain
                acts.append(torch.empty(M, lp.out_ld, device=pos.device, dtype=torch.float32)
                            if keep_all or idx in plan.outputs else None)
                masks.append(torch.empty(M, 32, device=pos.device, dtype=torch.uint8)
                             if keep_all and lp.relu and plan.consumed[idx] and lp.N <= 256 else None)
            col_t = {li: torch.empty(M, device=pos.device, dtype=torch.float32) for li, _ in plan.column_outputs}
            # deferred encodings (render_raw) are generated by the kernel itself, their rows stored by
            # the first layer that reads them
            if comp is not None:
                B = M // comp.S
                rgb = torch.empty(B, 3, device=pos.device, dtype=torch.float32)
                w = torch.empty(B, comp.S, device=pos.device, dtype=torch.float32)
                comp.coef = (torch.empty(M, 8, device=pos.device, dtype=torch.float32)
                             if keep_all else None)
            fused.run(M, pos, dirs, dir_rd, acts, masks, col_t, (K.deferred(pos), K.deferred(dirs)),
                      comp=(comp, rgb, w, composite_sigma_layer(plan)) if comp is not None else None,
                      passes=passes(prec))
            K.mark_filled(pos)
            K.mark_filled(dirs)
            cols = tuple(col_t[li] for li, _ in plan.column_outputs)
            ctx.fused_forward = True
        else:
            K.materialize(pos)
            K.materialize(dirs)
            for idx, lp in enumerate(plan.layers):
                lp.pack(prec)
                segs = []
                for s in lp.sources:
                    t, rd = _src_tensor(s, pos, dirs, acts, dir_rd)
                    segs.append((t, s.k_seg, rd))
                out = torch.empty(M, lp.out_ld, device=pos.device, dtype=torch.float32)
                # Gaussian layers: the GEMM writes the pre-activation z (kept for the backward) and,
                # in split precision, exp(-z^2 v) into the layer's output from the same epilogue;
                # otherwise nerf_gauss_act_fwd applies the activation in a second pass
                target = torch.empty_like(out) if lp.gauss is not None else out
                if (GAUSS_EPILOGUE and lp.gauss is not None and is_split(prec) and lp.N > 32 and lp.residual < 0
                        and not lp.relu and K.linear_gauss_x3(segs, M, lp.Wpx, lp.Kp, lp.N, target, lp.gauss, bias=lp.module.bias,
                                              y=out)):
                    pre.append(target)
                    acts.append(out)
                    masks.append(None)
                    continue
                epi = NERF_EPI_BIAS | (NERF_EPI_RELU if lp.relu else 0) | (NERF_EPI_TANH if lp.tanh else 0)
                mask = None
                if lp.relu and plan.consumed[idx] and lp.N <= 256:
                    # the ReLU-backward mask of this output as bits (32 bytes a row): the input-
                    # gradient GEMMs read it instead of the fp32 activation
                    mask = torch.empty(M, 32, device=pos.device, dtype=torch.uint8)
                    epi |= NERF_EPI_MASKOUT
                if lp.residual >= 0:
                    # out = residual + (x W^T + b): the accumulate epilogue adds onto the copied residual
                    rc = lp.residual_cols
                    target[:, rc:].zero_()
                    target[:, :rc].copy_(acts[lp.residual][:, :rc])
                    epi |= NERF_EPI_ACCUM
                lp.gemm(prec, segs, M, False, lp.N, lp.module.bias, target, epi, aux=mask)
                if lp.gauss is not None:
                    K.gauss_act_fwd(target, lp.N, lp.gauss, out)
                    if lp.out_ld > lp.N:
                        out[:, lp.N:].zero_()
                    pre.append(target)
                acts.append(out)
                masks.append(mask)
        if CAPTURE is not None:
            CAPTURE.append((list(acts), list(masks)))
        ctx.masks = masks
        ctx.prec = prec
        ctx.plan = plan
        sink = GRAD_SINK
        ctx.sink = sink if (sink is not None and not plan.infer and sink.claim(plan.linear_params())) else None
        ctx.M = M
        ctx.dir_rd = dir_rd
        ctx.has_dirs = dirs is not None
        ctx.n_pos_cols = pos.shape[1]
        ctx.n_dir_cols = dirs.shape[1] if dirs is not None else 0
        if any(a is None for a in acts):
            ctx.save_for_backward(pos)     # no backward can run (no input needed a gradient)
        else:
            ctx.save_for_backward(pos, dirs if dirs is not None else pos, *acts, *pre)
        if cols is None:
            cols = tuple(acts[li][:, c].contiguous() for li, c in plan.column_outputs)
        if comp is not None:
            ctx.comp = comp
            ctx.mark_non_differentiable(w)
            return tuple(acts[i] for i in plan.outputs) + cols + (rgb, w)
        return tuple(acts[i] for i in plan.outputs) + cols

    @staticmethod
    def backward(ctx, *grads):
        plan: MLPPlan = ctx.plan
        M = ctx.M
        saved = ctx.saved_tensors
        pos = saved[0]
        dirs = saved[1] if ctx.has_dirs else None
        L = len(plan.layers)
        acts = list(saved[2:2 + L])
        pre_it = iter(saved[2 + L:])
        pre = [next(pre_it) if lp.gauss is not None else None for lp in plan.layers]
        dev = pos.device
        dY: list[torch.Tensor | None] = [None] * L
        owned = [True] * L       # False: dY[i] is autograd's incoming tensor (never written in place)
        comp = ctx.comp
        g_rgb = None
        if comp is not None:
            n_out = len(plan.outputs) + len(plan.column_outputs)
            g_rgb = grads[n_out]
            grads = grads[:n_out]
            if g_rgb is not None:
                g_rgb = g_rgb.contiguous()
        col_grads: list[list[tuple[int, torch.Tensor]]] = [[] for _ in range(L)]
        for (li, c), g in zip(plan.column_outputs, grads[len(plan.outputs):]):
            if g is not None:
                col_grads[li].append((c, g))
        for idx, g in zip(plan.outputs, grads[:len(plan.outputs)]):
            if g is None:
                continue
            if g.shape != (M, plan.layers[idx].out_ld):
                raise RuntimeError(f"unexpected gradient shape {tuple(g.shape)} for MLP output {idx}")
            # outputs that also feed a later layer are accumulated into: never write autograd's tensor
            dY[idx] = g.contiguous().clone() if plan.consumed[idx] else g.contiguous()
            owned[idx] = plan.consumed[idx]
        need_pos = ctx.needs_input_grad[2]
        need_dir = ctx.needs_input_grad[3]
        dpos = None
        ddir = None
        layer_grads: list[list[torch.Tensor]] = [[] for _ in range(L)]
        gauss_done: list[torch.Tensor | None] = [None] * L   # inverse-std gradients formed in an epilogue

        # the input-gradient chain in one launch (csrc/mlp_fused.hip): every dY[l], l < L-1, from
        # the head gradient through the stored ReLU bits, when nothing else feeds the backward
        # (a column output's gradient joins the chain as one more k-block and is added to its
        # layer's stored gradient below, as in the layer-by-layer path)
        chain_ok = (ctx.fused_forward and mlp_fused.dgrad_eligible(plan, M)
                    and mlp_fused.FusedInputGrad.layout(plan, need_pos, need_dir) is not None)
        # fused compositing: the chain forms the head / density gradient rows itself from the
        # forward's coefficients and grad_rgb (and stores them for the weight gradients) when they
        # are the only gradients; otherwise they are formed here and join the others
        comp_chain = (g_rgb is not None and chain_ok and all(d is None for d in dY)
                      and not any(col_grads))
        if g_rgb is not None and not comp_chain:
            sl = composite_sigma_layer(plan)
            gh, gs = composite_grads_torch(comp, g_rgb, sl >= 0)
            head = plan.layers[L - 1]
            if dY[L - 1] is None:
                dY[L - 1] = torch.zeros(M, head.out_ld, device=dev, dtype=torch.float32)
            elif not owned[L - 1]:
                dY[L - 1] = dY[L - 1].clone()
            owned[L - 1] = True
            dY[L - 1][:, 0:3] += gh
            if sl < 0:
                dY[L - 1][:, 3] += gs
            else:
                col_grads[sl].append((dict(plan.column_outputs)[sl], gs))
        chain = chain_ok and (comp_chain or (
            all(dY[i] is None for i in range(L - 1)) and dY[L - 1] is not None
            and all(len(col_grads[li]) == 1 for li, _ in plan.column_outputs)))
        if chain:
            key = (dev, bool(need_pos), bool(need_dir))
            fd = plan.fused_dgrad.get(key)
            if fd is None:
                fd = plan.fused_dgrad[key] = mlp_fused.FusedInputGrad(plan, dev, need_pos, need_dir)
            g_cols = {}
            comp_rt = None
            if comp_chain:
                g_head = None
                dY[L - 1] = torch.empty(M, plan.layers[L - 1].out_ld, device=dev, dtype=torch.float32)
                if plan.layers[L - 1].out_ld > 4:
                    dY[L - 1][:, 4:].zero_()
            else:
                g_head = dY[L - 1]
                for li, _ in plan.column_outputs:
                    g4 = torch.zeros(M, 4, device=dev, dtype=torch.float32)
                    g4[:, 0] = col_grads[li][0][1].reshape(-1)
                    g_cols[li] = g4
            sl = composite_sigma_layer(plan)
            for l in range(L - 1):
                dY[l] = torch.empty(M, plan.layers[l].out_ld, device=dev, dtype=torch.float32)
                if plan.layers[l].out_ld > 256 and plan.layers[l].N > 256:
                    if comp_chain and l == sl and plan.layers[l].out_ld == 260:
                        continue              # the chain writes the density column 256 (+ zeros to 259)
                    dY[l][:, 256:].zero_()    # the chain fills the register-fed 256 columns
            if comp_chain:
                comp_rt = (comp, g_rgb, dY[L - 1], dY[sl][:, 256:] if sl >= 0 else None, sl)
            # encoding-input gradients (pose refinement): one buffer per step that produces them
            x_out = {}
            for (l, _, _, _, x, *_rest) in fd.steps:
                if x is not None:
                    x_out[l] = torch.empty(M, x.k_pad, device=dev, dtype=torch.float32)
            fd.run(M, g_head, dY, ctx.masks, g_cols, x_out, comp=comp_rt, passes=passes(ctx.prec))
            for (l, _, _, _, x, *_rest) in fd.steps:
                if x is None:
                    continue
                if x.kind == "pos":
                    dpos = x_out[l] if dpos is None else dpos.add_(x_out[l])
                else:
                    ddir = x_out[l] if ddir is None else ddir.add_(x_out[l])

        # one workspace sized for the largest weight-gradient launch
        ws_bytes = 0
        for lp in plan.layers:
            ws_bytes = max(ws_bytes, K.linear_wgrad_workspace_bytes(M, (lp.N + 3) // 4 * 4, lp.Kp))
        workspace = torch.empty((ws_bytes + 3) // 4, device=dev, dtype=torch.float32)

        for li in range(L - 1, -1, -1):
            lp = plan.layers[li]
            if col_grads[li]:
                # gradients of the column outputs, added after every consumer's contribution
                if dY[li] is None:
                    dY[li] = torch.zeros(M, lp.out_ld, device=dev, dtype=torch.float32)
                elif not owned[li]:
                    dY[li] = dY[li].clone()
                for c, g in col_grads[li]:
                    dY[li][:, c] += g
            dZ = dY[li]
            w = lp.module.weight
            sink = ctx.sink
            if dZ is None:
                if sink is not None:
                    for t in (w, lp.module.bias):
                        g, acc = sink.target(t)
                        if not acc:
                            g.zero_()
                        sink.landed(t)
                    layer_grads[li] = [None, None]
                else:
                    layer_grads[li] = [torch.zeros_like(w), torch.zeros_like(lp.module.bias)]
                if lp.gauss is not None:
                    layer_grads[li].append(torch.zeros_like(lp.gauss))
                continue
            gs = None
            if gauss_done[li] is not None:
                gs = gauss_done[li]          # dY[li] already is dL/dz (the consumer's epilogue)
            elif lp.gauss is not None:
                # dY -> dZ through the Gaussian activation (+ the inverse-std gradient)
                gs = torch.empty_like(lp.gauss)
                dz = dZ if owned[li] else torch.empty_like(dZ)
                K.gauss_act_bwd(dZ, pre[li], lp.N, lp.gauss, dz, gs)
                dZ = dz
            if lp.residual >= 0:
                r, rc = lp.residual, lp.residual_cols
                if dY[r] is None:
                    dY[r] = torch.zeros(M, plan.layers[r].out_ld, device=dev, dtype=torch.float32)
                dY[r][:, :rc] += dZ[:, :rc]
            segs = []
            for s in lp.sources:
                t, rd = _src_tensor(s, pos, dirs, acts, ctx.dir_rd)
                segs.append((t, s.k_seg, rd))
            # ---- weight and bias gradients
            N4 = (lp.N + 3) // 4 * 4
            # the true row count: 257 (density + features) runs as one 256 x 256 tile + a row
            nrow = lp.N if (lp.N == 257 and WGRAD_ROW257) else N4
            merge = sink is not None and is_split(ctx.prec) and MERGE_PASSES and gs is None
            prev = sink.stash.pop((id(plan), li), (None, None))[0] if merge else None
            if merge and prev is None and sink.remaining(w) >= 2:
                # another pass of this field lands its contribution later in this backward: its
                # weight gradient runs once over both passes' rows (one launch, one reduce); the
                # sink flushes the stash alone if that pass never comes
                sink.stash[(id(plan), li)] = ((dZ, segs, M, nrow, N4, lp, passes(ctx.prec)), _flush_wgrad)
                layer_grads[li] = [None, None]
            else:
                if sink is not None:
                    gW, acc = sink.target(w)
                    gb, acc_b = sink.target(lp.module.bias)
                    if acc != acc_b:
                        raise RuntimeError("direct gradient sink: weight and bias of one layer out of step")
                else:
                    gW, gb, acc = torch.empty_like(w), torch.empty_like(lp.module.bias), False
                rsplit = None
                wblocks = [(prev[0], prev[1], prev[2]), (dZ, segs, M)] if prev is not None else [(dZ, segs, M)]
                if is_split(ctx.prec) and nrow == N4:
                    rsplit = _ray_split(wblocks, N4)
                npass = passes(ctx.prec)
                tsplit = _tile_split(segs, nrow) if rsplit is None and is_split(ctx.prec) else None
                if rsplit is not None:
                    _wgrad_rays(wblocks, N4, lp, workspace, gW, gb, acc, rsplit, npass)
                elif tsplit is not None:
                    _wgrad_tiles(wblocks, nrow, N4, lp, workspace, gW, gb, acc, tsplit, npass)
                elif prev is not None:
                    pdZ, psegs, pM = prev[0], prev[1], prev[2]
                    ws = _wgrad_workspace(workspace, M + pM, N4, lp.Kp)
                    K.linear_wgrad_x3_rows([(pdZ, psegs, pM), (dZ, segs, M)], nrow, ws, passes=npass)
                    K.linear_wgrad_reduce(M + pM, N4, lp.Kp, lp.N, ws, lp.col_map, gW, gb, accumulate=acc)
                elif is_split(ctx.prec):
                    K.linear_wgrad_x3(dZ, nrow, segs, M, workspace, passes=npass)
                    K.linear_wgrad_reduce(M, N4, lp.Kp, lp.N, workspace, lp.col_map, gW, gb, accumulate=acc)
                else:
                    K.linear_wgrad(dZ, N4, segs, M, workspace)
                    K.linear_wgrad_reduce(M, N4, lp.Kp, lp.N, workspace, lp.col_map, gW, gb, accumulate=acc)
                if sink is not None:
                    for _ in range(2 if prev is not None else 1):     # the stashed pass's too
                        sink.landed(w)
                        sink.landed(lp.module.bias)
                    gW = gb = None
                layer_grads[li] = [gW, gb] + ([gs] if gs is not None else [])
            # ---- input gradients
            if chain:
                continue
            lp.pack(ctx.prec, forward=False)
            a_seg = [(dZ, lp.out_ld, 1)]
            for s, koff in zip(lp.sources, lp.koffs):
                if s.kind == "act":
                    j = s.layer
                    prod = plan.layers[j]
                    if (GAUSS_EPILOGUE and prod.gauss is not None and plan.contributors[j] == 1 and dY[j] is None
                            and not prod.relu and is_split(ctx.prec) and s.k_valid > 32):
                        # sole consumer: dL/dz of the Gaussian layer straight from this GEMM's epilogue
                        dz = torch.empty(M, prod.out_ld, device=dev, dtype=torch.float32)
                        gsj = torch.empty_like(prod.gauss)
                        if K.linear_gauss_x3(a_seg, M, lp.Wtx, lp.ldwt, s.k_valid, dz, prod.gauss, z=pre[j],
                                             grad_inv_std=gsj, w_row_offset=koff):
                            dY[j] = dz
                            gauss_done[j] = gsj
                            continue
                    epi = 0
                    aux = None
                    if prod.tanh:
                        epi |= NERF_EPI_TANH_BWD       # * (1 - y^2) from the stored activation
                        aux = acts[j]
                    if prod.relu:
                        # (the fused forward's bits are in the NERF_FUSED_MASK layout, which only
                        # the fused chain reads: this path takes the stored activation instead)
                        if ctx.masks[j] is not None and not ctx.fused_forward:
                            epi |= NERF_EPI_MASK | NERF_EPI_MASKBITS
                            aux = ctx.masks[j]
                        else:
                            epi |= NERF_EPI_MASK
                            aux = acts[j]
                    fresh = dY[j] is None
                    if fresh:
                        dY[j] = torch.empty(M, prod.out_ld, device=dev, dtype=torch.float32)
                    else:
                        epi |= NERF_EPI_ACCUM
                    lp.gemm(ctx.prec, a_seg, M, True, s.k_valid, None, dY[j], epi, aux=aux, row_offset=koff)
                    if fresh and prod.out_ld > s.k_valid:
                        dY[j][:, s.k_valid:].zero_()     # columns this consumer does not read
                elif s.kind == "pos" and need_pos:
                    if dpos is None:
                        dpos = torch.empty(M, s.k_pad, device=dev, dtype=torch.float32)
                        epi = 0
                    else:
                        epi = NERF_EPI_ACCUM
                    lp.gemm(ctx.prec, a_seg, M, True, s.k_pad, None, dpos, epi, row_offset=koff)
                elif s.kind == "dir" and need_dir:
                    if ddir is None:
                        ddir = torch.empty(M, s.k_pad, device=dev, dtype=torch.float32)
                        epi = 0
                    else:
                        epi = NERF_EPI_ACCUM
                    lp.gemm(ctx.prec, a_seg, M, True, s.k_pad, None, ddir, epi, row_offset=koff)
        if ddir is not None and ctx.dir_rd > 1:
            ddir = ddir.view(-1, ctx.dir_rd, ddir.shape[1]).sum(dim=1)
        # the packed gradients span pad32 columns; the inputs may be narrower (e.g. [M, 4])
        if dpos is not None and dpos.shape[1] != ctx.n_pos_cols:
            dpos = dpos[:, :ctx.n_pos_cols]
        if ddir is not None and ddir.shape[1] != ctx.n_dir_cols:
            ddir = ddir[:, :ctx.n_dir_cols]
        param_grads = [g for lg in layer_grads for g in lg]
        return (None, None, dpos, ddir, None, *param_grads)


def nerf_model_plan(n_segments: int, model_segments: nn.ModuleList, model_color: nn.Sequential,
                    hidden_dim: int, pos_dim: int, dir_dim: int, delayed_direction: bool,
                    delayed_density: bool) -> tuple[MLPPlan, int, int]:
    """Lower NerfModel (barf/model_interpolation_architecture.py:33-161).

    Segment i input = [z_{i-1} | dir (if not delayed_direction) | pos]; inside a
    segment every Linear but the last is followed by ReLU; the last one is
    followed by ReLU only between segments.  Head input = [z_last[:, :D] | dir
    (if delayed_direction)] -> Linear -> ReLU -> Linear.
    Returns (plan, index of the last segment layer, index of the head output layer).
    """
    layers: list[LayerPlan] = []
    pos_src = Source("pos", pos_dim, K.pad32(pos_dim))
    dir_src = Source("dir", dir_dim, K.pad32(dir_dim))
    prev = -1
    for i in range(n_segments):
        seg = model_segments[i]
        linears = [m for m in seg.modules() if isinstance(m, nn.Linear)] if isinstance(seg, nn.Sequential) \
            else [seg]
        for j, lin in enumerate(linears):
            srcs: list[Source] = []
            if j == 0:
                if prev >= 0:
                    srcs.append(Source("act", hidden_dim, K.pad32(hidden_dim), prev))
                if not delayed_direction:
                    srcs.append(dir_src)
                srcs.append(pos_src)
            else:
                srcs.append(Source("act", hidden_dim, K.pad32(hidden_dim), len(layers) - 1))
            last_in_seg = j == len(linears) - 1
            relu = (not last_in_seg) or (i < n_segments - 1)
            layers.append(LayerPlan(lin, srcs, relu))
        prev = len(layers) - 1
    z_last = prev
    head0, head1 = model_color[0], model_color[2]
    srcs = [Source("act", hidden_dim, K.pad32(hidden_dim), z_last)]
    if delayed_direction:
        srcs.append(dir_src)
    layers.append(LayerPlan(head0, srcs, True))
    layers.append(LayerPlan(head1, [Source("act", head0.out_features, K.pad32(head0.out_features), len(layers) - 1)],
                            False))
    head_out = len(layers) - 1
    # without delayed density, sigma is column hidden_dim of the last segment output: exposed as
    # its own [M] output so the compositor never touches (or differentiates) the 257-wide buffer
    cols = [] if delayed_density else [(z_last, hidden_dim)]
    return MLPPlan(layers, [z_last, head_out], cols), z_last, head_out
