"""Lowering of a field-MLP plan onto the fused forward kernel (csrc/mlp_fused.hip).

``nerf_mlp_fused_fwd`` runs every Linear (+ bias + ReLU) of a NerfModel
(barf/model_interpolation_architecture.py:96-141) in one launch, keeping each wave's
activations in registers between layers.  This module decides whether a plan fits the
kernel, builds the packed weight image (MFMA-fragment order, split hi/lo bf16, biases) and
the per-layer descriptors, and launches it.  Outputs are exactly those of the layer-by-layer
forward in mlp.py (every layer's output, the ReLU mask bits, the density column), so the
backward is unchanged.

Fragment order (mirrors the kernel header): chunk (layer, nb) holds output rows 32 nb .. +31;
for every 32-deep k-block kb and 16-row half bb, lane l (s = l & 15, g = l >> 4) element j is
W[32 nb + 16 bb + s][k(kb, g, j)] with
  k = 32 kb + 16 (j >> 2) + 4 g + (j & 3)          register-fed input (previous layer output)
  k = seg_offset + 32 kh + 8 g + j                  HBM-fed segment block kh (encodings)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from . import kernels as K

def _pack_image(f) -> None:
    """Rebuild a fused image from the plan's current parameters (one gather launch, ~2.6 MB for
    NerfModel).  Runs before EVERY launch that reads the image: a cache keyed on the parameters'
    version counters misses ``p.data`` updates and fused optimizers, and would then train on stale
    weights without any error (in training the weights change every step anyway)."""
    ps = []
    for lp in f.plan.layers:
        ps += [lp.module.weight, lp.module.bias]
    arr = (ctypes.c_void_p * len(ps))(*[p.detach().contiguous().data_ptr() for p in ps])
    st = _lib.load().nerf_fused_pack(arr, len(ps), f.map_src.data_ptr(), f.map_dst.data_ptr(), f.map_src.numel(),
                                     f.image.data_ptr(), K._stream(f.device))
    _lib.check(st, "nerf_fused_pack")


FUSED_TYPES = {(0, 1): 1, (0, 2): 2, (4, 0): 3, (8, 0): 6, (8, 1): 7, (8, 2): 8}   # (kbr, kbh) -> type
ENABLED = os.environ.get("NERF_FUSED", "1") != "0"     # A/B switch (bench, tests)


def _layer_shape(plan, idx):
    """(kbr, hbm sources, act source) of layer idx, or None if the kernel cannot run it."""
    lp = plan.layers[idx]
    if lp.gauss is not None or lp.residual >= 0:
        return None
    acts = [s for s in lp.sources if s.kind == "act"]
    hbm = [s for s in lp.sources if s.kind != "act"]
    if idx == 0:
        if acts:
            return None
        kbr = 0
    else:
        if len(acts) != 1 or lp.sources[0] is not acts[0] or acts[0].layer != idx - 1:
            return None
        if acts[0].k_valid not in (128, 256):
            return None
        kbr = acts[0].k_valid // 32
    if len(hbm) > 2 or any(s.kind not in ("pos", "dir") for s in hbm):
        return None
    kbh = sum(s.k_pad // 32 for s in hbm)
    if (kbr, kbh) not in FUSED_TYPES:
        return None
    return kbr, hbm


def eligible(plan, M: int) -> bool:
    if not ENABLED or len(plan.layers) > _lib.NERF_FUSED_MAX_LAYERS or M >= (1 << 30):
        return False
    if len(plan.layers) * 2 > _lib.NERF_FUSED_MAX_SRCS:
        return False
    cols = {}
    for li, c in plan.column_outputs:
        if c % 32 or li in cols:
            return False
        cols[li] = c
    for idx, lp in enumerate(plan.layers):
        if _layer_shape(plan, idx) is None:
            return False
        N = lp.module.out_features
        if (N + 31) // 32 > 9 or M * lp.out_ld * 4 >= (1 << 31):
            return False
        if idx + 1 < len(plan.layers) and plan.layers[idx + 1].sources[0].kind == "act" and N > 288:
            return False
    return True


class FusedForward:
    """Packed image + static descriptors of one plan on one device."""

    def __init__(self, plan, device):
        self.plan = plan
        self.device = device
        self.layers = []          # (kbr, kbh, hbm sources, nb, units, img_off, bias_off)
        shapes = []
        off = 0
        for idx, lp in enumerate(plan.layers):
            kbr, hbm = _layer_shape(plan, idx)
            kbh = sum(s.k_pad // 32 for s in hbm)
            nb = (lp.module.out_features + 31) // 32
            units = 4 * (kbr + kbh)
            shapes.append((kbr, kbh, hbm, nb, units, off))
            off += nb * units * 1024
        src_codes, dst_codes = [], []
        for idx, lp in enumerate(plan.layers):
            kbr, kbh, hbm, nb, units, img_off = shapes[idx]
            self.layers.append((kbr, kbh, hbm, nb, units, img_off, off))
            s, d = self._maps(idx, lp, kbr, hbm, nb, units, img_off, off)
            src_codes.append(s)
            dst_codes.append(d)
            off += nb * 128
        self.image_bytes = off
        self.image = torch.zeros(off // 2, dtype=torch.bfloat16, device=device)
        self.map_src = torch.from_numpy(np.concatenate(src_codes).astype(np.int32)).to(device)
        self.map_dst = torch.from_numpy(np.concatenate(dst_codes).astype(np.int32)).to(device)

    @staticmethod
    def _maps(idx, lp, kbr, hbm, nb, units, off, bias_off):
        """Gather map of one layer: source codes (tensor << 24 | element, -1 = 0) and
        destinations (bf16 index of hi, or ~fp32 word for raw bias words)."""
        N, K_orig = lp.module.out_features, lp.module.in_features
        tw, tb = 2 * idx, 2 * idx + 1
        # original weight column offsets of the sources (plan order, k_valid wide)
        orig = {}
        o = 0
        for s in lp.sources:
            orig[id(s)] = o
            o += s.k_valid
        lane = np.arange(64)
        srow, grp = lane & 15, lane >> 4
        j = np.arange(8)
        kb_total = kbr + sum(s.k_pad // 32 for s in hbm)
        col = np.full((kb_total, 64, 8), -1, dtype=np.int64)       # weight column per (kb, lane, j)
        for kb in range(kbr):
            col[kb] = 32 * kb + 16 * (j[None, :] >> 2) + 4 * grp[:, None] + (j[None, :] & 3)
        kb = kbr
        for s in hbm:
            for kh in range(s.k_pad // 32):
                local = 32 * kh + 8 * grp[:, None] + j[None, :]
                col[kb] = np.where(local < s.k_valid, orig[id(s)] + local, -1)
                kb += 1
        srcs, dsts = [], []
        for c in range(nb):
            base = off + c * units * 1024
            for bb in range(2):
                n = 32 * c + 16 * bb + srow                          # [64]
                nn = np.broadcast_to(n[None, :, None], col.shape)
                valid = (col >= 0) & (nn < N)
                code = np.where(valid, (tw << 24) + nn * K_orig + col, -1)
                dst = (base + np.arange(kb_total)[:, None, None] * 4096 + bb * 2048) // 2 + \
                    lane[None, :, None] * 8 + j[None, None, :]
                srcs.append(code.reshape(-1))
                dsts.append(np.broadcast_to(dst, col.shape).reshape(-1))
            nbias = 32 * c + np.arange(32)
            srcs.append(np.where(nbias < N, (tb << 24) + nbias, -1))
            dsts.append(~(bias_off // 4 + nbias))
        return np.concatenate(srcs), np.concatenate(dsts)

    def pack(self):
        _pack_image(self)

    def run(self, M: int, pos: torch.Tensor, dirs: torch.Tensor | None, dir_rd: int, acts, masks, col_outs):
        """Launch on the current stream.  acts[l]: [M, out_ld] fp32 or None (not stored),
        masks[l]: [M, 32] uint8 or None, col_outs: {layer: [M] fp32}."""
        self.pack()
        L = len(self.plan.layers)
        descs = (_lib.NerfFusedLayer * L)()
        flops = 0.0
        nbytes = 0.0
        for idx, lp in enumerate(self.plan.layers):
            kbr, kbh, hbm, nb, units, off, bias_off = self.layers[idx]
            d = descs[idx]
            d.type = FUSED_TYPES[(kbr, kbh)]
            d.N = lp.module.out_features
            d.nb = nb
            d.relu = 1 if lp.relu else 0
            d.nseg = len(hbm)
            for si, s in enumerate(hbm):
                t = pos if s.kind == "pos" else dirs
                d.seg_kb[si] = s.k_pad // 32
                d.seg_k[si] = s.k_seg
                d.seg_rd[si] = 1 if s.kind == "pos" else dir_rd
                d.seg_rows[si] = t.shape[0]
                d.seg_ld[si] = t.stride(0)
                d.seg_ptr[si] = t.data_ptr()
            d.chunk_units = units
            d.col_idx = -1
            # a layer without a tensor (inference: not an exposed output) has its stores dropped
            d.out = acts[idx].data_ptr() if acts[idx] is not None else None
            d.ldo = acts[idx].stride(0) if acts[idx] is not None else 0
            d.mask = masks[idx].data_ptr() if masks[idx] is not None else None
            if idx in col_outs:
                d.col_out = col_outs[idx].data_ptr()
                d.col_idx = dict(self.plan.column_outputs)[idx]
            d.img_off = off
            d.bias_off = bias_off
            flops += 2.0 * M * lp.module.out_features * lp.module.in_features
            # algorithmic bytes: HBM-fed encodings read, stored outputs / mask bits / columns written
            nbytes += sum(4.0 * d.seg_k[si] * d.seg_rows[si] for si in range(d.nseg))
            nbytes += (4.0 * M * acts[idx].shape[1] if acts[idx] is not None else 0.0) \
                + (32.0 * M if masks[idx] is not None else 0.0) + (4.0 * M if idx in col_outs else 0.0)
        end = K.TIMER.bracket("mlp_fused_fwd", flops, nbytes + self.image.numel() * self.image.element_size(),
                              fn="mlp_fused_fwd_kernel") \
            if K.TIMER is not None else None
        st = _lib.load().nerf_mlp_fused_fwd(descs, L, self.image.data_ptr(), M, K._stream(self.device))
        if end is not None:
            end.record()
        _lib.check(st, "nerf_mlp_fused_fwd")


# ---------------------------------------------------------------------------------------------
# Input-gradient chain of the backward on the same kernel: steps l = L-1 .. 1, step l maps the
# gradient w.r.t. layer l's output (dL/dz_l, B operand) through W_l^T to the gradient w.r.t. its
# register-fed input, times the ReLU bits of layer l-1 (mask_in) = dL/dz_{l-1}.  The chain starts
# from the head gradient in HBM; every step's output is stored for the weight gradients.
# ---------------------------------------------------------------------------------------------
def dgrad_eligible(plan, M: int) -> bool:
    """NerfModel plans whose backward needs only the register-fed chain (no encoding gradients;
    the caller checks that and which outputs carry gradients).  A column output is allowed on a
    257-wide layer at column 256 (the density of NerfModel without delayed density): its gradient
    enters the chain as one HBM-fed k-block."""
    if not ENABLED or not eligible(plan, M):
        return False
    cols = dict(plan.column_outputs)
    L = len(plan.layers)
    for li, c in cols.items():
        if plan.layers[li].N != 257 or c != 256 or li == L - 1 or plan.layers[li].relu:
            return False
    for l in range(1, L):
        lp = plan.layers[l]
        act = lp.sources[0]
        if act.kind != "act" or act.layer != l - 1 or act.k_valid not in (128, 256):
            return False
        if l < L - 1 and not (lp.N in (128, 256) or (l in cols and lp.N == 257)):
            return False
        if l == L - 1 and lp.N > 32:
            return False
        if plan.layers[l - 1].relu and plan.layers[l - 1].N > 256:
            return False
    return True


class FusedInputGrad:
    """Packed W^T image + static step table of the input-gradient chain of one plan."""

    runs = 0                      # launches so far (tests check the chain actually ran)

    @staticmethod
    def layout(plan, need_pos: bool, need_dir: bool):
        """Steps (layer l, kbr, kbh, n1 chained chunks, extra source or None) of the chain, or None
        if the plan needs encoding gradients the kernel cannot route (at most one encoding input
        per layer may need its gradient, written to the step's second output)."""
        L = len(plan.layers)
        cols = dict(plan.column_outputs)

        def extra(lp):
            xs = [s for s in lp.sources[1:] if (s.kind == "pos" and need_pos) or (s.kind == "dir" and need_dir)]
            return xs
        steps = []
        for l in range(L - 1, 0, -1):
            lp = plan.layers[l]
            kbr, kbh = (0, 1) if l == L - 1 else (lp.N // 32, 1 if l in cols else 0)
            xs = extra(lp)
            if len(xs) > 1:
                return None
            steps.append((l, kbr, kbh, lp.sources[0].k_valid // 32, xs[0] if xs else None))
        lp0 = plan.layers[0]
        xs = [s for s in lp0.sources if (s.kind == "pos" and need_pos) or (s.kind == "dir" and need_dir)]
        if len(xs) > 1 or (xs and lp0.N not in (128, 256)):
            return None
        if xs:
            steps.append((0, lp0.N // 32, 0, 0, xs[0]))
        return steps

    def __init__(self, plan, device, need_pos: bool = False, need_dir: bool = False):
        self.plan = plan
        self.device = device
        self.steps = []           # (l, kbr, kbh, n1, extra, n_out, nb, units, img_off, bias_off)
        shapes = []
        off = 0
        for (l, kbr, kbh, n1, x) in self.layout(plan, need_pos, need_dir):
            nb = n1 + (x.k_pad // 32 if x is not None else 0)
            units = 4 * (kbr + kbh)
            shapes.append((l, kbr, kbh, n1, x, nb, units, off))
            off += nb * units * 1024
        src_codes, dst_codes = [], []
        for (l, kbr, kbh, n1, x, nb, units, img_off) in shapes:
            self.steps.append((l, kbr, kbh, n1, x, 32 * nb, nb, units, img_off, off))
            s, d = self._maps(plan.layers[l], l, kbr, kbh, n1, x, nb, units, img_off, off)
            src_codes.append(s)
            dst_codes.append(d)
            off += nb * 128
        self.image_bytes = off
        self.image = torch.zeros(off // 2, dtype=torch.bfloat16, device=device)
        self.map_src = torch.from_numpy(np.concatenate(src_codes).astype(np.int32)).to(device)
        self.map_dst = torch.from_numpy(np.concatenate(dst_codes).astype(np.int32)).to(device)

    @staticmethod
    def _maps(lp, l, kbr, kbh, n1, x, nb, units, off, bias_off):
        """A fragment (row i = input feature k of layer l, column = its output n) = W_l[n][k];
        n permuted like the previous step's accumulator layout when register-fed, natural when
        it is an HBM-fed gradient (head output, density column); rows of chunks >= n1 are the
        columns of the encoding input x; biases zero."""
        N, K_orig = lp.module.out_features, lp.module.in_features
        lane = np.arange(64)
        srow, grp = lane & 15, lane >> 4
        j = np.arange(8)
        kb_total = kbr + kbh
        nidx = np.full((kb_total, 64, 8), -1, dtype=np.int64)
        for kb in range(kbr):
            nidx[kb] = 32 * kb + 16 * (j[None, :] >> 2) + 4 * grp[:, None] + (j[None, :] & 3)
        for kh in range(kbh):
            # HBM-fed gradient columns follow the register-fed ones (natural order)
            local = 32 * kbr + 32 * kh + 8 * grp[:, None] + j[None, :]
            nidx[kbr + kh] = np.where(local < N, local, -1)
        orig = {}
        o = 0
        for s_ in lp.sources:
            orig[id(s_)] = o
            o += s_.k_valid
        act_valid = lp.sources[0].k_valid if lp.sources[0].kind == "act" else 0
        srcs, dsts = [], []
        for c in range(nb):
            base = off + c * units * 1024
            for bb in range(2):
                if c < n1:
                    k = 32 * c + 16 * bb + srow
                    kcol = np.where(k < act_valid, k, -1)
                else:
                    local = 32 * (c - n1) + 16 * bb + srow
                    kcol = np.where(local < x.k_valid, orig[id(x)] + local, -1)
                kk = np.broadcast_to(kcol[None, :, None], nidx.shape)
                valid = (nidx >= 0) & (nidx < N) & (kk >= 0)
                code = np.where(valid, ((2 * l) << 24) + nidx * K_orig + kk, -1)
                dst = (base + np.arange(kb_total)[:, None, None] * 4096 + bb * 2048) // 2 + \
                    lane[None, :, None] * 8 + j[None, None, :]
                srcs.append(code.reshape(-1))
                dsts.append(np.broadcast_to(dst, nidx.shape).reshape(-1))
            srcs.append(np.full(32, -1))
            dsts.append(~(bias_off // 4 + 32 * c + np.arange(32)))
        return np.concatenate(srcs), np.concatenate(dsts)

    def pack(self):
        _pack_image(self)

    def run(self, M: int, g_head: torch.Tensor, dY, masks, g_cols=None, x_out=None):
        """g_head: [M, ld] gradient of the last layer's output; g_cols: {layer: [M, 4] buffer whose
        column 0 is the gradient of the layer's column output}; x_out: {layer: [M, k_pad] buffer for
        the gradient of the layer's encoding input}.  Fills dY[l] ([M, out_ld] fp32, the columns of
        the register-fed chain) for l = L-2 .. 0 on the current stream."""
        g_cols = g_cols or {}
        x_out = x_out or {}
        self.pack()
        S = len(self.steps)
        descs = (_lib.NerfFusedLayer * S)()
        flops = 0.0
        nbytes = 0.0
        for i, (l, kbr, kbh, n1, x, n_out, nb, units, img_off, bias_off) in enumerate(self.steps):
            lp = self.plan.layers[l]
            d = descs[i]
            d.type = FUSED_TYPES[(kbr, kbh)]
            d.N = n_out
            d.nb = nb
            d.relu = 0
            d.nseg = 1 if kbh else 0
            if kbh:
                src = g_head if kbr == 0 else g_cols[l]
                d.seg_kb[0] = 1
                d.seg_k[0] = (lp.N + 3) // 4 * 4 if kbr == 0 else 4
                d.seg_rd[0] = 1
                d.seg_rows[0] = src.shape[0]
                d.seg_ld[0] = src.stride(0)
                d.seg_ptr[0] = src.data_ptr()
            d.chunk_units = units
            d.col_idx = -1
            if l >= 1:
                d.out = dY[l - 1].data_ptr()
                d.ldo = dY[l - 1].stride(0)
                mk = masks[l - 1] if self.plan.layers[l - 1].relu else None
                d.mask_in = mk.data_ptr() if mk is not None else None
            else:                                      # the last step only produces encoding gradients
                d.out = x_out[l].data_ptr()
                d.ldo = x_out[l].stride(0)
                d.mask_in = None
            d.mask = None
            d.col_out = None
            if x is not None:
                d.out2 = x_out[l].data_ptr()
                d.ldo2 = x_out[l].stride(0)
                d.n1 = n1
            d.img_off = img_off
            d.bias_off = bias_off
            flops += 2.0 * M * lp.module.out_features * n_out
            # algorithmic bytes: HBM-fed gradients and ReLU bits read, dY / encoding gradients written
            nbytes += (4.0 * d.seg_k[0] * d.seg_rows[0] if kbh else 0.0) + (32.0 * M if d.mask_in else 0.0)
            nbytes += 4.0 * M * min(d.ldo, n_out) + (4.0 * M * d.ldo2 if x is not None else 0.0)
        end = K.TIMER.bracket("mlp_fused_dgrad", flops, nbytes + self.image.numel() * self.image.element_size(),
                              fn="mlp_fused_fwd_kernel") \
            if K.TIMER is not None else None
        st = _lib.load().nerf_mlp_fused_fwd(descs, S, self.image.data_ptr(), M, K._stream(self.device))
        if end is not None:
            end.record()
        _lib.check(st, "nerf_mlp_fused_fwd (input-gradient chain)")
        FusedInputGrad.runs += 1
