"""Lowering of a field-MLP plan onto the fused forward kernel (csrc/mlp_fused.hip).

``nerf_mlp_fused_fwd`` runs every Linear (+ bias + ReLU) of a NerfModel
(barf/model_interpolation_architecture.py:96-141) in one launch, keeping each wave's
activations in registers between layers.  This module decides whether a plan fits the
kernel, builds the packed weight image (MFMA-fragment order, split hi/lo bf16, biases) and
the per-layer descriptors, and launches it.  Outputs are exactly those of the layer-by-layer
forward in mlp.py (every layer's output, the ReLU mask bits, the density column), so the
backward is unchanged.

Image layout (mirrors the kernel header): per layer, 16-row output chunks c (rows 16 c .. 16 c + 15);
for every 32-deep k-block one A fragment of v_mfma_f32_16x16x32_bf16 as [hi 64 lanes x 16 B][lo 64
lanes x 16 B]; lane l (s = l & 15, g = l >> 4) element j is W[16 c + s][k(kb, g, j)] with
  k = 32 kb + 16 (j >> 2) + 4 g + (j & 3)          register-fed input (previous layer output)
  k = seg_offset + 32 kh + 8 g + j                  HBM-fed segment block kh (encodings)
The register-fed blocks of a chunk are contiguous ([c][kb], 2 KB each: one LDS-DMA stream), the
HBM-fed ones live in a second region ([c][kh]) and the biases in a third ([c][16] fp32).
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


def _flags(passes: int) -> int:
    """nerf_mlp_fused_run flags of a pass count (3: the 3 x bf16 split, 1: NERF_FUSED_BF16)."""
    if passes not in (1, 3):
        raise ValueError(f"fused MLP: passes must be 1 or 3 (got {passes})")
    return _lib.NERF_FUSED_BF16 if passes == 1 else 0


FUSED_TYPES = {(0, 1): 1, (0, 2): 2, (4, 0): 3, (8, 0): 6, (8, 1): 7, (8, 2): 8}   # (kbr, kbh) -> type
ENABLED = os.environ.get("NERF_FUSED", "1") != "0"     # A/B switch (bench, tests)
# a per-ray encoding read by a later layer comes from registers captured at the tile start; tests
# turn this off (NERF_FUSED_CAPTURE=0 or the module flag) to check that the library refuses the HBM
# read-back instead (the ordering rule)
CAPTURE_PER_RAY = os.environ.get("NERF_FUSED_CAPTURE", "1") != "0"


def _layer_shape(plan, idx):
    """(kbr, hbm sources, act source) of layer idx, or None if the kernel cannot run it."""
    lp = plan.layers[idx]
    if lp.gauss is not None or lp.tanh or lp.residual >= 0:
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


def _fragment_maps(n16, kbr, kbh, row_of, red_reg, red_hbm, elem, img_off, hbm_off, bias_off, bias_code):
    """Gather maps (source code: tensor << 24 | element, -1 = 0; destination: bf16 index of hi, or
    ~fp32 word) of one layer's image: row_of(c) -> [16] weight rows of 16-row chunk c (-1 absent),
    red_reg(kb) / red_hbm(kh) -> [64, 8] reduction indices of a register- / HBM-fed block (-1
    absent), elem(rows[64,1], red[64,8]) -> codes (-1 where either is absent), bias_code(rows[16])."""
    lane = np.arange(64)
    srow = lane & 15
    jj = np.arange(8)
    srcs, dsts = [], []
    for c in range(n16):
        rows = row_of(c)                                   # [16]
        r = rows[srow][:, None]                            # [64, 1]
        for kb in range(kbr):
            base = (img_off + (c * kbr + kb) * 2048) // 2
            srcs.append(elem(r, red_reg(kb)).reshape(-1))
            dsts.append((base + lane[:, None] * 8 + jj[None, :]).reshape(-1))
        for kh in range(kbh):
            base = (hbm_off + (c * kbh + kh) * 2048) // 2
            srcs.append(elem(r, red_hbm(kh)).reshape(-1))
            dsts.append((base + lane[:, None] * 8 + jj[None, :]).reshape(-1))
        srcs.append(bias_code(rows))
        dsts.append(~(bias_off // 4 + 16 * c + np.arange(16)))
    return np.concatenate(srcs), np.concatenate(dsts)


def _red_reg(kb):
    """Reduction index of register-fed k-block kb, lane (s, g) element j: the previous layer's
    accumulator order 32 kb + 16 (j >> 2) + 4 g + (j & 3)."""
    lane = np.arange(64)
    g = (lane >> 4)[:, None]
    j = np.arange(8)[None, :]
    return 32 * kb + 16 * (j >> 2) + 4 * g + (j & 3)


def _layout_offsets(shapes):
    """Byte offsets of each layer's register-fed, HBM-fed and bias regions: (n16, kbr, kbh) per
    layer -> [(img_off, hbm_off, bias_off)], total bytes."""
    offs = []
    off = 0
    for n16, kbr, kbh in shapes:
        offs.append([off, 0, 0])
        off += n16 * kbr * 2048
    for i, (n16, kbr, kbh) in enumerate(shapes):
        offs[i][1] = off
        off += n16 * kbh * 2048
    for i, (n16, kbr, kbh) in enumerate(shapes):
        offs[i][2] = off
        off += n16 * 64
    return [tuple(o) for o in offs], off


class FusedForward:
    """Packed image + static descriptors of one plan on one device."""

    def __init__(self, plan, device):
        self.plan = plan
        self.device = device
        self.layers = []          # (kbr, kbh, hbm sources, nb, n16, img_off, hbm_off, bias_off)
        shapes = []
        for idx, lp in enumerate(plan.layers):
            kbr, hbm = _layer_shape(plan, idx)
            kbh = sum(s.k_pad // 32 for s in hbm)
            shapes.append(((lp.module.out_features + 15) // 16, kbr, kbh))
        offs, total = _layout_offsets(shapes)
        src_codes, dst_codes = [], []
        for idx, lp in enumerate(plan.layers):
            kbr, hbm = _layer_shape(plan, idx)
            n16, _, kbh = shapes[idx]
            nb = (lp.module.out_features + 31) // 32
            img_off, hbm_off, bias_off = offs[idx]
            self.layers.append((kbr, kbh, hbm, nb, n16, img_off, hbm_off, bias_off))
            s_, d_ = self._maps(idx, lp, kbr, hbm, n16, img_off, hbm_off, bias_off)
            src_codes.append(s_)
            dst_codes.append(d_)
        self.image_bytes = total
        self.image = torch.zeros(total // 2, dtype=torch.bfloat16, device=device)
        self.map_src = torch.from_numpy(np.concatenate(src_codes).astype(np.int32)).to(device)
        self.map_dst = torch.from_numpy(np.concatenate(dst_codes).astype(np.int32)).to(device)

    @staticmethod
    def _maps(idx, lp, kbr, hbm, n16, img_off, hbm_off, bias_off):
        N, K_orig = lp.module.out_features, lp.module.in_features
        tw, tb = 2 * idx, 2 * idx + 1
        orig = {}
        o = 0
        for s in lp.sources:
            orig[id(s)] = o
            o += s.k_valid
        lane = np.arange(64)
        g = (lane >> 4)[:, None]
        j = np.arange(8)[None, :]
        hbm_cols = []
        for s in hbm:
            for kh in range(s.k_pad // 32):
                local = 32 * kh + 8 * g + j
                hbm_cols.append(np.where(local < s.k_valid, orig[id(s)] + local, -1))

        def row_of(c):
            n = 16 * c + np.arange(16)
            return np.where(n < N, n, -1)

        def elem(r, red):
            ok = (r >= 0) & (red >= 0)
            return np.where(ok, (tw << 24) + r * K_orig + red, -1)

        return _fragment_maps(n16, kbr, len(hbm_cols), row_of, _red_reg, lambda kh: hbm_cols[kh], elem,
                              img_off, hbm_off, bias_off, lambda rows: np.where(rows >= 0, (tb << 24) + rows, -1))

    def pack(self):
        _pack_image(self)

    def run(self, M: int, pos: torch.Tensor, dirs: torch.Tensor | None, dir_rd: int, acts, masks, col_outs,
            gens=(None, None), comp=None, passes: int = 3):
        """Launch on the current stream.  acts[l]: [M, out_ld] fp32 or None (not stored),
        masks[l]: [M, 32] uint8 or None, col_outs: {layer: [M] fp32}.  gens: the DeferredEncoding
        of pos / dirs or None: generated in-kernel at every tile start (kernels.encode_fwd(defer=True))
        and stored into the tensor, which later layers read; the first layer reads them from LDS.
        comp: (CompositeSpec, rgb [B, 3], weights [B, S], sigma layer) — the rays composited at the
        end of every tile (nerf_mlp_fused_render), coefficients into spec.coef when it is set.
        passes: 3 (3 x bf16 split products) or 1 (one bf16 pass: matmul precision "medium")."""
        self.pack()
        L = len(self.plan.layers)
        descs = (_lib.NerfFusedLayer * L)()
        encs = (_lib.NerfFusedEncoding * 2)()
        gen_of = {}
        nbytes = 0.0
        # Ordering rule (csrc/mlp_fused.hip fused_launch): a later layer reads generated rows back from
        # HBM only when its own wave stored them (per-sample rows); a per-ray encoding read by a later
        # layer comes from the registers captured at the tile start (one 32-column block), else it is
        # filled before the launch.
        reg_kind = None
        for e, (kind, g) in enumerate((("pos", gens[0]), ("dir", gens[1]))):
            if g is None:
                continue
            later = [s for idx in range(1, L) for s in self.layers[idx][2] if s.kind == kind]
            if not any(s.kind == kind for idx in range(L) for s in self.layers[idx][2]):
                K.materialize(pos if kind == "pos" else dirs)      # not read by the kernel
                continue
            per_ray = g.spec.per_ray and (dir_rd if kind == "dir" else 1) > 1
            if later and per_ray and CAPTURE_PER_RAY and (reg_kind is not None or any(s.k_pad != 32 for s in later)):
                K.materialize(pos if kind == "pos" else dirs)      # filled by the encoding launch
                continue
            if later and per_ray and CAPTURE_PER_RAY:
                reg_kind = kind
            ctypes.memmove(ctypes.byref(encs[e]), ctypes.byref(g.spec), ctypes.sizeof(g.spec))
            if kind == "dir":
                encs[e].samples_per_ray = dir_rd
            gen_of[kind] = e + 1
            # generated at every tile start and stored: rows written once, the inputs read
            # (t_start [, t_end] per sample, o, d [, pw] per ray; directions per ray)
            t = pos if kind == "pos" else dirs
            nbytes += 4.0 * t.stride(0) * t.shape[0]
            nbytes += (8.0 * M + 28.0 * encs[e].n_rays) if not encs[e].per_ray else 12.0 * encs[e].n_rays
            if encs[e].params.kind == 2:
                # hash-grid features: 8 corners x F fp32 gathered per (sample, level)
                nbytes += 32.0 * M * encs[e].out_dim
        flops = 0.0
        for idx, lp in enumerate(self.plan.layers):
            kbr, kbh, hbm, nb, n16, off, hbm_off, bias_off = self.layers[idx]
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
                if idx == 0 and s.kind in gen_of:
                    # the first layer takes the rows generated at the tile start straight from LDS
                    d.seg_gen[si] = gen_of[s.kind]
                elif s.kind == reg_kind:
                    # a per-ray encoding: the block captured in registers at the tile start
                    d.seg_gen[si] = gen_of[s.kind]
                else:
                    # algorithmic bytes: an HBM-fed encoding read (generated ones: the rows the kernel
                    # stored at the tile start)
                    nbytes += 4.0 * d.seg_k[si] * d.seg_rows[si]
            d.chunk_units = 2 * kbr
            d.col_idx = -1
            # a layer without a tensor (inference: not an exposed output) has its stores dropped
            d.out = acts[idx].data_ptr() if acts[idx] is not None else None
            d.ldo = acts[idx].stride(0) if acts[idx] is not None else 0
            d.mask = masks[idx].data_ptr() if masks[idx] is not None else None
            if idx in col_outs:
                d.col_out = col_outs[idx].data_ptr()
                d.col_idx = dict(self.plan.column_outputs)[idx]
            d.img_off = off
            d.hbm_off = hbm_off
            d.bias_off = bias_off
            flops += 2.0 * M * lp.module.out_features * lp.module.in_features
            # algorithmic bytes: stored outputs / mask bits / columns written
            nbytes += (4.0 * M * acts[idx].shape[1] if acts[idx] is not None else 0.0) \
                + (32.0 * M if masks[idx] is not None else 0.0) + (4.0 * M if idx in col_outs else 0.0)
        cdesc = None
        if comp is not None:
            spec, rgb, w, sl = comp
            cdesc = _lib.NerfFusedComposite()
            cdesc.dist = spec.dist.data_ptr()
            cdesc.rgb = rgb.data_ptr()
            cdesc.weights = w.data_ptr() if w is not None else None
            cdesc.coef = spec.coef.data_ptr() if spec.coef is not None else None
            cdesc.samples_per_ray = spec.S
            cdesc.head_layer = L - 1
            cdesc.sigma_layer = sl
            cdesc.scale_a, cdesc.scale_b, cdesc.density_shift = spec.sa, spec.sb, spec.shift
            # algorithmic bytes: interval lengths in; rgb, weights, coefficients out
            nbytes += 4.0 * M + 12.0 * (M // spec.S) + (4.0 * M if w is not None else 0.0) \
                + (32.0 * M if spec.coef is not None else 0.0)
        end = K.TIMER.bracket("mlp_fused_fwd", flops, nbytes + self.image.numel() * self.image.element_size(),
                              fn="mlp_fused_kernel<0>" if passes == 3 else "mlp_fused_kernel<2>") \
            if K.TIMER is not None else None
        st = _lib.load().nerf_mlp_fused_run(descs, L, self.image.data_ptr(), M, encs if gen_of else None,
                                            ctypes.byref(cdesc) if cdesc is not None else None,
                                            _flags(passes), K._stream(self.device))
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
        self.steps = []           # (l, kbr, kbh, n1, extra, n_out, nb, img_off, hbm_off, bias_off)
        lay = self.layout(plan, need_pos, need_dir)
        shapes = []
        for (l, kbr, kbh, n1, x) in lay:
            nb = n1 + (x.k_pad // 32 if x is not None else 0)
            shapes.append((2 * nb, kbr, kbh))
        offs, total = _layout_offsets(shapes)
        src_codes, dst_codes = [], []
        for (l, kbr, kbh, n1, x), (n16, _, _), (img_off, hbm_off, bias_off) in zip(lay, shapes, offs):
            nb = n16 // 2
            self.steps.append((l, kbr, kbh, n1, x, 32 * nb, nb, img_off, hbm_off, bias_off))
            s_, d_ = self._maps(plan.layers[l], l, kbr, kbh, n1, x, n16, img_off, hbm_off, bias_off)
            src_codes.append(s_)
            dst_codes.append(d_)
        self.image_bytes = total
        self.image = torch.zeros(total // 2, dtype=torch.bfloat16, device=device)
        self.map_src = torch.from_numpy(np.concatenate(src_codes).astype(np.int32)).to(device)
        self.map_dst = torch.from_numpy(np.concatenate(dst_codes).astype(np.int32)).to(device)

    @staticmethod
    def _maps(lp, l, kbr, kbh, n1, x, n16, img_off, hbm_off, bias_off):
        """A fragment (row = input feature k of layer l, reduction = its output n) = W_l[n][k]; n
        permuted like the previous step's accumulator layout when register-fed, natural when it is
        an HBM-fed gradient (head output, density column); rows of chunks >= 2 n1 are the columns of
        the encoding input x; biases zero."""
        N, K_orig = lp.module.out_features, lp.module.in_features
        lane = np.arange(64)
        g = (lane >> 4)[:, None]
        j = np.arange(8)[None, :]
        orig = {}
        o = 0
        for s_ in lp.sources:
            orig[id(s_)] = o
            o += s_.k_valid
        act_valid = lp.sources[0].k_valid if lp.sources[0].kind == "act" else 0

        def row_of(c):
            i = np.arange(16)
            if c < 2 * n1:
                k = 16 * c + i
                return np.where(k < act_valid, k, -1)
            local = 16 * (c - 2 * n1) + i
            return np.where(local < x.k_valid, orig[id(x)] + local, -1)

        def red_reg(kb):
            n = _red_reg(kb)
            return np.where(n < N, n, -1)

        def red_hbm(kh):
            n = 32 * kbr + 32 * kh + 8 * g + j
            return np.where(n < N, n, -1)

        def elem(r, red):
            ok = (r >= 0) & (red >= 0)
            return np.where(ok, ((2 * l) << 24) + red * K_orig + r, -1)

        return _fragment_maps(n16, kbr, kbh, row_of, red_reg, red_hbm, elem, img_off, hbm_off, bias_off,
                              lambda rows: np.full(16, -1))

    def pack(self):
        _pack_image(self)

    def run(self, M: int, g_head: torch.Tensor | None, dY, masks, g_cols=None, x_out=None, comp=None,
            passes: int = 3):
        """g_head: [M, ld] gradient of the last layer's output; g_cols: {layer: [M, 4] buffer whose
        column 0 is the gradient of the layer's column output}; x_out: {layer: [M, k_pad] buffer for
        the gradient of the layer's encoding input}.  Fills dY[l] ([M, out_ld] fp32, the columns of
        the register-fed chain) for l = L-2 .. 0 on the current stream.  comp: (CompositeSpec,
        grad_rgb [B, 3], head-gradient rows [M, >=4], density-gradient rows (a [M, >=4] view) or
        None, sigma layer) — the head and density blocks are formed in-kernel from the fused
        compositing's coefficients (seg_gen 3 / 4) and stored to those rows."""
        g_cols = g_cols or {}
        x_out = x_out or {}
        self.pack()
        S = len(self.steps)
        descs = (_lib.NerfFusedLayer * S)()
        flops = 0.0
        nbytes = 0.0
        for i, (l, kbr, kbh, n1, x, n_out, nb, img_off, hbm_off, bias_off) in enumerate(self.steps):
            lp = self.plan.layers[l]
            d = descs[i]
            d.type = FUSED_TYPES[(kbr, kbh)]
            d.N = n_out
            d.nb = nb
            d.relu = 0
            d.nseg = 1 if kbh else 0
            if kbh and comp is not None:
                # the composite's head (first step) / density (the density layer's step) gradient
                coef = comp[0].coef
                d.seg_kb[0] = 1
                d.seg_k[0] = 8
                d.seg_rd[0] = 1
                d.seg_rows[0] = coef.shape[0]
                d.seg_ld[0] = 8
                d.seg_ptr[0] = coef.data_ptr()
                d.seg_gen[0] = 3 if kbr == 0 else 4
            elif kbh:
                src = g_head if kbr == 0 else g_cols[l]
                d.seg_kb[0] = 1
                d.seg_k[0] = (lp.N + 3) // 4 * 4 if kbr == 0 else 4
                d.seg_rd[0] = 1
                d.seg_rows[0] = src.shape[0]
                d.seg_ld[0] = src.stride(0)
                d.seg_ptr[0] = src.data_ptr()
            d.chunk_units = 2 * kbr
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
            d.hbm_off = hbm_off
            d.bias_off = bias_off
            flops += 2.0 * M * lp.module.out_features * n_out
            # algorithmic bytes: HBM-fed gradients and ReLU bits read, dY / encoding gradients written
            nbytes += (4.0 * d.seg_k[0] * d.seg_rows[0] if kbh else 0.0) + (32.0 * M if d.mask_in else 0.0)
            nbytes += 4.0 * M * min(d.ldo, n_out) + (4.0 * M * d.ldo2 if x is not None else 0.0)
        cdesc = None
        if comp is not None:
            spec, g_rgb, gh, gsig, sl = comp
            cdesc = _lib.NerfFusedComposite()
            cdesc.grad_rgb = g_rgb.data_ptr()
            cdesc.grad_head = gh.data_ptr()
            cdesc.ld_head = gh.stride(0)
            cdesc.grad_sigma = gsig.data_ptr() if gsig is not None else None
            cdesc.ld_sigma = gsig.stride(0) if gsig is not None else 0
            cdesc.samples_per_ray = spec.S
            cdesc.head_layer = len(self.plan.layers) - 1
            cdesc.sigma_layer = sl
            # algorithmic bytes beyond the coefficient rows counted above: grad_rgb, the rows stored
            nbytes += 12.0 * (M // spec.S) + 16.0 * M * (2 if gsig is not None else 1)
        end = K.TIMER.bracket("mlp_fused_dgrad", flops, nbytes + self.image.numel() * self.image.element_size(),
                              fn="mlp_fused_kernel<1>" if passes == 3 else "mlp_fused_kernel<3>") \
            if K.TIMER is not None else None
        st = _lib.load().nerf_mlp_fused_run(descs, S, self.image.data_ptr(), M, None,
                                            ctypes.byref(cdesc) if cdesc is not None else None, _flags(passes),
                                            K._stream(self.device))
        if end is not None:
            end.record()
        _lib.check(st, "nerf_mlp_fused_fwd (input-gradient chain)")
        FusedInputGrad.runs += 1
