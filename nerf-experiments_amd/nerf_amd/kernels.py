"""Validated Python entry points for every C-ABI kernel.

Each function checks device, dtype, contiguity and shapes (raising ``ValueError``
like the reference's own asserts, e.g. positional_encodings.py:52,183 and
model_interpolation.py:175,285), allocates outputs with the PyTorch caching
allocator and launches on ``torch.cuda.current_stream()``.  No host
synchronisation happens anywhere in this module.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import torch

from . import _lib
from ._lib import NerfPEParams, NerfSeg


class KernelTimer:
    """Optional HIP-event bracketing of kernel launches (used by bench.py).

    Events are recorded on the same stream the kernel is launched on (torch's
    current stream, which is the stream passed to the C-ABI), so
    elapsed_time() is the kernel's device duration.  Records (tag, flops, algorithmic
    HBM bytes, start, end, kernel function).  ``tag`` names the role of a launch (e.g. the
    fused forward vs the input-gradient chain); ``fn`` is the HIP kernel function it runs, the
    name rocprofv3's kernel trace reports, so summary(by="fn") lines up with the rocprof stats."""

    def __init__(self):
        self.records = []

    def bracket(self, tag: str, flops: float = 0.0, nbytes: float = 0.0, fn: str | None = None, launches: int = 1):
        """launches: kernel launches inside the bracket (a wide layer's column blocks), so that the
        per-launch averages match rocprofv3's"""
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record()
        self.records.append((tag, flops, nbytes, start, end, fn or tag, launches))
        return end

    def summary(self, by: str = "tag"):
        out = {}
        for *_, e, _fn, _n in self.records:
            e.synchronize()                     # (every end event recorded: durations are final)
        for tag, flops, nbytes, s, e, fn, n in self.records:
            ms = s.elapsed_time(e)
            d = out.setdefault(fn if by == "fn" else tag,
                               {"launches": 0, "flops": 0.0, "bytes": 0.0, "ms": 0.0, "tags": set()})
            d["launches"] += n
            d["flops"] += flops
            d["bytes"] += nbytes
            d["ms"] += ms
            d["tags"].add(tag)
        for d in out.values():
            d["tags"] = sorted(d["tags"])
        return out


TIMER: KernelTimer | None = None


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _require_cuda_f32(name: str, t: torch.Tensor) -> None:
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must live on a ROCm device (got {t.device}); nerf_amd has no CPU path")
    if t.dtype != torch.float32:
        raise ValueError(f"{name} must be float32 (got {t.dtype})")


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


def pad128(n: int) -> int:
    return (n + 127) // 128 * 128


# ----------------------------------------------------------------------------- composite
def composite_fwd(density: torch.Tensor, density_stride: int, color: torch.Tensor, color_stride: int,
                  dist: torch.Tensor, n_rays: int, samples_per_ray: int, scale_a: float, scale_b: float,
                  act: bool, density_shift: float = 0.0, want_weights: bool = True):
    _require_cuda_f32("density", density)
    _require_cuda_f32("color", color)
    _require_cuda_f32("dist", dist)
    if not dist.is_contiguous() or dist.numel() != n_rays * samples_per_ray:
        raise ValueError("dist must be contiguous with n_rays*samples_per_ray elements")
    dev = dist.device
    rgb = torch.empty(n_rays, 3, device=dev, dtype=torch.float32)
    w = torch.empty(n_rays, samples_per_ray, device=dev, dtype=torch.float32) if want_weights else None
    n = n_rays * samples_per_ray
    # algorithmic bytes: sigma, rgb, delta in (+ weights out) per sample, rgb out per ray
    end = TIMER.bracket("composite_fwd", nbytes=n * (20 + (4 if want_weights else 0)) + 12 * n_rays,
                        fn="composite_fwd_kernel") \
        if TIMER is not None else None
    st = _lib.load().nerf_composite_fwd(_ptr(density), density_stride, _ptr(color), color_stride, _ptr(dist),
                                        n_rays, samples_per_ray, scale_a, scale_b, int(act), density_shift,
                                        _ptr(rgb), _ptr(w), _stream(dev))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_composite_fwd")
    return rgb, w


def composite_bwd(density, density_stride, color, color_stride, dist, n_rays, samples_per_ray, scale_a, scale_b,
                  act, density_shift, grad_rgb, grad_weights, grad_density, gd_stride, grad_color, gc_stride):
    grad_rgb = grad_rgb.contiguous()
    if grad_weights is not None:
        grad_weights = grad_weights.contiguous()
    n = n_rays * samples_per_ray
    # algorithmic bytes: sigma, rgb, delta (+ dL/dw) in, dL/dsigma, dL/drgb out per sample; dL/drgb in per ray
    nb = n * (20 + (4 if grad_weights is not None else 0) + (4 if grad_density is not None else 0)
              + (12 if grad_color is not None else 0)) + 12 * n_rays
    end = TIMER.bracket("composite_bwd", nbytes=nb, fn="composite_bwd_kernel") if TIMER is not None else None
    st = _lib.load().nerf_composite_bwd(_ptr(density), density_stride, _ptr(color), color_stride, _ptr(dist),
                                        n_rays, samples_per_ray, scale_a, scale_b, int(act), density_shift,
                                        _ptr(grad_rgb), _ptr(grad_weights), _ptr(grad_density), gd_stride,
                                        _ptr(grad_color), gc_stride, _stream(dist.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_composite_bwd")


# ----------------------------------------------------------------------------- sampling
def sample_uniform(n_rays: int, samples_per_ray: int, near: float, far: float, stratified: bool,
                   offset_size: float, seed: int, counter: int, device: torch.device):
    t0 = torch.empty(n_rays, samples_per_ray, device=device, dtype=torch.float32)
    t1 = torch.empty_like(t0)
    st = _lib.load().nerf_sample_uniform(n_rays, samples_per_ray, near, far, int(stratified), offset_size,
                                         seed, counter, _ptr(t0), _ptr(t1), _stream(device))
    _lib.check(st, "nerf_sample_uniform")
    return t0, t1


def ray_batch(indices: torch.Tensor, H: int, W: int, focal: float, c2w: torch.Tensor, noise_rot, noise_trans,
              images: torch.Tensor, blur: tuple[int, int, int, float, float] | None, want_raw_colors: bool,
              status: torch.Tensor):
    """nerf_ray_batch: (o_raw, o_noisy, d_raw, d_noisy, colors_raw or None, colors_pair or None, img_idx).
    blur = (mode, lo, hi, coef_lo, coef_hi) or None (no pair output)."""
    dev = indices.device
    B = indices.shape[0]
    n_img, n_sigma = c2w.shape[0], images.shape[-2]
    for name, t in (("indices", indices), ("c2w", c2w), ("images", images)):
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    if indices.dtype != torch.int64 or images.shape[:3] != (n_img, H, W) or images.shape[-1] != 3:
        raise ValueError("indices int64 [B]; images [n_img, H, W, n_sigma, 3]")
    f = dict(device=dev, dtype=torch.float32)
    o_raw, d_raw = torch.empty(B, 3, **f), torch.empty(B, 3, **f)
    o_noisy, d_noisy = torch.empty(B, 3, **f), torch.empty(B, 3, **f)
    craw = torch.empty(B, n_sigma, 3, **f) if want_raw_colors else None
    cpair = torch.empty(B, 2, 3, **f) if blur is not None else None
    img_idx = torch.empty(B, device=dev, dtype=torch.int64)
    mode, lo, hi, ca, cb = blur if blur is not None else (0, 0, 0, 0.0, 0.0)
    st = _lib.load().nerf_ray_batch(_ptr(indices), B, H, W, focal, _ptr(c2w), _ptr(noise_rot), _ptr(noise_trans),
                                    n_img, _ptr(images), n_sigma, mode, lo, hi, ca, cb, _ptr(o_raw), _ptr(o_noisy),
                                    _ptr(d_raw), _ptr(d_noisy), _ptr(craw), _ptr(cpair), _ptr(img_idx),
                                    _ptr(status), _stream(dev))
    _lib.check(st, "nerf_ray_batch")
    return o_raw, o_noisy, d_raw, d_noisy, craw, cpair, img_idx


def resample_pdf(t_coarse: torch.Tensor, weights: torch.Tensor, dist_coarse: torch.Tensor, n_samples: int,
                 mode: int, near: float, far: float, seed: int, counter: int, status: torch.Tensor | None = None):
    for name, t in (("t_coarse", t_coarse), ("weights", weights), ("distances_coarse", dist_coarse)):
        _require_cuda_f32(name, t)
    if t_coarse.dim() != 2 or weights.shape != t_coarse.shape or dist_coarse.shape != t_coarse.shape:
        raise ValueError("t_coarse, weights and distances_coarse must share shape (batch_size, n_bins)")
    t_coarse, weights, dist_coarse = t_coarse.contiguous(), weights.contiguous(), dist_coarse.contiguous()
    n_rays, n_bins = t_coarse.shape
    if n_samples < n_bins:
        raise ValueError("n_samples must be >= the number of coarse bins")
    dev = t_coarse.device
    t0 = torch.empty(n_rays, n_samples, device=dev, dtype=torch.float32)
    t1 = torch.empty_like(t0)
    if status is None:
        status = torch.zeros(1, device=dev, dtype=torch.int32)
    st = _lib.load().nerf_resample_pdf(_ptr(t_coarse), _ptr(weights), _ptr(dist_coarse), n_rays, n_bins,
                                       n_samples, mode, near, far, seed, counter, _ptr(t0), _ptr(t1),
                                       _ptr(status), _stream(dev))
    _lib.check(st, "nerf_resample_pdf")
    return t0, t1, status


# ----------------------------------------------------------------------------- encodings
def make_pe_params(kind: int, levels: int, include_identity: bool, scale: float, query: int = 1,
                   pixel_width_sigma: float = 0.0, distribute_variance: bool = False, pw_mode: int = 2,
                   mask: Sequence[float] | None = None) -> NerfPEParams:
    if levels > 16:
        raise ValueError("levels > 16 is not supported")
    p = NerfPEParams()
    p.kind = kind
    p.levels = levels
    p.include_identity = int(bool(include_identity))
    p.query = query
    p.scale = scale
    p.pixel_width_sigma = pixel_width_sigma
    p.distribute_variance = int(bool(distribute_variance))
    p.pw_mode = pw_mode
    if mask is not None:
        p.use_mask = 1
        for i, m in enumerate(mask):
            p.mask[i] = float(m)
    else:
        p.use_mask = 0
    return p


def encode_fwd(params: NerfPEParams, out_dim: int, *, x=None, xdir=None, ray_o=None, ray_d=None, t_start=None,
               t_end=None, pixel_width=None, n_samples: int, samples_per_ray: int = 1, n_rays: int = 0,
               out_ld: int | None = None, device=None, defer: bool = False) -> torch.Tensor:
    """[n_samples, out_ld] encoding (nerf_encode_fwd).  defer=True: when the encoding can be generated
    inside the fused field-MLP kernel (ray-mode positions, or per-ray Fourier features of
    directions), the rows are left to that kernel: the tensor is returned unfilled, carrying a
    DeferredEncoding that the consumer either hands to the kernel or fills (see materialize)."""
    ld = out_ld if out_ld is not None else pad32(out_dim)
    for name, t in (("x", x), ("dir", xdir), ("ray_origs", ray_o), ("ray_dirs", ray_d), ("t_start", t_start),
                    ("t_end", t_end), ("pixel_width", pixel_width)):
        if t is not None:
            _require_cuda_f32(name, t)
            if not t.is_contiguous():
                raise ValueError(f"{name} must be contiguous")
    out = torch.empty(n_samples, ld, device=device, dtype=torch.float32)

    def fill(out):
        end = None
        if TIMER is not None:
            # algorithmic bytes: the encoding's out_dim columns written, its inputs read once
            per_sample = 4 * out_dim
            if x is not None:
                per_sample += 12 + (12 if params.kind == 1 else 0) + (12 if params.kind == 1 else 0)
                per_ray = 0
            else:
                per_sample += 4 + (4 if (params.query == 1 or params.kind == 1) else 0)
                per_ray = 24 + (4 if params.kind == 1 else 0)
            end = TIMER.bracket("encode_fwd", nbytes=n_samples * per_sample + n_rays * per_ray,
                                fn="encode_fwd_lds_kernel" if ld <= 128 else "encode_fwd_kernel")
        st = _lib.load().nerf_encode_fwd(ctypes.byref(params), _ptr(x), _ptr(xdir), _ptr(ray_o), _ptr(ray_d),
                                         _ptr(t_start), _ptr(t_end), _ptr(pixel_width), n_samples, samples_per_ray,
                                         n_rays, _ptr(out), ld, _stream(out.device))
        if end is not None:
            end.record()
        _lib.check(st, "nerf_encode_fwd")

    if defer and n_samples > 0 and (x is None or (xdir is None and params.kind == 0)):
        if os.environ.get("NERF_POISON_DEFERRED", "0") == "1":
            # tests (tests/conftest.py): rows read before the kernel wrote them come out NaN every time
            out.fill_(float("nan"))
        e = _lib.NerfFusedEncoding()
        e.params = params
        if x is None:
            e.ray_o, e.ray_d, e.t_start, e.t_end = _ptr(ray_o), _ptr(ray_d), _ptr(t_start), _ptr(t_end)
            e.pixel_width = _ptr(pixel_width)
            e.samples_per_ray, e.n_rays, e.per_ray = samples_per_ray, n_rays, 0
        else:
            # per-row features of x (directions): generated per sample from ray m / samples_per_ray,
            # the divisor being the consumer's (set when the kernel is launched)
            e.ray_d = _ptr(x)
            e.samples_per_ray, e.n_rays, e.per_ray = 1, n_samples, 1
        e.out, e.ld, e.out_dim = _ptr(out), ld, out_dim
        # keep holds the inputs whose pointers the spec carries; NOT out itself (the tensor owns the
        # spec: a reference back to it would be a cycle holding the rows' HBM until the cycle GC)
        out._nerf_deferred = DeferredEncoding(e, (x, ray_o, ray_d, t_start, t_end, pixel_width), fill)
        return out
    fill(out)
    return out


class DeferredEncoding:
    """The pending rows of an encoding output: ``spec`` (nerf_fused_encoding: what the fused field
    MLP needs to generate them in-kernel; its input pointers stay valid through ``keep``, its output
    pointer through the tensor that owns this object) and ``fill(out)`` (the stand-alone encoding
    launch, for any other consumer).  Deferral is internal to NerfModel.render_raw /
    render_composite → MLPFunction, which either hands the spec to the fused kernel or materializes
    the rows first; any other reader must call ``materialize`` before touching the rows."""

    __slots__ = ("spec", "keep", "fill")

    def __init__(self, spec, keep, fill):
        self.spec, self.keep, self.fill = spec, keep, fill


def deferred(t) -> "DeferredEncoding | None":
    return getattr(t, "_nerf_deferred", None) if t is not None else None


def materialize(t) -> None:
    """Fill a deferred encoding's rows now (no-op for an ordinary tensor)."""
    d = deferred(t)
    if d is not None:
        t._nerf_deferred = None
        d.fill(t)


def mark_filled(t) -> None:
    """The fused kernel has written a deferred encoding's rows."""
    if deferred(t) is not None:
        t._nerf_deferred = None


def encode_bwd(params: NerfPEParams, x: torch.Tensor, grad_out: torch.Tensor, dx: torch.Tensor | None = None,
               accumulate: bool = False) -> torch.Tensor:
    n = x.shape[0]
    if dx is None:
        dx = torch.empty(n, 3, device=x.device, dtype=torch.float32)
    if grad_out.stride(1) != 1:
        grad_out = grad_out.contiguous()
    st = _lib.load().nerf_encode_bwd(ctypes.byref(params), _ptr(x), _ptr(grad_out), grad_out.stride(0), n,
                                     _ptr(dx), int(accumulate), _stream(x.device))
    _lib.check(st, "nerf_encode_bwd")
    return dx


def encode_bwd_integrated(params: NerfPEParams, x: torch.Tensor, xdir: torch.Tensor, t_start: torch.Tensor,
                          t_end: torch.Tensor, pixel_width: torch.Tensor, grad_out: torch.Tensor, want_dx: bool,
                          want_ddir: bool):
    """(dx, ddir) of an integrated encoding; per-sample t_start / t_end / pixel_width rows."""
    n = x.shape[0]
    dx = torch.empty(n, 3, device=x.device, dtype=torch.float32) if want_dx else None
    ddir = torch.empty(n, 3, device=x.device, dtype=torch.float32) if want_ddir else None
    if grad_out.stride(1) != 1:
        grad_out = grad_out.contiguous()
    st = _lib.load().nerf_encode_bwd_integrated(ctypes.byref(params), _ptr(x), _ptr(xdir), _ptr(t_start),
                                                _ptr(t_end), _ptr(pixel_width), _ptr(grad_out), grad_out.stride(0),
                                                n, _ptr(dx), _ptr(ddir), 0, _stream(x.device))
    _lib.check(st, "nerf_encode_bwd_integrated")
    return dx, ddir


def encode_bwd_rays(params: NerfPEParams, ray_o: torch.Tensor, ray_d: torch.Tensor, t_start: torch.Tensor,
                    t_end: torch.Tensor, pixel_width: torch.Tensor | None, grad_out: torch.Tensor,
                    samples_per_ray: int, want_do: bool, want_dd: bool):
    """(dL/d origins, dL/d directions) [n_rays, 3] of a ray-mode encoding."""
    n_rays = ray_o.shape[0]
    d_o = torch.empty(n_rays, 3, device=ray_o.device, dtype=torch.float32) if want_do else None
    d_d = torch.empty(n_rays, 3, device=ray_o.device, dtype=torch.float32) if want_dd else None
    if grad_out.stride(1) != 1:
        grad_out = grad_out.contiguous()
    st = _lib.load().nerf_encode_bwd_rays(ctypes.byref(params), _ptr(ray_o), _ptr(ray_d), _ptr(t_start),
                                          _ptr(t_end), _ptr(pixel_width), _ptr(grad_out), grad_out.stride(0), n_rays,
                                          samples_per_ray, _ptr(d_o), _ptr(d_d), 0, _stream(ray_o.device))
    _lib.check(st, "nerf_encode_bwd_rays")
    return d_o, d_d


# ----------------------------------------------------------------------------- optimizer
def adam_step(entries, beta1: float, beta2: float, eps: float, device) -> None:
    """entries: (param, grad, exp_avg, exp_avg_sq, step_size, bc2_sqrt, weight_decay) of fp32
    contiguous device tensors; one nerf_adam_step launch per NERF_ADAM_MAX_TENSORS entries."""
    lib = _lib.load()
    cap = _lib.NERF_ADAM_MAX_TENSORS
    for c in range(0, len(entries), cap):
        chunk = entries[c:c + cap]
        b = _lib.NerfAdamBatch()
        b.n_tensors = len(chunk)
        b.beta1, b.beta2, b.eps = beta1, beta2, eps
        b.one_minus_beta1, b.one_minus_beta2 = 1 - beta1, 1 - beta2
        for i, (p, g, m, v, step, bc2s, wd) in enumerate(chunk):
            for name, t in (("param", p), ("grad", g), ("exp_avg", m), ("exp_avg_sq", v)):
                _require_cuda_f32(name, t)
                if not t.is_contiguous() or t.numel() != p.numel():
                    raise ValueError(f"adam: {name} must be contiguous with the parameter's size")
            b.param[i], b.grad[i], b.exp_avg[i], b.exp_avg_sq[i] = p.data_ptr(), g.data_ptr(), m.data_ptr(), \
                v.data_ptr()
            b.numel[i] = p.numel()
            b.step_size[i], b.bc2_sqrt[i], b.weight_decay[i] = step, bc2s, wd
        _lib.check(lib.nerf_adam_step(ctypes.byref(b), _stream(device)), "nerf_adam_step")


# ----------------------------------------------------------------------------- gaussian activation
def gauss_act_fwd(z: torch.Tensor, N: int, inv_std: torch.Tensor, y: torch.Tensor) -> None:
    _require_cuda_f32("inv_standard_deviation", inv_std)
    end = TIMER.bracket("gauss_act_fwd", 0.0, 8.0 * z.shape[0] * N, fn="gauss_fwd_kernel") \
        if TIMER is not None else None
    st = _lib.load().nerf_gauss_act_fwd(_ptr(z), z.stride(0), _ptr(inv_std), z.shape[0], N, _ptr(y), y.stride(0),
                                        _stream(z.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_gauss_act_fwd")


def gauss_act_bwd(grad_y: torch.Tensor, z: torch.Tensor, N: int, inv_std: torch.Tensor, grad_z: torch.Tensor,
                  grad_inv_std: torch.Tensor) -> None:
    M = z.shape[0]
    lib = _lib.load()
    ws = torch.empty(max(1, (int(lib.nerf_gauss_act_workspace(M, N)) + 7) // 8), device=z.device,
                     dtype=torch.float64)
    end = TIMER.bracket("gauss_act_bwd", 0.0, 12.0 * M * N, fn="gauss_bwd_kernel") if TIMER is not None else None
    st = lib.nerf_gauss_act_bwd(_ptr(grad_y), grad_y.stride(0), _ptr(z), z.stride(0), _ptr(inv_std), M, N,
                                _ptr(grad_z), grad_z.stride(0), _ptr(grad_inv_std), 0, _ptr(ws),
                                ws.numel() * 8, _stream(z.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_gauss_act_bwd")


# ----------------------------------------------------------------------------- linear layers
def make_segs(segs: Sequence[tuple[torch.Tensor, int, int]]):
    """segs: (tensor, k, row_div) with k % 4 == 0 valid columns; the tensor's row
    stride is its ld.  In the packed weight layout each segment occupies
    pad32(k) columns."""
    arr = (NerfSeg * len(segs))()
    for i, (t, k, rd) in enumerate(segs):
        if t.stride(1) != 1:
            raise ValueError("linear operand segments must be row-major")
        arr[i].ptr = t.data_ptr()
        arr[i].ld = t.stride(0)
        arr[i].k = k
        arr[i].row_div = rd
    return arr


def _segs_bytes(segs, M: int) -> float:
    """Algorithmic bytes of a segmented fp32 operand: every row of every segment read once."""
    return sum(4.0 * k * ((M + rd - 1) // rd) for _, k, rd in segs)


def linear_fwd(segs, M: int, W: torch.Tensor, ldw: int, N: int, bias: torch.Tensor | None, out: torch.Tensor,
               epilogue: int, aux: torch.Tensor | None = None, w_row_offset: int = 0) -> None:
    arr = make_segs(segs)
    wptr = W.data_ptr() + w_row_offset * ldw * 4
    end = TIMER.bracket("linear_nt", 2.0 * M * N * ldw, _segs_bytes(segs, M) + 4.0 * M * N + 4.0 * N * ldw,
                        fn="linear_nt_kernel") \
        if TIMER is not None else None
    st = _lib.load().nerf_linear_fwd(arr, len(segs), M, wptr, ldw, N, _ptr(bias), _ptr(out), out.stride(0),
                                     epilogue, _ptr(aux), aux.stride(0) if aux is not None else 0,
                                     _stream(out.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_linear_fwd")


def linear_wgrad(dY: torch.Tensor, N4: int, segs, M: int, workspace: torch.Tensor) -> None:
    arr = make_segs(segs)
    kt = sum(k for _, k, _ in segs)
    # algorithmic bytes: dY and X read once, dW written once (the split-M slabs are the kernel's)
    end = TIMER.bracket("linear_wgrad", 2.0 * M * N4 * kt, 4.0 * M * N4 + _segs_bytes(segs, M) + 4.0 * N4 * kt,
                        fn="linear_wgrad_kernel") \
        if TIMER is not None else None
    st = _lib.load().nerf_linear_wgrad(_ptr(dY), dY.stride(0), N4, arr, len(segs), M, _ptr(workspace),
                                       workspace.numel() * workspace.element_size(), _stream(dY.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_linear_wgrad")


def linear_wgrad_workspace_bytes(M: int, N4: int, K: int) -> int:
    return int(_lib.load().nerf_linear_wgrad_workspace(M, N4, K))


def linear_wgrad_reduce(M: int, N4: int, K: int, n_valid: int, workspace: torch.Tensor, col_map: torch.Tensor,
                        dW: torch.Tensor, db: torch.Tensor | None, accumulate: bool = False) -> None:
    st = _lib.load().nerf_linear_wgrad_reduce(M, N4, K, n_valid, _ptr(workspace), _ptr(col_map), _ptr(dW),
                                              dW.stride(0), _ptr(db), int(accumulate), _stream(dW.device))
    _lib.check(st, "nerf_linear_wgrad_reduce")


# nerf_linear_fwd_x3 / nerf_linear_gauss_x3 run layers wider than 256 outputs as column blocks on
# the 256-row tile kernel unless NERF_NT_NBLOCK=0 (read once by the library, mirrored here for the
# timer's kernel names)
NT_NBLOCK = os.environ.get("NERF_NT_NBLOCK", "1") != "0"


def _nt_x3_fn(N: int, epilogue: int = 0) -> str:
    """The kernel function nerf_linear_fwd_x3 / nerf_linear_gauss_x3 launches for N outputs."""
    if epilogue & (_lib.NERF_EPI_NARROW_TILE | _lib.NERF_EPI_TANH | _lib.NERF_EPI_TANH_BWD):
        return "linear_nt_x3_kernel"
    wide_ok = NT_NBLOCK and not epilogue & (_lib.NERF_EPI_MASKBITS | _lib.NERF_EPI_MASKOUT)
    return "linear_nt_x3_glds_kernel" if N <= 256 or wide_ok else "linear_nt_x3_kernel"


def _nt_x3_launches(N: int, epilogue: int = 0) -> int:
    return (N + 255) // 256 if _nt_x3_fn(N, epilogue) == "linear_nt_x3_glds_kernel" else 1


def linear_fwd_x3(segs, M: int, Wx: torch.Tensor, ldw: int, N: int, bias: torch.Tensor | None,
                  out: torch.Tensor, epilogue: int, aux: torch.Tensor | None = None, w_row_offset: int = 0) -> None:
    """3 x bf16 split-precision variant of linear_fwd; Wx holds the interleaved hi|lo
    weights of nerf_pack_weight_x3 ([rows][ldw/32][hi 32 | lo 32] bf16)."""
    arr = make_segs(segs)
    off = w_row_offset * ldw * 2 * 2
    end = TIMER.bracket("linear_nt_x3", 2.0 * M * N * ldw, _segs_bytes(segs, M) + 4.0 * M * N + 4.0 * N * ldw,
                        fn=_nt_x3_fn(N, epilogue), launches=_nt_x3_launches(N, epilogue)) \
        if TIMER is not None else None
    st = _lib.load().nerf_linear_fwd_x3(arr, len(segs), M, Wx.data_ptr() + off, ldw, N, _ptr(bias), _ptr(out),
                                        out.stride(0), epilogue, _ptr(aux), aux.stride(0) if aux is not None else 0,
                                        _stream(out.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_linear_fwd_x3")


def linear_gauss_x3(segs, M: int, Wx: torch.Tensor, ldw: int, N: int, out: torch.Tensor, inv_std: torch.Tensor, *,
                    bias: torch.Tensor | None = None, y: torch.Tensor | None = None, z: torch.Tensor | None = None,
                    grad_inv_std: torch.Tensor | None = None, w_row_offset: int = 0) -> bool:
    """Split-precision linear layer with the Gaussian activation fused into its epilogue
    (nerf_linear_gauss_x3).  Forward (y given): out = z = x W^T + b, y = exp(-z^2 (s^2 + 1e-6)).
    Input gradient (z, grad_inv_std given): out = dL/dz of the layer whose pre-activation is z,
    from the product (= dL/dy), and grad_inv_std = its inverse-std gradient.  Returns False when the
    shapes need the unfused path (N % 4, alignment)."""
    _require_cuda_f32("inv_standard_deviation", inv_std)
    arr = make_segs(segs)
    off = w_row_offset * ldw * 2 * 2
    fwd = y is not None
    lib = _lib.load()
    ws = None
    if not fwd:
        ws = torch.empty(max(1, (int(lib.nerf_linear_gauss_workspace(M, N)) + 7) // 8), device=out.device,
                         dtype=torch.float64)
    nbytes = _segs_bytes(segs, M) + 4.0 * N * ldw + (8.0 * M * N if fwd else 12.0 * M * N)
    end = TIMER.bracket("linear_gauss_x3" if fwd else "linear_gauss_bwd_x3", 2.0 * M * N * ldw, nbytes,
                        fn=_nt_x3_fn(N), launches=_nt_x3_launches(N)) \
        if TIMER is not None else None
    st = lib.nerf_linear_gauss_x3(arr, len(segs), M, Wx.data_ptr() + off, ldw, N, _ptr(bias), _ptr(out),
                                  out.stride(0), _lib.NERF_GAUSS_FWD if fwd else _lib.NERF_GAUSS_BWD,
                                  _ptr(inv_std), _ptr(y), y.stride(0) if fwd else 0, _ptr(z),
                                  z.stride(0) if z is not None else 0, _ptr(grad_inv_std), 0, _ptr(ws),
                                  ws.numel() * 8 if ws is not None else 0, _stream(out.device))
    if end is not None:
        end.record()
    if st == _lib.NERF_ERR_UNSUPPORTED:
        return False
    _lib.check(st, "nerf_linear_gauss_x3")
    return True


# the single-tile layers' weight-gradient kernel the library runs (NERF_WGRAD_TR=0: the LDS-DMA stream
# kernel, default the register-staged transposed-read kernel; the same switch is read by the library),
# for the timer's per-function grouping
WGRAD_TILE_FN = ("linear_wgrad_x3_stream_kernel" if os.environ.get("NERF_WGRAD_TR", "1") == "0"
                 else "linear_wgrad_x3_tr_kernel")


def linear_wgrad_x3(dY: torch.Tensor, N4: int, segs, M: int, workspace: torch.Tensor, passes: int = 3) -> None:
    """Split-precision weight-gradient slabs (nerf_linear_wgrad_x3).  N4 is the row count: rounded
    up to 4 over a padded dY, or the true count (257: one 256 x 256 tile + a vector-ALU row); the
    workspace and the reduce take it rounded up to 4.  passes: 3 (3 x bf16 split) or 1 (one bf16
    pass, matmul precision "medium")."""
    arr = make_segs(segs)
    kt = sum(k for _, k, _ in segs)
    # algorithmic bytes: dY and X read once, dW written once (the split-M slabs are the kernel's)
    # the C side runs one 256 x 256 tile per M split when the layer fits it (nerf_linear_wgrad_x3)
    kpad = sum(pad32(k) for _, k, _ in segs)
    wide = (N4 > 128 or kpad > 128) and N4 <= 257 and kpad <= 256
    end = TIMER.bracket("linear_wgrad_x3", 2.0 * M * N4 * kt, 4.0 * M * N4 + _segs_bytes(segs, M) + 4.0 * N4 * kt,
                        fn=WGRAD_TILE_FN if wide else
                        ("linear_wgrad_smalln_kernel" if N4 <= 16 else "linear_wgrad_x3_kernel")) \
        if TIMER is not None else None
    st = _lib.load().nerf_linear_wgrad_x3(_ptr(dY), dY.stride(0), N4, arr, len(segs), M, _ptr(workspace),
                                          workspace.numel() * workspace.element_size(), passes, _stream(dY.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_linear_wgrad_x3")


def linear_wgrad_x3_rows(blocks, N4: int, workspace: torch.Tensor, passes: int = 3) -> None:
    """Split-precision weight-gradient slabs over two blocks of rows summed into one gradient
    (nerf_linear_wgrad_x3_rows): blocks = [(dY, segs, M), (dY1, segs1, M1)], the segments of the
    same widths; the workspace and the reduce take M + M1."""
    (dY, segs, M), (dY1, segs1, M1) = blocks
    if any(k != k1 for (_, k, _), (_, k1, _) in zip(segs, segs1)) or len(segs) != len(segs1):
        raise ValueError("linear_wgrad_x3_rows: the blocks' segments differ in width")
    a0, a1 = make_segs(segs), make_segs(segs1)
    kt = sum(k for _, k, _ in segs)
    kpad = sum(pad32(k) for _, k, _ in segs)
    wide = (N4 > 128 or kpad > 128) and N4 <= 257 and kpad <= 256
    end = TIMER.bracket("linear_wgrad_x3", 2.0 * (M + M1) * N4 * kt,
                        4.0 * (M + M1) * N4 + _segs_bytes(segs, M) + _segs_bytes(segs1, M1) + 4.0 * N4 * kt,
                        fn=WGRAD_TILE_FN if wide else
                        ("linear_wgrad_smalln_kernel" if N4 <= 16 else "linear_wgrad_x3_kernel")) \
        if TIMER is not None else None
    st = _lib.load().nerf_linear_wgrad_x3_rows(_ptr(dY), dY.stride(0), a0, M, _ptr(dY1), dY1.stride(0), a1, M1,
                                               len(segs), N4, _ptr(workspace),
                                               workspace.numel() * workspace.element_size(), passes,
                                               _stream(dY.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_linear_wgrad_x3_rows")


def linear_wgrad_x3_rays(blocks, N4: int, workspace: torch.Tensor, raysum: torch.Tensor, S0: int, S1: int,
                        passes: int = 3) -> None:
    """linear_wgrad_x3_rows (streamed single-tile kernel) that also writes the per-ray sums of dY into
    raysum [B0 + B1, N4] (nerf_linear_wgrad_x3_rays); blocks as linear_wgrad_x3_rows, M1 may be 0."""
    (dY, segs, M), (dY1, segs1, M1) = blocks
    a0, a1 = make_segs(segs), make_segs(segs1)
    kt = sum(k for _, k, _ in segs)
    if raysum.shape[1] != N4 or not raysum.is_contiguous():
        raise ValueError("linear_wgrad_x3_rays: raysum must be contiguous [rays, N4]")
    end = TIMER.bracket("linear_wgrad_x3", 2.0 * (M + M1) * N4 * kt,
                        4.0 * (M + M1) * N4 + _segs_bytes(segs, M) + _segs_bytes(segs1, M1) + 4.0 * N4 * kt
                        + 4.0 * raysum.numel(), fn=WGRAD_TILE_FN) \
        if TIMER is not None else None
    st = _lib.load().nerf_linear_wgrad_x3_rays(_ptr(dY), dY.stride(0), a0, M, _ptr(dY1), dY1.stride(0), a1, M1,
                                               len(segs), N4, _ptr(workspace),
                                               workspace.numel() * workspace.element_size(), _ptr(raysum), S0, S1,
                                               passes, _stream(dY.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_linear_wgrad_x3_rays")


def pack_weight_x3(W: torch.Tensor, col_map: torch.Tensor, Kp: int, Wpx: torch.Tensor | None,
                   Wtx: torch.Tensor | None, ldwt: int) -> None:
    N, K_orig = W.shape
    st = _lib.load().nerf_pack_weight_x3(_ptr(W), N, K_orig, _ptr(col_map), Kp, _ptr(Wpx), _ptr(Wtx), ldwt,
                                         _stream(W.device))
    _lib.check(st, "nerf_pack_weight_x3")


def interleave_x3(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """[rows][ld] hi / lo planes -> the interleaved [rows][ld/32][hi 32 | lo 32] layout."""
    r, ld = hi.shape
    return torch.stack((hi.reshape(r, ld // 32, 32), lo.reshape(r, ld // 32, 32)), dim=2).reshape(r, 2 * ld)


def pack_weight(W: torch.Tensor, col_map: torch.Tensor, Kp: int, Wp: torch.Tensor | None,
                Wt: torch.Tensor | None, ldwt: int) -> None:
    N, K_orig = W.shape
    st = _lib.load().nerf_pack_weight(_ptr(W), N, K_orig, _ptr(col_map), Kp, _ptr(Wp), _ptr(Wt), ldwt,
                                      _stream(W.device))
    _lib.check(st, "nerf_pack_weight")


# ----------------------------------------------------------------------------- hash grid (a9)
INGP_PRIMES = (1, 2654435761, 805459861)


def make_hashgrid_params(levels: int, table_size: int, features: int, res, query: int = 1, *,
                         primes=INGP_PRIMES, normalize: bool = True) -> _lib.NerfHashgridParams:
    if not 1 <= levels <= _lib.NERF_HASHGRID_MAX_LEVELS:
        raise ValueError(f"levels must be in [1, {_lib.NERF_HASHGRID_MAX_LEVELS}] (got {levels})")
    if not 1 <= features <= _lib.NERF_HASHGRID_MAX_FEATURES:
        raise ValueError(f"n_features must be in [1, {_lib.NERF_HASHGRID_MAX_FEATURES}] (got {features})")
    if len(res) != levels or any(not 1 <= int(r) <= (1 << 20) for r in res):
        raise ValueError(f"need {levels} resolutions in [1, 2^20] (got {list(res)})")
    if not 1 <= table_size or levels * table_size * features >= 2 ** 31:
        raise ValueError(f"table_size {table_size} out of range")
    if len(primes) != 3 or any(not -2 ** 63 <= int(q) < 2 ** 63 for q in primes):
        raise ValueError("primes must be three int64 values")
    p = _lib.NerfHashgridParams()
    p.levels, p.table_size, p.features, p.query = levels, table_size, features, query
    p.normalize = int(bool(normalize))
    for i, q in enumerate(primes):
        p.primes[i] = int(q)
    for i, r in enumerate(res):
        p.res[i] = int(r)
    return p


def hashgrid_level_rows(resolution: int, table_size: int) -> int:
    """Rows of one level's table: (r + 1)^3 when bijective, else table_size (nerf_hashgrid_table_rows)."""
    n = (int(resolution) + 1) ** 3
    return n if n <= table_size else table_size


def hashgrid_table_rows(params) -> int:
    return sum(hashgrid_level_rows(params.res[l], params.table_size) for l in range(params.levels))


def _hashgrid_inputs(params, n_samples, x, ray_o, ray_d, t_start, t_end, samples_per_ray):
    """Validate the position inputs of nerf_hashgrid_fwd / _bwd: explicit [n, 3] points, or rays
    ([B, 3] origins / directions, [B * samples_per_ray] intervals) covering n_samples."""
    for name, t in (("x", x), ("ray_o", ray_o), ("ray_d", ray_d), ("t_start", t_start), ("t_end", t_end)):
        if t is not None:
            _require_cuda_f32(name, t)
            if not t.is_contiguous():
                raise ValueError(f"{name} must be contiguous")
    if x is not None:
        if x.dim() != 2 or x.shape[1] != 3 or x.shape[0] < n_samples:
            raise ValueError(f"x must be [>= {n_samples}, 3] (got {tuple(x.shape)})")
        return
    if ray_o is None or ray_d is None or t_start is None or (params.query != 0 and t_end is None):
        raise ValueError("ray mode needs ray_o, ray_d, t_start (and t_end for midpoint queries)")
    if samples_per_ray < 1:
        raise ValueError("samples_per_ray must be >= 1")
    rays = (n_samples + samples_per_ray - 1) // samples_per_ray
    for name, t in (("ray_o", ray_o), ("ray_d", ray_d)):
        if t.numel() < 3 * rays:
            raise ValueError(f"{name} must hold {rays} rays")
    for name, t in (("t_start", t_start), ("t_end", t_end)):
        if t is not None and t.numel() < n_samples:
            raise ValueError(f"{name} must hold {n_samples} samples")


def _hashgrid_table_check(name: str, params, table: torch.Tensor) -> None:
    _require_cuda_f32(name, table)
    rows = hashgrid_table_rows(params)
    if not table.is_contiguous() or table.numel() != rows * params.features:
        raise ValueError(f"{name} must be a contiguous packed table of {rows} x {params.features} floats "
                         f"(got {tuple(table.shape)})")


# the kernels the library runs (NERF_HG_FWD: 1 (default) the level grid, 2 64-sample tiles with whole
# output rows, 0 one thread per (sample, level); NERF_HG_BWD: 0 (default) the per-item grid on the
# rows, 1 the per-item grid over grad_out restaged level-major, 2 the persistent part walk over it —
# the same switches are read by the library; tile / restaging for F in {1, 2, 4} and <= 16 levels;
# measured on a 1.31 M-sample batch, profiles/r04e/hg_*.txt: forward 361 / 375 / 764 us, backward
# 2807 / 3042 / 5586 us)
_HG_FWD = os.environ.get("NERF_HG_FWD", "1")[:1]
HASHGRID_FWD_FN = {"0": "hashgrid_fwd_kernel", "2": "hashgrid_fwd_tile_kernel"}.get(_HG_FWD, "hashgrid_fwd_level_kernel")
# the backward's event bracket covers the whole call; named by its kernel when one kernel does the
# work, else (the default bucketed form: restage, bijective-level walk, two bucket passes) by the call
HASHGRID_BWD_FN = ("hashgrid_bwd_walk_kernel" if os.environ.get("NERF_HG_BWD", "0")[:1] == "2"
                   else "nerf_hashgrid_bwd" if os.environ.get("NERF_HG_BUCKET", "1")[:1] != "0"
                   else "hashgrid_bwd_kernel")


def hashgrid_fwd(params, table: torch.Tensor, out: torch.Tensor, *, x=None, ray_o=None, ray_d=None, t_start=None,
                 t_end=None, n_samples: int, samples_per_ray: int = 1) -> None:
    _hashgrid_table_check("table", params, table)
    _require_cuda_f32("out", out)
    if out.dim() != 2 or out.stride(1) != 1 or out.shape[0] < n_samples or out.shape[1] < params.levels * params.features:
        raise ValueError("out must be a row-major [n, >= levels * features] tensor")
    _hashgrid_inputs(params, n_samples, x, ray_o, ray_d, t_start, t_end, samples_per_ray)
    # algorithmic bytes: 8 corners x F fp32 gathered + F fp32 written per (sample, level)
    end = TIMER.bracket("hashgrid_fwd", 0.0, 8.0 * n_samples * params.levels * params.features * 4
                        + 4.0 * n_samples * params.levels * params.features, fn=HASHGRID_FWD_FN) \
        if TIMER is not None else None
    st = _lib.load().nerf_hashgrid_fwd(ctypes.byref(params), _ptr(x), _ptr(ray_o), _ptr(ray_d), _ptr(t_start),
                                       _ptr(t_end), n_samples, samples_per_ray, table.data_ptr(), out.data_ptr(),
                                       out.stride(0), _stream(table.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_hashgrid_fwd")


def hashgrid_workspace_bytes(params, n_samples: int | None = None) -> int:
    """nerf_hashgrid_workspace(params), or with n_samples nerf_hashgrid_workspace_n: room for the ray
    form's float4 position records (computed once per backward instead of in every part walk) and
    grad_out restaged level-major as well.  The library's own sizes, not a restatement of them."""
    lib = _lib.load()
    size = lib.nerf_hashgrid_workspace(ctypes.byref(params)) if n_samples is None \
        else lib.nerf_hashgrid_workspace_n(ctypes.byref(params), int(n_samples))
    if size == 0:
        raise ValueError("invalid hash-grid parameters")
    return int(size)


def hashgrid_bwd_pos(params, table: torch.Tensor, grad_out: torch.Tensor, *, x=None, ray_o=None, ray_d=None,
                     t_start=None, t_end=None, n_samples: int, samples_per_ray: int = 1, want_o: bool = True,
                     want_d: bool = True):
    """Position gradient through the hash grid (nerf_hashgrid_bwd_pos): grad_x [n, 3] for explicit
    positions, else (grad_o, grad_d) [n_rays, 3] (None where not wanted) for ray-mode samples."""
    _require_cuda_f32("grad_out", grad_out)
    _hashgrid_table_check("table", params, table)
    if grad_out.dim() != 2 or grad_out.stride(1) != 1 or grad_out.shape[0] < n_samples \
            or grad_out.shape[1] < params.levels * params.features:
        raise ValueError(f"grad_out must be a row-major [>= {n_samples}, >= {params.levels * params.features}] "
                         f"tensor (got {tuple(grad_out.shape)})")
    _hashgrid_inputs(params, n_samples, x, ray_o, ray_d, t_start, t_end, samples_per_ray)
    dev = grad_out.device
    lib = _lib.load()
    if x is not None:
        gx = torch.empty(n_samples, 3, device=dev, dtype=torch.float32)
        st = lib.nerf_hashgrid_bwd_pos(ctypes.byref(params), _ptr(x), None, None, None, None, n_samples, 1,
                                       table.data_ptr(), grad_out.data_ptr(), grad_out.stride(0), gx.data_ptr(),
                                       None, None, 0, None, 0, _stream(dev))
        _lib.check(st, "nerf_hashgrid_bwd_pos")
        return gx
    rays = n_samples // samples_per_ray
    go = torch.empty(rays, 3, device=dev, dtype=torch.float32) if want_o else None
    gd = torch.empty(rays, 3, device=dev, dtype=torch.float32) if want_d else None
    ws = torch.empty(max(1, n_samples * 3), device=dev, dtype=torch.float32)
    st = lib.nerf_hashgrid_bwd_pos(ctypes.byref(params), None, _ptr(ray_o), _ptr(ray_d), _ptr(t_start), _ptr(t_end),
                                   n_samples, samples_per_ray, table.data_ptr(), grad_out.data_ptr(),
                                   grad_out.stride(0), None, _ptr(go), _ptr(gd), 0, ws.data_ptr(),
                                   ws.numel() * 4, _stream(dev))
    _lib.check(st, "nerf_hashgrid_bwd_pos")
    return go, gd


def hashgrid_bwd(params, grad_out: torch.Tensor, grad_table: torch.Tensor, workspace: torch.Tensor, *, x=None,
                 ray_o=None, ray_d=None, t_start=None, t_end=None, n_samples: int, samples_per_ray: int = 1,
                 accumulate: bool = False) -> None:
    _require_cuda_f32("grad_out", grad_out)
    _hashgrid_table_check("grad_table", params, grad_table)
    if grad_out.dim() != 2 or grad_out.stride(1) != 1 or grad_out.shape[0] < n_samples \
            or grad_out.shape[1] < params.levels * params.features:
        raise ValueError(f"grad_out must be a row-major [>= {n_samples}, >= {params.levels * params.features}] "
                         f"tensor (got {tuple(grad_out.shape)})")
    _hashgrid_inputs(params, n_samples, x, ray_o, ray_d, t_start, t_end, samples_per_ray)
    need = hashgrid_workspace_bytes(params)
    if workspace.device != grad_out.device or not workspace.is_contiguous() \
            or workspace.numel() * workspace.element_size() < need or workspace.data_ptr() % 256:
        raise ValueError(f"workspace must be a contiguous, 256-byte aligned device buffer of >= {need} bytes")
    # algorithmic work: F fp32 gradients read and 8 corners x F 8-byte fixed-point adds per (sample, level)
    end = TIMER.bracket("hashgrid_bwd", 0.0, 8.0 * n_samples * params.levels * params.features * 8
                        + 4.0 * n_samples * params.levels * params.features, fn=HASHGRID_BWD_FN) \
        if TIMER is not None else None
    st = _lib.load().nerf_hashgrid_bwd(ctypes.byref(params), _ptr(x), _ptr(ray_o), _ptr(ray_d), _ptr(t_start),
                                       _ptr(t_end), n_samples, samples_per_ray, grad_out.data_ptr(),
                                       grad_out.stride(0), grad_table.data_ptr(), int(accumulate),
                                       workspace.data_ptr(), workspace.numel() * workspace.element_size(),
                                       _stream(grad_out.device))
    if end is not None:
        end.record()
    _lib.check(st, "nerf_hashgrid_bwd")


# ----------------------------------------------------------------------------- pose alignment
def kabsch(p_from: torch.Tensor, p_to: torch.Tensor, remove_outliers: bool = True, error: bool = False):
    """nerf_kabsch: (R [3, 3], t [1, 3], c [] (, mean aligned distance [])) on the device."""
    for name, x in (("point_cloud_from", p_from), ("point_cloud_to", p_to)):
        _require_cuda_f32(name, x)
    p_from, p_to = p_from.contiguous(), p_to.contiguous()
    n = p_from.shape[0]
    if not 3 <= n <= _lib.NERF_KABSCH_MAX_POINTS:
        raise ValueError(f"kabsch needs 3 .. {_lib.NERF_KABSCH_MAX_POINTS} points (got {n})")
    out = torch.empty(14, device=p_from.device, dtype=torch.float32)
    st = _lib.load().nerf_kabsch(p_from.data_ptr(), p_to.data_ptr(), n, int(remove_outliers), out.data_ptr(),
                                 out.data_ptr() + 36, out.data_ptr() + 48, out.data_ptr() + 52 if error else None,
                                 _stream(p_from.device))
    _lib.check(st, "nerf_kabsch")
    R, t, c = out[:9].view(3, 3), out[9:12].view(1, 3), out[12]
    return (R, t, c, out[13]) if error else (R, t, c)


# ----------------------------------------------------------------------------- camera refinement
def _check_pose_inputs(rotation, translation, img_idx, o, d):
    for name, x in (("rotation", rotation), ("translation", translation), ("o", o), ("d", d)):
        _require_cuda_f32(name, x)
    if img_idx.device != o.device or img_idx.dtype != torch.int64:
        raise ValueError("img_idx must be an int64 tensor on the rays' device")
    n_img = rotation.shape[0]
    if rotation.shape != (n_img, 3) or translation.shape != (n_img, 3):
        raise ValueError("rotation / translation must be [n_images, 3]")
    B = img_idx.numel()
    if o.shape != (B, 3) or d.shape != (B, 3):
        raise ValueError(f"o / d must be [{B}, 3] (one row per image index)")


# above this many (image, ray) pairs the pose backward buckets the rays by image first (a stable
# device argsort + searchsorted, no host sync): each workgroup then reads only its own rays
POSE_BUCKET_MIN_WORK = 1 << 22


def pose_ray_buckets(idx: torch.Tensor, n_images: int):
    """(ray_order, image_start): ray indices stably sorted by image, and each image's first position."""
    order = torch.argsort(idx, stable=True)
    start = torch.searchsorted(idx[order].contiguous(),
                               torch.arange(n_images + 1, device=idx.device, dtype=torch.int64))
    return order.contiguous(), start.contiguous()


class _PoseRays(torch.autograd.Function):
    """CameraExtrinsics.forward on nerf_pose_rays_fwd / _bwd (csrc/camera.hip)."""

    @staticmethod
    def forward(ctx, rotation, translation, img_idx, o, d, magic):
        rotation, translation = rotation.contiguous(), translation.contiguous()
        idx, o, d = img_idx.reshape(-1).contiguous(), o.contiguous(), d.contiguous()
        B = idx.numel()
        new_o = torch.empty(B, 3, device=o.device, dtype=torch.float32)
        new_d = torch.empty_like(new_o)
        R = torch.empty(B, 3, 3, device=o.device, dtype=torch.float32)
        t = torch.empty_like(new_o)
        _lib.check(_lib.load().nerf_pose_rays_fwd(rotation.data_ptr(), translation.data_ptr(), rotation.shape[0],
                                                  idx.data_ptr(), o.data_ptr(), d.data_ptr(), B, float(magic),
                                                  new_o.data_ptr(), new_d.data_ptr(), R.data_ptr(), t.data_ptr(),
                                                  _stream(o.device)), "nerf_pose_rays_fwd")
        ctx.save_for_backward(rotation, idx, d, R)
        ctx.magic = magic
        ctx.set_materialize_grads(False)          # unused outputs reach the kernel as NULL
        return new_o, new_d, R, t

    @staticmethod
    def backward(ctx, g_o, g_d, g_R, g_t):
        rotation, idx, d, R = ctx.saved_tensors
        B = idx.numel()
        grads = [None] * 6
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            gr = [None if g is None else g.contiguous() for g in (g_o, g_d, g_R, g_t)]
            g_rot = torch.empty_like(rotation)
            g_trans = torch.empty_like(rotation)
            order = start = None
            if rotation.shape[0] * B > POSE_BUCKET_MIN_WORK:
                order, start = pose_ray_buckets(idx, rotation.shape[0])
            _lib.check(_lib.load().nerf_pose_rays_bwd(rotation.data_ptr(), rotation.shape[0], idx.data_ptr(),
                                                      d.data_ptr(), B, float(ctx.magic), *[_ptr(g) for g in gr],
                                                      _ptr(order), _ptr(start), g_rot.data_ptr(), g_trans.data_ptr(),
                                                      _stream(d.device)),
                       "nerf_pose_rays_bwd")
            grads[0], grads[1] = g_rot, g_trans
        if ctx.needs_input_grad[3]:
            grads[3] = g_o
        if ctx.needs_input_grad[4] and g_d is not None:          # d new_d / d d = R^T
            grads[4] = torch.bmm(R.transpose(1, 2), g_d.unsqueeze(-1)).squeeze(-1)
        return tuple(grads)


def pose_rays(rotation, translation, img_idx, o, d, magic: float = 1.0):
    """(new_o [B,3], new_d [B,3], R [B,3,3], t [B,3]) of CameraExtrinsics.forward, differentiable
    in rotation / translation (and o / d)."""
    _check_pose_inputs(rotation, translation, img_idx, o, d)
    return _PoseRays.apply(rotation, translation, img_idx, o, d, magic)


# ----------------------------------------------------------------------------- proposal sampler
def prop_cdf(w: torch.Tensor) -> torch.Tensor:
    """[R, K] weights -> [R, K+1] cdf (0, exclusive sums, 1) — nerf_prop_cdf."""
    _require_cuda_f32("weights", w)
    R, Kb = w.shape
    if w.stride(1) != 1:
        w = w.contiguous()
    cdf = torch.empty(R, Kb + 1, device=w.device, dtype=torch.float32)
    _lib.check(_lib.load().nerf_prop_cdf(w.data_ptr(), w.stride(0), R, Kb, cdf.data_ptr(), cdf.stride(0),
                                         _stream(w.device)), "nerf_prop_cdf")
    return cdf


def prop_sample(vals: torch.Tensor, cdf: torch.Tensor, n: int, stratified: bool, seed: int, transform: int,
                near: float, far: float):
    """Inverse-cdf sampling of n intervals per ray: (s edges, t edges), each [R, n+1] — nerf_prop_sample."""
    for name, t in (("vals", vals), ("cdf", cdf)):
        _require_cuda_f32(name, t)
        if t.stride(1) != 1:
            raise ValueError(f"{name} must be row-major")
    R, E = vals.shape
    if cdf.shape != (R, E) or E > _lib.NERF_PROP_MAX_EDGES or n + 1 > _lib.NERF_PROP_MAX_EDGES:
        raise ValueError(f"vals / cdf must be [R, K+1] with K+1 and n+1 <= {_lib.NERF_PROP_MAX_EDGES}")
    s = torch.empty(R, n + 1, device=vals.device, dtype=torch.float32)
    t = torch.empty_like(s)
    _lib.check(_lib.load().nerf_prop_sample(vals.data_ptr(), vals.stride(0), cdf.data_ptr(), cdf.stride(0), R, E - 1,
                                            n, int(stratified), seed, 0, transform, float(near), float(far),
                                            s.data_ptr(), t.data_ptr(), s.stride(0), _stream(vals.device)),
               "nerf_prop_sample")
    return s, t


def prop_loss(q_vals, q_cdf, k_vals, k_cdf, eps: float, grad_scale: float = 0.0, want_loss: bool = True,
              want_grad: bool = False):
    """Interlevel loss of query vs key intervals: (per-ray loss sums [R] or None, d/d key weights [R, K] or None)."""
    for name, t in (("q_vals", q_vals), ("q_cdf", q_cdf), ("k_vals", k_vals), ("k_cdf", k_cdf)):
        _require_cuda_f32(name, t)
        if t.dim() != 2 or t.stride(1) != 1:
            raise ValueError(f"{name} must be a row-major [R, edges] tensor")
    if q_cdf.shape != q_vals.shape or k_cdf.shape != k_vals.shape:
        raise ValueError("each cdf must have its edges' shape [R, edges]")
    if q_cdf.stride(0) != q_vals.stride(0) or k_cdf.stride(0) != k_vals.stride(0):
        raise ValueError("each cdf must share its edges' row stride")
    if q_vals.shape[0] != k_vals.shape[0]:
        raise ValueError("query and key intervals must cover the same rays")
    R, E = q_vals.shape
    Kb = k_vals.shape[1] - 1
    if E < 2 or Kb < 1 or E > _lib.NERF_PROP_MAX_EDGES or Kb + 1 > _lib.NERF_PROP_MAX_EDGES:
        raise ValueError(f"edge counts must lie in [2, {_lib.NERF_PROP_MAX_EDGES}]")
    lr = torch.empty(R, device=q_vals.device, dtype=torch.float32) if want_loss else None
    gw = torch.empty(R, Kb, device=q_vals.device, dtype=torch.float32) if want_grad else None
    _lib.check(_lib.load().nerf_prop_loss(q_vals.data_ptr(), q_cdf.data_ptr(), q_vals.stride(0), k_vals.data_ptr(),
                                          k_cdf.data_ptr(), k_vals.stride(0), R, E - 1, Kb, float(eps), _ptr(lr),
                                          float(grad_scale), _ptr(gw), gw.stride(0) if gw is not None else 0,
                                          _stream(q_vals.device)), "nerf_prop_loss")
    return lr, gw
