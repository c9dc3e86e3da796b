"""ctypes binding of the C-ABI library ``libnerf_amd.so`` (include/nerf_amd.h).

This is the binding a maintainer of the reference would add:
plain pointers, sizes and a ``hipStream_t`` per call.  ``torch`` must be imported
first so that the library binds to the same ``libamdhip64.so.7`` (same SONAME)
that PyTorch-ROCm already loaded — device pointers and streams are then shared.

There is no fallback: if the library is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before the HIP library, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NERF_AMD_LIB", os.path.join(_HERE, "libnerf_amd.so"))

c_f = ctypes.c_float
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_vp = ctypes.c_void_p
c_sz = ctypes.c_size_t

NERF_EPI_BIAS = 1
NERF_EPI_RELU = 2
NERF_EPI_MASK = 4
NERF_EPI_ACCUM = 8
NERF_EPI_MASKBITS = 16
NERF_EPI_MASKOUT = 32
NERF_EPI_NO_PERSIST = 256
NERF_EPI_NARROW_TILE = 512
NERF_EPI_TANH = 4096
NERF_EPI_TANH_BWD = 8192
NERF_ERR_UNSUPPORTED = -2
NERF_FUSED_BF16 = 1
NERF_KABSCH_MAX_POINTS = 4096
NERF_PROP_MAX_EDGES = 512
NERF_GAUSS_FWD = 0
NERF_GAUSS_BWD = 1


class NerfSeg(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("ld", c_i64), ("k", c_i32), ("row_div", c_i32)]


class NerfPEParams(ctypes.Structure):
    _fields_ = [
        ("kind", c_i32),
        ("levels", c_i32),
        ("include_identity", c_i32),
        ("query", c_i32),
        ("scale", c_f),
        ("pixel_width_sigma", c_f),
        ("distribute_variance", c_i32),
        ("pw_mode", c_i32),
        ("use_mask", c_i32),
        ("mask", c_f * 16),
    ]


NERF_ADAM_MAX_TENSORS = 48


class NerfAdamBatch(ctypes.Structure):
    _fields_ = [
        ("n_tensors", c_i32),
        ("beta1", c_f),
        ("beta2", c_f),
        ("eps", c_f),
        ("one_minus_beta1", c_f),
        ("one_minus_beta2", c_f),
        ("param", c_vp * NERF_ADAM_MAX_TENSORS),
        ("grad", c_vp * NERF_ADAM_MAX_TENSORS),
        ("exp_avg", c_vp * NERF_ADAM_MAX_TENSORS),
        ("exp_avg_sq", c_vp * NERF_ADAM_MAX_TENSORS),
        ("numel", c_i64 * NERF_ADAM_MAX_TENSORS),
        ("step_size", c_f * NERF_ADAM_MAX_TENSORS),
        ("bc2_sqrt", c_f * NERF_ADAM_MAX_TENSORS),
        ("weight_decay", c_f * NERF_ADAM_MAX_TENSORS),
    ]


NERF_FUSED_MAX_LAYERS = 16
NERF_FUSED_MAX_SRCS = 64


class NerfFusedLayer(ctypes.Structure):
    _fields_ = [
        ("type", c_i32),
        ("N", c_i32),
        ("nb", c_i32),
        ("relu", c_i32),
        ("nseg", c_i32),
        ("seg_kb", c_i32 * 2),
        ("seg_k", c_i32 * 2),
        ("seg_rd", c_i32 * 2),
        ("seg_rows", c_i32 * 2),
        ("chunk_units", c_i32),
        ("col_idx", c_i32),
        ("seg_ld", c_i64 * 2),
        ("seg_ptr", c_vp * 2),
        ("out", c_vp),
        ("ldo", c_i64),
        ("mask", c_vp),
        ("col_out", c_vp),
        ("img_off", c_i64),
        ("bias_off", c_i64),
        ("mask_in", c_vp),
        ("out2", c_vp),
        ("ldo2", c_i64),
        ("n1", c_i32),
        ("hbm_off", c_i32),
        ("seg_gen", c_i32 * 2),
    ]


class NerfFusedEncoding(ctypes.Structure):
    _fields_ = [
        ("params", NerfPEParams),
        ("ray_o", c_vp),
        ("ray_d", c_vp),
        ("t_start", c_vp),
        ("t_end", c_vp),
        ("pixel_width", c_vp),
        ("out", c_vp),
        ("ld", c_i64),
        ("n_rays", c_i64),
        ("samples_per_ray", c_i32),
        ("per_ray", c_i32),
        ("out_dim", c_i32),
        ("reserved", c_i32),
        ("hash", c_vp),
        ("hash_table", c_vp),
    ]


class NerfFusedComposite(ctypes.Structure):
    _fields_ = [
        ("dist", c_vp),
        ("rgb", c_vp),
        ("weights", c_vp),
        ("coef", c_vp),
        ("grad_rgb", c_vp),
        ("grad_head", c_vp),
        ("ld_head", c_i64),
        ("grad_sigma", c_vp),
        ("ld_sigma", c_i64),
        ("samples_per_ray", c_i32),
        ("head_layer", c_i32),
        ("sigma_layer", c_i32),
        ("scale_a", c_f),
        ("scale_b", c_f),
        ("density_shift", c_f),
        ("reserved", c_i32),
    ]


NERF_HASHGRID_MAX_LEVELS = 32
NERF_HASHGRID_MAX_FEATURES = 8


class NerfHashgridParams(ctypes.Structure):
    _fields_ = [
        ("levels", c_i32),
        ("table_size", c_i32),
        ("features", c_i32),
        ("query", c_i32),
        ("normalize", c_i32),
        ("reserved", c_i32),
        ("primes", c_i64 * 3),
        ("res", c_i32 * NERF_HASHGRID_MAX_LEVELS),
    ]

# name -> (restype, argtypes)
_SIGNATURES = {
    "nerf_abi_version": (c_i32, []),
    "nerf_status_string": (ctypes.c_char_p, [c_i32]),
    "nerf_composite_fwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i32, c_f, c_f, c_i32, c_f,
                                   c_vp, c_vp, c_vp]),
    "nerf_composite_bwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i32, c_f, c_f, c_i32, c_f,
                                   c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "nerf_sample_uniform": (c_i32, [c_i64, c_i32, c_f, c_f, c_i32, c_f, c_u64, c_u64, c_vp, c_vp, c_vp]),
    "nerf_resample_pdf": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_f, c_f, c_u64, c_u64,
                                  c_vp, c_vp, c_vp, c_vp]),
    "nerf_encode_fwd": (c_i32, [ctypes.POINTER(NerfPEParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                c_i64, c_i32, c_i64, c_vp, c_i64, c_vp]),
    "nerf_encode_bwd": (c_i32, [ctypes.POINTER(NerfPEParams), c_vp, c_vp, c_i64, c_i64, c_vp, c_i32, c_vp]),
    "nerf_encode_bwd_integrated": (c_i32, [ctypes.POINTER(NerfPEParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_i64, c_i64, c_vp, c_vp, c_i32, c_vp]),
    "nerf_encode_bwd_rays": (c_i32, [ctypes.POINTER(NerfPEParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                     c_i64, c_i32, c_vp, c_vp, c_i32, c_vp]),
    "nerf_encode_rays": (c_i32, [ctypes.POINTER(NerfPEParams), c_vp, c_i64, c_vp, c_i64, c_vp]),
    "nerf_adam_step": (c_i32, [ctypes.POINTER(NerfAdamBatch), c_vp]),
    "nerf_ray_batch": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_f, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_i32, c_i32,
                               c_i32, c_f, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nerf_gauss_act_workspace": (c_sz, [c_i64, c_i32]),
    "nerf_gauss_act_fwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "nerf_gauss_act_bwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i32,
                                   c_vp, c_sz, c_vp]),
    "nerf_linear_fwd": (c_i32, [ctypes.POINTER(NerfSeg), c_i32, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp, c_i64,
                                c_i32, c_vp, c_i64, c_vp]),
    "nerf_linear_wgrad_workspace": (c_sz, [c_i64, c_i32, c_i32]),
    "nerf_linear_wgrad": (c_i32, [c_vp, c_i64, c_i32, ctypes.POINTER(NerfSeg), c_i32, c_i64, c_vp, c_sz, c_vp]),
    "nerf_linear_wgrad_reduce": (c_i32, [c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp]),
    "nerf_pack_weight": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp]),
    "nerf_linear_fwd_x3": (c_i32, [ctypes.POINTER(NerfSeg), c_i32, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp,
                                   c_i64, c_i32, c_vp, c_i64, c_vp]),
    "nerf_linear_gauss_workspace": (c_sz, [c_i64, c_i32]),
    "nerf_linear_gauss_x3": (c_i32, [ctypes.POINTER(NerfSeg), c_i32, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp, c_i64,
                                     c_i32, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_sz, c_vp]),
    "nerf_linear_wgrad_x3": (c_i32, [c_vp, c_i64, c_i32, ctypes.POINTER(NerfSeg), c_i32, c_i64, c_vp, c_sz, c_i32,
                                     c_vp]),
    "nerf_linear_wgrad_x3_rows": (c_i32, [c_vp, c_i64, ctypes.POINTER(NerfSeg), c_i64, c_vp, c_i64,
                                          ctypes.POINTER(NerfSeg), c_i64, c_i32, c_i32, c_vp, c_sz, c_i32, c_vp]),
    "nerf_linear_wgrad_x3_rays": (c_i32, [c_vp, c_i64, ctypes.POINTER(NerfSeg), c_i64, c_vp, c_i64,
                                          ctypes.POINTER(NerfSeg), c_i64, c_i32, c_i32, c_vp, c_sz, c_vp, c_i32,
                                          c_i32, c_i32, c_vp]),
    "nerf_pack_weight_x3": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp]),
    "nerf_mlp_fused_fwd": (c_i32, [ctypes.POINTER(NerfFusedLayer), c_i32, c_vp, c_i64,
                                   ctypes.POINTER(NerfFusedEncoding), c_vp]),
    "nerf_mlp_fused_render": (c_i32, [ctypes.POINTER(NerfFusedLayer), c_i32, c_vp, c_i64,
                                      ctypes.POINTER(NerfFusedEncoding), ctypes.POINTER(NerfFusedComposite), c_vp]),
    "nerf_mlp_fused_run": (c_i32, [ctypes.POINTER(NerfFusedLayer), c_i32, c_vp, c_i64, ctypes.POINTER(NerfFusedEncoding),
                                   ctypes.POINTER(NerfFusedComposite), c_i32, c_vp]),
    "nerf_struct_size": (c_i64, [c_i32]),
    "nerf_build_flags": (c_i32, []),
    "nerf_fused_pack": (c_i32, [ctypes.POINTER(c_vp), c_i32, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "nerf_hashgrid_fwd": (c_i32, [ctypes.POINTER(NerfHashgridParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32,
                                  c_vp, c_vp, c_i64, c_vp]),
    "nerf_kabsch": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nerf_pose_rays_fwd": (c_i32, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_f, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nerf_pose_rays_bwd": (c_i32, [c_vp, c_i32, c_vp, c_vp, c_i64, c_f, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_vp]),
    "nerf_prop_cdf": (c_i32, [c_vp, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "nerf_prop_sample": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_i32, c_i32, c_u64, c_u64, c_i32, c_f,
                                 c_f, c_vp, c_vp, c_i64, c_vp]),
    "nerf_prop_loss": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_i32, c_i32, c_f, c_vp, c_f, c_vp,
                               c_i64, c_vp]),
    "nerf_hashgrid_workspace": (c_sz, [ctypes.POINTER(NerfHashgridParams)]),
    "nerf_hashgrid_workspace_n": (c_sz, [ctypes.POINTER(NerfHashgridParams), c_i64]),
    "nerf_hashgrid_table_rows": (c_i64, [ctypes.POINTER(NerfHashgridParams), c_i32]),
    "nerf_hashgrid_bwd": (c_i32, [ctypes.POINTER(NerfHashgridParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32,
                                  c_vp, c_i64, c_vp, c_i32, c_vp, c_sz, c_vp]),
    "nerf_hashgrid_bwd_pos": (c_i32, [ctypes.POINTER(NerfHashgridParams), c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32,
                                      c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_vp, c_sz, c_vp]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES.keys())
# argument structs in nerf_struct_size's order (their sizes are checked against the library at load)
STRUCTS = (NerfPEParams, NerfFusedLayer, NerfFusedEncoding, NerfHashgridParams, NerfAdamBatch, NerfSeg,
           NerfFusedComposite)

_lib = None


def load(path: str | None = None):
    """Load (once) and return the ctypes handle.  Raises if the library is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"nerf_amd: HIP library not found at {p}. Build it with `make -C nerf-experiments_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback.")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nerf_abi_version() != 10:
        raise RuntimeError("nerf_amd: ABI version mismatch between Python binding and libnerf_amd.so")
    for which, st in enumerate(STRUCTS):
        if lib.nerf_struct_size(which) != ctypes.sizeof(st):
            raise RuntimeError(f"nerf_amd: {st.__name__} layout differs from libnerf_amd.so's")
    flags = lib.nerf_build_flags()
    if flags != 0 and os.environ.get("NERF_ALLOW_DIAG_BUILD") != "1":
        # NERF_*_DIAG_* ablation builds drop work and return wrong results by construction; only
        # the profiling tools opt in (NERF_ALLOW_DIAG_BUILD=1), never the product path or a test
        raise RuntimeError(f"nerf_amd: {p} is a diagnostic build (nerf_build_flags = {flags:#x}); "
                           "rebuild with `make -C nerf-experiments_amd`")
    if path is None:
        _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().nerf_status_string(status).decode()
        raise RuntimeError(f"{what} failed with status {status}: {msg}")
