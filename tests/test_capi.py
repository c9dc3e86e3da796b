"""C-ABI library: loads without a GPU, exports exactly what include/nerf_amd.h
declares, and rejects bad arguments with a status (no compute launched)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "nerf_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nerf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ("nerf_composite_fwd", "nerf_composite_bwd", "nerf_resample_pdf", "nerf_sample_uniform",
                 "nerf_encode_fwd", "nerf_encode_bwd", "nerf_linear_fwd", "nerf_linear_wgrad",
                 "nerf_linear_wgrad_reduce", "nerf_pack_weight"):
        assert name in fns


def test_library_exports_every_header_symbol():
    from nerf_amd import _lib
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert sorted(_lib.EXPORTED_SYMBOLS) == header_functions()


def test_exported_dynamic_symbols_with_nm():
    import subprocess
    from nerf_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    syms = set(re.findall(r"\b(nerf_[a-z0-9_]+)\b", out))
    assert set(header_functions()) <= syms


def test_abi_version_and_status_strings():
    from nerf_amd import _lib
    lib = _lib.load()
    assert lib.nerf_abi_version() == 10
    assert lib.nerf_status_string(0) == b"ok"
    assert b"invalid" in lib.nerf_status_string(-1)
    assert b"workspace" in lib.nerf_status_string(-4)


def test_product_build_has_no_diagnostic_flags():
    """the shipped library was built with no NERF_*_DIAG_* ablation switch."""
    from nerf_amd import _lib
    assert _lib.load().nerf_build_flags() == 0


def test_every_diagnostic_switch_is_reported():
    """Every NERF_*_DIAG_* macro a kernel source tests is in common.h's list that feeds
    nerf_build_flags (a new switch not listed there would ship unnoticed)."""
    csrc = os.path.join(ROOT, "nerf-experiments_amd", "csrc")
    common = open(os.path.join(csrc, "common.h")).read()
    listed = set(re.findall(r"defined\((NERF_\w*DIAG\w*)\)", common))
    used = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")) and f != "common.h":
            src = open(os.path.join(csrc, f)).read()
            used |= set(re.findall(r"\b(NERF_\w*_DIAG_\w+)\b", src))
            # any switch next to a "diagnostic" comment, whatever its name, must be a listed DIAG switch
            for line in src.splitlines():
                m = re.match(r"\s*#\s*if(?:n?def)?\s+(?:defined\()?(NERF_\w+)", line)
                if m and "diagnostic" in line:
                    assert "_DIAG_" in m.group(1), line
                    used.add(m.group(1))
    assert used and used <= listed, sorted(used - listed)


def test_load_refuses_a_diagnostic_build(tmp_path):
    """A library with a unit compiled under a diagnostic switch (here capi.hip, the cheapest unit to
    recompile, with NERF_FUSED_DIAG_NOSTORE; every unit reports through the same common.h macro)
    returns bit 0 from nerf_build_flags and load() refuses it unless NERF_ALLOW_DIAG_BUILD=1."""
    import subprocess
    from nerf_amd import _lib
    pkg = os.path.join(ROOT, "nerf-experiments_amd")
    objs = [os.path.join(pkg, "build", f) for f in sorted(os.listdir(os.path.join(pkg, "build")))
            if f.endswith(".o") and f != "capi.o"]
    capi = tmp_path / "capi_diag.o"
    base = ["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
            "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(pkg, "csrc")]
    r = subprocess.run(base + ["-DNERF_FUSED_DIAG_NOSTORE", "-c", os.path.join(pkg, "csrc", "capi.hip"),
                               "-o", str(capi)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    lib = tmp_path / "libnerf_amd_diag.so"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", str(lib),
                        *objs, str(capi)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    with pytest.raises(RuntimeError, match="diagnostic build"):
        _lib.load(str(lib))
    os.environ["NERF_ALLOW_DIAG_BUILD"] = "1"
    try:
        assert _lib.load(str(lib)).nerf_build_flags() == 1
    finally:
        del os.environ["NERF_ALLOW_DIAG_BUILD"]


def test_struct_layouts_match_the_library():
    """Every argument struct of the binding has the C struct's size (load() checks it too)."""
    import ctypes
    from nerf_amd import _lib
    lib = _lib.load()
    for which, st in enumerate(_lib.STRUCTS):
        assert lib.nerf_struct_size(which) == ctypes.sizeof(st), st.__name__
    assert lib.nerf_struct_size(len(_lib.STRUCTS)) == -1
    # field offsets the fused kernel reads from its kernel arguments
    assert _lib.NerfFusedLayer.seg_gen.offset == ctypes.sizeof(_lib.NerfFusedLayer) - 8
    assert _lib.NerfFusedEncoding.out.offset == ctypes.sizeof(_lib.NerfPEParams) + 5 * 8 + 4


def test_argument_validation_returns_status_without_launch():
    from nerf_amd import _lib
    lib = _lib.load()
    # null pointers / bad sizes are rejected before anything touches the device
    assert lib.nerf_composite_fwd(None, 1, None, 3, None, 5, 64, 3.0, 1.0, 0, 0.0, None, None, None) == -1
    assert lib.nerf_composite_fwd(None, 1, None, 3, None, 0, 64, 3.0, 1.0, 0, 0.0, None, None, None) == 0
    assert lib.nerf_resample_pdf(None, None, None, 4, 64, 128, 0, 0.0, 1.0, 0, 0, None, None, None, None) == -1
    seg = (_lib.NerfSeg * 1)()
    seg[0].ptr = None
    assert lib.nerf_linear_fwd(seg, 1, 10, None, 32, 4, None, None, 4, 0, None, 0, None) == -1
    seg[0].ptr = 16
    seg[0].ld = 32
    seg[0].k = 6          # not a multiple of 4
    seg[0].row_div = 1
    assert lib.nerf_linear_fwd(seg, 1, 10, 16, 32, 4, None, 16, 4, 0, None, 0, None) == -1
    assert lib.nerf_linear_wgrad(16, 8, 6, seg, 1, 10, None, 0, None) == -1   # N % 4 != 0
    p = _lib.NerfPEParams()
    p.levels = 20
    assert lib.nerf_encode_fwd(ctypes.byref(p), None, None, None, None, None, None, None, 10, 1, 10, 16, 64,
                               None) == -1
    p.levels = 10
    p.kind = 0   # the integrated backward needs kind 1
    assert lib.nerf_encode_bwd_integrated(ctypes.byref(p), 16, 16, 16, 16, 16, 16, 64, 10, 16, None, 0, None) == -1
    p.kind = 1
    assert lib.nerf_encode_bwd_integrated(ctypes.byref(p), None, 16, 16, 16, 16, 16, 64, 10, 16, None, 0,
                                          None) == -1
    assert lib.nerf_encode_bwd_integrated(ctypes.byref(p), 16, 16, 16, 16, 16, 16, 64, 0, 16, None, 0, None) == 0
    # Gaussian activation: strides narrower than N, missing workspace
    assert lib.nerf_gauss_act_fwd(16, 8, 16, 10, 16, 16, 16, None) == -1
    assert lib.nerf_gauss_act_fwd(None, 16, None, 0, 16, None, 16, None) == 0
    assert lib.nerf_gauss_act_workspace(1000, 64) >= 64 * 8
    assert lib.nerf_gauss_act_bwd(16, 16, 16, 16, 16, 10, 16, 16, 16, 16, 0, None, 0, None) == -4
    # linear + Gaussian epilogue: bad mode, empty batch, N not a multiple of 4 (-> unfused path),
    # backward without workspace
    assert lib.nerf_linear_gauss_x3(None, 0, 10, 256, 32, 8, None, 256, 8, 2, 256, 256, 8, None, 0, None, 0,
                                    None, 0, None) == -1
    assert lib.nerf_linear_gauss_x3(None, 0, 0, 256, 32, 8, None, 256, 8, 0, 256, 256, 8, None, 0, None, 0,
                                    None, 0, None) == 0
    assert lib.nerf_linear_gauss_x3(None, 0, 10, 256, 32, 6, None, 256, 8, 0, 256, 256, 8, None, 0, None, 0,
                                    None, 0, None) == -2
    assert lib.nerf_linear_gauss_x3(None, 0, 10, 256, 32, 8, None, 256, 8, 1, 256, None, 0, 256, 8, 256, 0,
                                    None, 0, None) == -4
    assert lib.nerf_linear_gauss_workspace(1000, 64) >= 8 * 64 * 8
    # Kabsch: too few / too many points, missing outputs
    assert lib.nerf_kabsch(16, 16, 2, 1, 16, 16, 16, None, None) == -1
    assert lib.nerf_kabsch(16, 16, 5000, 1, 16, 16, 16, None, None) == -1
    assert lib.nerf_kabsch(16, 16, 10, 1, None, 16, 16, None, None) == -1
    # proposal sampler: too many edges, bad transform, lindisp with near 0, no outputs; empty batches
    assert lib.nerf_prop_sample(16, 600, 16, 600, 4, 599, 8, 0, 0, 0, 1, 2.0, 7.0, 16, 16, 16, None) == -1
    assert lib.nerf_prop_sample(16, 65, 16, 65, 4, 64, 8, 0, 0, 0, 2, 2.0, 7.0, 16, 16, 16, None) == -1
    assert lib.nerf_prop_sample(16, 65, 16, 65, 4, 64, 8, 0, 0, 0, 1, 0.0, 7.0, 16, 16, 16, None) == -1
    assert lib.nerf_prop_sample(16, 65, 16, 65, 0, 64, 8, 0, 0, 0, 1, 2.0, 7.0, 16, 16, 16, None) == 0
    assert lib.nerf_prop_loss(16, 16, 193, 16, 16, 65, 4, 192, 64, 1e-7, None, 0.0, None, 0, None) == -1
    assert lib.nerf_prop_cdf(16, 63, 4, 64, 16, 65, None) == -1
    assert lib.nerf_prop_cdf(None, 64, 0, 64, None, 65, None) == 0
    # ray-mode encoding backward: missing rays / outputs
    p.kind = 0
    assert lib.nerf_encode_bwd_rays(ctypes.byref(p), None, 16, 16, 16, None, 16, 64, 4, 8, 16, 16, 0, None) == -1
    assert lib.nerf_encode_bwd_rays(ctypes.byref(p), 16, 16, 16, 16, None, 16, 64, 4, 8, None, None, 0, None) == -1
    assert lib.nerf_encode_bwd_rays(ctypes.byref(p), 16, 16, 16, 16, None, 16, 64, 0, 8, 16, 16, 0, None) == 0
    # fused Adam: table bounds and null pointers
    b = _lib.NerfAdamBatch()
    b.n_tensors = 49
    assert lib.nerf_adam_step(ctypes.byref(b), None) == -1
    b.n_tensors = 1
    b.numel[0] = 10
    assert lib.nerf_adam_step(ctypes.byref(b), None) == -1
    b.numel[0] = 0
    assert lib.nerf_adam_step(ctypes.byref(b), None) == 0


def test_check_raises_with_message():
    from nerf_amd import _lib
    with pytest.raises(RuntimeError, match="invalid argument"):
        _lib.check(-1, "nerf_test")


def test_missing_library_fails_loudly(tmp_path):
    from nerf_amd import _lib
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load(str(tmp_path / "absent.so"))


def test_fused_forward_rejects_bad_generated_segments_without_launch():
    """nerf_mlp_fused_fwd with in-kernel encodings: checked like nerf_encode_fwd before any launch."""
    import ctypes
    from nerf_amd import _lib
    lib = _lib.load()
    img = ctypes.create_string_buffer(4096)
    out = ctypes.create_string_buffer(64 * 32 * 4 + 16)
    aligned = ctypes.addressof(out) + (-ctypes.addressof(out)) % 16
    L = (_lib.NerfFusedLayer * 2)()
    d = L[0]
    d.type, d.N, d.nb, d.relu, d.nseg = 1, 16, 1, 1, 1
    d.seg_kb[0], d.seg_k[0], d.seg_rd[0], d.seg_rows[0], d.seg_ld[0] = 1, 32, 1, 64, 32
    d.seg_ptr[0] = aligned
    d.chunk_units, d.col_idx, d.img_off, d.hbm_off, d.bias_off = 0, -1, 0, 0, 2048
    d.seg_gen[0] = 1
    enc = (_lib.NerfFusedEncoding * 2)()
    e = enc[0]
    e.params.kind, e.params.levels, e.params.include_identity, e.params.scale = 0, 5, 0, 1.0
    buf = ctypes.create_string_buffer(4096)
    e.ray_o = e.ray_d = e.t_start = ctypes.addressof(buf)
    e.n_rays, e.samples_per_ray, e.per_ray, e.out_dim = 8, 8, 0, 30
    e.out, e.ld = aligned, 32

    def call(n_layers=1, encs=enc):
        return lib.nerf_mlp_fused_fwd(L, n_layers, img, 64, encs, None)
    # no encodings array for a generated segment
    assert call(encs=None) == -1
    # out_dim inconsistent with the parameters
    e.out_dim = 31
    assert call() == -1
    e.out_dim = 30
    # fewer rays x samples than rows
    e.n_rays = 7
    assert call() == -1
    e.n_rays = 8
    # a per-ray (direction) encoding must be plain Fourier features
    e.per_ray, e.params.kind = 1, 1
    assert call() == -1
    e.per_ray, e.params.kind = 0, 0
    # the rows must be stored: no, misaligned or too narrow output rows
    e.out = None
    assert call() == -1
    e.out, e.ld = aligned + 4, 32
    assert call() == -1
    e.out, e.ld = aligned, 28
    assert call() == -1
    e.ld = 32
    # generator index out of range; a generated segment read by a later layer or in the chain
    d.seg_gen[0] = 3
    assert call() == -1
    d.seg_gen[0] = 9
    assert call() == -1
    d.seg_gen[0] = 0
    L[1] = L[0]
    L[1].type, L[1].seg_gen[0] = 7, 1
    assert call(2) == -1
    d.seg_gen[0] = 1
    d.mask_in = ctypes.addressof(buf)
    d.relu = 0
    assert call() == -1
