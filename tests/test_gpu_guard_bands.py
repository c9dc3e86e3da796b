"""Stray-store guard bands around every output of the fused field-MLP kernels
(mlp_fused_kernel<0> forward, <1> input-gradient chain), the weight-gradient kernels
(linear_wgrad_x3_*, linear_wgrad_smalln) and their slab reduce, over one full training step
(forward, backward, optimizer) of the mip workload (C3's shared coarse / fine field,
barf/model_interpolation.py:356-414, barf/model_interpolation_architecture.py:96-141) and of the
ingp workload (C5, NaiveINGP), in split precision ("high") and for mip also in one bf16 pass
("medium").

Every device buffer the nerf_amd host code allocates with `torch.empty` / `torch.empty_like`
(layer outputs, ReLU bits, density columns, dY rows, encoding rows and their gradients, compositing
weights / coefficients, weight-gradient slab workspaces, weight gradients) is carved out of a larger
allocation whose bytes are all set to a sentinel, with a 4 KB guard region on each side.  After the
step:
* every guard byte still holds the sentinel (a store before the first or past the last row of any
  buffer — e.g. the round-5 chain pair-store variant whose chunk -1 offsets wrapped to the 128 bytes
  before each dY row — lands there);
* for every layer output a fused launch named in its descriptors (`out` [M][ldo], `out2` [M][ldo2]),
  the pad columns between the layer's columns and the row stride hold either the sentinel (never
  written) or zero (the zero-padded weight rows' outputs), never data — except the columns another
  output of the same launch is declared to write (the composite descriptor's head / density
  gradient rows, which the chain stores into columns 256.. of the 257-wide layer's dY).
The sentinel pattern fills memory torch.empty leaves undefined anyway: the product never reads it.
"""
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

SENT = 0xA5
GUARD = 4096


class _GuardedTorch:
    """Stand-in for the `torch` module inside nerf_amd: device allocations come with guard bands."""

    def __init__(self):
        self.allocs = []      # (flat uint8 buffer, offset of the view, view bytes)

    def __getattr__(self, name):
        return getattr(torch, name)

    def _guarded(self, shape, dtype, device):
        shape = tuple(int(s) for s in shape)
        n = 1
        for s in shape:
            n *= s
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        buf = torch.empty(nbytes + 2 * GUARD, dtype=torch.uint8, device=device)
        buf.fill_(SENT)
        self.allocs.append((buf, GUARD, nbytes))
        # a base tensor (not an autograd view) on the buffer's storage: the product code sets Python
        # attributes on its buffers and returns them from autograd Functions, which treat views apart
        esz = torch.empty((), dtype=dtype).element_size()
        stride, acc = [], 1
        for dim in reversed(shape):
            stride.append(acc)
            acc *= dim
        t = torch.empty(0, dtype=dtype, device=device)
        t.set_(buf.untyped_storage(), GUARD // esz, shape, tuple(reversed(stride)))
        return t

    def empty(self, *size, device=None, dtype=None, requires_grad=False, **kw):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            size = tuple(size[0])
        dev = torch.device(device) if device is not None else torch.device("cpu")
        if dev.type != "cuda" or kw:
            return torch.empty(*size, device=device, dtype=dtype, requires_grad=requires_grad, **kw)
        t = self._guarded(size, dtype or torch.get_default_dtype(), dev)
        return t.requires_grad_(requires_grad) if requires_grad else t

    def empty_like(self, t, dtype=None, device=None, requires_grad=False, **kw):
        dev = torch.device(device) if device is not None else t.device
        if dev.type != "cuda" or kw or not t.is_contiguous():
            return torch.empty_like(t, dtype=dtype, device=device, requires_grad=requires_grad, **kw)
        out = self._guarded(t.shape, dtype or t.dtype, dev)
        return out.requires_grad_(requires_grad) if requires_grad else out

    def owner(self, ptr):
        for buf, off, nbytes in self.allocs:
            base = buf.data_ptr() + off
            if base <= ptr < base + max(nbytes, 1):
                return buf, off, nbytes
        return None


def _install(monkeypatch):
    gt = _GuardedTorch()
    for name, mod in list(sys.modules.items()):
        if not name.startswith("nerf_amd") or mod is None:
            continue
        for attr in ("torch", "th"):
            if getattr(mod, attr, None) is torch:
                monkeypatch.setattr(mod, attr, gt)
    return gt


def _record_fused_outputs(monkeypatch, lib):
    """Wrap the fused entry points: (pointer, rows, row stride, written columns) of every layer
    output.  Every other entry point is wrapped too, to count the calls the step made."""
    regions, calls = [], {}
    extra = []     # 4-column outputs of the composite descriptor (head / density gradient rows): (ptr, ld)

    def wrap(fname):
        fn = getattr(lib, fname)
        fused = fname.startswith("nerf_mlp_fused_")

        def call(*args):
            calls[fname] = calls.get(fname, 0) + 1
            if fused:
                layers, n_layers, M = args[0], args[1], args[3]
                for i in range(int(n_layers)):
                    L = layers[i]
                    ncols = min(32 * L.n1, L.N) if L.out2 else L.N
                    if L.out and ncols > 0:          # (n1 = 0: every chunk goes to out2, none to out)
                        regions.append((fname, i, int(L.out), int(M), int(L.ldo), ncols))
                    if L.out2:
                        regions.append((fname, i, int(L.out2), int(M), int(L.ldo2), L.N - 32 * L.n1))
                comp = args[5] if fname != "nerf_mlp_fused_fwd" and len(args) > 6 else None
                c = getattr(comp, "_obj", None)
                if c is not None:
                    for ptr, ld in ((c.grad_head, c.ld_head), (c.grad_sigma, c.ld_sigma)):
                        if ptr:
                            extra.append((int(ptr), int(ld)))
            return fn(*args)

        monkeypatch.setattr(lib, fname, call)

    from nerf_amd import _lib as libmod
    for f in libmod._SIGNATURES:
        wrap(f)
    return regions, calls, extra


def _check(gt, regions, extra=()):
    torch.cuda.synchronize()
    assert gt.allocs, "no guarded allocation: the nerf_amd modules were not patched"
    bad = []
    for buf, off, nbytes in gt.allocs:
        lo, hi = buf[:off], buf[off + nbytes:]
        for part, where in ((lo, "before"), (hi, "after")):
            if part.numel() and not bool((part == SENT).all()):
                idx = torch.nonzero(part != SENT)
                bad.append(f"{where} a {nbytes}-byte buffer: {idx.numel()} bytes changed")
    assert not bad, "stores outside their buffers:\n" + "\n".join(bad[:20])
    seen = 0
    sent_f = torch.tensor([SENT] * 4, dtype=torch.uint8).view(torch.float32).item()
    for fname, layer, ptr, rows, ld, ncols in regions:
        if ld <= ncols:
            continue
        own = gt.owner(ptr)
        if own is None:
            continue
        buf, off, nbytes = own
        start = ptr - (buf.data_ptr() + off)
        assert start % 4 == 0 and start + rows * ld * 4 <= nbytes, (fname, layer, "region outside its buffer")
        view = buf[off + start:off + start + rows * ld * 4].view(torch.float32).view(rows, ld)
        # columns another output of the same launch writes (the chain's density-gradient rows are
        # columns 256.. of the 257-wide layer's dY, written from the composite descriptor)
        keep = torch.ones(ld - ncols, dtype=torch.bool, device=view.device)
        for eptr, eld in extra:
            off = eptr - ptr
            if eld == ld and 4 * ncols <= off < 4 * ld and off % 4 == 0:
                c0 = off // 4 - ncols
                keep[c0:c0 + 4] = False
        pad = view[:, ncols:][:, keep]
        bits = pad.contiguous().view(torch.int32)
        ok = (bits == torch.tensor([SENT] * 4, dtype=torch.uint8).view(torch.int32).to(bits.device)) | (pad == 0)
        assert bool(ok.all()), (f"{fname} layer {layer}: pad columns {ncols}..{ld - 1} hold data "
                                f"(first bad row {int(torch.nonzero(~ok)[0, 0])}; sentinel {sent_f})")
        seen += 1
    return seen


def _step(name, monkeypatch, rays):
    import importlib
    import pkgutil

    import bench
    import nerf_amd
    for m in pkgutil.iter_modules(nerf_amd.__path__):      # every module whose `torch` gets patched
        if not m.name.startswith("lib"):                     # (not the HIP library itself)
            importlib.import_module("nerf_amd." + m.name)
    nerf_amd._lib.load()
    gt = _install(monkeypatch)
    regions, calls, extra = _record_fused_outputs(monkeypatch, nerf_amd._lib.load())
    monkeypatch.setitem(bench.WORKLOADS, name, dict(bench.WORKLOADS[name], rays=rays))
    dev = torch.device("cuda", 0)
    _, _, opt, loss_fn, _ = bench.build_workload(name, dev, 0)
    loss = loss_fn()
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    assert torch.isfinite(loss).item()
    n_regions = _check(gt, regions, extra)
    return gt, regions, n_regions, calls


@pytest.mark.parametrize("name,precision", [("mip", "high"), ("mip", "medium"), ("ingp", "high")])
def test_guard_bands_full_step(name, precision, monkeypatch):
    # the fused kernels run in split ("high": mlp_fused_kernel<0> / <1>) or single-pass ("medium":
    # <2> / <3>) precision; torch's default "highest" takes the fp32 layer-by-layer GEMMs instead
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    try:
        gt, regions, n_pad, calls = _step(name, monkeypatch, 1024)
    finally:
        torch.set_float32_matmul_precision(old)
    # the step ran the fused forward and chain (layer outputs recorded) and guarded their buffers
    assert calls.get("nerf_mlp_fused_run", 0) >= 2, calls
    assert any(f == "nerf_mlp_fused_run" for f, *_ in regions), calls
    assert len(gt.allocs) > 20
    assert n_pad > 0, "no fused layer output with pad columns was checked"
