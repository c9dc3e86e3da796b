"""Stray-store guard bands around every output of the fused field-MLP kernels
(mlp_fused_kernel<0> forward, <1> input-gradient chain), the weight-gradient kernels
(linear_wgrad_x3_*, linear_wgrad_smalln) and their slab reduce, over one full training step
(forward, backward, optimizer) of the mip workload (C3's shared coarse / fine field,
barf/model_interpolation.py:356-414, barf/model_interpolation_architecture.py:96-141) and of the
ingp workload (C5, NaiveINGP).

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
  written) or zero (the zero-padded weight rows' outputs), never data.
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
        return buf[GUARD:GUARD + nbytes].view(dtype).view(shape)

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
    """Wrap the fused entry points: (pointer, rows, row stride, written columns) of every layer output."""
    regions = []

    def wrap(fname):
        fn = getattr(lib, fname)

        def call(layers, n_layers, image, M, *rest):
            for i in range(int(n_layers)):
                L = layers[i]
                if L.out:
                    ncols = min(32 * L.n1, L.N) if L.out2 else L.N
                    regions.append((fname, i, int(L.out), int(M), int(L.ldo), ncols))
                if L.out2:
                    regions.append((fname, i, int(L.out2), int(M), int(L.ldo2), L.N - 32 * L.n1))
            return fn(layers, n_layers, image, M, *rest)

        monkeypatch.setattr(lib, fname, call)

    for f in ("nerf_mlp_fused_fwd", "nerf_mlp_fused_render", "nerf_mlp_fused_run"):
        wrap(f)
    return regions


def _check(gt, regions):
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
        pad = view[:, ncols:]
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
    regions = _record_fused_outputs(monkeypatch, nerf_amd._lib.load())
    monkeypatch.setitem(bench.WORKLOADS, name, dict(bench.WORKLOADS[name], rays=rays))
    dev = torch.device("cuda", 0)
    _, _, opt, loss_fn, _ = bench.build_workload(name, dev, 0)
    loss = loss_fn()
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    assert torch.isfinite(loss).item()
    n_regions = _check(gt, regions)
    return gt, regions, n_regions


@pytest.mark.parametrize("name", ["mip", "ingp"])
def test_guard_bands_full_step(name, monkeypatch):
    gt, regions, n_pad = _step(name, monkeypatch, 1024)
    # the step ran the fused forward and chain (layer outputs recorded) and guarded their buffers
    assert any(f == "nerf_mlp_fused_run" for f, *_ in regions)
    assert len(gt.allocs) > 20
    assert n_pad > 0, "no fused layer output with pad columns was checked"
