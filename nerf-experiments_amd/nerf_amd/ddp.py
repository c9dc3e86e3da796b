"""Ray-batch data parallelism: one process per GPU, the gradient mean as the only exchange.

Rays are independent through sampling, encoding, the field MLP, compositing and
resampling, so every rank renders its own ray shard and the only
exchange is the mean of the parameter gradients (~2.6 MB fp32 for NerfModel) per
step over RCCL ("nccl" backend = RCCL on ROCm; xGMI on one node).  The reference
itself is single-device (run_barf.py:103-148).

``BucketedGradAllReduce`` (what bench.py uses) launches one asynchronous all-reduce
per gradient bucket from post-accumulate-grad hooks while the backward pass is still
running; with ``direct=True`` it is also the field MLPs' gradient sink (nerf_amd.mlp.GRAD_SINK):
each layer's weight gradient is reduced straight into its bucket view inside the MLP's backward,
so buckets launch layer by layer while the remaining weight-gradient kernels run.
``GradAllReduce`` is the one-collective-after-backward form.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReduce:
    """Averages ``.grad`` of ``params`` across the process group with ONE collective.

    The gradients are concatenated into one flat fp32 bucket (a single copy kernel) followed by
    one "has a gradient" flag per parameter, reduced in place, scaled by 1/world, and every
    parameter's ``.grad`` becomes a view of its slice of the bucket — no copy back.  A parameter
    without a gradient contributes zeros so every rank issues the same collective; a parameter
    that NO rank produced a gradient for ends with ``.grad = None``, as with one process and as
    torch DDP leaves it, so the optimizer skips it on every rank (no momentum or weight-decay
    drift).  Deciding that needs the reduced flags on the host: the read happens only on a rank
    that itself lacks some gradient (if every local gradient exists, every reduced flag is >= 1)."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.sizes = [p.numel() for p in self.params]
        self.numel = sum(self.sizes)

    def __call__(self) -> None:
        if not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        missing = [p.grad is None for p in self.params]
        ref = self.params[0]
        grads = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in self.params]
        flags = torch.tensor([0.0 if m else 1.0 for m in missing], dtype=ref.dtype).to(ref.device, non_blocking=True)
        flat = torch.cat(grads + [flags])
        dist.all_reduce(flat, group=self.group)
        flat.div_(world)
        parts = flat.split(self.sizes + [len(self.params)])
        used = None
        if any(missing):
            used = (parts[-1] > 0).tolist()       # host read of the reduced flags (only here)
        for i, (p, g) in enumerate(zip(self.params, parts[:-1])):
            p.grad = g.view_as(p) if used is None or used[i] else None


class _Bucket:
    __slots__ = ("params", "offsets", "flat", "flags_at", "ready", "pending", "handle", "launched")

    def __init__(self, params, device, dtype):
        self.params = params
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += p.numel()
        self.flags_at = off
        # gradients, then one "has a gradient" flag per parameter
        self.flat = torch.zeros(off + len(params), device=device, dtype=dtype)
        self.ready = [False] * len(params)
        self.pending = len(params)
        self.handle = None
        self.launched = False

    def view(self, j):
        p = self.params[j]
        return self.flat[self.offsets[j]:self.offsets[j] + p.numel()].view_as(p)


class BucketedGradAllReduce:
    """Gradient mean across the process group, overlapped with the backward pass.

    Parameters are split into buckets of about ``bucket_bytes`` in REVERSE registration order (the
    order backward produces their gradients).  A post-accumulate-grad hook moves each gradient into
    its bucket (no copy when ``.grad`` already is the bucket view, as after
    ``zero_grad(set_to_none=False)``) and, once a bucket is complete, launches its all-reduce
    asynchronously (RCCL runs it on its own stream while backward continues).  Buckets launch
    strictly in bucket order on every rank, so the collective sequence matches across ranks even when
    gradients arrive in different orders.  ``finish()`` (after ``backward()``, before the optimizer)
    launches the buckets still incomplete — a parameter without a local gradient contributes zeros
    and a 0 flag — waits for all of them and leaves every ``.grad`` as a view of its reduced bucket;
    a parameter that NO rank produced a gradient for ends with ``.grad = None`` on every rank, as
    with one process (the reduced flags are read on the host only by a rank that itself lacked a
    gradient).  Gradients are pre-scaled by 1/world and summed.  One backward per ``finish()``.
    With world size 1 (or no process group) and ``direct=False`` every method is a no-op and
    ``.grad`` is untouched.

    ``direct=True`` also installs this object as the field MLPs' gradient sink
    (``nerf_amd.mlp.GRAD_SINK``): every MLP forward recorded for autograd ``claim``s its layers'
    weights and biases (one expected contribution each per use), and the MLP backward writes each
    layer's gradient straight into ``target(p)`` — the bucket view, or ``.grad`` at world size 1 —
    accumulating in the slab reduce when an earlier pass of the step already landed, then calls
    ``landed(p)``; the last expected landing marks the parameter ready, so its bucket can start its
    all-reduce while the MLP's remaining weight-gradient kernels run.  Those parameters never pass
    through autograd's accumulation (the backward returns None for them), and a field used twice
    per step costs no extra add.  This holds at world size 1 too: the sink is installed, the MLP
    weight gradients bypass autograd accumulation and any user gradient hooks on those
    parameters, and ``finish()`` must still be called after every backward (it flushes held-back
    weight gradients and resets the per-step claims).  A forward that claims parameters after
    gradients of the previous backward have landed, without a ``finish()`` in between, raises."""

    def __init__(self, params, bucket_bytes: int = 1 << 20, group=None, direct: bool = False,
                 force: bool = False):
        seen, plist = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                plist.append(p)
        self.params = plist
        self.group = group
        # force: run the buckets and their collectives even in a world of one process (the all-reduce
        # is then the identity: tests/test_gpu_rccl.py drives RCCL through this path on one GPU)
        self.active = dist.is_available() and dist.is_initialized() and (dist.get_world_size(group) > 1 or force)
        self.world = dist.get_world_size(group) if self.active else 1
        self.buckets: list[_Bucket] = []
        self._where = {}
        self._next = 0
        self._hooks = []
        self.direct = direct
        self._owned = {id(p) for p in plist}
        self._expected: dict[int, int] = {}
        self._arrived: dict[int, int] = {}
        # (MLP, layer) -> ((dY, X, rows, ...), flush): a weight gradient held back for the other
        # pass of a field used twice per step (nerf_amd.mlp: one launch over both passes' rows)
        self.stash: dict = {}
        if direct:
            from . import mlp
            if mlp.GRAD_SINK is not None and mlp.GRAD_SINK is not self:
                raise RuntimeError("another direct gradient sink is installed; remove() it first")
            mlp.GRAD_SINK = self
        if not self.active:
            return
        cur, cur_bytes = [], 0
        for p in reversed(plist):
            if cur and (cur_bytes + p.numel() * p.element_size() > bucket_bytes
                        or p.device != cur[0].device or p.dtype != cur[0].dtype):
                self.buckets.append(_Bucket(cur, cur[0].device, cur[0].dtype))
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += p.numel() * p.element_size()
        if cur:
            self.buckets.append(_Bucket(cur, cur[0].device, cur[0].dtype))
        for bi, b in enumerate(self.buckets):
            for j, p in enumerate(b.params):
                self._where[id(p)] = (bi, j)
                self._hooks.append(p.register_post_accumulate_grad_hook(self._hook))

    # -- direct gradient sink (nerf_amd.mlp.GRAD_SINK) --------------------------------------------
    def claim(self, params) -> bool:
        """One more expected contribution for each of ``params`` this step (all must be ours)."""
        if not all(id(p) in self._owned for p in params):
            return False
        if self._arrived:
            raise RuntimeError("BucketedGradAllReduce: a forward claimed parameters after the previous "
                               "backward's gradients landed; call finish() after every backward()")
        for p in params:
            self._expected[id(p)] = self._expected.get(id(p), 0) + 1
        return True

    def target(self, p):
        """(tensor the next contribution of p is written into, accumulate onto it?)."""
        first = self._arrived.get(id(p), 0) == 0
        if self.active:
            bi, j = self._where[id(p)]
            b = self.buckets[bi]
            if b.launched or b.ready[j]:
                raise RuntimeError("BucketedGradAllReduce: a gradient arrived after its bucket was launched; "
                                   "call finish() after every backward()")
            v = b.view(j)
            if first:
                g = p.grad
                if g is None:
                    return v, False
                if g.data_ptr() != v.data_ptr():
                    v.copy_(g)
            return v, True
        if first and p.grad is None:
            p.grad = torch.empty_like(p)
            return p.grad, False
        if p.grad is None:
            raise RuntimeError("BucketedGradAllReduce: .grad was cleared between two contributions of one "
                               "step (zero_grad inside a step, or a skipped finish())")
        return p.grad, True

    def remaining(self, p) -> int:
        """Contributions of p still expected this step (claimed, not yet landed)."""
        return self._expected.get(id(p), 0) - self._arrived.get(id(p), 0)

    def landed(self, p) -> None:
        k = id(p)
        n = self._arrived.get(k, 0) + 1
        self._arrived[k] = n
        if n == self._expected.get(k, 0) and self.active:
            bi, j = self._where[k]
            b = self.buckets[bi]
            p.grad = b.view(j)
            b.ready[j] = True
            b.pending -= 1
            self._launch_ready()

    def _hook(self, p) -> None:
        # the hook also fires when a backward returned no gradient for p (.grad untouched): the
        # direct sink's parameters (their gradients land through target / landed) and unused ones
        if id(p) in self._expected or p.grad is None:
            return
        bi, j = self._where[id(p)]
        b = self.buckets[bi]
        if b.launched or b.ready[j]:
            raise RuntimeError("BucketedGradAllReduce: a gradient arrived twice in one step; call finish() "
                               "after every backward()")
        v = b.view(j)
        if p.grad.data_ptr() != v.data_ptr():
            v.copy_(p.grad)
            p.grad = v
        b.ready[j] = True
        b.pending -= 1
        self._launch_ready()

    def _launch(self, b: _Bucket) -> None:
        # the "has a gradient" flags: one fill when every parameter is ready, else one host->device
        # copy of the whole flag row (not a launch per missing parameter)
        if all(b.ready):
            b.flat[b.flags_at:].fill_(1.0)
        else:
            flags = torch.tensor([1.0 if r else 0.0 for r in b.ready], dtype=b.flat.dtype)
            b.flat[b.flags_at:].copy_(flags.to(b.flat.device, non_blocking=True))
        if self.world > 1:
            b.flat.mul_(1.0 / self.world)
        b.handle = dist.all_reduce(b.flat, group=self.group, async_op=True)
        b.launched = True

    def _launch_ready(self) -> None:
        while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def finish(self) -> None:
        # weight gradients held back for a pass whose backward never ran: computed alone now
        pending, self.stash = list(self.stash.values()), {}
        for entry, flush in pending:
            flush(entry, self)
        arrived = self._arrived
        self._expected, self._arrived = {}, {}
        if not self.active:
            return
        missing = []
        for b in self.buckets[self._next:]:
            for j, p in enumerate(b.params):
                if not b.ready[j]:
                    if arrived.get(id(p), 0) > 0:
                        # direct contributions landed, fewer than claimed (a claimed forward whose
                        # backward never ran): what landed is the gradient
                        b.ready[j] = True
                        continue
                    b.view(j).zero_()
                    missing.append((b, j))
            self._launch(b)
        self._next = len(self.buckets)
        for b in self.buckets:
            b.handle.wait()
        used = None
        if missing:
            used = {(id(b), j): f > 0 for b in {id(b): b for b, _ in missing}.values()
                    for j, f in enumerate(b.flat[b.flags_at:].tolist())}
        for b in self.buckets:
            for j, p in enumerate(b.params):
                if used is not None and not used.get((id(b), j), True):
                    p.grad = None
                else:
                    p.grad = b.view(j)
            b.ready = [False] * len(b.params)
            b.pending = len(b.params)
            b.handle = None
            b.launched = False
        self._next = 0

    __call__ = finish

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.direct:
            from . import mlp
            if mlp.GRAD_SINK is self:
                mlp.GRAD_SINK = None


def shard_rays(n_global: int, rank: int, world: int) -> slice:
    """Contiguous shard of a global ray batch (sizes differ by at most one ray)."""
    base, rem = divmod(n_global, world)
    start = rank * base + min(rank, rem)
    return slice(start, start + base + (1 if rank < rem else 0))
