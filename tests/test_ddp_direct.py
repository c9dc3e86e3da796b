"""The direct gradient sink (BucketedGradAllReduce(direct=True), nerf_amd.mlp.GRAD_SINK) on bench.py's
mip step shape, rehearsed on CPU with gloo at world size 2.

Each rank builds the mip workload's objects as bench.build_workload("mip") does — the masked IPE /
BARF encoders, NerfModel(4, 256, delayed direction, 2 segments), NerfInterpolation with the same
model as proposal and radiance field, configure_optimizers() (torch Adam on the host; FusedAdam on a
GPU) — and runs coarse 64 + fine 128 samples per ray through the CPU oracle (the HIP path has no
CPU mode).  The field MLP runs inside a test Function that follows MLPFunction's direct-sink
protocol exactly: each recorded forward claims the layers' weights and biases, the backward writes
each layer's gradient into sink.target(p) (accumulating on the second pass) in reverse layer order
and calls sink.landed(p), returning None to autograd.  Checked: buckets start their all-reduce
from inside the last pass's backward before every parameter has landed (the overlap), the reduced
gradients equal the single-process full batch, and two Adam steps give the full-batch parameters."""
import os
import socket
import sys
import traceback

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B_GLOBAL, K_COARSE, S_FINE = 8, 64, 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup_env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    # groups this module initialises itself rendezvous through a file (no TCP port to race for);
    # bench.init_distributed (env://) keeps MASTER_PORT
    os.environ["NERF_GLOO_RDV"] = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"nerf_gloo_{port}_{world}")
    for p in (ROOT, os.path.join(ROOT, "nerf-experiments_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.set_num_threads(2)


def _mip_workload():
    """bench.build_workload("mip")'s renderer, on the host."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
    pos.pixel_width_sigma = 0.0
    dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
    model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
    ren = NerfInterpolation(2.0, 8.0, model, S_FINE, "stratified_uniform", -1.0, "middle", model, K_COARSE)
    return ren


class _OracleMLP(torch.autograd.Function):
    """The field MLP through the oracle, with MLPFunction's direct gradient-sink protocol."""

    @staticmethod
    def forward(ctx, names, pos_pe, dir_pe, *params):
        from nerf_amd import mlp
        from oracle import nerf_oracle as O
        local = [p.detach().requires_grad_(True) for p in params]
        with torch.enable_grad():
            dens, rgb = O.nerf_model_forward(dict(zip(names, local)), pos_pe, dir_pe, 2, 4, True, False)
        ctx.graph = (local, dens, rgb)
        ctx.params = params
        sink = mlp.GRAD_SINK
        ctx.sink = sink if sink is not None and sink.claim(params) else None
        return dens.detach(), rgb.detach()

    @staticmethod
    def backward(ctx, g_dens, g_rgb):
        local, dens, rgb = ctx.graph
        grads = torch.autograd.grad((dens, rgb), local, (g_dens, g_rgb), allow_unused=True)
        grads = [torch.zeros_like(p) if g is None else g for p, g in zip(local, grads)]
        if ctx.sink is None:
            return (None, None, None) + tuple(grads)
        for p, g in reversed(list(zip(ctx.params, grads))):      # last layer first, as MLPFunction
            t, acc = ctx.sink.target(p)
            if acc:
                t.add_(g)
            else:
                t.copy_(g)
            ctx.sink.landed(p)
        return (None, None, None) + (None,) * len(ctx.params)


def _batch():
    g = torch.Generator().manual_seed(5)
    o = torch.randn(B_GLOBAL, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 4.0])
    d = torch.nn.functional.normalize(torch.randn(B_GLOBAL, 3, generator=g) * 0.2
                                      - torch.tensor([0.0, 0.0, 1.0]), dim=1)
    pw = torch.full((B_GLOBAL, 1), 1 / 1111.1)
    target = torch.rand(B_GLOBAL, 3, generator=g)
    jitter = torch.rand(B_GLOBAL, K_COARSE, generator=g)
    offset = torch.rand(B_GLOBAL, 1, generator=g)
    return o, d, pw, target, jitter, offset


def _loss(ren, sl):
    """The mip training loss (coarse + fine MSE, shared field) of rays `sl` of the global batch."""
    from oracle import nerf_oracle as O
    o, d, pw, target, jitter, offset = (x[sl] for x in _batch())
    model = ren.model_radiance
    names, params = zip(*model.named_parameters())
    B = o.shape[0]
    near, far = ren.near_sphere_normalized, ren.far_sphere_normalized
    ones10 = torch.ones(10)

    def color(t0, t1, n):
        pos, dirs = O.compute_positions(o, d, t0, t1, "middle")
        N = B * n
        pos_pe = O.integrated_pe(pos.reshape(N, 3), dirs.reshape(N, 3), pw.repeat(1, n).view(N, 1),
                                 t0.reshape(N, 1), t1.reshape(N, 1), 10, 1.0, True, True, 0.0, mask=ones10)
        dir_pe = O.barf_pe(dirs.reshape(N, 3), 4, 4.0, True, 1.0)
        dens, rgb = _OracleMLP.apply(names, pos_pe, dir_pe, *params)
        return O.render_rays(dens.view(B, n), rgb.view(B, n, 3), t1 - t0, 3.0, 1 / 3)

    interval = (far - near) / K_COARSE
    t = O.linspace_t(near, far, K_COARSE).unsqueeze(0).repeat(B, 1) + jitter * interval - offset * interval
    t0, t1 = O.intervals(t, far)
    rgb_c, w = color(t0, t1, K_COARSE)
    f0, f1, _ = O.sample_t_pdf_weighted_batched(t0, w.detach(), t1 - t0, S_FINE, far)
    rgb_f, _ = color(f0, f1, S_FINE)
    return torch.nn.functional.mse_loss(rgb_f, target) + torch.nn.functional.mse_loss(rgb_c, target)


def _worker(rank, world, port, q):
    try:
        _setup_env(rank, world, port)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="file://" + os.environ["NERF_GLOO_RDV"], rank=rank,
                                world_size=world)
        from nerf_amd import mlp
        from nerf_amd.ddp import BucketedGradAllReduce, shard_rays
        ren = _mip_workload()
        opt = ren.configure_optimizers()["optimizer"]
        assert type(opt) is torch.optim.Adam and opt.param_groups[0]["eps"] == 1e-5
        ar = BucketedGradAllReduce(list(ren.parameters()), bucket_bytes=256 * 1024, direct=True)
        assert mlp.GRAD_SINK is ar and len(ar.buckets) >= 4
        landed_at_launch = []
        orig_launch = ar._launch

        def spy(b):
            landed_at_launch.append(sum(ar._arrived.values()))
            orig_launch(b)
        ar._launch = spy
        # single-process full batch, plain autograd (no sink)
        ref = _mip_workload()
        opt_ref = ref.configure_optimizers()["optimizer"]
        sl = shard_rays(B_GLOBAL, rank, world)
        n_params = len(list(ren.parameters()))
        for it in range(2):
            opt.zero_grad(set_to_none=True)
            loss = _loss(ren, sl)
            landed_at_launch.clear()
            loss.backward()
            # every bucket was launched from inside the backward; the first one a few layers into
            # the last pass, while most parameters' last contributions had not landed yet (two
            # passes: two landings per parameter)
            assert ar._next == len(ar.buckets) and all(b.launched for b in ar.buckets)
            assert landed_at_launch[0] <= n_params + 8 and landed_at_launch[-1] == 2 * n_params, landed_at_launch
            ar.finish()
            mlp.GRAD_SINK, saved = None, mlp.GRAD_SINK
            try:
                opt_ref.zero_grad(set_to_none=True)
                _loss(ref, slice(None)).backward()
            finally:
                mlp.GRAD_SINK = saved
            for (name, p), pr in zip(ren.named_parameters(), ref.parameters()):
                assert p.grad is not None, name
                torch.testing.assert_close(p.grad, pr.grad, atol=1e-7, rtol=2e-4, msg=f"step {it}: {name}")
                b = ar.buckets[ar._where[id(p)][0]]
                assert p.grad.untyped_storage().data_ptr() == b.flat.untyped_storage().data_ptr(), name
            opt.step()
            opt_ref.step()
        for (name, p), pr in zip(ren.named_parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), pr.detach(), atol=1e-6, rtol=1e-5, msg=name)
        ar.remove()
        assert mlp.GRAD_SINK is None
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_direct_sink_mip_step_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    rdv = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"nerf_gloo_{port}_{world}")   # see _setup_env
    if os.path.exists(rdv):
        os.unlink(rdv)
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=400) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    if os.path.exists(rdv):
        os.unlink(rdv)
    for r in range(world):
        assert res[r] == "ok", f"rank {r}:\n{res[r]}"


def test_direct_sink_world1_accumulates_into_grad():
    """Without a process group the sink writes .grad directly: first contribution written,
    later ones accumulated; a pre-existing .grad is accumulated onto (torch semantics)."""
    for p in (ROOT, os.path.join(ROOT, "nerf-experiments_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from nerf_amd import mlp
    from nerf_amd.ddp import BucketedGradAllReduce
    w = torch.nn.Parameter(torch.ones(2, 3))
    ar = BucketedGradAllReduce([w], direct=True)
    try:
        assert ar.claim([w]) and ar.claim([w])
        t, acc = ar.target(w)
        assert not acc and t is w.grad
        t.copy_(torch.full((2, 3), 2.0))
        ar.landed(w)
        t, acc = ar.target(w)
        assert acc
        t.add_(1.0)
        ar.landed(w)
        ar.finish()
        assert torch.equal(w.grad, torch.full((2, 3), 3.0))
        assert ar.claim([w])
        t, acc = ar.target(w)
        assert acc and t is w.grad                     # not zeroed: accumulates as autograd would
        assert not ar.claim([torch.nn.Parameter(torch.ones(1))])   # not ours
    finally:
        ar.remove()
    assert mlp.GRAD_SINK is None
