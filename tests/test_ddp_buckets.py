"""Bucketed, backward-overlapped gradient all-reduce (nerf_amd.ddp.BucketedGradAllReduce) and
bench.py's world>1 harness, rehearsed on CPU with the gloo backend at world size 2.

The model is NerfModel-shaped (nerf_amd.NerfModel's own parameters, two segments, delayed
direction, run through the CPU oracle's NerfModel forward so autograd reaches the real
Parameters in backward order), plus a parameter only rank 1 uses and one no rank uses.  Each rank
checks against a single-process full-batch reference computed in the same process."""
import os
import socket
import sys
import traceback

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    torch.set_num_threads(1)


def _model():
    from nerf_amd import FourierFeatures, NerfModel
    torch.manual_seed(0)
    m = NerfModel(4, 64, True, False, 2, FourierFeatures(10, 6.283185307179586), FourierFeatures(4, 1.0))
    only1 = torch.nn.Parameter(torch.ones(5))
    unused = torch.nn.Parameter(torch.ones(3))
    return m, only1, unused


def _loss(m, only1, rank, world, sl, with_only1=True):
    from oracle import nerf_oracle as O
    g = torch.Generator().manual_seed(7)
    n = 96
    pos = torch.randn(n, m.position_encoder.output_dim, generator=g)
    dirs = torch.randn(n, m.direction_encoder.output_dim, generator=g)
    target = torch.rand(n, 3, generator=g)
    sd = dict(m.named_parameters())
    dens, rgb = O.nerf_model_forward(sd, pos[sl], dirs[sl], 2, 4, True, False)
    loss = (((rgb - target[sl]) ** 2).sum() + 0.1 * dens.sum()) / n * world
    if with_only1 and rank == 1:
        loss = loss + (only1 * 2.0).sum()
    return loss


def _params(m, only1, unused):
    return list(m.parameters()) + [only1, unused]


def _worker_grads(rank, world, port, q):
    try:
        _setup_env(rank, world, port)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="file://" + os.environ["NERF_GLOO_RDV"], rank=rank,
                                world_size=world)
        from nerf_amd.ddp import BucketedGradAllReduce, shard_rays
        m, only1, unused = _model()
        ar = BucketedGradAllReduce(_params(m, only1, unused), bucket_bytes=48 * 1024)
        assert len(ar.buckets) >= 3, len(ar.buckets)
        # reference: full batch on one process; only1's mean gradient is (0 + 2) / 2
        mr, o1r, _ = _model()
        _loss(mr, o1r, 0, 1, slice(None), with_only1=False).backward()
        sl = shard_rays(96, rank, world)
        for it in range(2):                       # second step: .grad already are bucket views
            for p in _params(m, only1, unused):
                if it == 0:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.zero_()
            _loss(m, only1, rank, world, sl).backward()
            ar.finish()
            for (name, p), pr in zip(m.named_parameters(), mr.parameters()):
                assert p.grad is not None, name
                torch.testing.assert_close(p.grad, pr.grad, atol=1e-6, rtol=1e-5, msg=name)
                b = ar.buckets[ar._where[id(p)][0]]
                assert p.grad.untyped_storage().data_ptr() == b.flat.untyped_storage().data_ptr(), name
            torch.testing.assert_close(only1.grad, torch.ones(5))
            assert unused.grad is None
        # a second backward before finish() is refused
        _loss(m, only1, rank, world, sl).backward(retain_graph=False)
        try:
            _loss(m, only1, rank, world, sl).backward()
            raise AssertionError("double backward accepted")
        except RuntimeError as e:
            assert "arrived twice" in str(e)
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))


def _worker_adam(rank, world, port, q):
    """Three torch.optim.Adam steps with DP over two shards == three full-batch steps on one
    process (zero_grad alternating set_to_none True / False)."""
    try:
        _setup_env(rank, world, port)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="file://" + os.environ["NERF_GLOO_RDV"], rank=rank,
                                world_size=world)
        from nerf_amd.ddp import BucketedGradAllReduce, shard_rays
        m, only1, unused = _model()
        opt = torch.optim.Adam(_params(m, only1, unused), lr=1e-3, eps=1e-5)
        ar = BucketedGradAllReduce(_params(m, only1, unused), bucket_bytes=64 * 1024)
        mr, o1r, ur = _model()
        optr = torch.optim.Adam(_params(mr, o1r, ur), lr=1e-3, eps=1e-5)
        sl = shard_rays(96, rank, world)
        for it in range(3):
            opt.zero_grad(set_to_none=(it % 2 == 0))
            _loss(m, only1, rank, world, sl).backward()
            ar.finish()
            opt.step()
            optr.zero_grad(set_to_none=(it % 2 == 0))
            loss = _loss(mr, o1r, 0, 1, slice(None), with_only1=False) + (o1r * 1.0).sum()
            loss.backward()
            optr.step()
        for (name, p), pr in zip(m.named_parameters(), mr.parameters()):
            torch.testing.assert_close(p.detach(), pr.detach(), atol=1e-6, rtol=1e-5, msg=name)
        torch.testing.assert_close(only1.detach(), o1r.detach())
        torch.testing.assert_close(unused.detach(), torch.ones(3))      # never stepped
        assert unused not in opt.state or len(opt.state[unused]) == 0
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))


def _worker_bench(rank, world, port, q):
    """bench.py's world>1 setup, timed loop (barriers, max over ranks) and teardown on gloo."""
    try:
        _setup_env(rank, world, port)
        import bench
        from nerf_amd.ddp import BucketedGradAllReduce, shard_rays
        w, r, lr, dist = bench.init_distributed("gloo")
        assert (w, r, lr) == (world, rank, rank) and dist is not None and dist.get_world_size() == world
        m, only1, unused = _model()
        opt = torch.optim.Adam(_params(m, only1, unused), lr=1e-3, eps=1e-5)
        ar = BucketedGradAllReduce(_params(m, only1, unused))
        sl = shard_rays(96, rank, world)
        started = []

        def step():
            opt.zero_grad(set_to_none=True)
            loss = _loss(m, only1, rank, world, sl)
            loss.backward()
            ar.finish()
            opt.step()
            return loss

        elapsed, loss = bench.run_timed(step, 3, 1, dist, lambda: None, torch.device("cpu"),
                                        lambda: started.append(True))
        assert started == [True] and elapsed > 0 and torch.isfinite(loss)
        t = torch.tensor([elapsed], dtype=torch.float64)
        ts = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(ts, t)
        assert all(float(x) == elapsed for x in ts)        # every rank reports the max
        bench.teardown(dist)
        import torch.distributed as tdist
        assert not tdist.is_initialized()
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))


def _run(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    rdv = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"nerf_gloo_{port}_{world}")   # see _setup_env
    if os.path.exists(rdv):
        os.unlink(rdv)
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    if os.path.exists(rdv):
        os.unlink(rdv)
    for r in range(world):
        assert res[r] == "ok", f"rank {r}:\n{res[r]}"


def test_bucketed_allreduce_nerfmodel_grads_gloo_world2():
    _run(_worker_grads)


def test_bucketed_allreduce_adam_matches_full_batch_gloo_world2():
    _run(_worker_adam)


def test_bench_distributed_harness_gloo_world2():
    _run(_worker_bench)


def test_bucketed_allreduce_is_noop_without_process_group():
    sys.path.insert(0, os.path.join(ROOT, "nerf-experiments_amd"))
    from nerf_amd.ddp import BucketedGradAllReduce
    p = torch.nn.Parameter(torch.ones(3))
    ar = BucketedGradAllReduce([p])
    (p * 2).sum().backward()
    g = p.grad
    ar.finish()
    assert p.grad is g and not ar.buckets
