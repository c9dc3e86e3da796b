"""Ray-batch DP on CPU with the gloo backend, world size 2: the gradient
all-reduce produces the mean gradient on every rank, and DP over two shards
equals the full-batch gradient of a shared model (the multi-GPU bench path)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    """A rendezvous for the gloo group: a fresh file (file:// init, no TCP port to race for)."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="nerf_gloo_")
    os.close(fd)
    os.unlink(path)
    return path


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "nerf-experiments_amd"))
        from nerf_amd.ddp import GradAllReduce, shard_rays
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
        g = torch.Generator().manual_seed(42)
        x = torch.randn(64, 6, generator=g)
        y = torch.randn(64, 3, generator=g)
        sl = shard_rays(64, rank, world)
        loss = torch.nn.functional.mse_loss(model(x[sl]), y[sl], reduction="sum") / 64 * world
        loss.backward()
        GradAllReduce(model.parameters())()
        flat = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
        q.put((rank, flat))
    finally:
        dist.destroy_process_group()


def _worker_unused(rank, world, port, q):
    """A parameter used by one rank only keeps its gradient (mean over ranks); a parameter no rank
    used ends with grad None on every rank, as with one process."""
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "nerf-experiments_amd"))
        from nerf_amd.ddp import GradAllReduce
        a = torch.nn.Parameter(torch.ones(4))
        b = torch.nn.Parameter(torch.ones(3))       # rank 1 only
        c = torch.nn.Parameter(torch.ones(2))       # nobody
        loss = (a * (rank + 1)).sum() + ((b * 2).sum() if rank == 1 else 0)
        loss.backward()
        GradAllReduce([a, b, c])()
        q.put((rank, a.grad.clone(), None if b.grad is None else b.grad.clone(), c.grad is None))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_unused_parameters_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_unused, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (ga, gb, cnone) for r, ga, gb, cnone in (q.get(timeout=120) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    if os.path.exists(port):
        os.unlink(port)
    for r in (0, 1):
        ga, gb, cnone = res[r]
        assert torch.allclose(ga, torch.full((4,), 1.5))
        assert gb is not None and torch.allclose(gb, torch.full((3,), 1.0))
        assert cnone


def test_grad_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    if os.path.exists(port):
        os.unlink(port)
    # reference: full-batch gradient on one process
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    g = torch.Generator().manual_seed(42)
    x = torch.randn(64, 6, generator=g)
    y = torch.randn(64, 3, generator=g)
    torch.nn.functional.mse_loss(model(x), y, reduction="sum").div(64).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    assert torch.allclose(res[0], res[1])
    assert torch.allclose(res[0], ref, atol=1e-6)
