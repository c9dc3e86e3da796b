"""RCCL on the hardware: a process group with the "nccl" backend (= RCCL on ROCm) in a
world of one rank on cuda:0, and the bench's mip training step (C3: shared coarse / fine NerfModel,
barf/model_interpolation.py:356-414) with its gradients reduced through BucketedGradAllReduce
(direct=True, force=True: ~1 MiB buckets whose RCCL all-reduces are launched from the backward's
post-accumulate hooks and the direct weight-gradient sink, on RCCL's stream, while backward runs).
In a world of one the all-reduce is the identity, so two steps must leave every parameter bitwise
equal to the same two steps without any process group — the collective path (bucket views, flags,
1/world scaling, async handles, finish) changes nothing but where the gradients live.  The driver's
multi-GPU runs use the same path with one rank per GPU; the CPU suite covers world size 2 with gloo
(tests/test_ddp_direct.py, tests/test_ddp_buckets.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _two_steps(collective: bool):
    import bench
    from nerf_amd.ddp import BucketedGradAllReduce
    dev = torch.device("cuda", 0)
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        ren, modules, opt, loss_fn, _ = bench.build_workload("mip", dev, 0)
        ar = BucketedGradAllReduce([p for m in modules for p in m.parameters()], direct=True, force=collective)
        torch.manual_seed(1234)          # the same stratified-sampling draws in both runs
        assert ar.active == collective and (not collective or len(ar.buckets) >= 2)
        for _ in range(2):
            opt.zero_grad(set_to_none=True)
            loss = loss_fn()
            loss.backward()
            ar.finish()
            opt.step()
        ar.remove()
        torch.cuda.synchronize()
        return [p.detach().clone() for m in modules for p in m.parameters()], float(loss.item())
    finally:
        torch.set_float32_matmul_precision(old)


def test_rccl_bucketed_allreduce_world_one_equals_no_group(monkeypatch):
    import bench
    monkeypatch.setitem(bench.WORKLOADS, "mip", dict(bench.WORKLOADS["mip"], rays=1024))
    ref, ref_loss = _two_steps(False)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        # one bare RCCL all-reduce first (the library initialises and runs on this GPU)
        t = torch.arange(8, dtype=torch.float32, device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), torch.arange(8, dtype=torch.float32))
        got, loss = _two_steps(True)
    finally:
        dist.destroy_process_group()
    assert loss == ref_loss
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
