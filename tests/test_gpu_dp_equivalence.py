"""Ray-batch data parallelism on the real kernels: two processes, each with half of a batch, reduce
their weight gradients through BucketedGradAllReduce(direct=True) — the field MLP's weight gradients
land straight in the buckets from the slab reduce (per-ray, small-N and merged-pass routes included)
and the buckets are all-reduced as they complete — and the result equals one process's gradient of
the whole batch (rays are independent, the gradient mean is the only exchange).  The
ranks share the one GPU over gloo (the driver's multi-GPU runs use RCCL, one GPU per rank; the CPU
suite's tests/test_ddp_direct.py covers the same protocol on the oracle forward).  Equidistant
samples and the deterministic resample, so both runs see the same samples per ray; tolerance 1e-5
of each gradient's scale (summation order).  Two workloads: mip (C3's shared coarse / fine field)
and barf (C4: per-image CameraExtrinsics refining the rays, whose rotation / translation
gradients come back through the ray-mode encoding backward and pose_rays_bwd and are all-reduced
through the post-accumulate-grad hooks beside the MLP's direct buckets;
barf/model_camera_extrinsics.py:77-85, barf/model_barf.py:29-92), and ingp (C5: NaiveINGP, the
hash-grid tables' fixed-point gradients reduced beside the two fields' direct buckets;
3d-ingp/model.py:195-519 as VERDICT r3 quotes it)."""
import os
import sys
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nerf-experiments_amd")
B = 512


def _setup(dev, workload="mip"):
    """(modules whose parameters are reduced, loss of a ray slice)."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(3)
    o = (torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]),
                                      dim=1).to(dev)
    pw = torch.full((B,), 1 / 1111.1, device=dev)
    c = torch.rand(B, 3, generator=g).to(dev)
    if workload == "mip":
        pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
        pos.pixel_width_sigma = 0.0
        dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
        model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
        ren = NerfInterpolation(2.0, 8.0, model, 128, "equidistant", 0.0, "middle", model, 64).to(dev)

        def loss(sl):
            return ren.training_loss(o[sl], d[sl], pw[sl], c[sl])[0]
        return [ren], loss
    if workload == "ingp":
        # C5: NaiveINGP (separate coarse / fine fields sharing the hash grid, whose table gradient is
        # the fixed-point scatter reduced through the post-accumulate-grad buckets); coarse t
        # equidistant so both runs see the same samples, 64 + 192 fine samples from the deterministic
        # resample
        from nerf_amd.model_ingp import FourierFeatures, INGPEncoding, NaiveINGP
        ren = NaiveINGP(2, 7, 192, 64, INGPEncoding(1600, 16, 2 ** 16, 2, 16), FourierFeatures(4), 8, 256).to(dev)
        S = ren.samples_per_ray_coarse
        t = torch.linspace(2.0, 7.0 - 5.0 / S, S, device=dev).repeat(B, 1).contiguous()
        ren._sample_t_coarse = lambda batch_size: t[:batch_size]

        def loss(sl):
            return ren.training_loss(o[sl], d[sl], c[sl])[0]
        return [ren], loss
    # barf (bench.py --workload barf): coarse-to-fine masked PE mid-schedule, 128 equidistant
    # samples, rays refined by the per-image extrinsics of 16 views
    from nerf_amd.model_camera_extrinsics import CameraExtrinsics
    pos = BarfPositionalEncoding(10, 10.0, 0, 1, True, 1.0)
    dirs = BarfPositionalEncoding(4, 4.0, 0, 1, True, 1.0)
    pos.update_alpha(0.55)
    dirs.update_alpha(0.55)
    model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-5, 200000)
    ren = NerfInterpolation(2.0, 8.0, model, 128, "equidistant", 0.0, "middle").to(dev)
    extr = CameraExtrinsics(16, 1e-3, 1e-5, 200000).to(dev)
    with torch.no_grad():
        extr.rotation.copy_(torch.randn(extr.rotation.shape, generator=g) * 0.02)
        extr.translation.copy_(torch.randn(extr.translation.shape, generator=g) * 0.02)
    img = torch.randint(0, 16, (B,), generator=g).to(dev)

    def loss(sl):
        o2, d2, _, _ = extr(img[sl], o[sl], d[sl])
        return ren.training_loss(o2, d2, pw[sl], c[sl])[0]
    return [ren, extr], loss


def _grads(modules, loss, sl):
    from nerf_amd.ddp import BucketedGradAllReduce
    params = [p for m in modules for p in m.parameters()]
    ar = BucketedGradAllReduce(params, direct=True)
    try:
        loss(sl).backward()
        ar.finish()
        torch.cuda.synchronize()
        return {f"{i}.{n}": p.grad.detach().cpu().clone() for i, m in enumerate(modules)
                for n, p in m.named_parameters() if p.grad is not None}
    finally:
        ar.remove()


def _worker(rank, world, init_file, out_file, workload):
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=world)
    try:
        torch.set_float32_matmul_precision("high")
        dev = torch.device("cuda", 0)
        modules, loss = _setup(dev, workload)
        n = B // world
        g = _grads(modules, loss, slice(rank * n, (rank + 1) * n))
        if rank == 0:
            torch.save(g, out_file)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("workload", ["mip", "barf", "ingp"])
def test_two_ranks_equal_the_whole_batch(workload):
    with tempfile.TemporaryDirectory() as tmp:
        init_file, out_file = os.path.join(tmp, "rdzv"), os.path.join(tmp, "g.pt")
        mp.spawn(_worker, args=(2, init_file, out_file, workload), nprocs=2, join=True)
        dp = torch.load(out_file, weights_only=True)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        modules, loss = _setup(torch.device("cuda", 0), workload)
        ref = _grads(modules, loss, slice(0, B))
    finally:
        torch.set_float32_matmul_precision(prev)
    assert dp.keys() == ref.keys() and len(ref) > 0
    if workload == "barf":
        assert any(k.startswith("1.") for k in ref)          # the camera extrinsics were reduced
    for n in ref:
        scale = ref[n].abs().max().clamp_min(1e-30)
        assert (dp[n] - ref[n]).abs().max() <= 1e-5 * scale, n
