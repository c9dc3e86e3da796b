"""The direct gradient sink on the GPU at world size 1 (bench.py's default).

Per-pass weight gradients (NERF_MERGE_PASSES=0 semantics): the mip step's field MLP gradients
written by the slab reduce into .grad (accumulate epilogue for the second pass) are bitwise the
gradients autograd's accumulation gives (the same fp32 add of the two passes' rounded sums), and
the 27 separate adds of the shared field disappear.

Merged passes (the default in split precision): the first backward stashes each layer's rows and
the second runs one weight-gradient launch over both passes' rows — the same products, summed in
one fp32 split-M order instead of two: equal to autograd's within 1e-5 of each gradient's scale.
A stash whose partner pass never runs its backward is flushed by finish(): the gradient of the one
pass that ran, bitwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mip(dev):
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    torch.manual_seed(0)
    pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
    pos.pixel_width_sigma = 0.0
    dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
    model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
    return NerfInterpolation(2.0, 8.0, model, 128, "stratified_uniform", -1.0, "middle", model, 64).to(dev)


def _batch(dev):
    g = torch.Generator().manual_seed(3)
    B = 512
    o = (torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]),
                                      dim=1).to(dev)
    pw = torch.full((B,), 1 / 1111.1, device=dev)
    c = torch.rand(B, 3, generator=g).to(dev)
    return o, d, pw, c


@pytest.mark.parametrize("precision", ["high", "highest"])
def test_direct_sink_matches_autograd_bitwise(precision):
    from nerf_amd import mlp
    from nerf_amd.ddp import BucketedGradAllReduce
    dev = torch.device("cuda", 0)
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    merge = mlp.MERGE_PASSES
    mlp.MERGE_PASSES = False
    try:
        ren = _mip(dev)
        g = torch.Generator().manual_seed(3)
        B = 512
        o = (torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
        d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]),
                                          dim=1).to(dev)
        pw = torch.full((B,), 1 / 1111.1, device=dev)
        c = torch.rand(B, 3, generator=g).to(dev)
        grads = []
        for direct in (False, True):
            ar = BucketedGradAllReduce(list(ren.parameters()), direct=direct)
            try:
                for p in ren.parameters():
                    p.grad = None
                torch.manual_seed(11)                 # same stratification draws
                loss, _ = ren.training_loss(o, d, pw, c)
                loss.backward()
                ar.finish()
                grads.append({n: p.grad.clone() for n, p in ren.named_parameters()})
            finally:
                ar.remove()
        assert mlp.GRAD_SINK is None
        for n in grads[0]:
            assert torch.equal(grads[0][n], grads[1][n]), n
    finally:
        mlp.MERGE_PASSES = merge
        torch.set_float32_matmul_precision(old)


def _grads(ren, dev, direct, merge, passes="both"):
    from nerf_amd import mlp
    from nerf_amd.ddp import BucketedGradAllReduce
    o, d, pw, c = _batch(dev)
    saved = mlp.MERGE_PASSES
    mlp.MERGE_PASSES = merge
    ar = BucketedGradAllReduce(list(ren.parameters()), direct=direct)
    try:
        for p in ren.parameters():
            p.grad = None
        torch.manual_seed(11)
        if passes == "both":
            loss, _ = ren.training_loss(o, d, pw, c)
        else:
            # both passes run forward (two claims), only the fine one reaches the loss
            rgb_f, rgb_c = ren(o, d, pw)
            loss = torch.nn.functional.mse_loss(rgb_f, c) + 0.0 * rgb_c.detach().sum()
        loss.backward()
        ar.finish()
        torch.cuda.synchronize()
        return {n: p.grad.clone() for n, p in ren.named_parameters() if p.grad is not None}
    finally:
        ar.remove()
        mlp.MERGE_PASSES = saved


def test_merged_passes_match_autograd():
    dev = torch.device("cuda", 0)
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        ren = _mip(dev)
        ref = _grads(ren, dev, direct=False, merge=False)
        got = _grads(ren, dev, direct=True, merge=True)
        assert ref.keys() == got.keys()
        for n in ref:
            scale = ref[n].abs().max().clamp_min(1e-30)
            assert ((got[n] - ref[n]).abs().max() <= 1e-5 * scale).item(), n
        # a claimed pass without a backward: the stash is flushed alone, bitwise the per-pass result
        one_ref = _grads(ren, dev, direct=True, merge=False, passes="fine")
        one_got = _grads(ren, dev, direct=True, merge=True, passes="fine")
        assert one_ref.keys() == one_got.keys()
        for n in one_ref:
            assert torch.equal(one_ref[n], one_got[n]), n
    finally:
        torch.set_float32_matmul_precision(old)
