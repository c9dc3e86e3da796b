"""The direct gradient sink on the GPU at world size 1 (bench.py's default): the mip step's field
MLP gradients written by the slab reduce into .grad (accumulate epilogue for the second pass) are
bitwise the gradients autograd's accumulation gives (the same fp32 add of the two passes' rounded
sums), and the 27 separate adds of the shared field disappear."""
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


@pytest.mark.parametrize("precision", ["high", "highest"])
def test_direct_sink_matches_autograd_bitwise(precision):
    from nerf_amd import mlp
    from nerf_amd.ddp import BucketedGradAllReduce
    dev = torch.device("cuda", 0)
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
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
        torch.set_float32_matmul_precision(old)
