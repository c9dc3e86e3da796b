"""The fused forward on 32-sample waves (NERF_FUSED_W32=1: mlp_fused32_kernel, one wave per SIMD on
v_mfma_f32_32x32x16_bf16; csrc/mlp_fused.hip) — the checks of test_gpu_fused.py,
test_gpu_fused_composite.py and test_gpu_fused_encoding.py with the switch on, plus the two forward
kernels against each other.

Same image, descriptors and outputs as the 16-sample kernel; the fp32 sums run in another order
(biases first, 16-deep k-steps), so rows agree within the split-precision bar of test_gpu_fused.py
(1e-4 of the layer's max |value|) and ReLU bits wherever the activation is not within 1e-5 of zero.
Within one kernel the contracts stay bitwise: the fused composite's rgb / weights equal the
stand-alone compositing of the same kernel's heads (S = 16 .. 256: two rays per wave at S = 16, one
ray over two tiles at S = 256), and in-kernel encodings equal the encoding launches'."""
import numpy as np
import pytest
import torch

import test_gpu_fused as F
import test_gpu_fused_composite as FC
import test_gpu_fused_encoding as FE

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import nerf_amd
    nerf_amd._lib.load()
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    yield
    torch.set_float32_matmul_precision(prev)


@pytest.fixture(autouse=True)
def _w32(monkeypatch):
    monkeypatch.setenv("NERF_FUSED_W32", "1")


@pytest.mark.parametrize("name,M,rd", [("n2v", 4096 * 64, 64), ("n2v", 1000, 1), ("barf", 4096 * 8 + 37, 1),
                                       ("barf", 64, 64), ("n2v", 3 * 64 + 5, 1)])
def test_w32_forward_matches_layerwise(name, M, rd):
    F.test_fused_forward_matches_layerwise(name, M, rd)


def test_w32_against_the_16_sample_kernel(monkeypatch):
    """Both forward kernels on the same rows: every layer output within the bar, ReLU bits equal
    away from zero — and not bitwise equal (the switch selects another kernel)."""
    model = F._model("n2v").to(DEV)
    g = torch.Generator(device=DEV).manual_seed(21)
    M, rd = 4096 * 16 + 77, 1
    pos_pe = torch.zeros(M, 64, device=DEV)
    pos_pe[:, :63] = torch.rand(M, 63, device=DEV, generator=g) * 2 - 1
    dir_pe = torch.zeros(M, 32, device=DEV)
    dir_pe[:, :27] = torch.rand(M, 27, device=DEV, generator=g) * 2 - 1
    plan = model._get_plan()
    plan.to_device(torch.device(DEV))
    monkeypatch.setenv("NERF_FUSED_W32", "0")
    _, a16, m16, _ = F._run(model, pos_pe, dir_pe, rd, True)
    monkeypatch.setenv("NERF_FUSED_W32", "1")
    _, a32, m32, _ = F._run(model, pos_pe, dir_pe, rd, True)
    differs = False
    for li, (x, y) in enumerate(zip(a16, a32)):
        n = plan.layers[li].N
        scale = max(1.0, x[:, :n].abs().max().item())
        err = (x[:, :n] - y[:, :n]).abs().max().item()
        assert err <= 1e-4 * scale, (li, err, scale)
        differs = differs or not torch.equal(x[:, :n], y[:, :n])
        if y.shape[1] > n:
            assert (y[:, n:] == 0).all()
        ma, mb = m16[li], m32[li]
        assert (ma is None) == (mb is None)
        if ma is None:
            continue
        order = F._fused_mask_order()
        bits_a = np.unpackbits(ma.cpu().numpy(), axis=1, bitorder="little")[:, order]
        bits_b = np.unpackbits(mb.cpu().numpy(), axis=1, bitorder="little")[:, order]
        act = x[:, :n].cpu().numpy()
        near0 = np.abs(act) <= 1e-5 * max(1.0, np.abs(act).max())
        assert not ((bits_a[:, :n] != bits_b[:, :n]) & ~near0).any(), li
        # bits past N are zero in both layouts' unused nibbles
        if n < 256:
            assert (bits_b[:, n:] == bits_a[:, n:]).all(), li
    assert differs


def test_w32_forward_vs_oracle_subset():
    F.test_fused_forward_vs_oracle_subset()


@pytest.mark.parametrize("n_rays,S,delayed", [(4096, 64, False), (4096, 128, False), (37, 64, False),
                                              (301, 32, False), (75, 16, False), (203, 128, True),
                                              (1024, 256, False), (37, 256, False), (45, 256, True)])
def test_w32_fused_composite_bitwise_and_gradients(n_rays, S, delayed):
    FC.test_fused_composite_forward_bitwise_and_gradients(n_rays, S, delayed)


@pytest.mark.parametrize("kind,n_rays,S,query,pw_mode", [
    ("mip", 4096, 64, 1, 0), ("mip", 37, 65, 1, 2), ("barf", 129, 3, 1, 0), ("n2v", 1000, 7, 0, 0),
    ("ingp_dirs", 64, 64, 0, 0)])
def test_w32_generated_encodings_bitwise(kind, n_rays, S, query, pw_mode):
    FE.test_generated_encodings_bitwise(kind, n_rays, S, query, pw_mode)


@pytest.mark.parametrize("kind", ["mip", "barf"])
def test_w32_generated_encodings_training_step_bitwise(kind):
    FE.test_generated_encodings_training_step_bitwise(kind)
