"""The full-view render (NerfInterpolation.render_image, the reference's image logger loop:
barf/image_logger.py:155-206 — batches of rays through forward, the fine rgb clipped to [0, 1]) on the
C3 mip configuration: every batch goes through nerf_mlp_fused_render (no stand-alone encoding or
compositing launch), and the image equals forward() of the same rays batch by batch
(bitwise: the same launches on the same inputs; equidistant samples, so no random draws)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_render_image_is_forward_per_batch_on_the_fused_path():
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    from nerf_amd import kernels as K
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
        pos.pixel_width_sigma = 0.0
        dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
        model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
        ren = NerfInterpolation(2.0, 8.0, model, 128, "equidistant", 0.0, "middle", model, 64).to(dev)
        g = torch.Generator().manual_seed(2)
        n = 5000                                   # two batches of 4096 rays, the second ragged
        o = (torch.randn(n, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
        d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]),
                                          dim=1).to(dev)
        pw = torch.full((n, 1), 1 / 1111.1, device=dev)
        timer, saved = K.KernelTimer(), K.TIMER
        K.TIMER = timer
        try:
            img = ren.render_image(o, d, pw, batch_size=4096)
        finally:
            K.TIMER = saved
        ks = timer.summary()
        assert "encode_fwd" not in ks and "composite_fwd" not in ks, sorted(ks)
        assert ks["mlp_fused_fwd"]["launches"] == 4               # coarse + fine per batch
        with torch.no_grad():
            ref = torch.cat([ren(o[i:i + 4096], d[i:i + 4096], pw[i:i + 4096])[0].clip(0, 1)
                             for i in range(0, n, 4096)])
        assert torch.equal(img, ref)
        assert img.min() >= 0 and img.max() <= 1
    finally:
        torch.set_float32_matmul_precision(prev)


def test_render_image_default_batch_stays_on_the_fused_path():
    """With the default 65536-ray batch the passes' rows would pass the fused launch's 32-bit
    addressing (mlp_fused.eligible); render_image halves its batch until they fit, so the full view
    still launches no stand-alone encoding or compositing kernel (bench.py's frame_render)."""
    from nerf_amd import BarfPositionalEncoding, IntegratedBarfFourierFeatures, NerfInterpolation, NerfModel
    from nerf_amd import kernels as K
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("high")
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        pos = IntegratedBarfFourierFeatures(10, 10, 1.28, 6.4, True, 1.0, True)
        pos.pixel_width_sigma = 0.0
        dirs = BarfPositionalEncoding(4, 4, 1.28, 6.4, True, 1.0)
        model = NerfModel(4, 256, True, False, 2, pos, dirs, 5e-4, 1e-4, 200000)
        ren = NerfInterpolation(2.0, 8.0, model, 128, "equidistant", 0.0, "middle", model, 64).to(dev)
        g = torch.Generator().manual_seed(3)
        n = 20000
        o = (torch.randn(n, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, 4.0])).to(dev)
        d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g) * 0.2 - torch.tensor([0.0, 0.0, 1.0]),
                                          dim=1).to(dev)
        timer, saved = K.KernelTimer(), K.TIMER
        K.TIMER = timer
        try:
            img = ren.render_image(o, d, 1 / 1111.1)
        finally:
            K.TIMER = saved
        ks = timer.summary()
        assert "encode_fwd" not in ks and "composite_fwd" not in ks and "linear_nt_x3" not in ks, sorted(ks)
        assert ks["mlp_fused_fwd"]["launches"] == 6               # 3 batches of 8192 rays x 2 passes
        assert torch.isfinite(img).all() and img.min() >= 0 and img.max() <= 1
    finally:
        torch.set_float32_matmul_precision(prev)
