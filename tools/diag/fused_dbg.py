"""Debug helper: where the fused forward differs from the layer-by-layer path."""
import sys
import torch
sys.path[:0] = ["/root/repo", "/root/repo/nerf-experiments_amd", "/root/repo/tests"]
import test_gpu_fused as T  # noqa: E402
import nerf_amd  # noqa: E402
nerf_amd._lib.load()
torch.set_float32_matmul_precision("high")
for M in (64 * 256, 64 * 512, 4096 * 64):
    rd = 64
    model = T._model("n2v").to("cuda")
    g = torch.Generator(device="cuda").manual_seed(11)
    pos_pe = torch.zeros(M, 64, device="cuda")
    pos_pe[:, :60] = torch.rand(M, 60, device="cuda", generator=g) * 2 - 1
    dir_pe = torch.zeros(M // rd, 32, device="cuda")
    dir_pe[:, :24] = torch.rand(M // rd, 24, device="cuda", generator=g) * 2 - 1
    plan = model._get_plan()
    plan.to_device(torch.device("cuda"))
    _, a_ref, _, _ = T._run(model, pos_pe, dir_pe, rd, False)
    _, a_fus, _, _ = T._run(model, pos_pe, dir_pe, rd, True)
    for li in (0, 1, 2, 5, 11):
        n = plan.layers[li].N
        x, y = a_ref[li][:, :n], a_fus[li][:, :n]
        bad = ((x - y).abs() > 1e-4 * max(1.0, x.abs().max().item())).nonzero()
        rows = bad[:, 0].unique()
        cols = bad[:, 1].unique()
        print(f"M={M} layer {li}: nbad {bad.shape[0]} rows {rows.numel()} rows%64 {(rows % 64).unique()[:8].tolist()} "
              f"tiles {(rows // 64).unique()[:6].tolist()} cols {cols.min().item() if cols.numel() else -1}.."
              f"{cols.max().item() if cols.numel() else -1} ({cols.numel()})")
