"""Debug helper: compare the fused forward's ReLU mask bits with the layer-by-layer path."""
import sys
import numpy as np
import torch
sys.path[:0] = ["/root/repo", "/root/repo/nerf-experiments_amd", "/root/repo/tests"]
import test_gpu_fused as T  # noqa: E402
import nerf_amd  # noqa: E402
nerf_amd._lib.load()
torch.set_float32_matmul_precision("high")
M, rd = 64 * 256, 64
model = T._model("n2v").to("cuda")
g = torch.Generator(device="cuda").manual_seed(11)
pos_pe = torch.zeros(M, 64, device="cuda")
pos_pe[:, :60] = torch.rand(M, 60, device="cuda", generator=g) * 2 - 1
dir_pe = torch.zeros(M // rd, 32, device="cuda")
dir_pe[:, :24] = torch.rand(M // rd, 24, device="cuda", generator=g) * 2 - 1
_, a_ref, m_ref, _ = T._run(model, pos_pe, dir_pe, rd, False)
_, a_fus, m_fus, _ = T._run(model, pos_pe, dir_pe, rd, True)
ma = m_ref[0].cpu().numpy().view(np.uint32)
mb = m_fus[0].cpu().numpy().view(np.uint32)
for row in (0, 1, 17, 63):
    print(row, [f"{x:08x}" for x in ma[row]], [f"{x:08x}" for x in mb[row]])
diff = (ma != mb)
print("rows with diff", diff.any(1).sum(), "words with diff", diff.sum(0))
