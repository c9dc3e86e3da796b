"""Practical HBM rates on this GPU for the roofline discussion: a write-only
stream (torch fill_ of 4 GiB), a read-only stream (sum of 4 GiB) and a copy (4 GiB read + 4 GiB
written), each timed with HIP events over 10 repetitions after a warm-up.  Prints one JSON line."""
import json

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


n = (4 << 30) // 4
x = torch.empty(n, device="cuda", dtype=torch.float32)
y = torch.empty_like(x)
x.fill_(1.0)
out = torch.empty((), device="cuda")
w = timed(lambda: x.fill_(2.0))
r = timed(lambda: torch.sum(x, dim=0, out=out))
c = timed(lambda: y.copy_(x))
gb = 4 * n / 1e9
print(json.dumps({"write_only_TBs": gb / w / 1e3, "read_only_TBs": gb / r / 1e3, "copy_TBs_read_plus_write": 2 * gb / c / 1e3,
                  "bytes_per_pass": 4 * n}))
