"""HBM calibration on the box: torch copy / fill / read (sum) of cfg2-sized buffers, GB/s."""
import json
import torch

def timed(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3

n = 57_600_000  # cfg2 outputs (f32)
x = torch.rand(n, device="cuda")
y = torch.empty_like(x)
res = {}
t = timed(lambda: y.copy_(x)); res["copy_TBps"] = 2 * 4 * n / t / 1e12
t = timed(lambda: y.fill_(1.0)); res["fill_TBps"] = 4 * n / t / 1e12
t = timed(lambda: x.sum()); res["sum_TBps"] = 4 * n / t / 1e12
print(json.dumps({k: round(v, 3) for k, v in res.items()}))
