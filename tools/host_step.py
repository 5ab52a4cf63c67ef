"""Host-side cost of one bench step (Reset, process_device, flush_device) with the GPU kept busy:
per-call host microseconds, without and with library profiling events."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import torch, gar
frames, ch = 600 * 44100, 2
x = torch.rand((frames, ch), device="cuda") - 0.5
r = gar.New(gar.Config(44100, 48000, ch, gar.QualityHigh, ComputeDtype=gar.F32))
n = gar.lib().gar_device_output_size(r._h, frames)
y = torch.empty((n, ch), device="cuda")
yf = torch.empty((8192, ch), device="cuda")
for prof in (False, True):
    r.profile(prof)
    for _ in range(3):
        r.Reset(); r.process_device(x, out=y); r.flush_device(out=yf)
    torch.cuda.synchronize()
    t = {"reset": 0.0, "process": 0.0, "flush": 0.0}
    K = 20
    t0 = time.perf_counter()
    for _ in range(K):
        a = time.perf_counter(); r.Reset()
        b = time.perf_counter(); r.process_device(x, out=y)
        c = time.perf_counter(); r.flush_device(out=yf)
        d = time.perf_counter()
        t["reset"] += b - a; t["process"] += c - b; t["flush"] += d - c
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print({"profile": prof, **{k: round(v / K * 1e6, 1) for k, v in t.items()}, "host_us_per_step": round((t1 - t0) / K * 1e6, 1),
           "gpu_us_per_step": round((t2 - t0) / K * 1e6, 1)})
    if prof:
        for k in range(6):
            r.profile_read(k)
