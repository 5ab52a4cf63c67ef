"""Streaming probe: 4096-frame process_device calls (stereo f32 44.1k->48k High by default), us per call."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import torch  # noqa: E402
import gar  # noqa: E402
C, chunk, n = int(os.environ.get("P_CH", 2)), int(os.environ.get("P_CHUNK", 4096)), int(os.environ.get("P_N", 600))
x = (torch.rand((chunk * n, C), device="cuda") - 0.5)
r = gar.New(gar.Config(44100, 48000, C, gar.QualityHigh, ComputeDtype=gar.F32))
y = torch.empty((int(chunk * n * 48000 / 44100) + 64 * (n + 1), C), device="cuda")
def run():
    r.Reset(); o = 0
    for i in range(n):
        o += r.process_device(x[i * chunk:(i + 1) * chunk], out=y[o:]).shape[0]
run(); torch.cuda.synchronize()
t0 = time.perf_counter(); run(); torch.cuda.synchronize(); dt = time.perf_counter() - t0
print(f"us_per_call {dt / n * 1e6:.2f}")
