"""cfg5 chunked path probe: per-call time of 4800-frame process_device calls (8 ch f64 96k->44.1k
VeryHigh), kernel time by kind (library events), first launch geometries (GAR_BG_TRACE=1)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import torch  # noqa: E402
import gar  # noqa: E402
ir, orr, C = float(os.environ.get("P_IN", 96000)), float(os.environ.get("P_OUT", 44100)), int(os.environ.get("P_CH", 8))
chunk, nchunks = int(os.environ.get("P_CHUNK", 4800)), int(os.environ.get("P_N", 1200))
cd = getattr(gar, os.environ.get("P_DT", "F64"))
x = (torch.rand((chunk * nchunks, C), device="cuda", dtype=torch.float64 if cd == gar.F64 else torch.float32) - 0.5)
r = gar.New(gar.Config(ir, orr, C, gar.QualityVeryHigh, ComputeDtype=cd))
y = torch.empty((int(chunk * nchunks * orr / ir) + 64 * (nchunks + 1), C), dtype=x.dtype, device="cuda")
def run():
    r.Reset(); o = 0
    for i in range(nchunks):
        j = 0 if os.environ.get("P_REUSE") else i  # P_REUSE: every call reads the same chunk (cache / TLB warm)
        o += r.process_device(x[j * chunk:(j + 1) * chunk], out=y[o:]).shape[0]
    return o
run(); torch.cuda.synchronize()
r.profile(True)
for k in range(6): r.profile_read(k)
t0 = time.perf_counter(); run(); torch.cuda.synchronize(); dt = time.perf_counter() - t0
print(f"calls {nchunks} us_per_call {dt / nchunks * 1e6:.2f} msamples_per_s {chunk * nchunks * C / dt / 1e6:.1f}")
for k in range(6):
    ms, n = r.profile_read(k)
    if n: print(f"kind {k}: {n} launches, {ms / n * 1000:.2f} us per launch, {ms / nchunks * 1000:.2f} us per call")
r.profile(False)
t0 = time.perf_counter(); run(); torch.cuda.synchronize(); dt = time.perf_counter() - t0
print(f"no-profile: us_per_call {dt / nchunks * 1e6:.2f} msamples_per_s {chunk * nchunks * C / dt / 1e6:.1f}")
