"""One process: the poly bench workload (stereo f32 16k->44.1k QualityHigh, x != 0) a few times (for rocprofv3)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import torch  # noqa: E402
import gar  # noqa: E402
frames = int(float(os.environ.get("KB_SECONDS", "600")) * 16000)
x = (torch.rand((frames, 2), device="cuda") - 0.5)
r = gar.New(gar.Config(16000, 44100, 2, gar.QualityHigh, ComputeDtype=gar.F32))
y = torch.empty((int(frames * 44100 / 16000) + 4096, 2), device="cuda")
for _ in range(int(os.environ.get("KB_REPS", "2"))):
    r.Reset()
    r.process_device(x, out=y)
torch.cuda.synchronize()
print("ok")
