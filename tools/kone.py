"""One process: resample the bench workload a few times (env GAR_HX_* knobs apply); for rocprofv3 runs."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import torch  # noqa: E402
import gar  # noqa: E402
frames = int(float(os.environ.get("KB_SECONDS", "600")) * 44100)
ch = int(os.environ.get("KB_CH", "2"))
rin, rout = float(os.environ.get("KB_IN", "44100")), float(os.environ.get("KB_OUT", "48000"))
q = int(os.environ.get("KB_Q", "3"))
x = (torch.rand((frames, ch), device="cuda") - 0.5)
r = gar.New(gar.Config(rin, rout, ch, q, ComputeDtype=gar.F32))
n = gar.lib().gar_device_output_size(r._h, frames)
y = torch.empty((n, ch), device="cuda")
for _ in range(int(os.environ.get("KB_REPS", "3"))):
    r.Reset()
    r.process_device(x, out=y)
torch.cuda.synchronize()
print("ok")
