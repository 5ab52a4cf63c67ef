"""Debug: which outputs of a loud (1e30-scaled) stream come out non-finite."""
import os, sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go-audio-resampler_amd"), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
import numpy as np, torch, gar
from helpers import signal
x = (signal(40000, 2, 44100, seed=7) * float(sys.argv[1] if len(sys.argv) > 1 else 1e30)).astype(np.float32)
r = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=gar.F32))
xd = torch.from_numpy(x).cuda()
y = r.process_device(xd).cpu().numpy()
bad = np.nonzero(~np.isfinite(y))
print("process:", y.shape, "nonfinite", len(bad[0]), bad[0][:20], bad[1][:20], y[bad][:5])
f = r.flush_device().cpu().numpy()
bad = np.nonzero(~np.isfinite(f))
print("flush:", f.shape, "nonfinite", len(bad[0]), bad[0][:20])
print("sample vals", y[1000:1003], y[-3:])
