"""Output bits of one library build vs another on the same input (A/B correctness of kernel variants).
usage: GAR_LIB_PATH=<lib> python tools/bitcmp.py <out.npy> [ch] [seconds] [in_rate] [out_rate]
Writes the float32 output of one one-shot Process + Flush of a seeded stream (device API)."""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go-audio-resampler_amd")]
import torch
import gar

out = sys.argv[1]
ch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
sec = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
ir = float(sys.argv[4]) if len(sys.argv) > 4 else 44100.0
orr = float(sys.argv[5]) if len(sys.argv) > 5 else 48000.0
frames = int(sec * ir)
g = torch.Generator(device="cuda").manual_seed(7)
x = (torch.rand((frames, ch), device="cuda", generator=g) - 0.5) * 1.8
r = gar.New(gar.Config(ir, orr, ch, 3 if orr > ir else 4, ComputeDtype=gar.F32))
y = r.process_device(x)
yf = r.flush_device()
torch.cuda.synchronize()
np.save(out, torch.cat([y, yf]).cpu().numpy())
print("saved", out, tuple(y.shape), tuple(yf.shape))
