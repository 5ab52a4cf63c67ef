import os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd"), os.path.join(ROOT, "tests")]
import torch, gar
from oracle import oracle as O
from helpers import signal
O.build()
for (i, o) in [(48000, 44100), (44100, 48000), (96000, 48000)]:
    x = signal(i // 2, 1, i, seed=3)[:, 0].astype(np.float32)
    e32 = O.Engine(i, o, O.HIGH, f32=True)
    w_p = e32.process(x); w_f = e32.flush()
    r = gar.NewEngineFloat32(i, o, gar.QualityHigh)
    gp = np.asarray(r.ProcessFloat32(x)); gf = np.asarray(r.Flush()) if hasattr(r, "Flush") else None
    print(i, o, "info", r.GetInfo() if hasattr(r, "GetInfo") else None)
    print(" process", len(gp), len(w_p), "nan", np.isnan(gp).sum(), "first nan", np.argmax(np.isnan(gp)) if np.isnan(gp).any() else -1,
          "rms", np.sqrt(np.nanmean((gp[:len(w_p)] - w_p[:len(gp)]) ** 2)))
    if gf is not None:
        print(" flush", len(gf), len(w_f), "nan", np.isnan(gf).sum(), np.where(np.isnan(gf))[0][:10],
              "rms", np.sqrt(np.nanmean((gf[:len(w_f)] - w_f[:len(gf)]) ** 2)))
    d = gar.design_engine(float(i), float(o), gar.Engine24Bit)[0]
    print(" geom", {k: getattr(d, k) for k, _ in d._fields_})
