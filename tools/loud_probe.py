"""Loud samples (|x| >= 16) on the float32 split path, stage kind by stage kind (engine seam) and for
the New-path pipelines the sweep flagged: RMS against the oracle next to exact-f32's."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np  # noqa: E402
import gar  # noqa: E402
from helpers import oracle_new, rms, signal  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()


def sig(n, rate, ch=1):
    x = signal(n, ch, rate, seed=5)
    x[3000:3040, 0] *= 1e5
    x[7000, 0] = 40.0
    return x.astype(np.float32).astype(np.float64)


for ir, orr, q in [(8000, 16000, 3), (11025, 22050, 3), (16000, 32000, 3), (44100, 88200, 3), (8000, 11025, 3),
                   (96000, 48000, 3), (44100, 48000, 3), (22050, 44100, 4), (16000, 48000, 3)]:
    x = sig(12000, ir)[:, 0]
    out = {}
    for dt in ("F32", "F32_EXACT"):
        r = gar.EngineNewResampler(ir, orr, q, getattr(gar, dt))
        out[dt] = np.concatenate([r.ProcessFloat32(x.astype(np.float32)), r.Flush()]).astype(np.float64)
    e = O.Engine(ir, orr, q)
    w = np.concatenate([e.process(x), e.flush()])
    print(f"engine {ir}->{orr} q{q}: F32 {rms(out['F32'], w):.3g} exact {rms(out['F32_EXACT'], w):.3g}", flush=True)
CH = int(os.environ.get("LP_CH", "1"))
for ir, orr, p in [(8000, 176400, "High"), (8000, 88200, "High"), (8000, 48000, "High"), (11025, 96000, "High"),
                   (8000, 16000, "High"), (44100, 48000, "High"), (16000, 11025, "High")]:
    x = sig(12000, ir, CH)
    want = oracle_new(O, ir, orr, x, getattr(O, "P_" + p.upper()))
    res = {}
    for dt in ("F32", "F32_EXACT"):
        r = gar.New(gar.Config(ir, orr, CH, getattr(gar, "Quality" + p), ComputeDtype=getattr(gar, dt)))
        st = [(round(r.stage_geometry(j)[0], 4), int(r.stage_geometry(j)[1].kind)) for j in range(r.num_stages())]
        outs = r.ProcessMulti([x[:, c] for c in range(CH)])
        tails = r.FlushMulti()
        res[dt] = max(rms(np.concatenate([outs[c], tails[c]]), want[c]) for c in range(CH))
    print(f"New {CH}ch {ir}->{orr} {p} stages {st}: F32 {res['F32']:.3g} exact {res['F32_EXACT']:.3g}", flush=True)
