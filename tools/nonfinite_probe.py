"""Non-finite input samples (Inf / NaN) through every compute dtype and stage kind: where the device
output is NaN / +-Inf against the oracle (the reference's loops over the true taps only)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gar  # noqa: E402
from helpers import oracle_new, signal  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()
for ir, orr, preset in [(96000, 48000, "QualityVeryHigh"), (44100, 48000, "QualityHigh"), (22050, 44100, "QualityHigh"),
                        (16000, 11025, "QualityHigh"), (48000, 16000, "QualityMedium")]:
    x = signal(12000, 2, ir, seed=3).astype(np.float32).astype(np.float64)
    x[5000, 0] = np.inf
    x[7000, 1] = np.nan
    want = oracle_new(O, ir, orr, x, getattr(O, "P_" + preset[7:].upper()))
    for dt in ("F64", "F32", "F32_EXACT"):
        r = gar.New(gar.Config(ir, orr, 2, getattr(gar, preset), ComputeDtype=getattr(gar, dt)))
        tdt = torch.float64 if dt == "F64" else torch.float32
        xd = torch.from_numpy(x).to(tdt).cuda()
        got = torch.cat([r.process_device(xd), r.flush_device(dtype=tdt)]).double().cpu().numpy()
        row = []
        for c in range(2):
            w = np.asarray(want[c])
            g = got[:, c]
            row.append(f"c{c} nan g/w {int(np.isnan(g).sum())}/{int(np.isnan(w).sum())} inf g/w {int(np.isinf(g).sum())}/{int(np.isinf(w).sum())}"
                       f" nan-only-g {int((np.isnan(g) & ~np.isnan(w)).sum())} nonfin-only-w {int((~np.isfinite(w) & np.isfinite(g)).sum())}")
        print(f"{ir}->{orr} {preset[7:]} {dt}: " + " | ".join(row), flush=True)
