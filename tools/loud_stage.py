"""Where the float32 split path goes wrong on loud samples (odd channel counts): error runs of two
identical runs against the oracle, per channel.  LP_CH channels, LP_CASE 'ir,or,Preset'."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np  # noqa: E402
import gar  # noqa: E402
from helpers import oracle_new, signal  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()
CH = int(os.environ.get("LP_CH", "3"))
ir, orr, p = os.environ.get("LP_CASE", "8000,88200,High").split(",")
ir, orr = int(ir), int(orr)
x = signal(12000, CH, ir, seed=5)
x[3000:3040, 0] *= 1e5
x[7000, 0] = 40.0
x = x.astype(np.float32).astype(np.float64)
want = oracle_new(O, ir, orr, x, getattr(O, "P_" + p.upper()))


def runs(mask):
    idx = np.flatnonzero(mask)
    if not len(idx):
        return []
    cut = np.flatnonzero(np.diff(idx) > 1)
    starts = np.r_[idx[0], idx[cut + 1]]
    ends = np.r_[idx[cut], idx[-1]]
    return list(zip(starts.tolist(), ends.tolist()))


for rep in range(2):
    r = gar.New(gar.Config(ir, orr, CH, getattr(gar, "Quality" + p), ComputeDtype=gar.F32))
    if rep == 0:
        print("stages", [(round(r.stage_geometry(j)[0], 4), int(r.stage_geometry(j)[1].kind))
                         for j in range(r.num_stages())], flush=True)
    outs = r.ProcessMulti([x[:, c] for c in range(CH)])
    tails = r.FlushMulti()
    for c in range(CH):
        g = np.concatenate([outs[c], tails[c]])
        w = np.asarray(want[c])
        tol = 1e-3 * max(1.0, np.abs(w).max())
        bad = np.abs(g - w) > tol
        rr = runs(bad)
        print(f"rep{rep} c{c}: n={len(g)} bad={int(bad.sum())} runs={len(rr)} first={rr[:12]}", flush=True)
