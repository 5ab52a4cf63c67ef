"""One engine-seam case (gar_new_engine_quality): where the output departs from the oracle's engine.
SP_CASE 'ir,or,q,dtype[,chunk]'."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np  # noqa: E402
import gar  # noqa: E402
from helpers import chunk_sizes, signal  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()
f = os.environ.get("SP_CASE", "11025,176400,2,F64").split(",")
ir, orr, q, dtype = int(f[0]), int(f[1]), int(f[2]), f[3]
chunk = int(f[4]) if len(f) > 4 else None
frames = int(os.environ.get("SP_FRAMES", "9000"))
x = signal(frames, 1, ir, seed=ir + 3 * orr + q)[:, 0]
for rep in range(2):
    r = gar.EngineNewResampler(ir, orr, q, getattr(gar, dtype))
    e = O.Engine(ir, orr, q)
    parts, want, s, lens = [], [], 0, []
    for n in (chunk_sizes(frames, chunk) if chunk else [frames]):
        seg = x[s:s + n]
        parts.append(r.Process(seg) if dtype == "F64" else r.ProcessFloat32(seg.astype(np.float32)))
        want.append(e.process(seg))
        lens.append((len(parts[-1]), len(want[-1])))
        s += n
    parts.append(r.Flush())
    want.append(e.flush())
    lens.append((len(parts[-1]), len(want[-1])))
    got = np.concatenate(parts).astype(np.float64)
    w = np.concatenate(want)
    d = np.abs(got - w)
    bad = np.flatnonzero(~(d <= 1e-9))
    print(f"rep{rep} lens {lens[:3]}..{lens[-2:]} n={len(got)} bad={len(bad)}", flush=True)
    if len(bad):
        print("  first/last bad", bad[:8].tolist(), bad[-4:].tolist(), "got", got[bad[:4]].tolist(),
              "want", w[bad[:4]].tolist(), flush=True)
