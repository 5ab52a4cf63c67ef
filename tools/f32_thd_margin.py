"""THD of the float32 HIP paths (split-f16 F32, exact F32_EXACT) against the reference's own float32
engine (the oracle's Resampler[float32] restatement) on every GPU quality case: prints the margin
(HIP THD - reference float32 THD, dB; negative = the HIP output is cleaner) so the tolerance in
tests/test_quality.py can be set from measurements.  GPU box only."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np  # noqa: E402
import quality as Q  # noqa: E402
from oracle import oracle as O  # noqa: E402
import gar  # noqa: E402

O.build()
worst = {}
for ir, orr, name in Q.THD_CASES:
    q = Q.ENGINE_Q[name]

    def o32(x):
        e = O.Engine(ir, orr, q, f32=True)
        x = np.asarray(x, dtype=np.float32)
        return np.concatenate([e.process(x), e.flush()]).astype(np.float64)
    t_o = Q.thd_internal(o32, ir, orr)
    row = [f"{name:8s} {ir}->{orr}", f"ref f32 {t_o:8.2f}"]
    for dt in ("F32", "F32_EXACT"):
        def g(x, dt=dt):
            r = gar.EngineNewResampler(ir, orr, q, getattr(gar, dt))
            return np.concatenate([r.ProcessFloat32(np.asarray(x, np.float32)), r.Flush()]).astype(np.float64)
        t_g = Q.thd_internal(g, ir, orr)
        row.append(f"{dt} {t_g:8.2f} ({t_g - t_o:+.2f})")
        worst[dt] = max(worst.get(dt, -1e9), t_g - t_o)
    print("  ".join(row), flush=True)
print("worst margin (dB):", {k: round(v, 3) for k, v in worst.items()})
