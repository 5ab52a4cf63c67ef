import os, sys
sys.path[:0] = ["/root/repo/tests", "/root/repo", "/root/repo/go-audio-resampler_amd"]
os.environ.pop("GAR_SWEEP_SEED", None)
import numpy as np, torch
import test_gpu_sweep as T
import gar
from oracle import oracle as O
from helpers import signal, oracle_new, chunk_sizes, rms
O.build()
want_ids = sys.argv[1:]
for case in T.LOUD:
    ir, orr, preset, ch, nonfinite, chunk, s0 = case
    cid = f"{ir}-{orr}-{preset[7:]}-{ch}ch-{'nf' if nonfinite else 'loud'}-{chunk}"
    if cid not in want_ids: continue
    rng = np.random.default_rng(s0)
    frames = 12000
    x = signal(frames, ch, ir, seed=s0 % 1000)
    for _ in range(int(rng.integers(1, 5))):
        c, t = int(rng.integers(ch)), int(rng.integers(frames - 100))
        x[t:t + int(rng.integers(1, 100)), c] *= float(rng.choice([40.0, 1000.0, 1e5]))
    if nonfinite:
        for v in (np.inf, -np.inf, np.nan)[: int(rng.integers(1, 4))]:
            x[int(rng.integers(frames)), int(rng.integers(ch))] = v
    x = x.astype(np.float32).astype(np.float64)
    def run(dtype, ck):
        r = gar.New(gar.Config(ir, orr, ch, getattr(gar, preset), ComputeDtype=dtype))
        st = [(r.stage_geometry(j)[0], int(r.stage_geometry(j)[1].kind)) for j in range(r.num_stages())]
        xd = torch.from_numpy(np.ascontiguousarray(x)).float().cuda()
        parts, s = [], 0
        for n in (chunk_sizes(frames, ck) if ck else [frames]):
            parts.append(r.process_device(xd[s:s + n]).clone()); s += n
        parts.append(r.flush_device(dtype=torch.float32).clone())
        torch.cuda.synchronize()
        return torch.cat(parts).double().cpu().numpy(), st
    got, st = run(gar.F32, chunk)
    one, _ = run(gar.F32, None)
    ex, _ = run(gar.F32_EXACT, None)
    f64, _ = run(gar.F64, None) if False else (None, None)
    want = oracle_new(O, ir, orr, x, getattr(O, "P_" + preset[7:].upper()))
    print("==", cid, "stages", st)
    for c in range(ch):
        w = np.asarray(want[c])
        nan_g, nan_w, nan_e = np.isnan(got[:, c]), np.isnan(w), np.isnan(ex[:, c])
        inf_g, inf_w = np.isinf(got[:, c]), np.isinf(w)
        d = got[:, c] != one[:, c]
        d &= ~(np.isnan(got[:, c]) & np.isnan(one[:, c]))
        if nan_g.any() or nan_w.any() or d.any():
            print(f" c{c}: nan got {nan_g.sum()} want {nan_w.sum()} exact {nan_e.sum()} | inf got {inf_g.sum()} want {inf_w.sum()} | nan got&~want {int((nan_g & ~nan_w).sum())} want&~got {int((nan_w & ~nan_g).sum())}"
                  f" | chunk!=one {int(d.sum())} first {int(np.argmax(d)) if d.any() else -1} maxrel {float(np.nanmax(np.abs(got[d, c] - one[d, c]) / np.maximum(np.abs(one[d, c]), 1e-30))) if d.any() else 0:.3g}"
                  f" | |x| loud rows {int((np.abs(x[:, c]) >= 16).sum())}")
