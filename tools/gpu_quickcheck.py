"""Quick GPU parity sweep used during development (not collected by pytest)."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np, torch
import gar
from oracle import oracle as O

def sig(n, ch, rate, seed=4242):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / rate
    return np.stack([0.7*np.sin(2*np.pi*440*t + 0.3*c) + 0.2*np.sin(2*np.pi*1750*t+c) + 0.1*(rng.random(n)-0.5) for c in range(ch)], axis=1)

def rms(a, b):
    return float(np.sqrt(np.mean((a-b)**2))) if len(a) else 0.0

def engine_case(i, o, preset, n, f32=False):
    x = sig(n, 1, i)[:, 0]
    q = O.lib().o_preset_to_engine_quality(preset)
    e = O.Engine(i, o, q)
    want = np.concatenate([e.process(x), e.flush()])
    got = gar.ResampleMono(x, i, o, preset)
    print(f"engine {i}->{o} p{preset}: len {len(got)} vs {len(want)} rms {rms(got, want) if len(got)==len(want) else 'LEN'}", flush=True)

def new_case(i, o, preset, n, ch, dtype, chunk=None):
    x = sig(n, ch, i)
    ref = O.NewResampler(i, o, ch, preset)
    xin = x.astype(np.float32).astype(np.float64) if dtype == gar.F32 else x
    r = gar.New(gar.Config(i, o, ch, preset, ComputeDtype=dtype))
    tdt = torch.float32 if dtype == gar.F32 else torch.float64
    xd = torch.from_numpy(x).to(tdt).cuda()
    outs = []
    if chunk is None:
        outs.append(r.process_device(xd))
    else:
        for s in range(0, n, chunk):
            outs.append(r.process_device(xd[s:s+chunk]))
    outs.append(r.flush_device(dtype=tdt))
    y = torch.cat(outs).double().cpu().numpy()
    worst = 0
    for c in range(ch):
        want = np.concatenate([ref.process(xin[:, c], c), ref.flush(c)])
        if len(want) != y.shape[0]:
            print("LEN MISMATCH", len(want), y.shape); return
        worst = max(worst, rms(y[:, c], want))
    print(f"new {i}->{o} p{preset} ch{ch} dt{dtype} chunk{chunk}: len {y.shape[0]} worst rms {worst:.3e}", flush=True)

if __name__ == "__main__":
    engine_case(44100, 48000, gar.QualityHigh, 44100)
    engine_case(48000, 44100, gar.QualityHigh, 20000)
    engine_case(16000, 44100, gar.QualityHigh, 16000)
    engine_case(48000, 96000, gar.QualityHigh, 10000)
    engine_case(96000, 48000, gar.QualityHigh, 10000)
    new_case(44100, 48000, gar.QualityHigh, 44100, 2, gar.F32)
    new_case(44100, 48000, gar.QualityHigh, 44100, 2, gar.F32, chunk=4096)
    new_case(48000, 44100, gar.QualityVeryHigh, 48000, 16, gar.F32)
    new_case(96000, 44100, gar.QualityVeryHigh, 96000, 8, gar.F64, chunk=4800)
    new_case(44100, 48000, gar.QualityHigh, 44100, 2, gar.F64)
