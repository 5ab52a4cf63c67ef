import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-audio-resampler_amd")]
import numpy as np, torch, gar
from oracle import oracle as O
from gpu_quickcheck import sig

def run(i, o, preset, n, ch, dtype, chunks, flush=True):
    x = sig(n, ch, i)
    ref = O.NewResampler(i, o, ch, preset)
    xin = x.astype(np.float32).astype(np.float64) if dtype == gar.F32 else x
    r = gar.New(gar.Config(i, o, ch, preset, ComputeDtype=dtype))
    tdt = torch.float32 if dtype == gar.F32 else torch.float64
    xd = torch.from_numpy(x).to(tdt).cuda()
    outs = []; s = 0; bounds=[]
    for cn in chunks:
        y = r.process_device(xd[s:s+cn]); outs.append(y); s += cn; bounds.append(sum(len(q) for q in outs))
    if flush:
        outs.append(r.flush_device(dtype=tdt)); bounds.append(sum(len(q) for q in outs))
    y = torch.cat(outs).double().cpu().numpy()
    for c in range(ch):
        want = np.concatenate([ref.process(xin[:s, c], c)] + ([ref.flush(c)] if flush else []))
        if len(want) != y.shape[0]:
            print("  LEN", len(want), y.shape); return
        err = np.abs(y[:, c] - want)
        bad = np.nonzero(err > 1e-4)[0]
        tag = f"{i}->{o} p{preset} ch{ch} dt{dtype} chunks{chunks[:3]}.. flush{flush} c{c}"
        if len(bad):
            print(f"  BAD {tag}: n={len(want)} nbad={len(bad)} first={bad[0]} last={bad[-1]} bounds={bounds} maxerr={err.max():.3g}")
        else:
            print(f"  ok  {tag}: maxerr={err.max():.3g}")
    sys.stdout.flush()

run(44100, 48000, 3, 20000, 1, gar.F32, [20000], flush=False)
run(44100, 48000, 3, 20000, 1, gar.F32, [10000, 10000], flush=False)
run(44100, 48000, 3, 20000, 1, gar.F32, [20000], flush=True)
run(44100, 48000, 3, 20000, 2, gar.F32, [10000, 10000], flush=False)
run(44100, 48000, 3, 20000, 1, gar.F64, [20000], flush=True)
run(44100, 48000, 3, 20000, 2, gar.F64, [20000], flush=False)
run(44100, 48000, 3, 20000, 2, gar.F64, [20000], flush=True)
run(48000, 44100, 4, 20000, 16, gar.F32, [20000], flush=False)
run(48000, 44100, 4, 20000, 16, gar.F32, [20000], flush=True)
run(48000, 44100, 4, 20000, 1, gar.F32, [20000], flush=True)
run(48000, 44100, 4, 20000, 1, gar.F32, [5000, 15000], flush=False)
run(48000, 96000, 3, 20000, 2, gar.F32, [10000, 10000], flush=True)
run(96000, 48000, 3, 20000, 2, gar.F64, [10000, 10000], flush=True)
