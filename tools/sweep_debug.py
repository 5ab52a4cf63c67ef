"""Isolate a failing sweep case (tests/test_gpu_sweep.py): one-shot vs chunked device runs in F32 / F64
against the oracle, per knob setting given as JSON env dicts on the command line (each in a child)."""
import json
import os
import subprocess
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json
sys.path[:0] = [%r, %r, %r]
import numpy as np, torch, gar
from helpers import signal, oracle_new, rms, chunk_sizes
from oracle import oracle as O
O.build()
ir, orr, preset, ch, frames, chunk = json.loads(os.environ["SD_CASE"])
x = signal(frames, ch, ir, seed=ir + orr + ch).astype(np.float32).astype(np.float64)
want = oracle_new(O, ir, orr, x, getattr(O, "P_" + preset[7:].upper()))
res = {}
for dt in os.environ.get("SD_DT", "F32,F64").split(","):
    tdt = torch.float64 if dt == "F64" else torch.float32
    for ck in (None, chunk):
        r = gar.New(gar.Config(ir, orr, ch, getattr(gar, preset), ComputeDtype=getattr(gar, dt)))
        if ck is None and dt == "F32":
            res["stages"] = [(r.stage_geometry(j)[0], int(r.stage_geometry(j)[1].kind)) for j in range(r.num_stages())]
        xd = torch.from_numpy(np.ascontiguousarray(x)).to(tdt).cuda()
        parts, s, sizes = [], 0, []
        for n in (chunk_sizes(frames, ck) if ck else [frames]):
            y = r.process_device(xd[s:s + n]).clone(); parts.append(y); sizes.append(y.shape[0]); s += n
        parts.append(r.flush_device(dtype=tdt).clone()); sizes.append(parts[-1].shape[0])
        torch.cuda.synchronize()
        got = torch.cat(parts).double().cpu().numpy()
        e = [rms(got[:, c], want[c]) if got.shape[0] == len(want[c]) else -1 for c in range(ch)]
        bad = np.nonzero(np.abs(got[:, 0] - want[0]) > 1e-4)[0] if got.shape[0] == len(want[0]) else []
        res[f"{dt}-{'chunk' if ck else 'one'}"] = {"rms": max(e), "n": got.shape[0], "first_bad": int(bad[0]) if len(bad) else None,
                                                   "nbad": int(len(bad)), "sizes": sizes[:6]}
        if ck is None:
            ref_one = got
        elif got.shape == ref_one.shape:
            diff = np.nonzero((got != ref_one).any(axis=1))[0]
            res[f"{dt}-chunk"]["bits_differ_rows"] = int(len(diff))
            res[f"{dt}-chunk"]["first_diff_row"] = int(diff[0]) if len(diff) else None
print(json.dumps(res))
''' % (ROOT, os.path.join(ROOT, "go-audio-resampler_amd"), os.path.join(ROOT, "tests"))

case = sys.argv[1]
for cfg in json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]:
    env = dict(os.environ, SD_CASE=case, **{k: str(v) for k, v in cfg.items()})
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    print(json.dumps(cfg), line[-1] if line else p.stderr[-800:], flush=True)
    if os.environ.get("SD_STDERR"):
        print(p.stderr[-12000:], flush=True)
