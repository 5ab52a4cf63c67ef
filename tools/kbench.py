"""Sweep bg_kernel launch knobs on the bench workload (one process, interleaved rounds).
Env knobs are read once per process by the library, so each config runs in a child process."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json, time
sys.path[:0] = [%r, %r]
import numpy as np, torch, gar
frames = int(float(os.environ.get("KB_SECONDS", "600")) * 44100)
ch = int(os.environ.get("KB_CH", "2"))
rin, rout = float(os.environ.get("KB_IN", "44100")), float(os.environ.get("KB_OUT", "48000"))
q = int(os.environ.get("KB_Q", "3"))
x = (torch.rand((frames, ch), device="cuda") - 0.5)
r = gar.New(gar.Config(rin, rout, ch, q, ComputeDtype=gar.F32))
n = gar.lib().gar_device_output_size(r._h, frames)
y = torch.empty((n, ch), device="cuda")
for _ in range(3):
    r.Reset(); r.process_device(x, out=y)
torch.cuda.synchronize()
r.profile(True); r.profile_read(0)
for _ in range(10):
    r.Reset(); r.process_device(x, out=y)
torch.cuda.synchronize()
ms, k = r.profile_read(0)
print(json.dumps({"ms": ms / k, "msamples_per_s": frames * ch / (ms / k) / 1e3}))
''' % (ROOT, os.path.join(ROOT, "go-audio-resampler_amd"))

def run(env):
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    out = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if not line:
        return {"err": out.stderr[-500:]}
    d = json.loads(line[-1])
    prof = [l for l in out.stderr.splitlines() if l.startswith(("hxs", "hxt", "hxq"))]
    if prof:
        d["prof"] = prof
    return d

if __name__ == "__main__":
    configs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
    for cfg in configs:
        print(json.dumps({"cfg": cfg, **run(cfg)}), flush=True)
