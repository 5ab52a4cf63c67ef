"""Golden fixtures: small per-sample vectors of the reference algorithm, made by
the CPU oracle (tests/golden/make_golden.py) and committed under tests/golden/.

The reference ships no per-sample golden outputs; these vectors
pin (1) the oracle against its own regressions and (2) the GPU path on exactly
the same inputs.  Inputs are regenerated from (generator, seed, n) -- numpy's
PCG64 stream is stable across versions.
"""
import json
import os

import numpy as np

from helpers import signal, sine

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# kind: "engine" (NewEngine/ResampleMono, engine.Resampler[float64]),
#       "engine32" (NewEngineFloat32), "new" (resampler.New, float64)
CASES = [
    dict(name="cfg1_mono_f64_44k1_48k_high", kind="engine", in_rate=44100, out_rate=48000, preset=3,
         gen="sine", n=44100, channels=1, ops=[["p", 44100], ["f"]]),
    dict(name="cfg2_stereo_44k1_48k_high_chunked", kind="new", in_rate=44100, out_rate=48000, preset=3,
         gen="signal", seed=4242, n=11025, channels=2, f32_input=True,
         ops=[["p", 4096], ["p", 4096], ["p", 2833], ["f"]]),
    dict(name="cfg3_4ch_48k_44k1_veryhigh", kind="new", in_rate=48000, out_rate=44100, preset=4,
         gen="signal", seed=11, n=9600, channels=4, f32_input=True, ops=[["p", 9600], ["f"]]),
    dict(name="cfg5_2ch_96k_44k1_veryhigh_4800", kind="new", in_rate=96000, out_rate=44100, preset=4,
         gen="signal", seed=5, n=19200, channels=2, ops=[["p", 4800]] * 4 + [["f"]]),
    dict(name="engine_16k_44k1_high_cubic_interp", kind="engine", in_rate=16000, out_rate=44100, preset=3,
         gen="signal", seed=3, n=4000, channels=1, ops=[["p", 4000], ["f"]]),
    dict(name="new_96k_16k_high_multistage", kind="new", in_rate=96000, out_rate=16000, preset=3,
         gen="signal", seed=9, n=24000, channels=1, ops=[["p", 24000], ["f"]]),
    dict(name="engine32_44k1_48k_high", kind="engine32", in_rate=44100, out_rate=48000, preset=3,
         gen="signal", seed=21, n=11025, channels=1, ops=[["p", 11025], ["f"]]),
    dict(name="engine_44k1_48k_process_after_flush", kind="engine", in_rate=44100, out_rate=48000, preset=3,
         gen="signal", seed=31, n=5000, channels=1, ops=[["p", 3000], ["f"], ["p", 2000], ["f"], ["f"]]),
]


def make_input(case):
    if case["gen"] == "sine":
        x = sine(case["n"], case["in_rate"])[:, None]
    else:
        x = signal(case["n"], case["channels"], case["in_rate"], case["seed"])
    if case.get("f32_input"):
        x = x.astype(np.float32).astype(np.float64)
    return x


def run_oracle(O, case):
    """Per channel: concatenation of every op's output (p = Process(n), f = Flush)."""
    x = make_input(case)
    outs = []
    if case["kind"] == "new":
        r = O.NewResampler(case["in_rate"], case["out_rate"], case["channels"], case["preset"])
    for c in range(case["channels"]):
        if case["kind"] in ("engine", "engine32"):
            q = O.lib().o_preset_to_engine_quality(case["preset"])
            e = O.Engine(case["in_rate"], case["out_rate"], q, f32=case["kind"] == "engine32")
            proc, fl = e.process, e.flush
        else:
            proc, fl = (lambda v, c=c: r.process(v, c)), (lambda c=c: r.flush(c))
        parts, s = [], 0
        for op in case["ops"]:
            if op[0] == "p":
                parts.append(np.asarray(proc(x[s:s + op[1], c]), dtype=np.float64))
                s += op[1]
            else:
                parts.append(np.asarray(fl(), dtype=np.float64))
        outs.append(np.concatenate(parts))
    return outs


def save(case, outs):
    os.makedirs(GOLDEN_DIR, exist_ok=True)
    np.savez_compressed(os.path.join(GOLDEN_DIR, case["name"] + ".npz"),
                        **{f"out_{c}": o for c, o in enumerate(outs)})


def load_all():
    res = []
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        manifest = json.load(f)
    for case in manifest["cases"]:
        z = np.load(os.path.join(GOLDEN_DIR, case["name"] + ".npz"))  # allow_pickle=False (default)
        res.append(dict(case, outputs=[z[f"out_{c}"] for c in range(case["channels"])]))
    return res
