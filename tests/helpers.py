"""Shared test helpers: deterministic signals, error metrics, oracle runners."""
import numpy as np

F32_RMS_TOL = 1e-6    # BASELINE.json north_star: float32 <= 1e-6 RMS vs the reference
F64_RMS_TOL = 1e-12   # float64 <= 1e-12 RMS


def signal(n, channels=1, rate=44100.0, seed=4242):
    """0.7 sin(440) + 0.2 sin(1750) + 0.1 (U - 0.5) per channel -- the generator
    shape of makeDeterministicInput (processinto_test.go:19-30); numpy RNG."""
    t = np.arange(n) / rate
    out = np.empty((n, channels))
    for c in range(channels):
        rng = np.random.default_rng(seed + c)
        p1, p2 = rng.random() * 2 * np.pi, rng.random() * 2 * np.pi
        out[:, c] = (0.7 * np.sin(2 * np.pi * 440 * t + p1) + 0.2 * np.sin(2 * np.pi * 1750 * t + p2)
                     + 0.1 * (rng.random(n) - 0.5))
    return out


def sine(n, rate, freq=1000.0):
    return np.sin(2 * np.pi * freq * np.arange(n) / rate)


def rms(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2))) if a.size else 0.0


def oracle_new(O, in_rate, out_rate, x, preset, chunks=None, flush=True):
    """Reference New(config) path over planar channels x[:, c]; returns list per channel."""
    ch = x.shape[1]
    r = O.NewResampler(in_rate, out_rate, ch, preset)
    outs = []
    for c in range(ch):
        parts = []
        if chunks is None:
            parts.append(r.process(x[:, c], c))
        else:
            s = 0
            for n in chunks:
                parts.append(r.process(x[s:s + n, c], c))
                s += n
        if flush:
            parts.append(r.flush(c))
        outs.append(np.concatenate(parts) if parts else np.zeros(0))
    return outs


def chunk_sizes(total, size):
    out = []
    while total > 0:
        out.append(min(size, total))
        total -= out[-1]
    return out
