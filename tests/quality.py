"""Quality measurements restated from the reference's own test helpers (test
infrastructure only).

* go_fft                 -- internal/engine/antialiasing_test.go:179-230 (iterative radix-2
                            Cooley-Tukey, twiddles advanced by repeated multiplication)
* thd_internal           -- internal/engine/quality_regression_test.go:292-344 (measureTHDInternal)
* snr_internal           -- quality_regression_test.go:346-422 (measureSNRInternal)
* ripple_internal        -- quality_regression_test.go:424-510 (measurePassbandRippleInternal)
* dc_gain_internal       -- quality_regression_test.go:56-99 (TestQualityRegression_DCGain body)
* precision_thd          -- internal/engine/precision_comparison_test.go:552-600 (precisionMeasureTHD)

Each takes a `run(x) -> y` callable (Process + Flush of a fresh resampler), so
the same measurement grades the CPU oracle and the HIP path.
"""
import numpy as np

# Published Go THD, 44.1k -> 48k, 1 kHz, engine presets (README.md:303-308)
README_THD_44K1_48K = {"Low": -142.28, "Medium": -129.79, "High": -155.58, "VeryHigh": -162.19}
# Published float64 THD of precision_comparison_test, 44.1k -> 48k High (README.md:363-366)
README_PRECISION_THD_F64_HIGH = -145.25
README_PRECISION_THD_F32_HIGH = -145.01

# Thresholds of quality_regression_test.go:26-53
MAX_RIPPLE = {"Quick": 5.5, "Low": 2.0, "Medium": 2.0, "High": 2.0, "VeryHigh": 2.0}
MAX_THD = {"Quick": -80.0, "Low": -130.0, "Medium": -129.0, "High": -140.0, "VeryHigh": -140.0}
MIN_SNR = {"Quick": 35.0, "Low": 35.0, "Medium": 35.0, "High": 35.0, "VeryHigh": 35.0}
DC_TOL = 0.001

# Test tables (quality_regression_test.go:58-66, :104-130, :156-180, :204-213)
DC_CASES = [(44100, 48000, "VeryHigh"), (48000, 44100, "VeryHigh"), (48000, 32000, "VeryHigh"),
            (48000, 96000, "VeryHigh"), (44100, 48000, "Quick"), (48000, 32000, "Quick")]
THD_CASES = [(44100, 48000, "VeryHigh"), (48000, 44100, "VeryHigh"), (48000, 32000, "VeryHigh"),
             (48000, 96000, "VeryHigh"), (44100, 48000, "High"), (48000, 32000, "High"),
             (44100, 48000, "Medium"), (48000, 32000, "Medium"), (44100, 48000, "Low"), (48000, 32000, "Low"),
             (44100, 48000, "Quick"), (48000, 32000, "Quick")]
SNR_CASES = [(44100, 48000, "VeryHigh"), (48000, 44100, "VeryHigh"), (48000, 32000, "VeryHigh"),
             (44100, 48000, "High"), (48000, 32000, "High"), (44100, 48000, "Medium"), (48000, 32000, "Medium"),
             (44100, 48000, "Low"), (48000, 32000, "Low"), (44100, 48000, "Quick"), (48000, 32000, "Quick")]
RIPPLE_CASES = [(44100, 48000, "VeryHigh"), (48000, 44100, "VeryHigh"), (48000, 32000, "VeryHigh"),
                (44100, 48000, "High"), (44100, 48000, "Medium"), (44100, 48000, "Low"), (44100, 48000, "Quick")]
ENGINE_Q = {"Quick": 0, "Low": 1, "Medium": 2, "High": 3, "VeryHigh": 4}


def go_fft(x):
    """fft() of antialiasing_test.go:179-230 (power-of-two n)."""
    x = np.asarray(x, dtype=complex)
    n = len(x)
    bits = int(np.log2(n))
    assert 1 << bits == n
    idx = np.arange(n)
    rev = np.zeros(n, dtype=np.int64)
    for j in range(bits):
        rev |= ((idx >> j) & 1) << (bits - 1 - j)
    r = np.empty(n, dtype=complex)
    r[rev] = x
    for s in range(1, bits + 1):
        m = 1 << s
        h = m // 2
        wm = complex(np.cos(-2 * np.pi / m), np.sin(-2 * np.pi / m))
        w = np.empty(h, dtype=complex)
        w[0] = 1
        for j in range(1, h):  # w *= wm, sequentially
            w[j] = w[j - 1] * wm
        r = r.reshape(-1, m)
        t = w * r[:, h:]
        u = r[:, :h].copy()
        r = np.concatenate([u + t, u - t], axis=1).reshape(-1)
    return r


def _hann_fft(y, fft_size):
    i = np.arange(fft_size)
    w = 0.5 * (1.0 - np.cos(2.0 * np.pi * i / (fft_size - 1)))
    buf = np.zeros(fft_size)
    m = min(fft_size, len(y))
    buf[:m] = np.asarray(y[:m], dtype=np.float64) * w[:m]
    return go_fft(buf)


def sine_input(in_rate, freq=1000.0, n=65536, amp=0.9):
    return amp * np.sin(2.0 * np.pi * freq * np.arange(n) / in_rate)


def thd_internal(run, in_rate, out_rate, freq=1000.0):
    """measureTHDInternal: 65,536-sample 0.9 sine, Hann, 16,384-point FFT, harmonics 2..10."""
    F = 16384
    X = _hann_fft(run(sine_input(in_rate, freq)), F)
    fb = int(freq / out_rate * F)
    fm = abs(X[fb])
    p = 0.0
    for h in range(2, 11):
        hf = freq * h
        if hf >= out_rate / 2.0:
            break
        hb = int(hf / out_rate * F)
        if hb < F // 2:
            p += abs(X[hb]) ** 2
    return 20 * np.log10(np.sqrt(p) / (fm + 1e-20) + 1e-20)


def snr_internal(run, in_rate, out_rate, freq=1000.0):
    """measureSNRInternal: signal = fundamental +-3 bins, noise = all other bins below
    Nyquist except +-2 bins around harmonics 2..10."""
    F = 16384
    X = _hann_fft(run(sine_input(in_rate, freq)), F)
    fb = int(freq / out_rate * F)
    sig = 0.0
    for b in range(-3, 4):
        if 0 < fb + b < F // 2:
            sig += abs(X[fb + b]) ** 2
    hbins = []
    for h in range(2, 11):
        hf = freq * h
        if hf >= out_rate / 2.0:
            break
        hbins.append(int(hf / out_rate * F))
    noise = 0.0
    for b in range(1, F // 2):
        if fb - 3 <= b <= fb + 3:
            continue
        if any(hb - 2 <= b <= hb + 2 for hb in hbins):
            continue
        noise += abs(X[b]) ** 2
    return 10 * np.log10(sig + 1e-20) - 10 * np.log10(noise + 1e-20)


def ripple_internal(run, in_rate, out_rate):
    """measurePassbandRippleInternal: 20-tone 0.05-amplitude multitone up to 0.9 of the
    lower Nyquist, peak level per tone (+-2 bins), peak-to-peak deviation in dB."""
    F = 16384
    pb = min(in_rate, out_rate) / 2.0 * 0.9
    freqs = []
    f = 500.0
    while f < pb and len(freqs) < 20:
        freqs.append(f)
        f += pb / 20
    t = np.arange(65536)
    x = np.zeros(65536)
    for fr in freqs:  # accumulated tone by tone, as the Go loop does
        x += 0.05 * np.sin(2.0 * np.pi * fr * t / in_rate)
    X = _hann_fft(run(x), F)
    levels = []
    for fr in freqs:
        b0 = int(fr / out_rate * F)
        peak = -200.0
        for b in range(-2, 3):
            if 0 < b0 + b < F // 2:
                peak = max(peak, 20 * np.log10(abs(X[b0 + b]) + 1e-20))
        levels.append(peak)
    dev = np.array(levels) - np.mean(levels)
    return float(dev.max() - dev.min())


def dc_gain_internal(run, n=20000):
    y = run(np.ones(n))
    a, b = len(y) // 4, 3 * len(y) // 4
    return float(np.mean(y[a:b]))


def precision_thd(y, freq, rate):
    """precisionMeasureTHD: 8192-point Hann window from the middle, harmonics 2..5 of the rounded bin."""
    F = 8192 if len(y) >= 16384 else 1024
    s = (len(y) - F) // 2
    X = _hann_fft(np.asarray(y[s:s + F]), F)
    fb = int(np.round(freq / (rate / F)))
    fm = abs(X[fb])
    hp = sum(abs(X[fb * h]) ** 2 for h in range(2, 6) if fb * h < F // 2)
    return 10 * np.log10(hp / fm ** 2)
