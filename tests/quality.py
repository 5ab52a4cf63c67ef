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


# ----------------------------------------------------------------------------- anti-aliasing / impulse
# internal/engine/antialiasing_test.go:21-27, quality_comparison_test.go:578-648
ANTIALIAS_SAMPLES = 32768
FFT_WINDOW = 8192
MIN_STOPBAND_ATT = 80.0
NOISE, MULTITONE, SWEEP, ALIAS_TONES = "noise", "multitone", "sweep", "alias_tones"


def antialias_signal(kind, rate, n=ANTIALIAS_SAMPLES):
    """generateAntialiasTestSignal (antialiasing_test.go:56-117)."""
    x = np.zeros(n)
    i = np.arange(n)
    if kind == NOISE:  # LCG, uint32 state
        st = 12345
        v = np.empty(n)
        for k in range(n):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            v[k] = float(st & 0x7FFFFFFF) / float(0x7FFFFFFF) * 2.0 - 1.0
        x = v * 0.5
    elif kind == MULTITONE:
        for f in (1000, 2000, 4000, 8000, 12000, 16000, 20000, 22000, 23000):
            if f < rate / 2.0 * 0.95:
                x += 0.1 * np.sin(2.0 * np.pi * f * i / rate)
    elif kind == SWEEP:
        f0, f1 = 100.0, rate * 0.45
        rate_s = (f1 - f0) / (n / rate)
        t = i / rate
        x = 0.7 * np.sin(2.0 * np.pi * (f0 * t + rate_s * t * t / 2.0))
    elif kind == ALIAS_TONES:  # 48->32 estimate of the output Nyquist (sampleRate / 3)
        f = rate / 3.0 + 1000
        while f < rate / 2.0 - 500:
            x += 0.1 * np.sin(2.0 * np.pi * f * i / rate)
            f += 1000
    return x


def alias_tones(in_rate, out_rate, n=ANTIALIAS_SAMPLES):
    """generateAliasTones (antialiasing_test.go:617-633): 0.1-amplitude tones from the output
    Nyquist + 1 kHz to the input Nyquist - 500 Hz, 1 kHz apart."""
    x = np.zeros(n)
    i = np.arange(n)
    f = out_rate / 2.0 + 1000
    while f < in_rate / 2.0 - 500:
        x += 0.1 * np.sin(2.0 * np.pi * f * i / in_rate)
        f += 1000
    return x


def compute_psd(sig, rate, fft_size=FFT_WINDOW):
    """computePSD (antialiasing_test.go:123-177): Welch, Hann (N-1), 50 % overlap, dB."""
    sig = np.asarray(sig, dtype=np.float64)
    nb = fft_size // 2 + 1
    freqs = np.arange(nb) * rate / fft_size
    w = 0.5 * (1.0 - np.cos(2.0 * np.pi * np.arange(fft_size) / (fft_size - 1)))
    acc = np.zeros(nb)
    nwin = 0
    for s in range(0, len(sig) - fft_size + 1, fft_size // 2):
        X = go_fft(sig[s:s + fft_size] * w)
        acc += np.abs(X[:nb]) ** 2
        nwin += 1
    power = acc / (nwin * fft_size * float(np.sum(w * w)))
    with np.errstate(divide="ignore"):
        psd = np.where(power > 1e-20, 10.0 * np.log10(np.maximum(power, 1e-300)), -200.0)
    return freqs, psd


def band_energy(freqs, psd, lo, hi):
    """measureBandEnergy (antialiasing_test.go:232-248)."""
    sel = (freqs >= lo) & (freqs < hi)
    if not sel.any():
        return -200.0
    return float(10.0 * np.log10(np.sum(10.0 ** (psd[sel] / 10.0)) / sel.sum()))


def peak_energy(freqs, psd, lo, hi):
    """measurePeakEnergy (antialiasing_test.go:250-262)."""
    sel = (freqs >= lo) & (freqs < hi)
    return float(max(-200.0, psd[sel].max())) if sel.any() else -200.0


def antialiasing(run, in_rate, out_rate, kind):
    """measureAntiAliasing (antialiasing_test.go:276-348): stopband (imaging region above the
    input Nyquist) attenuation of an upsampler; peak-based for multitone, average otherwise."""
    y = run(antialias_signal(kind, in_rate))
    f, p = compute_psd(y, out_rate)
    pb_end = in_rate / 2.0 * 0.9
    sb0, sb1 = in_rate / 2.0 + 1000, out_rate / 2.0 - 1000
    meas = peak_energy if kind == MULTITONE else band_energy
    return meas(f, p, 100, pb_end) - meas(f, p, sb0, sb1)


def downsampling_antialiasing(run, in_rate, out_rate):
    """measureDownsamplingAntiAliasing (antialiasing_test.go:635-699): alias tones' input
    peak minus the output's peak where they would fold ([out - in/2, out/2])."""
    x = alias_tones(in_rate, out_rate)
    y = run(x)
    fi, pi_ = compute_psd(x, in_rate)
    fo, po = compute_psd(y, out_rate)
    inp = peak_energy(fi, pi_, out_rate / 2.0 + 500, in_rate / 2.0 - 500)
    lo = max(out_rate - in_rate / 2.0, 100.0)
    return inp - peak_energy(fo, po, lo, out_rate / 2.0)


def impulse_response(run, n=8192):
    """measureImpulseResponse (quality_comparison_test.go:578-648): unit impulse at n/2;
    pre-ringing peak before the main peak, post-ringing peak from 10 samples after it (dB
    re the main peak), ring-out = last sample above -60 dB."""
    x = np.zeros(n)
    x[n // 2] = 1.0
    y = np.abs(np.asarray(run(x), dtype=np.float64))
    k = int(np.argmax(y))  # first maximum, as the Go loop's strict '>'
    m = y[k]
    pre = y[:k].max() if k > 0 else 0.0
    post = y[k + 10:].max() if k + 10 < len(y) else 0.0
    above = np.nonzero(y[k:] > m * 10 ** (-60.0 / 20.0))[0]
    return {"pre_ringing_db": float(20 * np.log10(pre / m + 1e-20)),
            "post_ringing_db": float(20 * np.log10(post / m + 1e-20)),
            "ringout_samples": int(above[-1]) if len(above) else 0, "peak_index": k}
