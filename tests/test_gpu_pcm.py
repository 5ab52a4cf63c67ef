"""GPU: integer PCM I/O -- int16 / int24-in-int32 / int32 samples converted
inside the resampling kernels, after cmd/resample-wav/main.go:444-543:

  input   x = F(float64(i) * (1 / maxVal))                      (deinterleaveInto, main.go:444-472)
  output  i = int(clamp(float64(y), -1, 1) * maxVal), truncating (interleaveInto, main.go:476-543)
  maxVal  32767 / 8388607 / 2147483647                           (main.go:54-56)

Parity bars:
  * bit-exact against the float path of the same kernels fed the same scaled floats, with the
    reference's output conversion applied on the host (fused loads/stores change nothing but
    the bytes moved);
  * against the CPU oracle fed the same scaled floats: |delta| <= 1 LSB (the f32 path's
    ~1e-7 error moves a truncation across an integer boundary for a small fraction of samples;
    for the float64 path the fraction is ~0), fraction bounded in each test;
  * chunked streaming == one shot (bit-exact), flush tails included.
"""
import numpy as np
import pytest

from helpers import F32_RMS_TOL, chunk_sizes, oracle_new, signal

pytestmark = pytest.mark.gpu

MAXV = {16: 32767.0, 24: 8388607.0, 32: 2147483647.0}


def to_pcm(x, bits):
    """Float signal in [-1, 1] -> integer samples (as a WAV file would hold them)."""
    return np.round(np.clip(x, -1, 1) * MAXV[bits] * 0.98).astype(np.int16 if bits == 16 else np.int32)


def scaled(pcm, bits):
    """float64(i) * (1 / maxVal) -- main.go:449-460 (invMaxVal = 1 / maxVal)."""
    return pcm.astype(np.float64) * (1.0 / MAXV[bits])


def from_float(y, bits):
    """int(clamp(float64(y), -1, 1) * maxVal) -- main.go:497-541 (Go int() truncates)."""
    v = np.clip(np.asarray(y, dtype=np.float64), -1.0, 1.0) * MAXV[bits]
    return np.trunc(v).astype(np.int64)


def run(gar, torch, x, in_rate, out_rate, preset, compute, chunks=None, bits=None, tdtype=None):
    """Process (+ chunks) + Flush on the device; x is a host array of tdtype."""
    ch = x.shape[1]
    r = gar.New(gar.Config(in_rate, out_rate, ch, preset, ComputeDtype=compute))
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    outs, s = [], 0
    for n in (chunks or [x.shape[0]]):
        outs.append(r.process_device(xd[s:s + n], pcm_bits=bits).clone())
        s += n
    outs.append(r.flush_device(dtype=xd.dtype, pcm_bits=bits).clone())
    torch.cuda.synchronize()
    return torch.cat(outs).cpu().numpy().astype(np.float64 if xd.dtype.is_floating_point else np.int64)


@pytest.mark.parametrize("bits", [16, 24, 32])
def test_pcm_fused_equals_float_path(gar, cuda, bits):
    """cfg2 geometry (stereo 44.1k -> 48k QualityHigh, float32 split-f16 path): the fused PCM
    kernel == the float kernel fed float32(float64(i)/maxVal), output converted on the host."""
    torch = cuda
    n = 3 * 44100 + 123
    pcm = to_pcm(signal(n, 2), bits)
    got = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F32, bits=bits)
    xf = scaled(pcm, bits).astype(np.float32)
    yf = run(gar, torch, xf, 44100, 48000, gar.QualityHigh, gar.F32)
    want = from_float(yf.astype(np.float32), bits)
    assert got.shape == want.shape
    assert np.array_equal(got, want), int(np.max(np.abs(got - want)))


@pytest.mark.parametrize("bits", [16, 24])
def test_pcm_vs_oracle(gar, cuda, O, bits):
    """PCM in -> PCM out vs the oracle fed the same scaled floats: within one LSB."""
    torch = cuda
    n = 2 * 44100
    pcm = to_pcm(signal(n, 2), bits)
    got = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F32, bits=bits)
    xs = scaled(pcm, bits).astype(np.float32).astype(np.float64)
    ref = oracle_new(O, 44100, 48000, xs, O.P_HIGH)
    for c in range(2):
        want = from_float(ref[c], bits)
        assert len(want) == got.shape[0]
        d = np.abs(got[:, c] - want)
        if bits == 16:
            # f32 arithmetic (~1e-7 of full scale) is far below the 16-bit LSB: a truncation moves
            # across an integer boundary for a small fraction of samples, by one LSB
            assert d.max() <= 1, d.max()
            assert np.mean(d != 0) < 0.002, np.mean(d != 0)
        else:
            # the 24-bit LSB (1.2e-7) is at the f32 error level: the BASELINE float32 bar applies
            # (RMS <= 1e-6 of full scale), plus a per-sample cap
            assert np.sqrt(np.mean(d.astype(np.float64) ** 2)) / MAXV[bits] <= F32_RMS_TOL
            assert d.max() <= 16, d.max()


def test_pcm_chunked_is_bit_identical(gar, cuda):
    """processinto_test.go:258-308 on the PCM path: ragged chunks == one shot, flush included."""
    torch = cuda
    n = 2 * 44100 + 777
    pcm = to_pcm(signal(n, 2, seed=7), 16)
    one = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F32, bits=16)
    rag = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F32, chunks=chunk_sizes(n, 4096 + 17), bits=16)
    assert np.array_equal(one, rag)


def test_pcm_staged_f64(gar, cuda, O):
    """float64 compute (bg_kernel, conversion staged by convert_kernel) == the float64 path with
    the conversion on the host, and == the oracle's conversion except at exact ties."""
    torch = cuda
    n = 44100
    pcm = to_pcm(signal(n, 2, seed=3), 16)
    got = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F64, bits=16)
    yf = run(gar, torch, scaled(pcm, 16), 44100, 48000, gar.QualityHigh, gar.F64)
    assert np.array_equal(got, from_float(yf, 16))
    ref = oracle_new(O, 44100, 48000, scaled(pcm, 16), O.P_HIGH)
    for c in range(2):
        d = np.abs(got[:, c] - from_float(ref[c], 16))
        assert d.max() <= 1 and np.mean(d != 0) < 1e-4


@pytest.mark.parametrize("ch", [1, 16])
def test_pcm_other_layouts(gar, cuda, ch):
    """Mono and 16-channel rows (gathered PCM loads) == the float path + host conversion."""
    torch = cuda
    n = 44100 + 5
    pcm = to_pcm(signal(n, ch, seed=11), 16)
    got = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F32, bits=16)
    yf = run(gar, torch, scaled(pcm, 16).astype(np.float32), 44100, 48000, gar.QualityHigh, gar.F32)
    assert np.array_equal(got, from_float(yf.astype(np.float32), 16))


def test_pcm_clipping(gar, cuda):
    """Full-scale square-ish input overshoots after resampling: outputs clip to +-maxVal
    exactly like interleaveInto's clamp (no wrap-around)."""
    torch = cuda
    n = 44100
    t = np.arange(n)
    sq = np.where((t // 50) % 2 == 0, 32767, -32767).astype(np.int16)
    pcm = np.stack([sq, -sq], axis=1)
    got = run(gar, torch, pcm, 44100, 48000, gar.QualityHigh, gar.F32, bits=16)
    assert got.max() == 32767 and got.min() == -32767
    yf = run(gar, torch, scaled(pcm, 16).astype(np.float32), 44100, 48000, gar.QualityHigh, gar.F32)
    assert np.abs(yf).max() > 1.0  # the float path does overshoot
    assert np.array_equal(got, from_float(yf.astype(np.float32), 16))
