"""GPU: the float32 compute path (split-f16 MFMA kernel, csrc/gar_hx.hpp) against
the oracle and against the exact-f32 MFMA kernel (GAR_F32_EXACT).

Tolerances: BASELINE.json north_star float32 <= 1e-6 RMS vs the reference.
The split path's error must also stay within 2x of exact-f32 arithmetic's
(it is in fact below it: 22-bit operands, f32 accumulation).
Edge cases: Inf/NaN and |x| >= 16 samples (exact f64 fallback of the outputs
whose windows hold one, two-stage for non-finite), extreme magnitudes, ragged
lengths, both directions, the DFT-only / decimator stages and chunked
streaming (bit-identical to one shot).
"""
import numpy as np
import pytest

from helpers import F32_RMS_TOL, chunk_sizes, oracle_new, rms, signal

pytestmark = pytest.mark.gpu


def run(gar, torch, in_rate, out_rate, x, preset, dtype, chunks=None):
    ch = x.shape[1]
    r = gar.New(gar.Config(in_rate, out_rate, ch, preset, ComputeDtype=dtype))
    xd = torch.from_numpy(np.ascontiguousarray(x)).float().cuda()
    outs, s = [], 0
    for n in (chunks or [x.shape[0]]):
        outs.append(r.process_device(xd[s:s + n]).clone())
        s += n
    outs.append(r.flush_device(dtype=torch.float32).clone())
    torch.cuda.synchronize()
    return torch.cat(outs).double().cpu().numpy()


CASES = [
    (44100, 48000, 2, "QualityHigh"),      # cfg2 geometry (fused composite)
    (48000, 44100, 5, "QualityVeryHigh"),  # cfg3 geometry, odd channel count
    (96000, 44100, 3, "QualityVeryHigh"),  # decimator + fused
    (22050, 44100, 1, "QualityHigh"),      # DFT-only (integer up)
    (48000, 16000, 2, "QualityMedium"),    # integer down (decimator)
    (44100, 96000, 4, "QualityLow"),       # halfband x2 + fused
]


@pytest.mark.parametrize("case", CASES)
def test_hx_vs_oracle_and_exact(gar, O, cuda, case):
    ir, orr, ch, q = case
    n = 30011  # ragged
    x = signal(n, ch, ir, seed=ir + ch).astype(np.float32).astype(np.float64)
    got = run(gar, cuda, ir, orr, x, getattr(gar, q), gar.F32)
    ex = run(gar, cuda, ir, orr, x, getattr(gar, q), gar.F32_EXACT)
    want = oracle_new(O, ir, orr, x, getattr(O, "P_" + q[7:].upper()))
    for c in range(ch):
        assert got.shape[0] == ex.shape[0] == len(want[c])
        e_hx, e_ex = rms(got[:, c], want[c]), rms(ex[:, c], want[c])
        assert e_hx <= F32_RMS_TOL, e_hx
        assert e_hx <= max(2.0 * e_ex, 1e-8), (e_hx, e_ex)


@pytest.mark.parametrize("chunk", [4096, 1001])
def test_hx_chunked_equals_oracle(gar, O, cuda, chunk):
    x = signal(50000, 2, 44100).astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32, chunk_sizes(50000, chunk))
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    for c in range(2):
        assert got.shape[0] == len(want[c])
        assert rms(got[:, c], want[c]) <= F32_RMS_TOL


@pytest.mark.parametrize("scale", [1e30, 3.0e4, 1e-6])
def test_hx_extreme_magnitudes(gar, O, cuda, scale):
    """|x| >= 16 takes the exact f64 path; quiet signals keep 22-bit operands down to
    |x| ~ 2^-26 (the lo halves are scaled apart): error stays relative to the level."""
    x = signal(40000, 2, 44100, seed=7)
    xs = (x * scale).astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 44100, 48000, xs, gar.QualityHigh, gar.F32)
    want = oracle_new(O, 44100, 48000, xs, O.P_HIGH)
    for c in range(2):
        assert np.all(np.isfinite(got[:, c]))
        assert rms(got[:, c] / scale, want[c] / scale) <= F32_RMS_TOL


def test_hx_tiny_signal_absolute_floor(gar, O, cuda):
    """Below |x| ~ 2^-26 the fixed split scale leaves an absolute floor of ~2^-47."""
    x = signal(20000, 2, 44100, seed=8) * 1e-30
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32)
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    for c in range(2):
        assert np.max(np.abs(got[:, c] - want[c])) <= 1e-13


def test_hx_mixed_levels(gar, O, cuda):
    """A loud channel beside a very quiet one."""
    x = signal(40000, 2, 44100, seed=9)
    x[:, 1] *= 1e-6
    x = x.astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32)
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    assert rms(got[:, 0], want[0]) <= F32_RMS_TOL
    assert rms(got[:, 1] * 1e6, want[1] * 1e6) <= F32_RMS_TOL


@pytest.mark.parametrize("chunks", [None, 4096, 997])
def test_hx_nonfinite_propagates(gar, O, cuda, chunks):
    """Inf / NaN samples: non-finite exactly where the reference is -- an Inf gives NaN
    where the two-stage reference sums +Inf and -Inf DFT outputs (the exact fallback
    runs the two stages), +-Inf where it does not -- and the oracle's values elsewhere;
    any chunking gives the same bits."""
    n = 60000
    x = signal(n, 2, 44100, seed=11).astype(np.float32).astype(np.float64)
    x[20000, 0] = np.inf
    x[41000, 1] = np.nan
    x[41500, 0] = -np.inf
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32, None if chunks is None else chunk_sizes(n, chunks))
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    for c in range(2):
        w = np.asarray(want[c])
        fin = np.isfinite(w)
        assert not fin.all()
        np.testing.assert_array_equal(np.isnan(got[:, c]), np.isnan(w))
        np.testing.assert_array_equal(np.isposinf(got[:, c]), np.isposinf(w))
        np.testing.assert_array_equal(np.isneginf(got[:, c]), np.isneginf(w))
        assert rms(got[fin, c], w[fin]) <= F32_RMS_TOL
    if chunks is not None:
        one = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32)
        np.testing.assert_array_equal(got, one)


@pytest.mark.parametrize("chunks", [None, 4096, 1231])
def test_hx_loud_samples(gar, O, cuda, chunks):
    """Finite samples beyond the split range (|x| >= 16: clipped/unnormalised audio) next
    to normal ones: outputs whose windows hold one are exact, the rest are split-f16,
    and the result does not depend on the chunking."""
    n = 50000
    x = signal(n, 2, 44100, seed=12).astype(np.float32).astype(np.float64)
    x[10000:10050, 0] *= 1000.0
    x[33333, 1] = -3.0e5
    x[45000:, 0] *= 40.0
    x = x.astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32, None if chunks is None else chunk_sizes(n, chunks))
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    ex = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32_EXACT)
    for c in range(2):
        assert got.shape[0] == len(want[c])
        # error at the level of exact-f32 arithmetic on the same (partly loud) signal
        assert rms(got[:, c], want[c]) <= max(3.0 * rms(ex[:, c], want[c]), F32_RMS_TOL)
        big = np.abs(np.asarray(want[c])) > 20
        if big.any():
            assert np.max(np.abs(got[big, c] - want[c][big]) / np.abs(want[c][big])) <= 1e-6
    if chunks is not None:
        one = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32)
        np.testing.assert_array_equal(got, one)


def test_hx_zero_input(gar, O, cuda):
    x = np.zeros((20000, 2))
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32)
    assert np.all(got == 0.0)


def test_hx_loud_many_columns(gar, O, cuda):
    """Loud samples (|x| >= 16) in several columns of one 16-column block and in many blocks of
    one launch (16 channels: ROW16 loads, every block holds loud columns): each output whose
    window holds one is recomputed exactly after the block (hxsFixup), for every column."""
    n, ch = 120000, 16
    x = signal(n, ch, 48000, seed=21).astype(np.float32).astype(np.float64)
    rng = np.random.default_rng(5)
    for c in range(ch):
        for t in rng.integers(0, n, size=6):
            x[t, c] = (1 if rng.random() < 0.5 else -1) * 10.0 ** rng.uniform(1.3, 5)
    x = x.astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 48000, 44100, x, gar.QualityVeryHigh, gar.F32)
    want = oracle_new(O, 48000, 44100, x, O.P_VERYHIGH)
    ex = run(gar, cuda, 48000, 44100, x, gar.QualityVeryHigh, gar.F32_EXACT)
    for c in range(ch):
        assert got.shape[0] == len(want[c])
        assert rms(got[:, c], want[c]) <= max(3.0 * rms(ex[:, c], want[c]), F32_RMS_TOL)
        big = np.abs(np.asarray(want[c])) > 20
        assert big.any()
        assert np.max(np.abs(got[big, c] - want[c][big]) / np.abs(want[c][big])) <= 1e-6


@pytest.mark.parametrize("chunk", [4096, 1500])
def test_hx_row16_small_launches_loud(gar, O, cuda, chunk):
    """16 channels fed in short calls: every launch is a small ROW16 launch (hxq_kernel: one
    workgroup per block and row-block group, history seam loaded through the history resource),
    with loud samples in many columns -- the same bits as the one-shot call, exact where loud."""
    n, ch = 40000, 16
    x = signal(n, ch, 48000, seed=23).astype(np.float32).astype(np.float64)
    rng = np.random.default_rng(9)
    for c in range(ch):
        for t in rng.integers(0, n, size=3):
            x[t, c] = (1 if rng.random() < 0.5 else -1) * 10.0 ** rng.uniform(1.3, 4)
    x = x.astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 48000, 44100, x, gar.QualityVeryHigh, gar.F32, chunk_sizes(n, chunk))
    one = run(gar, cuda, 48000, 44100, x, gar.QualityVeryHigh, gar.F32)
    np.testing.assert_array_equal(got, one)
    want = oracle_new(O, 48000, 44100, x, O.P_VERYHIGH)
    for c in range(ch):
        big = np.abs(np.asarray(want[c])) > 20
        assert big.any()
        assert np.max(np.abs(got[big, c] - want[c][big]) / np.abs(want[c][big])) <= 1e-6


@pytest.mark.parametrize("chunks", [None, 4096])
def test_hx_values_just_below_16(gar, O, cuda, chunks):
    """Samples in [15.996, 16): x * 2^12 rounds to f16 +-Inf there (65520 ties to even), so the split
    bound is 16 - 2^-8 -- at or above it a sample takes the exact path, just below it the split stays
    finite.  Every output finite and within the float32 bar of the oracle, any chunking the same bits."""
    n = 40000
    x = signal(n, 2, 44100, seed=13).astype(np.float32).astype(np.float64)
    vals = [15.99609375, 15.997, 15.9999, -15.99609375, -15.998, 15.996, -15.9960937, 15.99, 16.0]
    rng = np.random.default_rng(3)
    for i, v in enumerate(vals * 6):
        x[int(rng.integers(100, n - 100)), i % 2] = v
    x = x.astype(np.float32).astype(np.float64)
    got = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32, None if chunks is None else chunk_sizes(n, chunks))
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    ex = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32_EXACT)
    for c in range(2):
        assert np.all(np.isfinite(got[:, c]))
        assert rms(got[:, c], want[c]) <= max(3.0 * rms(ex[:, c], want[c]), F32_RMS_TOL)
    if chunks is not None:
        one = run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32)
        np.testing.assert_array_equal(got, one)


def test_hxt_expired_wait_is_a_device_error(gar, cuda, monkeypatch):
    """An expired progress wait of the streaming kernel (hxt_kernel) is an error, not output
    (VERDICT r04 item 2): the development knob GAR_HXT_FAULT=1 makes the compute waves' load count
    unreachable (and the poll bound short), the status word reaches the host, gar_synchronize and
    the next call return GAR_ERR_DEVICE naming hxt_kernel, and Reset recovers the handle."""
    torch = cuda
    frames = 44100 * 20  # a streaming (non-small) launch: hxt_kernel, stereo frames
    x = torch.from_numpy(signal(frames, 2, 44100, seed=7).astype(np.float32)).cuda()
    r = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=gar.F32))
    ref = r.process_device(x).clone()
    torch.cuda.synchronize()
    r.Reset()
    monkeypatch.setenv("GAR_HXT_FAULT", "1")
    r.process_device(x)  # asynchronous: enqueued fine
    with pytest.raises(gar.ErrDevice, match="hxt_kernel"):
        r.synchronize()
    monkeypatch.delenv("GAR_HXT_FAULT")
    with pytest.raises(gar.ErrDevice):  # poisoned until Reset
        r.process_device(x)
    r.Reset()
    again = r.process_device(x).clone()
    r.synchronize()
    assert torch.equal(again, ref)


@pytest.mark.parametrize("ch,dtype,mono_first", [(256, "F32", False), (64, "F64", False), (24, "F32", True)])
def test_large_host_calls_equal_device_stream(gar, cuda, ch, dtype, mono_first):
    """Host ProcessMulti calls large enough for the packing pool (AVX2 conversions, streaming
    stores into the caller's arrays, whole channels per job) return exactly the samples and counts
    of the same streams run through the device API in one call each (chunked == one-shot, stereo ==
    monos), including a handle whose channel 0 was advanced alone first (two channel groups), and
    FlushMulti afterwards."""
    import torch
    n = 2 * 4096 if ch >= 256 else 6 * 4096 + 77
    x = signal(n, ch, 44100, seed=ch).astype(np.float32).astype(np.float64)
    dt = getattr(gar, dtype)
    tdt = torch.float32 if dtype == "F32" else torch.float64
    rh = gar.New(gar.Config(44100, 48000, ch, gar.QualityHigh, ComputeDtype=dt))
    pre = 1000 if mono_first else 0
    got = [[] for _ in range(ch)]
    if mono_first:
        got[0].append(rh.Process(x[:pre, 0]))
    # channel 0 continues at frame pre, the others start at 0: every call gives all channels k frames
    lens = [n - pre] if ch >= 256 else [4096 * 5 + 11, n - pre - (4096 * 5 + 11)]
    s = 0
    for k in lens:
        res = rh.ProcessMulti([x[s + (pre if c == 0 else 0):s + (pre if c == 0 else 0) + k, c] for c in range(ch)])
        for c in range(ch):
            got[c].append(res[c])
        s += k
    tails = rh.FlushMulti()
    got = [np.concatenate(got[c] + [tails[c]]) for c in range(ch)]
    xd = torch.from_numpy(np.ascontiguousarray(x)).to(tdt).cuda()
    if mono_first:
        ref = []
        for c in range(ch):
            r1 = gar.New(gar.Config(44100, 48000, 1, gar.QualityHigh, ComputeDtype=dt))
            L = n if c == 0 else n - pre
            y = torch.cat([r1.process_device(xd[:L, c:c + 1].contiguous()), r1.flush_device(dtype=tdt)])
            ref.append(y[:, 0].double().cpu().numpy())
    else:
        rd = gar.New(gar.Config(44100, 48000, ch, gar.QualityHigh, ComputeDtype=dt))
        y = torch.cat([rd.process_device(xd), rd.flush_device(dtype=tdt)]).double().cpu().numpy()
        ref = [y[:, c] for c in range(ch)]
    torch.cuda.synchronize()
    for c in range(ch):
        assert got[c].shape == ref[c].shape, (c, got[c].shape, ref[c].shape)
        np.testing.assert_array_equal(got[c], ref[c])
