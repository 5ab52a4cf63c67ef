"""BASELINE.json configs at their full sizes on the GPU: exact output lengths,
RMS vs the oracle (full stream where the oracle finishes in seconds, channel
subsets otherwise) and size-independent properties (chunk invariance,
channel independence, linearity)."""
import numpy as np
import pytest

from helpers import F32_RMS_TOL, F64_RMS_TOL, chunk_sizes, oracle_new, rms, signal

pytestmark = pytest.mark.gpu


def synth_torch(torch, frames, channels, rate, seed):
    """Device-side generator of the same signal shape (fast for 10^9 samples)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    t = torch.arange(frames, device="cuda", dtype=torch.float64) / rate
    ph = torch.rand((2, channels), generator=g, device="cuda", dtype=torch.float64) * 2 * np.pi
    noise = torch.rand((frames, channels), generator=g, device="cuda", dtype=torch.float32) - 0.5
    x = (0.7 * torch.sin(2 * np.pi * 440 * t[:, None] + ph[0]) + 0.2 * torch.sin(2 * np.pi * 1750 * t[:, None] + ph[1]))
    return (x + 0.1 * noise.double()).float()


def test_cfg2_full_600s_stereo(gar, O, cuda):
    frames = 26_460_000
    x = signal(frames, 2, 44100, seed=4242).astype(np.float32)
    r = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=gar.F32))
    xd = cuda.from_numpy(x).cuda()
    y = cuda.cat([r.process_device(xd), r.flush_device()]).double().cpu().numpy()
    assert y.shape == (28_800_002, 2)                  # 28,799,730 + 272
    ref = O.NewResampler(44100, 48000, 2, O.P_HIGH)
    for c in range(2):
        want = np.concatenate([ref.process(x[:, c].astype(np.float64), c), ref.flush(c)])
        assert len(want) == y.shape[0]
        assert rms(y[:, c], want) <= F32_RMS_TOL
    # chunked (reference ProcessInto 4096-frame pattern) vs one shot on a 60 s prefix:
    # bit for bit (the split scale is a constant; processinto_test.go:258-308)
    m = 44100 * 60
    r.Reset()
    one = cuda.cat([r.process_device(xd[:m]), r.flush_device()]).double().cpu().numpy()
    r.Reset()
    outs = [r.process_device(xd[s:s + n]).clone() for s, n in zip(range(0, m, 4096), chunk_sizes(m, 4096))]
    outs.append(r.flush_device())
    got = cuda.cat(outs).double().cpu().numpy()
    np.testing.assert_array_equal(got, one)


@pytest.mark.parametrize("dtype", ["F32", "F32_EXACT", "F64"])
def test_cfg2_chunked_bit_exact(gar, cuda, dtype):
    """Every compute path: the reference's 4096-frame ProcessInto pattern == one shot, bit for bit."""
    m = 44100 * 10
    x = signal(m, 2, 44100, seed=99).astype(np.float32)
    xd = cuda.from_numpy(x).cuda()
    r = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=getattr(gar, dtype)))
    one = cuda.cat([r.process_device(xd), r.flush_device()]).cpu().numpy()
    r.Reset()
    outs = [r.process_device(xd[s:s + n]).clone() for s, n in zip(range(0, m, 4096), chunk_sizes(m, 4096))]
    outs.append(r.flush_device())
    np.testing.assert_array_equal(cuda.cat(outs).cpu().numpy(), one)


def test_cfg3_full_256ch_10s(gar, O, cuda):
    frames, ch = 480_000, 256
    xd = synth_torch(cuda, frames, ch, 48000, 3)
    r = gar.New(gar.Config(48000, 44100, ch, gar.QualityVeryHigh, ComputeDtype=gar.F32))
    y = cuda.cat([r.process_device(xd), r.flush_device()])
    assert y.shape[0] == 441_002
    x = xd.double().cpu().numpy()
    yc = y.double().cpu().numpy()
    for c in (0, 101, 255):
        want = oracle_new(O, 48000, 44100, x[:, c:c + 1], O.P_VERYHIGH)[0]
        assert rms(yc[:, c], want) <= F32_RMS_TOL
    # channel independence: one channel resampled alone is bit-identical
    solo = gar.New(gar.Config(48000, 44100, 1, gar.QualityVeryHigh, ComputeDtype=gar.F32))
    s = cuda.cat([solo.process_device(xd[:, 101:102].contiguous()), solo.flush_device()]).cpu().numpy()
    np.testing.assert_array_equal(s[:, 0], y[:, 101].cpu().numpy())


def test_northstar_256ch_44k1_48k_60s(gar, O, cuda):
    """north_star workload: 256-channel float32 44.1k->48k QualityHigh, 60 s, one Process + Flush
    (the ROW16 streaming kernel): exact length, a channel subset vs the oracle over the whole
    stream, the reference's 4096-frame ProcessInto pattern == one shot bit for bit (small-launch
    kernel vs streaming kernel), and a channel resampled alone == its column of the 256."""
    frames, ch = 2_646_000, 256
    xd = synth_torch(cuda, frames, ch, 44100, 256)
    r = gar.New(gar.Config(44100, 48000, ch, gar.QualityHigh, ComputeDtype=gar.F32))
    y = cuda.cat([r.process_device(xd), r.flush_device()])
    assert y.shape[0] == 2_880_002                  # 44100 -> 48000 over 60 s + the flush tail
    x = xd[:, [0, 77, 255]].double().cpu().numpy()
    yc = y[:, [0, 77, 255]].double().cpu().numpy()
    for j in range(3):
        want = oracle_new(O, 44100, 48000, x[:, j:j + 1], O.P_HIGH)[0]
        assert len(want) == y.shape[0]
        assert rms(yc[:, j], want) <= F32_RMS_TOL
    m = 44100 * 5
    r.Reset()
    one = cuda.cat([r.process_device(xd[:m]), r.flush_device()]).cpu().numpy()
    r.Reset()
    outs = [r.process_device(xd[s:s + n]).clone() for s, n in zip(range(0, m, 4096), chunk_sizes(m, 4096))]
    outs.append(r.flush_device())
    np.testing.assert_array_equal(cuda.cat(outs).cpu().numpy(), one)
    solo = gar.New(gar.Config(44100, 48000, 1, gar.QualityHigh, ComputeDtype=gar.F32))
    s = cuda.cat([solo.process_device(xd[:, 77:78].contiguous()), solo.flush_device()]).cpu().numpy()
    np.testing.assert_array_equal(s[:, 0], y[:, 77].cpu().numpy())


def test_cfg4_full_1024_stereo_streams(gar, O, cuda):
    streams, frames = 1024, 441_000
    xd = synth_torch(cuda, frames, 2 * streams, 44100, 4)
    r = gar.NewBatch(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=gar.F32), streams)
    y = cuda.cat([r.process_device(xd), r.flush_device()])
    assert y.shape == (480_002, 2048)
    for s in (0, 517, 1023):
        x = xd[:, 2 * s:2 * s + 2].double().cpu().numpy()
        want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
        for c in range(2):
            assert rms(y[:, 2 * s + c].double().cpu().numpy(), want[c]) <= F32_RMS_TOL
    # linearity across streams: resample(a + b) == resample(a) + resample(b) within f32 rounding
    r2 = gar.NewBatch(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=gar.F32), 1)
    a, b = xd[:, 0:2].contiguous(), xd[:, 2:4].contiguous()
    ya = cuda.cat([r2.process_device(a), r2.flush_device()]); r2.Reset()
    yb = cuda.cat([r2.process_device(b), r2.flush_device()]); r2.Reset()
    yab = cuda.cat([r2.process_device(a + b), r2.flush_device()])
    assert float(((yab - ya - yb).double() ** 2).mean().sqrt()) <= 2 * F32_RMS_TOL


def test_cfg5_full_8ch_f64_60s_chunked(gar, O, cuda):
    frames = 5_760_000
    x = signal(frames, 8, 96000, seed=5)
    r = gar.New(gar.Config(96000, 44100, 8, gar.QualityVeryHigh, ComputeDtype=gar.F64))
    xd = cuda.from_numpy(x).cuda()
    outs = [r.process_device(xd[s:s + n]) for s, n in zip(range(0, frames, 4800), chunk_sizes(frames, 4800))]
    outs.append(r.flush_device(dtype=cuda.float64))
    y = cuda.cat(outs).cpu().numpy()
    ideal = frames * 44100 // 96000
    assert ideal - 64 <= y.shape[0] <= ideal + 256
    want = oracle_new(O, 96000, 44100, x[:, 3:4], O.P_VERYHIGH, chunks=chunk_sizes(frames, 4800))[0]
    assert len(want) == y.shape[0]
    assert rms(y[:, 3], want) <= F64_RMS_TOL
