"""GPU parity: every sample the MI355X path produces vs the CPU oracle (the
reference's algorithm) on identical inputs, through the C-ABI.

Tolerances (BASELINE.json north_star): float32 <= 1e-6 RMS, float64 <= 1e-12
RMS; output lengths must match exactly.  Invariants the reference tests as
bit-identities are asserted bit-identical here too.
"""
import numpy as np
import pytest

import golden_cases
from helpers import F32_RMS_TOL, F64_RMS_TOL, chunk_sizes, oracle_new, rms, signal, sine

pytestmark = pytest.mark.gpu


def dev_run(gar, torch, in_rate, out_rate, x, preset, dtype, chunks=None, flush=True, io_dtype=None):
    """resampler.New over the device API; x [n, ch] float64 host array."""
    ch = x.shape[1]
    r = gar.New(gar.Config(in_rate, out_rate, ch, preset, ComputeDtype=dtype))
    tdt = io_dtype or (torch.float32 if dtype == gar.F32 else torch.float64)
    xd = torch.from_numpy(np.ascontiguousarray(x)).to(tdt).cuda()
    outs, s = [], 0
    for n in (chunks or [x.shape[0]]):
        outs.append(r.process_device(xd[s:s + n]).clone())
        s += n
    if flush:
        outs.append(r.flush_device(dtype=tdt).clone())
    torch.cuda.synchronize()
    return torch.cat(outs).double().cpu().numpy()


def check(got, want, tol):
    assert got.shape[0] == len(want), (got.shape, len(want))
    err = rms(got, want)
    assert err <= tol, err
    return err


# ---- BASELINE configs at reduced length (full sizes: test_gpu_fullsize.py) --
def test_cfg1_resample_mono_f64(gar, O, cuda):
    x = sine(44100, 44100)
    got = gar.ResampleMono(x, 44100, 48000, gar.QualityHigh)
    want = O.resample_mono(x, 44100, 48000, O.P_HIGH)
    assert len(got) == len(want) == 48002
    assert rms(got, want) <= F64_RMS_TOL


@pytest.mark.parametrize("chunk", [None, 4096, 777])
def test_cfg2_stereo_f32_44k1_48k(gar, O, cuda, chunk):
    x = signal(88200, 2, 44100).astype(np.float32).astype(np.float64)
    chunks = chunk_sizes(88200, chunk) if chunk else None
    got = dev_run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32, chunks)
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    for c in range(2):
        check(got[:, c], want[c], F32_RMS_TOL)


def test_cfg3_256ch_f32_48k_44k1(gar, O, cuda):
    x = signal(24000, 256, 48000, seed=100).astype(np.float32).astype(np.float64)
    got = dev_run(gar, cuda, 48000, 44100, x, gar.QualityVeryHigh, gar.F32)
    want = oracle_new(O, 48000, 44100, x[:, ::17], O.P_VERYHIGH)
    for k, c in enumerate(range(0, 256, 17)):
        check(got[:, c], want[k], F32_RMS_TOL)


def test_cfg4_batched_stereo_streams(gar, O, cuda):
    streams, n = 64, 22050
    x = signal(n, 2 * streams, 44100, seed=7).astype(np.float32).astype(np.float64)
    r = gar.NewBatch(gar.Config(44100, 48000, 2, gar.QualityHigh, ComputeDtype=gar.F32), streams)
    xd = cuda.from_numpy(x.astype(np.float32)).cuda()
    got = cuda.cat([r.process_device(xd[:10000]), r.process_device(xd[10000:]), r.flush_device()]).double().cpu().numpy()
    for s in (0, 31, 63):
        want = oracle_new(O, 44100, 48000, x[:, 2 * s:2 * s + 2], O.P_HIGH)
        for c in range(2):
            check(got[:, 2 * s + c], want[c], F32_RMS_TOL)


def test_cfg5_8ch_f64_96k_44k1_multistage(gar, O, cuda):
    n = 48000
    x = signal(n, 8, 96000, seed=55)
    chunks = chunk_sizes(n, 4800)
    got = dev_run(gar, cuda, 96000, 44100, x, gar.QualityVeryHigh, gar.F64, chunks)
    want = oracle_new(O, 96000, 44100, x, O.P_VERYHIGH, chunks=chunks)
    for c in range(8):
        check(got[:, c], want[c], F64_RMS_TOL)


# ---- every engine kind / ratio family --------------------------------------
ENGINE_CASES = [
    (44100, 48000), (48000, 44100),                  # DFTx2 + polyphase, fused MFMA FIR
    (16000, 44100), (22050, 16000), (44100, 32000),  # frac != 0: staged + live cubic interpolation
    (48000, 96000), (48000, 192000),                 # integer up: DFT only
    (96000, 48000), (48000, 16000),                  # integer down: decimator
    (44100, 44100),                                  # factor-1 pass-through
    (48000, 200),                                    # extreme down (polyphase rebase quirk path)
]


@pytest.mark.parametrize("i,o", ENGINE_CASES)
@pytest.mark.parametrize("preset", [0, 1, 3])
def test_engine_f64_vs_oracle(gar, O, cuda, i, o, preset):
    x = signal(int(i * 0.3) + 17, 1, i, seed=i % 97)[:, 0]
    r = gar.NewEngine(i, o, preset)
    e = O.Engine(i, o, O.lib().o_preset_to_engine_quality(preset))
    for n in (1000, 1, 0, len(x) - 1001):
        seg = x[:n] if n else x[:0]
        x = x[n:]
        got, want = r.Process(seg), e.process(seg)
        check(got, want, F64_RMS_TOL)
    check(r.Flush(), e.flush(), F64_RMS_TOL)


@pytest.mark.parametrize("i,o", [(44100, 48000), (48000, 44100), (16000, 44100), (96000, 48000)])
def test_engine_float32_vs_oracle(gar, O, cuda, i, o):
    """NewEngineFloat32 (convenience.go:329): float32 engine vs the float32 and float64 restatements."""
    x = signal(i // 2, 1, i, seed=3)[:, 0].astype(np.float32)
    got = gar.ResampleMonoFloat32(x, i, o, gar.QualityHigh)
    e32 = O.Engine(i, o, O.HIGH, f32=True)
    want32 = np.concatenate([e32.process(x), e32.flush()])
    check(got, want32, F32_RMS_TOL)
    e64 = O.Engine(i, o, O.HIGH)
    want64 = np.concatenate([e64.process(x.astype(np.float64)), e64.flush()])
    check(got, want64, F32_RMS_TOL)


@pytest.mark.parametrize("i,o,preset", [(96000, 16000, 3), (192000, 48000, 4), (48000, 8000, 3), (8000, 96000, 4),
                                        (44100, 44200, 3), (88200, 16000, 1)])
def test_new_path_multistage_f64(gar, O, cuda, i, o, preset):
    x = signal(i // 2, 2, i, seed=1)
    chunks = chunk_sizes(i // 2, 4800)
    got = dev_run(gar, cuda, i, o, x, preset, gar.F64, chunks)
    want = oracle_new(O, i, o, x, preset, chunks=chunks)
    for c in range(2):
        check(got[:, c], want[c], F64_RMS_TOL)


def test_golden_fixtures(gar, O, cuda):
    for case in golden_cases.load_all():
        x = golden_cases.make_input(case)
        for c in range(case["channels"]):
            if case["kind"] == "new":
                r = gar.New(gar.Config(case["in_rate"], case["out_rate"], 1, case["preset"]))
                proc, fl = r.Process, r.Flush
            elif case["kind"] == "engine":
                r = gar.NewEngine(case["in_rate"], case["out_rate"], case["preset"])
                proc, fl = r.Process, r.Flush
            else:
                r = gar.NewEngineFloat32(case["in_rate"], case["out_rate"], case["preset"])
                proc, fl = r.ProcessFloat32, r.Flush
            parts, s = [], 0
            for op in case["ops"]:
                if op[0] == "p":
                    parts.append(np.asarray(proc(x[s:s + op[1], c]), np.float64))
                    s += op[1]
                else:
                    parts.append(np.asarray(fl(), np.float64))
            got = np.concatenate(parts)
            tol = F32_RMS_TOL if case["kind"] == "engine32" else F64_RMS_TOL
            check(got, case["outputs"][c], tol)


# ---- reference bit-identity invariants --------------------------------------
def test_process_into_equals_process(gar, cuda):  # processinto_test.go:36-104
    x = signal(30000, 1, 48000)[:, 0]
    a = gar.New(gar.Config(48000, 44100, 1, gar.QualityHigh))
    b = gar.New(gar.Config(48000, 44100, 1, gar.QualityHigh))
    for seg in np.array_split(x, 7):
        want = a.Process(seg)
        buf = np.empty(b.EstimateOutput(len(seg)))
        n = b.ProcessInto(seg, buf)
        np.testing.assert_array_equal(buf[:n], want)


@pytest.mark.parametrize("dtype", ["F32", "F32_EXACT", "F64"])
def test_chunking_is_bit_identical(gar, cuda, dtype):  # processinto_test.go:258-308
    """Any chunking == one shot, bit for bit, on every compute path (GAR_F32 included:
    its split scale is a constant, so an output depends only on its own window)."""
    dt = getattr(gar, dtype)
    x = signal(60000, 2, 44100)
    one = dev_run(gar, cuda, 44100, 48000, x, gar.QualityHigh, dt)
    for size in (4800, 4096, 333, 1):
        n = 60000 if size > 1 else 3000
        ref = one if size > 1 else dev_run(gar, cuda, 44100, 48000, x[:n], gar.QualityHigh, dt)
        np.testing.assert_array_equal(dev_run(gar, cuda, 44100, 48000, x[:n], gar.QualityHigh, dt,
                                              chunk_sizes(n, size)), ref)


@pytest.mark.parametrize("dtype", ["F32", "F32_EXACT", "F64"])
@pytest.mark.parametrize("case", [(8000, 11025, 1, "QualityMedium"), (16000, 44100, 2, "QualityHigh"),
                                  (64000, 176400, 2, "QualityLow"), (37800, 44100, 3, "QualityVeryHigh")])
def test_chunking_is_bit_identical_fractional_steps(gar, cuda, case, dtype):
    """Ratios whose polyphase step has fractional bits (poly_kernel, live cubic coefficients): any
    chunking == one shot, bit for bit (r05: the tap rotation used the launch-relative output index, so
    chunked and one-shot sums differed in the last bits -- found by the ragged-call sweep)."""
    ir, orr, ch, q = case
    dt = getattr(gar, dtype)
    x = signal(20011, ch, ir, seed=9)
    one = dev_run(gar, cuda, ir, orr, x, getattr(gar, q), dt)
    for size in (4096, 1111, 97):
        np.testing.assert_array_equal(dev_run(gar, cuda, ir, orr, x, getattr(gar, q), dt, chunk_sizes(20011, size)), one)


@pytest.mark.parametrize("case", [(48000, 44100, 5, "QualityVeryHigh"), (96000, 44100, 3, "QualityVeryHigh"),
                                  (22050, 44100, 1, "QualityHigh"), (44100, 96000, 4, "QualityLow")])
def test_chunking_is_bit_identical_f32_pipelines(gar, cuda, case):
    """GAR_F32 chunk invariance across the other engine kinds and multi-stage pipelines."""
    ir, orr, ch, q = case
    x = signal(30011, ch, ir, seed=5)
    one = dev_run(gar, cuda, ir, orr, x, getattr(gar, q), gar.F32)
    for size in (4096, 777):
        np.testing.assert_array_equal(dev_run(gar, cuda, ir, orr, x, getattr(gar, q), gar.F32,
                                              chunk_sizes(30011, size)), one)


def test_stereo_equals_two_monos(gar, cuda):  # convenience_stereo_test.go:40-106
    x = signal(20000, 2, 44100)
    both = dev_run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F64)
    for c in range(2):
        np.testing.assert_array_equal(dev_run(gar, cuda, 44100, 48000, x[:, c:c + 1], gar.QualityHigh, gar.F64)[:, 0],
                                      both[:, c])
    lo, ro = gar.ResampleStereo(x[:, 0], x[:, 1], 44100, 48000, gar.QualityHigh)
    np.testing.assert_array_equal(lo, gar.ResampleMono(x[:, 0], 44100, 48000, gar.QualityHigh))
    np.testing.assert_array_equal(ro, gar.ResampleMono(x[:, 1], 44100, 48000, gar.QualityHigh))


def test_reset_equals_fresh(gar, cuda):  # internal/engine/reset_state_test.go:97,321
    x = signal(12000, 1, 44100)[:, 0]
    r = gar.NewEngine(44100, 48000, gar.QualityHigh)
    first = np.concatenate([r.Process(x), r.Flush()])
    r.Process(x[:5000])
    r.Reset()
    again = np.concatenate([r.Process(x), r.Flush()])
    np.testing.assert_array_equal(first, again)


def test_process_multi_and_flush_multi(gar, O, cuda):  # parallel_test.go:12-89, flush_multi_test.go:88
    x = signal(20000, 3, 48000, seed=2)
    r = gar.New(gar.Config(48000, 44100, 3, gar.QualityHigh))
    outs = r.ProcessMulti([x[:, c] for c in range(3)])
    tails = r.FlushMulti()
    want = oracle_new(O, 48000, 44100, x, O.P_HIGH)
    for c in range(3):
        check(np.concatenate([outs[c], tails[c]]), want[c], F64_RMS_TOL)


def test_concurrent_handles_large_host_calls(gar, cuda):
    """Two threads drive two independent handles with host ProcessMulti calls large enough
    (> 1 MiB) to use the shared packing pool (ctypes releases the GIL): each thread's outputs
    equal the same calls made alone, bit for bit (Go resampler instances are independent)."""
    import threading
    xs = [signal(96000, 4, 48000, seed=s) for s in (11, 12)]

    def run(x, out, reps=4):
        r = gar.New(gar.Config(48000, 44100, 4, gar.QualityHigh, ComputeDtype=gar.F32))
        for _ in range(reps):
            r.Reset()
            res = r.ProcessMulti([x[:, c] for c in range(4)])
            out.append(np.concatenate(res + r.FlushMulti()))

    alone = [[], []]
    for k in range(2):
        run(xs[k], alone[k], reps=1)
    both = [[], []]
    th = [threading.Thread(target=run, args=(xs[k], both[k])) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for k in range(2):
        assert len(both[k]) == 4
        for got in both[k]:
            np.testing.assert_array_equal(got, alone[k][0])


def test_mono_call_on_multichannel_handle(gar, O, cuda):
    """Process advances channel 0 only (constant.go:88-95); ProcessMulti after it."""
    x = signal(9000, 2, 48000, seed=4)
    ref = O.NewResampler(48000, 44100, 2, O.P_HIGH)
    r = gar.New(gar.Config(48000, 44100, 2, gar.QualityHigh))
    check(r.Process(x[:3000, 0]), ref.process(x[:3000, 0], 0), F64_RMS_TOL)
    outs = r.ProcessMulti([x[3000:, 0], x[3000:, 1]])
    check(outs[0], ref.process(x[3000:, 0], 0), F64_RMS_TOL)
    check(outs[1], ref.process(x[3000:, 1], 1), F64_RMS_TOL)
    tails = r.FlushMulti()
    for c in range(2):
        check(tails[c], ref.flush(c), F64_RMS_TOL)


def test_process_after_flush_and_double_flush(gar, O, cuda):
    x = signal(9000, 1, 44100, seed=8)[:, 0]
    for (i, o) in ((44100, 48000), (48000, 44100), (16000, 44100), (96000, 48000)):
        r, e = gar.NewEngine(i, o, gar.QualityHigh), O.Engine(i, o, O.HIGH)
        seq = [("p", x[:4000]), ("f",), ("p", x[4000:6000]), ("f",), ("f",), ("p", x[6000:]), ("f",)]
        for op in seq:
            if op[0] == "p":
                check(r.Process(op[1]), e.process(op[1]), F64_RMS_TOL)
            else:
                check(r.Flush(), e.flush(), F64_RMS_TOL)


def test_edge_inputs(gar, O, cuda):
    """Empty input, inputs shorter than the filter, single samples (fuzz_test.go:73-132)."""
    for (i, o) in ((44100, 48000), (48000, 44100), (96000, 48000)):
        r, e = gar.NewEngine(i, o, gar.QualityHigh), O.Engine(i, o, O.HIGH)
        assert len(r.Process(np.zeros(0))) == 0 and len(r.Flush()) == 0   # never fed: no phantom tail
        for n in (1, 2, 3, 50, 1):
            seg = np.full(n, 0.25)
            check(r.Process(seg), e.process(seg), F64_RMS_TOL)
        check(r.Flush(), e.flush(), F64_RMS_TOL)
    for (i, o, n) in ((1.9195e6, 16033, 412), (1.296e6, 7350, 1080)):   # testdata/fuzz/FuzzResampleMono corpus
        y = gar.ResampleMono(sine(n, i), i, o, gar.QualityMedium)
        assert np.all(np.isfinite(y)) and len(y) > 0


def test_buffer_too_small_keeps_state_on_gpu(gar, cuda):  # processinto_test.go:176-227
    x = signal(10000, 1, 44100)[:, 0]
    a = gar.New(gar.Config(44100, 48000, 1, gar.QualityHigh))
    b = gar.New(gar.Config(44100, 48000, 1, gar.QualityHigh))
    with pytest.raises(gar.ErrBufferTooSmall):
        a.ProcessInto(x, np.empty(10))
    np.testing.assert_array_equal(a.Process(x), b.Process(x))


def test_device_api_float64_io_on_f32_compute(gar, O, cuda):
    """float64 device buffers into a float32-compute handle (dtype conversion in the loader)."""
    x = signal(30000, 2, 44100, seed=12)
    got = dev_run(gar, cuda, 44100, 48000, x, gar.QualityHigh, gar.F32, io_dtype=cuda.float64)
    want = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    for c in range(2):
        check(got[:, c], want[c], F32_RMS_TOL)


QUICK_CASES = [(44100, 48000), (48000, 44100), (16000, 44100), (96000, 8000), (8000, 96000), (44100, 44100),
               (22050, 16000)]


@pytest.mark.parametrize("i,o", QUICK_CASES)
def test_quick_cubic_new_path_streaming(gar, O, cuda, i, o):
    """QualityQuick (CubicStage, cubic.go:33-90; pipeline.go:115-121) through the device API in
    ragged chunks: exact output counts, float64 within 1e-12 of the oracle, float32 compute
    within 1e-6 of the oracle fed the same float32 samples."""
    x = signal(i // 3 + 5, 2, i, seed=7)
    chunks = [1, 2, 3, 4096, 1000, 0, 17]
    chunks += chunk_sizes(len(x) - sum(chunks), 4096)
    for dt, tdt, tol in ((gar.F64, cuda.float64, F64_RMS_TOL), (gar.F32, cuda.float32, F32_RMS_TOL)):
        xin = x if dt == gar.F64 else x.astype(np.float32).astype(np.float64)
        want = oracle_new(O, i, o, xin, 0, chunks=chunks)
        r = gar.New(gar.Config(i, o, 2, gar.QualityQuick, ComputeDtype=dt))
        xd = cuda.from_numpy(xin).to(device="cuda", dtype=tdt)
        outs, s = [], 0
        for n in chunks:
            outs.append(r.process_device(xd[s:s + n]) if n else xd[:0])
            s += n
        outs.append(r.flush_device(dtype=tdt))
        y = cuda.cat(outs).double().cpu().numpy()
        for c in range(2):
            assert y.shape[0] == len(want[c])
            assert rms(y[:, c], want[c]) <= tol


def test_quick_engine_float32(gar, O, cuda):
    """NewEngineFloat32 with QualityQuick: CubicStage[float32] (cubic.go:15-90)."""
    x = signal(30011, 1, 44100, seed=9)[:, 0].astype(np.float32)
    got = gar.ResampleMonoFloat32(x, 44100, 48000, gar.QualityQuick)
    e = O.Engine(44100, 48000, O.lib().o_preset_to_engine_quality(0), f32=True)
    want = np.concatenate([e.process(x), e.flush()])
    assert len(got) == len(want)
    assert rms(got, want) <= F32_RMS_TOL


@pytest.mark.parametrize("dtype", ["F64", "F32"])
@pytest.mark.parametrize("i,o,preset", [(44100, 48000, 3), (48000, 44100, 4), (96000, 44100, 4), (44100, 48000, 0)])
def test_new_path_process_float32_values(gar, O, cuda, i, o, preset, dtype):
    """New-path ProcessFloat32 / ProcessFloat32Into (constant.go:121-199): float32 in and out,
    the float64 pipeline in between; values within 1e-6 of the oracle fed the same float32
    samples, chunked Into calls identical to one-shot ProcessFloat32."""
    x = signal(i // 4 + 3, 1, i, seed=11)[:, 0].astype(np.float32)
    ref = O.NewResampler(i, o, 1, preset)
    want = np.concatenate([ref.process(x.astype(np.float64), 0), ref.flush(0)])
    r = gar.New(gar.Config(i, o, 1, preset, ComputeDtype=getattr(gar, dtype)))
    got = np.concatenate([r.ProcessFloat32(x), r.Flush()])
    assert got.dtype in (np.float32, np.float64)
    check(got.astype(np.float64), want, F32_RMS_TOL)
    r.Reset()
    outs = []
    for s, n in zip(range(0, len(x), 4096), chunk_sizes(len(x), 4096)):
        buf = np.empty(r.EstimateOutput(n), dtype=np.float32)
        k = r.ProcessFloat32Into(x[s:s + n], buf)
        outs.append(buf[:k].copy())
    outs.append(np.asarray(r.Flush(), dtype=np.float32))
    into = np.concatenate(outs)
    assert np.array_equal(into.astype(np.float32), got.astype(np.float32))
