"""C-ABI boundary and host state machine, CPU only (dry-run handles do the
reference's exact integer bookkeeping without touching a GPU)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from helpers import chunk_sizes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    hdr = open(os.path.join(ROOT, "include", "gar.h")).read()
    return set(re.findall(r"^\s*(?:gar_status|void|int64_t|int32_t|double|const char \*|gar_quality_spec)\s+\**"
                          r"(gar_\w+)\s*\(", hdr, re.M))


def test_library_exports_every_declared_symbol(gar):
    decl = header_symbols()
    assert len(decl) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", gar.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines()}
    assert decl <= syms, decl - syms
    assert set(gar.EXPORTED) <= syms
    # code object for gfx950 is embedded
    assert b"gfx950" in open(gar.LIB_PATH, "rb").read()


def _validate(gar, **kw):
    cfg = gar.Config(**kw)
    return gar.lib().gar_config_validate(C.byref(cfg))


def test_config_validate(gar):  # resample.go:168-214
    ok = dict(InputRate=44100, OutputRate=48000, Channels=2)
    assert _validate(gar, **ok) == 0
    assert _validate(gar, **dict(ok, InputRate=0)) == gar.INVALID_CONFIG
    assert _validate(gar, **dict(ok, OutputRate=-1)) == gar.INVALID_CONFIG
    assert _validate(gar, **dict(ok, Channels=0)) == gar.INVALID_CONFIG
    assert _validate(gar, **dict(ok, Channels=257)) == gar.INVALID_CONFIG
    assert _validate(gar, **dict(ok, Channels=256)) == 0
    assert _validate(gar, **dict(ok, OutputRate=44100 * 257)) == gar.INVALID_CONFIG
    assert _validate(gar, **dict(ok, OutputRate=44100 / 257)) == gar.INVALID_CONFIG
    bad = gar.QualitySpec(Preset=gar.QualityCustom, Precision=7, PhaseResponse=50, PassbandEnd=0.9, StopbandBegin=0.95)
    assert _validate(gar, **dict(ok, Quality=bad)) == gar.INVALID_CONFIG
    good = gar.QualitySpec(Preset=gar.QualityCustom, Precision=20, PhaseResponse=50, PassbandEnd=0.9, StopbandBegin=0.95)
    assert _validate(gar, **dict(ok, Quality=good)) == 0
    for field, val in (("PhaseResponse", 101), ("PassbandEnd", 1.0), ("StopbandBegin", 0.5)):
        q = gar.QualitySpec(Preset=gar.QualityCustom, Precision=20, PhaseResponse=50, PassbandEnd=0.9, StopbandBegin=0.95)
        setattr(q, field, val)
        assert _validate(gar, **dict(ok, Quality=q)) == gar.INVALID_CONFIG
    with pytest.raises(gar.ErrInvalidConfig):
        gar.New(gar.Config(0, 48000, DryRun=True))


def test_preset_specs(gar):  # resample.go:217-267
    want = {0: (8, 0.7, 1.0), 1: (16, 0.80, 0.95), 2: (16, 0.90, 0.98), 3: (24, 0.95, 0.99), 4: (32, 0.99, 0.995)}
    for p, (prec, pb, sb) in want.items():
        s = gar.GetPresetSpec(p)
        assert (s.Preset, s.Precision, s.PassbandEnd, s.StopbandBegin, s.PhaseResponse) == (p, prec, pb, sb, 50.0)


def test_new_expands_preset_into_config(gar):  # resample.go:282-284 mutates the caller's config
    cfg = gar.Config(44100, 48000, 1, gar.QualityVeryHigh, DryRun=True)
    h = C.c_void_p(0)
    assert gar.lib().gar_new(C.byref(cfg), C.byref(h)) == 0
    assert cfg.Quality.Precision == 32 and abs(cfg.Quality.StopbandBegin - 0.995) < 1e-12
    gar.lib().gar_free(h)


def test_quick_preset_builds_cubic_stage(gar, O):
    """QualityQuick: one CubicStage at the total ratio (pipeline.go:115-121, stages.go:21-23)."""
    g = gar.New(gar.Config(44100, 48000, 1, gar.QualityQuick, DryRun=True))
    ref = O.NewResampler(44100, 48000, 1, 0)
    assert g.GetLatency() == ref.latency()
    info = g.GetInfo()
    assert (info.FilterLength, info.Phases, bool(info.SIMDEnabled)) == (4, 0, False)  # cubic.go:119-137


ENGINE_PAIRS = [(44100, 48000), (48000, 44100), (48000, 96000), (96000, 48000), (48000, 16000), (16000, 44100),
                (22050, 16000), (44100, 32000), (8000, 48000), (44100, 44100), (48000, 200), (1000, 255000)]


@pytest.mark.parametrize("i,o", ENGINE_PAIRS)
@pytest.mark.parametrize("preset", [0, 1, 2, 3])
def test_engine_stream_lengths(gar, O, i, o, preset):
    """Every call returns exactly the reference's sample count: chunked Process,
    Flush, Process after Flush without Reset, repeated Flush, Reset."""
    rng = np.random.default_rng(0)
    e = O.Engine(i, o, O.lib().o_preset_to_engine_quality(preset))
    r = gar.NewEngineDry(i, o, preset)
    for step in ([1, 5, 100, 4096, 3, 20000, 0, 1], ["f", 777, "f", "f", 31, "reset", 5000, "f"]):
        for n in step:
            if n == "f":
                a, b = len(e.flush()), r.FlushSize()
                r.Flush()
            elif n == "reset":
                e.reset(), r.Reset()
                continue
            else:
                x = rng.standard_normal(n)
                a, b = len(e.process(x)), r.OutputSize(n)
                r.Process(x)
            assert a == b, (n, a, b)


@pytest.mark.parametrize("i,o", [(44100, 48000), (48000, 44100), (96000, 48000), (48000, 96000), (16000, 44100)])
@pytest.mark.parametrize("preset", [0, 3])
def test_engine_statistics(gar, O, i, o, preset):
    """GetStatistics (resampler.go:348-353) after every call of a chunked stream with flushes,
    an empty Process and a Reset equals the reference engine's samplesIn / samplesOut."""
    rng = np.random.default_rng(3)
    e = O.Engine(i, o, O.lib().o_preset_to_engine_quality(preset))
    r = gar.NewEngineDry(i, o, preset)
    assert r.GetStatistics() == {"samplesIn": 0, "samplesOut": 0}
    for n in [4096, 1, 0, 777, "f", 4800, "f", "reset", 333, 20000, "f"]:
        if n == "f":
            e.flush(), r.Flush()
        elif n == "reset":
            e.reset(), r.Reset()
        else:
            x = rng.standard_normal(n)
            e.process(x), r.Process(x)
        assert r.GetStatistics() == e.statistics(), n
    with pytest.raises(gar.ResamplerError):
        r.GetStatistics(channel=1)


def test_statistics_per_channel_group(gar):
    """A mono Process on a multi-channel handle advances channel 0 alone (constant.go:88-95):
    its counters move, the other channels' do not."""
    g = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, DryRun=True))
    g.ProcessMulti([np.zeros(1000), np.zeros(1000)])
    both = g.GetStatistics(0)
    assert both == g.GetStatistics(1) and both["samplesIn"] == 1000
    g.Process(np.zeros(500))
    assert g.GetStatistics(0)["samplesIn"] == 1500 and g.GetStatistics(1)["samplesIn"] == 1000
    g.Reset()
    assert g.GetStatistics(0) == {"samplesIn": 0, "samplesOut": 0} == g.GetStatistics(1)


NEW_PAIRS = [(44100, 48000), (48000, 44100), (96000, 44100), (96000, 16000), (192000, 48000), (48000, 8000),
             (88200, 16000), (44100, 44200), (16000, 48000), (8000, 96000)]


@pytest.mark.parametrize("i,o", NEW_PAIRS)
@pytest.mark.parametrize("preset", [0, 1, 2, 3, 4])
def test_new_path_stream_lengths(gar, O, i, o, preset):
    rng = np.random.default_rng(1)
    ref = O.NewResampler(i, o, 1, preset)
    g = gar.New(gar.Config(i, o, 1, preset, DryRun=True))
    for n in chunk_sizes(30017, 4800) + [0, 17]:
        x = rng.standard_normal(n)
        assert len(ref.process(x)) == g.OutputSize(n)
        g.Process(x)
    assert len(ref.flush()) == g.FlushSize()
    g.Flush()
    x = rng.standard_normal(999)
    assert len(ref.process(x)) == g.OutputSize(999)
    assert g.GetLatency() == ref.latency()
    assert g.GetRatio() == ref.ratio


@pytest.mark.parametrize("i,o,preset", [(44100, 48000, 3), (48000, 44100, 4), (96000, 44100, 4), (48000, 16000, 1)])
def test_estimate_output_is_upper_bound(gar, i, o, preset):  # processinto_test.go:311-453
    g = gar.New(gar.Config(i, o, 1, preset, DryRun=True))
    for n in [1, 7, 64, 1000, 4096, 4800, 48000] * 3:
        assert g.OutputSize(n) <= g.EstimateOutput(n)
        g.Process(np.zeros(n))
        assert g.EstimateOutput(n) == int(n * (o / i)) + 64


def test_buffer_too_small_does_not_advance_state(gar):  # processinto_test.go:176-227
    g = gar.New(gar.Config(44100, 48000, 1, gar.QualityHigh, DryRun=True))
    x = np.zeros(4096)
    g.Process(x)
    before = g.OutputSize(4096)
    small = np.zeros(g.EstimateOutput(4096) - 1)
    with pytest.raises(gar.ErrBufferTooSmall):
        g.ProcessInto(x, small)
    assert g.OutputSize(4096) == before
    with pytest.raises(gar.ErrBufferTooSmall):
        g.ProcessFloat32Into(x.astype(np.float32), np.zeros(len(small), np.float32))
    assert g.OutputSize(4096) == before


def test_channel_state_independence(gar, O):
    """Process (channel 0 only, constant.go:88-95) advances channel 0 alone;
    ProcessMulti then yields per-channel lengths exactly like the reference."""
    rng = np.random.default_rng(2)
    ref = O.NewResampler(48000, 44100, 3, O.P_HIGH)
    g = gar.New(gar.Config(48000, 44100, 3, gar.QualityHigh, DryRun=True))
    x0 = rng.standard_normal(1234)
    ref.process(x0, 0)
    g.Process(x0)
    xs = [rng.standard_normal(5000) for _ in range(3)]
    want = [len(ref.process(x, c)) for c, x in enumerate(xs)]
    got = [g.OutputSize(5000, c) for c in range(3)]
    assert got == want and got[0] != got[1]
    with pytest.raises(gar.ErrChannelMismatch):
        g.ProcessMulti(xs[:2])


def test_latency_and_info(gar, O):  # constant.go:407-485
    for (i, o, p) in [(44100, 48000, 3), (48000, 44100, 4), (96000, 44100, 4), (96000, 16000, 3)]:
        g = gar.New(gar.Config(i, o, 2, p, DryRun=True))
        assert g.GetLatency() == O.NewResampler(i, o, 2, p).latency()
        info = g.GetInfo()
        assert info.Algorithm == b"multi-stage" and info.Latency == g.GetLatency() and info.SIMDEnabled


def test_batch_handle_channel_count(gar):
    g = gar.NewBatch(gar.Config(44100, 48000, 2, gar.QualityHigh, DryRun=True), 1024)
    assert g.Channels == 2048
    with pytest.raises(gar.ErrInvalidConfig):
        gar.NewBatch(gar.Config(44100, 48000, 300, gar.QualityHigh, DryRun=True), 2)


def test_device_api_channel_mismatch(gar):
    """gar_process_device / gar_flush_device refuse a buffer whose channel count is not the
    handle's (ErrChannelMismatch, constant.go:205-207) before touching memory."""
    import ctypes as C
    r = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, DryRun=True))
    got = C.c_int64(0)
    rc = gar.lib().gar_process_device(r._h, None, gar.F32, 1, 1, 100, 3, None, gar.F32, 1, 1, 1000, C.byref(got), None)
    assert rc == gar.CHANNEL_MISMATCH
    rc = gar.lib().gar_flush_device(r._h, 1, None, gar.F32, 1, 1, 1000, C.byref(got), None)
    assert rc == gar.CHANNEL_MISMATCH
    rc = gar.lib().gar_process_device(r._h, None, gar.F32, 2, 1, -5, 2, None, gar.F32, 2, 1, 1000, C.byref(got), None)
    assert rc == gar.INVALID_ARGUMENT


def test_engine_quality_constructor_dry(gar):
    """gar_new_engine_quality maps engine.Quality directly (resampler.go:51): unknown values are ErrInvalidConfig."""
    import ctypes as C
    h = C.c_void_p(0)
    assert gar.lib().gar_new_engine_quality(44100.0, 48000.0, 42, gar.F64, C.byref(h)) == gar.INVALID_CONFIG
    assert not h.value


@pytest.mark.parametrize("i,o", [(44100, 48000), (48000, 44100), (96000, 44100), (16000, 44100), (48000, 96000)])
@pytest.mark.parametrize("preset", [0, 1, 3, 4])
def test_get_info_fields(gar, O, i, o, preset):
    """GetInfo (constant.go:452-485): algorithm, latency, and the primary stage's filter
    length / phases (StageAdapter.GetFilterLength/GetPhases, stage_adapter.go:98-119;
    CubicStage 4 / 0, cubic.go:119-132) against the oracle's stage designs."""
    g = gar.New(gar.Config(i, o, 2, preset, DryRun=True))
    ref = O.NewResampler(i, o, 1, preset)
    inf = g.GetInfo()
    assert inf.Algorithm == b"multi-stage"
    assert inf.Latency == ref.latency()
    s0 = ref.stage_info(0)
    if s0.kind == 0:
        assert (inf.FilterLength, inf.Phases) == (4, 0)
    else:
        want = (s0.dft_taps_per_phase * s0.dft_factor if s0.dft_factor > 1 else 0) + \
            s0.poly_taps_per_phase * s0.poly_phases
        assert (inf.FilterLength, inf.Phases) == (want, s0.poly_phases)
    assert inf.MemoryUsage == _ref_memory_usage(ref, 2)


def _ref_memory_usage(ref, channels, max_input_size=0):
    """MemoryUsage of a fresh reference handle (constant.go:457-468): per channel, the ring
    buffers' float64 capacity (8192, buffer 0 = MaxInputSize*2 when set: constant.go:72-78) plus
    StageAdapter.GetMemoryUsage (stage_adapter.go:66-96) -- DFT coefficients factor*taps + history
    cap 2*taps (dft_stage.go:142), polyphase bank `a` L*taps + history cap 2*taps
    (polyphase_stage.go:167), float64 elements; decimators and (Quick) cubic stages 64 B
    (cubicMemoryUsage)."""
    kinds, _ = ref.stages()
    per = sum((max_input_size * 2 if (j == 0 and max_input_size > 0) else 8192) * 8 for j in range(len(kinds) + 1))
    for j in range(len(kinds)):
        s = ref.stage_info(j)
        if s.kind == 0:
            per += 64
            continue
        if s.dft_factor > 1:
            per += (s.dft_factor * s.dft_taps_per_phase + 2 * s.dft_taps_per_phase) * 8
        if s.poly_phases > 0:
            per += (s.poly_phases * s.poly_taps_per_phase + 2 * s.poly_taps_per_phase) * 8
    return per * channels


def test_memory_usage_pinned(gar, O):
    """Hand-derived from the reference code for 44.1k->48k QualityHigh (Quality24Bit: DFT 2 x 200,
    polyphase 80 x 100) on 2 channels: buffers 2 x 8192 x 8, DFT 2*200*8 + 400*8, poly 80*100*8 + 200*8."""
    g = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, DryRun=True))
    assert g.GetInfo().MemoryUsage == 2 * (2 * 8192 * 8 + 3200 + 3200 + 64000 + 1600)
    g = gar.New(gar.Config(44100, 48000, 1, gar.QualityHigh, MaxInputSize=4096, DryRun=True))
    assert g.GetInfo().MemoryUsage == (4096 * 2 * 8 + 8192 * 8 + 3200 + 3200 + 64000 + 1600)


def test_device_api_sample_types(gar):
    """The device entry points accept float32/float64 and integer PCM (GAR_PCM16/24/32,
    resample-wav main.go:444-543) and refuse any other sample type before touching memory;
    a dry handle runs the PCM calls through the stream-length state machine."""
    import ctypes as C
    r = gar.New(gar.Config(44100, 48000, 2, gar.QualityHigh, DryRun=True))
    got = C.c_int64(0)
    for bad in (3, 8, 17, 64, -1):
        rc = gar.lib().gar_process_device(r._h, None, bad, 2, 1, 0, 2, None, gar.F32, 2, 1, 1000, C.byref(got), None)
        assert rc == gar.INVALID_ARGUMENT, bad
        rc = gar.lib().gar_flush_device(r._h, 2, None, bad, 2, 1, 1000, C.byref(got), None)
        assert rc == gar.INVALID_ARGUMENT, bad
    n = gar.lib().gar_device_output_size(r._h, 4410)
    for t in (gar.PCM16, gar.PCM24, gar.PCM32):
        r.Reset()
        rc = gar.lib().gar_process_device(r._h, C.c_void_p(1), t, 2, 1, 4410, 2, C.c_void_p(1), t, 2, 1, n, C.byref(got), None)
        assert rc == gar.GAR_OK and got.value == n
    assert gar._io_type.__doc__


def test_pcm_constants_match_header(gar):
    """gar.h GAR_PCM16/24/32 equal the Python mirror's codes (the bit depth)."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "gar.h")).read()
    m = re.search(r"GAR_PCM16 = (\d+), GAR_PCM24 = (\d+), GAR_PCM32 = (\d+)", hdr)
    assert m and tuple(int(v) for v in m.groups()) == (gar.PCM16, gar.PCM24, gar.PCM32)


@pytest.mark.parametrize("dtype", ["F64", "F32"])
@pytest.mark.parametrize("i,o,chunk", [(96000, 44100, 4800), (48000, 44100, 4096), (44100, 48000, 4096),
                                       (96000, 16000, 4800)])
def test_fused_stage_stays_fused_streaming(gar, dtype, i, o, chunk):
    """A DftPoly stage whose step has no fraction runs on its composite FIR plan (f64 and f32
    compute) and stays fused through ProcessMulti streaming of 4800/4096-frame chunks -- cfg5's
    48k->44.1k Quality32Bit stage included (a Pc=294 f64 plan did not fit; buildBgPlan now falls
    back to Pc=147).  Only Process after Flush switches it to stage-by-stage."""
    r = gar.New(gar.Config(i, o, 8, gar.QualityVeryHigh, ComputeDtype=getattr(gar, dtype), DryRun=True))
    nst = r.num_stages()
    assert nst >= 1
    fused_stages = [s for s in range(nst) if r.stage_state(s)[0]]
    assert fused_stages, "no fused stage"
    xs = [np.zeros(chunk) for _ in range(8)]
    for _ in range(25):
        r.ProcessMulti(xs)
        for s in fused_stages:
            assert r.stage_state(s) == (True, True)
    r.FlushMulti()
    r.ProcessMulti(xs)
    assert all(r.stage_state(s) == (True, False) for s in fused_stages)
    r.Reset()
    assert all(r.stage_state(s) == (True, True) for s in fused_stages)


@pytest.mark.parametrize("i,o,preset", [(96000, 44100, 4), (44100, 48000, 3), (96000, 16000, 3), (48000, 44100, 4)])
def test_stage_geometry_matches_oracle_pipeline(gar, O, i, o, preset):
    """gar_num_stages / gar_stage_geometry report the pipeline of pipeline.BuildPipeline
    (pipeline.go:104-183) and each stage's engine design, as the oracle builds them."""
    r = gar.New(gar.Config(i, o, 2, preset, DryRun=True))
    ref = O.NewResampler(i, o, 1, preset)
    kinds, ratios = ref.stages()
    assert r.num_stages() == len(kinds)
    for j in range(len(kinds)):
        ratio, g = r.stage_geometry(j)
        assert ratio == pytest.approx(ratios[j], rel=1e-15)
        s = ref.stage_info(j)
        assert g.kind == s.kind
        if s.dft_factor > 1:
            assert (g.dft_factor, g.dft_taps) == (s.dft_factor, s.dft_taps_per_phase)
        if s.poly_phases:
            assert (g.poly_phases, g.poly_taps, g.poly_step) == (s.poly_phases, s.poly_taps_per_phase, s.poly_step)
        if s.decim_factor:
            assert (g.decim_factor, g.decim_taps) == (s.decim_factor, s.decim_taps)


@pytest.mark.parametrize("i,o", [(44100, 48000), (96000, 8000), (44100, 44100), (48000, 96000), (48000, 44100)])
def test_quick_phase_walk_long_stream(gar, O, i, o):
    """QualityQuick phase walk over a long stream in ragged calls: every call's output count equals the
    reference's sequential float64 walk (cubic.go:42-61).  44.1k->48k, 96k->8k, 1:1 and 2x take the
    exact closed form (cntCubic: every f64 addition of the walk is exact there); 48k->44.1k walks."""
    rng = np.random.default_rng(7)
    e = O.Engine(i, o, O.lib().o_preset_to_engine_quality(0))
    r = gar.NewEngineDry(i, o, 0)
    total = 0
    while total < 3_000_000:
        n = int(rng.choice([1, 3, 4095, 4096, 65536, 250_000, 1_000_003]))
        x = np.zeros(n)
        assert r.OutputSize(n) == len(e.process(x)), (total, n)
        r.Process(x)
        total += n
    assert r.FlushSize() == len(e.flush())


def test_host_staging_pool_selftest(gar):
    """The host calls' conversion pool (spinning workers, (generation, index) job tickets, whole-channel
    jobs): several caller threads at once, every element checked (no GPU needed)."""
    import ctypes
    f = gar.lib().gar_dev_pool_selftest
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64]
    assert f(4, 20, 64, 8192) == 0      # many channels: whole channels per job
    assert f(3, 10, 3, 100000) == 0     # few channels: slices of channels
    assert f(8, 5, 256, 4096) == 0      # more caller threads than one job: the rest run inline
    assert f(2, 50, 2, 70000) == 0      # short jobs back to back: workers woken while spinning
    # caller t uses channels + t: the threads' job counts differ and cross 2 * workers (whole-channel
    # jobs vs channel slices), so consecutive jobs on the pool have different job counts
    assert f(6, 20, 12, 20000) == 0
    assert f(6, 20, 28, 12000) == 0


def test_host_pool_tsan():
    """ThreadSanitizer stress of the pool (tools/pool_tsan.cpp: callers with different job counts back
    to back, every index exactly once, nothing running after run() returns)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-audio-resampler_amd")
    r = subprocess.run(["make", "-s", "-C", root, "tsan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 bad" in r.stdout
