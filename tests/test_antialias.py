"""Anti-aliasing, anti-imaging and impulse-response QA, restated from the reference's
tests:

* antialiasing_test.go:430-466  TestAntiAliasing_Upsampling (engine QualityHigh, >= 80 dB)
* antialiasing_test.go:468-525  TestAntiAliasing_CompareWithSoxr (gap to libsoxr <= 60 dB, >= 80 dB)
* antialiasing_test.go:701-744  TestAntiAliasing_Downsampling (integer ratios >= 80 dB; others logged)
* antialiasing_test.go:746-796  TestAntiAliasing_Downsampling_CompareWithSoxr (48k->32k gap rule)
* quality_comparison_test.go:650-707  TestImpulseResponse_CompareWithSoxr (pre-ringing: warn > 6 dB)
* quality_comparison_test.go:709-790  TestRationalRatio_Quality (upsampling >= 60 dB; down logged)
* README.md:319  "Downsampling (48kHz -> 32kHz) ... THD below -190 dB across presets"

The libsoxr numbers are the reference's fixture (internal/engine/testdata/
soxr_reference_data.json -> tests/golden/soxr_reference_quality.json).

CPU: the oracle meets every threshold the reference asserts.  The reference's engine does
not low-pass non-integer downsampling at the output Nyquist (ComputePolyphaseFilterParams,
filter_params.go:489-511, takes the anti-imaging branch Fn = 1 when there is no pre-stage
and the 2x DFT stage runs first): alias tones pass at 0 dB for 48k->32k, which its own
tests log as "polyphase path limitation" (antialiasing_test.go:724-733,
quality_comparison_test.go:769-779).  Its CompareWithSoxr rule for 48k->32k therefore
fails for the reference design itself (that test skips without the libsoxr tool); it is
kept here as a strict xfail so a change of design shows up.

GPU: the same measurements on the HIP path -- float64 within 0.1 dB of the oracle (impulse:
same peak index and ring-out), float32 (split-f16 MFMA) no more than 3 dB worse than the
reference's own float32 engine -- on the engine seam and on the BASELINE New-path
geometries: cfg3's 48k->44.1k Quality32Bit stage and cfg5's 96k->48k decimator.
"""
import json
import os

import numpy as np
import pytest

import quality as Q

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "soxr_reference_quality.json")) as _f:
    SOXR = json.load(_f)

GPU_F64_DB = 0.1
GPU_F32_SLACK_DB = 3.0

UP_CASES = [(48000, 96000, Q.NOISE), (48000, 96000, Q.MULTITONE), (48000, 96000, Q.SWEEP),
            (44100, 88200, Q.NOISE), (44100, 96000, Q.NOISE)]                       # :430-441
DOWN_CASES = [(48000, 32000), (48000, 44100), (96000, 48000)]                        # :705-713
IMPULSE_CASES = [(44100, 48000), (48000, 44100), (48000, 96000), (96000, 48000), (48000, 32000),
                 (16000, 48000), (32000, 48000)]                                     # :651-662
RATIONAL_CASES = [(44100, 48000), (48000, 44100), (44100, 96000), (96000, 44100), (22050, 48000),
                  (48000, 22050)]                                                    # :711-722


def _eng(O, ir, orr, q, f32=False):
    def run(x):
        e = O.Engine(ir, orr, q, f32=f32)
        return np.concatenate([e.process(np.asarray(x, np.float32 if f32 else np.float64)), e.flush()]).astype(np.float64)
    return run


def _new(O, ir, orr, preset):
    def run(x):
        r = O.NewResampler(ir, orr, 1, preset)
        return np.concatenate([r.process(np.asarray(x, np.float64)), r.flush()])
    return run


def _new_f32_chain(O, ir, orr, x):
    """The New path's stage chain on the reference's float32 engine (VeryHigh -> Quality32Bit)."""
    q = O.lib().o_precision_to_engine_quality(32)
    _, ratios = O.NewResampler(ir, orr, 1, O.P_VERYHIGH).stages()
    y = np.asarray(x, np.float32)
    for r in ratios:
        e = O.Engine(48000.0, 48000.0 * r, q, f32=True)
        y = np.concatenate([e.process(y), e.flush()])
    return y.astype(np.float64)


# ----------------------------------------------------------------------------- CPU: oracle
@pytest.mark.parametrize("ir,orr,kind", UP_CASES)
def test_oracle_upsampling_antiimaging(O, ir, orr, kind):
    """TestAntiAliasing_Upsampling: engine QualityHigh, stopband attenuation >= 80 dB."""
    assert Q.antialiasing(_eng(O, ir, orr, O.HIGH), ir, orr, kind) >= Q.MIN_STOPBAND_ATT


@pytest.mark.parametrize("ir,orr,kind", [(48000, 96000, Q.NOISE), (48000, 96000, Q.MULTITONE),
                                         (44100, 88200, Q.NOISE), (44100, 96000, Q.NOISE)])
def test_oracle_antiimaging_vs_soxr_fixture(O, ir, orr, kind):
    """TestAntiAliasing_CompareWithSoxr's rule (soxr - go <= 60 dB, go >= 80 dB) against the
    fixture's libsoxr attenuation; the restated design lands within 10 dB of libsoxr."""
    soxr = SOXR["antialiasing"][f"{ir}_{orr}_{kind}"]
    go = Q.antialiasing(_eng(O, ir, orr, O.HIGH), ir, orr, kind)
    assert soxr - go <= 60.0 and go >= Q.MIN_STOPBAND_ATT
    assert soxr - go <= 10.0, (go, soxr)


@pytest.mark.parametrize("ir,orr", DOWN_CASES)
def test_oracle_downsampling_antialiasing(O, ir, orr):
    """TestAntiAliasing_Downsampling (engine QualityVeryHigh): integer ratios >= 80 dB; the
    non-integer ones are the reference's logged polyphase-path limitation (alias tones pass)."""
    att = Q.downsampling_antialiasing(_eng(O, ir, orr, O.VERYHIGH), ir, orr)
    if ir % orr == 0:
        assert att >= Q.MIN_STOPBAND_ATT
        # the fixture's libsoxr figure under the CompareWithSoxr gap rule
        assert SOXR["antialiasing"][f"{ir}_{orr}_alias_tones"] - att <= 60.0
    else:
        assert att < 20.0  # no anti-alias low-pass at the output Nyquist (module docstring)


@pytest.mark.xfail(strict=True, reason="the reference design itself fails its 48k->32k CompareWithSoxr rule "
                                       "(non-integer downsampling is not low-passed; module docstring)")
def test_oracle_downsampling_vs_soxr_48k_32k(O):
    """TestAntiAliasing_Downsampling_CompareWithSoxr (48k->32k, VeryHigh)."""
    att = Q.downsampling_antialiasing(_eng(O, 48000, 32000, O.VERYHIGH), 48000, 32000)
    assert SOXR["antialiasing"]["48000_32000_alias_tones"] - att <= 60.0 and att >= Q.MIN_STOPBAND_ATT


@pytest.mark.parametrize("ir,orr", RATIONAL_CASES)
def test_oracle_rational_ratio_quality(O, ir, orr):
    """TestRationalRatio_Quality (VeryHigh): upsampling stopband >= 60 dB; downsampling logged."""
    run = _eng(O, ir, orr, O.VERYHIGH)
    if orr > ir:
        assert Q.antialiasing(run, ir, orr, Q.NOISE) >= 60.0
    else:
        assert np.isfinite(Q.downsampling_antialiasing(run, ir, orr))
    assert Q.thd_internal(run, ir, orr) <= Q.MAX_THD["VeryHigh"]


@pytest.mark.parametrize("name", ["Quick", "Low", "Medium", "High", "VeryHigh"])
def test_oracle_downsampling_thd_readme(O, name):
    """README.md:319: 48k->32k THD below -190 dB across presets."""
    assert Q.thd_internal(_eng(O, 48000, 32000, Q.ENGINE_Q[name]), 48000, 32000) < -190.0


@pytest.mark.parametrize("ir,orr", IMPULSE_CASES)
def test_oracle_impulse_response(O, ir, orr):
    """measureImpulseResponse (VeryHigh): post-ringing below the main peak, ring-out within the
    filter's span; pre-ringing vs libsoxr is informational in the reference (a warning above
    6 dB), so only its sign is checked."""
    m = Q.impulse_response(_eng(O, ir, orr, O.VERYHIGH))
    assert m["post_ringing_db"] < -15.0 and m["pre_ringing_db"] < 0.0
    assert 0 < m["ringout_samples"] < 400
    key = f"impulse_{ir}_{orr}"
    if key in SOXR["quality"]:  # same order of ring-out as libsoxr
        assert abs(m["ringout_samples"] - SOXR["quality"][key]["ringout_samples"]) <= 60


def test_alias_signal_shapes():
    """The generators put their tones where the reference's comments say (48k->32k: 17..23 kHz)."""
    x = Q.alias_tones(48000, 32000)
    f, p = Q.compute_psd(x, 48000)
    peaks = f[(p > p.max() - 3)]
    assert 16900 < peaks.min() and peaks.max() < 23600
    n = Q.antialias_signal(Q.NOISE, 48000)
    assert abs(n).max() <= 0.5 and abs(np.mean(n)) < 0.01


# ----------------------------------------------------------------------------- GPU: HIP path
def _gpu_eng(gar, ir, orr, q, dtype):
    def run(x):
        r = gar.EngineNewResampler(ir, orr, q, dtype)
        if dtype == gar.F64:
            y = np.concatenate([r.Process(np.asarray(x, np.float64)), r.Flush()])
        else:
            y = np.concatenate([r.ProcessFloat32(np.asarray(x, np.float32)), r.Flush()])
        return y.astype(np.float64)
    return run


def _gpu_new(gar, ir, orr, dtype):
    def run(x):
        r = gar.New(gar.Config(ir, orr, 1, gar.QualityVeryHigh, ComputeDtype=dtype))
        if dtype == gar.F64:
            y = np.concatenate([r.Process(np.asarray(x, np.float64)), r.Flush()])
        else:
            y = np.concatenate([r.ProcessFloat32(np.asarray(x, np.float32)), r.Flush()])
        return y.astype(np.float64)
    return run


@pytest.mark.gpu
@pytest.mark.parametrize("ir,orr,kind", UP_CASES)
def test_gpu_upsampling_antiimaging(gar, O, cuda, ir, orr, kind):
    g64 = Q.antialiasing(_gpu_eng(gar, ir, orr, 3, gar.F64), ir, orr, kind)
    assert abs(g64 - Q.antialiasing(_eng(O, ir, orr, O.HIGH), ir, orr, kind)) <= GPU_F64_DB
    g32 = Q.antialiasing(_gpu_eng(gar, ir, orr, 3, gar.F32), ir, orr, kind)
    assert g32 >= Q.antialiasing(_eng(O, ir, orr, O.HIGH, f32=True), ir, orr, kind) - GPU_F32_SLACK_DB
    assert min(g64, g32) >= Q.MIN_STOPBAND_ATT


@pytest.mark.gpu
@pytest.mark.parametrize("ir,orr", DOWN_CASES + [(96000, 44100)])
@pytest.mark.parametrize("path", ["engine", "new"])
def test_gpu_downsampling_antialiasing(gar, O, cuda, ir, orr, path):
    """Engine seam (QualityVeryHigh) and the New path (Quality32Bit): 48k->44.1k is cfg3's
    stage, 96k->48k cfg5's decimator, 96k->44.1k all of cfg5."""
    if path == "engine":
        o64, o32 = _eng(O, ir, orr, O.VERYHIGH), _eng(O, ir, orr, O.VERYHIGH, f32=True)
        g64, g32 = _gpu_eng(gar, ir, orr, 4, gar.F64), _gpu_eng(gar, ir, orr, 4, gar.F32)
    else:
        o64 = _new(O, ir, orr, O.P_VERYHIGH)
        o32 = lambda x: _new_f32_chain(O, ir, orr, x)  # noqa: E731
        g64, g32 = _gpu_new(gar, ir, orr, gar.F64), _gpu_new(gar, ir, orr, gar.F32)
    want = Q.downsampling_antialiasing(o64, ir, orr)
    assert abs(Q.downsampling_antialiasing(g64, ir, orr) - want) <= GPU_F64_DB
    got32 = Q.downsampling_antialiasing(g32, ir, orr)
    assert got32 >= Q.downsampling_antialiasing(o32, ir, orr) - GPU_F32_SLACK_DB
    if ir % orr == 0:
        assert got32 >= Q.MIN_STOPBAND_ATT


@pytest.mark.gpu
@pytest.mark.parametrize("ir,orr", IMPULSE_CASES)
@pytest.mark.parametrize("path", ["engine", "new"])
def test_gpu_impulse_response(gar, O, cuda, ir, orr, path):
    if path == "engine":
        want = Q.impulse_response(_eng(O, ir, orr, O.VERYHIGH))
        runs = [_gpu_eng(gar, ir, orr, 4, gar.F64), _gpu_eng(gar, ir, orr, 4, gar.F32)]
    else:
        want = Q.impulse_response(_new(O, ir, orr, O.P_VERYHIGH))
        runs = [_gpu_new(gar, ir, orr, gar.F64), _gpu_new(gar, ir, orr, gar.F32)]
    for i, run in enumerate(runs):
        got = Q.impulse_response(run)
        assert got["peak_index"] == want["peak_index"]
        assert abs(got["ringout_samples"] - want["ringout_samples"]) <= (0 if i == 0 else 1)
        tol = GPU_F64_DB if i == 0 else 0.01 + 1e-3  # f32: 1e-7-level output error, far above -60 dB
        assert abs(got["pre_ringing_db"] - want["pre_ringing_db"]) <= tol
        assert abs(got["post_ringing_db"] - want["post_ringing_db"]) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("ir,orr", [(44100, 48000), (44100, 96000), (22050, 48000)])
def test_gpu_rational_ratio_upsampling(gar, O, cuda, ir, orr):
    g = Q.antialiasing(_gpu_eng(gar, ir, orr, 4, gar.F64), ir, orr, Q.NOISE)
    assert abs(g - Q.antialiasing(_eng(O, ir, orr, O.VERYHIGH), ir, orr, Q.NOISE)) <= GPU_F64_DB
    assert g >= 60.0
