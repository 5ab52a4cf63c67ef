"""Pins the CPU oracle against every known-answer test the reference holds for
this path (the reference ships no per-sample golden vectors -- SURVEY 8(c)).

Each test cites the reference test it restates (path:line in /root/reference).
"""
import math

import numpy as np
import pytest

from helpers import oracle_new, sine


# internal/mathutil/bessel_test.go:13-40
@pytest.mark.parametrize("x,expected,tol", [
    (0.0, 1.0, 1e-15), (0.5, 1.063483344, 1e-7), (1.0, 1.266065848, 1e-7), (2.0, 2.279585307, 1e-7),
    (3.0, 4.880792565, 1e-7), (3.75, 9.118945994, 1e-7), (4.0, 11.30192217, 1e-7), (5.0, 27.23987183, 1e-7),
    (10.0, 2815.716628, 1e-6), (20.0, 4.355826e7, 1e-1), (-0.5, 1.063483344, 1e-7), (-1.0, 1.266065848, 1e-7),
])
def test_bessel_i0_table(O, x, expected, tol):
    got = O.bessel_i0(x)
    assert abs(got - expected) / abs(expected) <= tol


def test_bessel_symmetry_monotonic(O):  # bessel_test.go:43-70
    for x in (0.1, 1.0, 2.5, 5.0, 10.0):
        assert abs(O.bessel_i0(x) - O.bessel_i0(-x)) <= 1e-10
    prev = O.bessel_i0(0)
    for x in np.arange(0.1, 10.0, 0.1):
        cur = O.bessel_i0(x)
        assert cur > prev
        prev = cur


def test_simdops_kats(O):  # internal/simdops/ops_test.go:25-70
    assert abs(O.dot([1, 2, 3], [4, 5, 6]) - 32) <= 1e-5
    np.testing.assert_allclose(O.convolve_valid([1, 2, 3, 4], [1, 0.5]), [2, 3.5, 5], atol=1e-5)
    np.testing.assert_allclose(O.convolve_valid([1, 2, 3, 4], [0, 2]), [4, 6, 8], atol=1e-5)
    assert abs(O.cubic_interp_dot([0.5, 0.5], [1, 2], [3, 4], [5, 6], [7, 8], 0.5) - 5.5625) <= 1e-5


# internal/engine/critical_functions_test.go:18-52
@pytest.mark.parametrize("ratio,expected", [
    (1.0, True), (2.0, True), (3.0, True), (4.0, True), (2.0000000001, True), (0.5, False), (0.333333, False),
    (1.5, False), (1.088435374, False), (0.91875, False), (2.1768707, False), (0.0, False), (0.999999, False),
    (0.9999999999, True), (1.0000000001, True),
])
def test_is_integer_ratio(O, ratio, expected):
    assert bool(O.lib().o_is_integer_ratio(ratio)) == expected


# critical_functions_test.go:58-100 (+ the exact L the SURVEY derives)
@pytest.mark.parametrize("ratio", [1.088435374, 0.91875, 1.0, 0.5, 0.25, 2.0])
def test_find_rational_approx(O, ratio):
    L, step = O.find_rational_approx(ratio)
    assert 64 <= L <= 256 and step > 0
    assert abs(step / L - 1 / ratio) / (1 / ratio) < 0.01


def test_rational_approx_exact_phases(O):
    assert O.find_rational_approx(48000.0 / 88200.0) == (80, 147)    # 44.1k->48k poly stage
    assert O.find_rational_approx(44100.0 / 96000.0) == (147, 320)   # 48k->44.1k poly stage


# critical_functions_test.go:103-165
def test_lsx_inv_f_resp(O):
    for drop, a in [(-0.01, 180), (-0.01, 140), (-0.01, 100), (-0.1, 180), (-1.0, 180), (-3.0, 180),
                    (-6.0, 180), (-0.01, 1.0), (-0.01, 300.0), (0.0, 180), (-20.0, 180)]:
        r = O.lib().o_lsx_inv_f_resp(drop, a)
        assert math.isfinite(r) and 0.0 <= r <= 1.0
    prev = -1
    for drop in (-0.001, -0.01, -0.1, -1.0, -3.0, -6.0):
        r = O.lib().o_lsx_inv_f_resp(drop, 180.0)
        assert r > prev
        prev = r


# critical_functions_test.go:170-310 (Fn normalisation from soxr cr.c)
@pytest.mark.parametrize("L,ratio,tio,pre,fn,up", [
    (147, 48000 / 44100, 44100 / 48000, True, 1.0, True),
    (147, 96000 / 44100, 44100 / 96000, True, 1.0, True),
    (160, 44100 / 48000, 48000 / 44100, False, 1.0, False),
    (1, 48000 / 96000, 96000 / 48000, False, 1.0, False),
    (2, 32000 / 48000, 48000 / 32000, False, 1.0, False),
    (160, 44100 / 48000, 48000 / 44100, True, 2.0 * 1.088, False),
    (1, 48000 / 96000, 96000 / 48000, True, 4.0, False),
])
def test_poly_params_fn(O, L, ratio, tio, pre, fn, up):
    p = O.compute_poly_params(L, ratio, tio, pre, 126.0, 0.912)
    assert bool(p.is_upsampling) == up
    assert abs(p.fn - fn) <= fn * 0.01
    if not up and pre:
        assert abs(p.fs_raw - (3.0 + abs(ratio - 1.0))) <= 0.01
    assert abs(p.fp - p.fp_raw / p.fn) <= 1e-4 and abs(p.fs - p.fs_raw / p.fn) <= 1e-4
    assert 0 < p.fc < 1


def test_decimation_normalisation():  # internal/filter/soxr_filter_test.go:270-282
    fpn, fsn = 0.913 / 2, 1.0 / 2
    assert abs(fpn - 0.4565) < 1e-4 and abs(fsn - 0.5) < 1e-4 and abs(0.5 * (fsn - fpn) - 0.02175) < 1e-4


# README.md:466-471 -- filter complexity table for 44.1k->48k engine presets
@pytest.mark.parametrize("q,dft_taps,poly_taps", [(1, 132, 32), (2, 132, 32), (3, 166, 64)])
def test_readme_filter_table(O, q, dft_taps, poly_taps):
    inf = O.Engine(44100, 48000, q).info()
    assert (inf.dft_factor, inf.dft_taps_per_phase, inf.poly_phases, inf.poly_taps_per_phase) == \
        (2, dft_taps, 80, poly_taps)


def test_dft_phase_dc_gain(O):  # critical_functions_test.go:397-419
    e = O.Engine(44100, 88200, O.HIGH)   # integer ratio -> DFT stage only
    for p in (0, 1):
        assert abs(e.coeffs(0, p).sum() - 1.0) < 0.01


def test_dc_gain_and_zero_in(O):  # critical_functions_test.go:445-490, regression_test.go:12-185
    for (i, o) in [(44100, 48000), (48000, 44100), (48000, 96000), (96000, 48000)]:
        e = O.Engine(i, o, O.HIGH)
        y = np.concatenate([e.process(np.ones(5000)), e.flush()])
        mid = y[len(y) // 4: 3 * len(y) // 4]
        assert abs(mid.mean() - 1.0) < 1e-3
        e = O.Engine(i, o, O.HIGH)
        z = np.concatenate([e.process(np.zeros(3000)), e.flush()])
        assert np.max(np.abs(z)) <= 1e-10


def test_cfg1_length(O):  # SURVEY 8 derived length; ResampleMono = Process + Flush (convenience.go:204-229)
    y = O.resample_mono(sine(44100, 44100), 44100, 48000, O.P_HIGH)
    assert len(y) == 48002
    assert np.all(np.isfinite(y))


def test_cfg3_geometry_length(O):
    x = sine(48000, 48000)[:, None]
    y = oracle_new(O, 48000, 44100, x, O.P_VERYHIGH)[0]
    assert len(y) == 44102


# flush_multistage_test.go:26-97: New path Process+Flush within [ideal-64, ideal+256]
@pytest.mark.parametrize("i,o", [(48000, 16000), (96000, 16000), (48000, 8000), (192000, 48000), (88200, 16000)])
def test_multistage_flush_lengths(O, i, o):
    n = i * 2
    x = np.random.default_rng(4242).standard_normal(n)[:, None] * 0.1
    y = oracle_new(O, i, o, x, O.P_HIGH)[0]
    ideal = round(n * o / i)
    assert ideal - 64 <= len(y) <= ideal + 256
    assert len(O.NewResampler(i, o, 1, O.P_HIGH).stages()[0]) >= 2


# internal/pipeline/pipeline_test.go:13-175 (stage types)
@pytest.mark.parametrize("ratio,prec,types", [
    (1.5, 8, [0]), (0.125, 16, [1, 1, 3]), (0.15, 16, [1, 1, 2]), (8.0, 16, [1, 1, 3]), (10.0, 16, [1, 1, 1, 2]),
    (44100 / 48000, 16, [3]), (48000 / 44100, 16, [3]), (1.5, 28, [3]),
])
def test_pipeline_stage_types(O, ratio, prec, types):
    t, _ = O.build_pipeline(ratio, prec)
    assert list(map(int, t)) == types


def test_bit_identities(O):
    """processinto_test.go:36-104/258-308, convenience_stereo_test.go:40-106,
    reset_state_test.go:97 -- chunking, stereo==two monos, Reset==fresh."""
    x = np.random.default_rng(7).standard_normal((9600, 2)) * 0.3
    one = oracle_new(O, 44100, 48000, x, O.P_HIGH)
    chunked = oracle_new(O, 44100, 48000, x, O.P_HIGH, chunks=[4800, 4800])
    for c in range(2):
        np.testing.assert_array_equal(one[c], chunked[c])
    mono = oracle_new(O, 44100, 48000, x[:, 1:2], O.P_HIGH)[0]
    np.testing.assert_array_equal(mono, one[1])
    r = O.NewResampler(44100, 48000, 1, O.P_HIGH)
    r.process(x[:, 0]); r.flush(); r.reset()
    again = np.concatenate([r.process(x[:, 1]), r.flush()])
    np.testing.assert_array_equal(again, one[1])


def test_golden_fixtures_reproduce(O):
    """The committed fixtures (tests/golden/make_golden.py) still come out of the oracle."""
    import golden_cases
    for case in golden_cases.load_all():
        got = golden_cases.run_oracle(O, case)
        want = case["outputs"]
        assert len(got) == len(want)
        for g, w in zip(got, want):
            np.testing.assert_allclose(g, w, rtol=0, atol=1e-13)
