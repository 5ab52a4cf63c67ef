"""Product host design (libgar.so, C++) vs the CPU oracle (C): coefficient
banks, geometry and the fused composite FIR.  No GPU needed."""
import numpy as np
import pytest

RATES = [(44100, 48000), (48000, 44100), (16000, 44100), (22050, 16000), (48000, 96000), (96000, 48000),
         (48000, 16000), (44100, 32000), (8000, 48000), (48000, 192000), (44100, 44100), (48000, 52244.89795918367)]
QUALS = [1, 2, 3, 4, 5, 6, 7, 8, 9]  # engine.Quality Low..Quality32Bit


@pytest.mark.parametrize("i,o", RATES)
@pytest.mark.parametrize("q", QUALS)
def test_banks_match_oracle(gar, O, i, o, q):
    g, b = gar.design_engine(i, o, q)
    e = O.Engine(i, o, q)
    inf = e.info()
    assert g.kind == inf.kind
    if g.kind in (1, 2):
        assert (g.dft_factor, g.dft_taps) == (inf.dft_factor, inf.dft_taps_per_phase)
        ref = np.concatenate([e.coeffs(0, p) for p in range(g.dft_factor)])
        np.testing.assert_array_equal(b["dft"], ref)
    if g.kind == 2:
        assert (g.poly_phases, g.poly_taps, g.poly_step) == (inf.poly_phases, inf.poly_taps_per_phase, inf.poly_step)
        for which, key in ((1, "a"), (2, "b"), (3, "c"), (4, "d")):
            np.testing.assert_array_equal(b[key], e.coeffs(which))
    if g.kind == 3:
        assert (g.decim_factor, g.decim_taps) == (inf.decim_factor, inf.decim_taps)
        np.testing.assert_array_equal(b["decim"], e.coeffs(5))


@pytest.mark.parametrize("i,o,q", [(44100, 48000, 7), (48000, 44100, 9), (44100, 48000, 3), (48000, 44100, 3),
                                   (48000, 32000, 7), (22050, 16000, 3), (44100, 96000, 9)])
def test_composite_fir_equals_stage_composition(gar, O, i, o, q):
    """The fused FIR row r equals a[ph] (poly bank) composed with the two DFT
    phases -- recomputed here in numpy from the *oracle's* banks."""
    rows, offs, g = gar.design_composite(i, o, q)
    e = O.Engine(i, o, q)
    inf = e.info()
    L, T2, S = inf.poly_phases, inf.poly_taps_per_phase, inf.poly_step >> 16
    T1 = inf.dft_taps_per_phase
    a = e.coeffs(1).reshape(L, T2)
    c = np.stack([e.coeffs(0, 0), e.coeffs(0, 1)])
    P = g.fir_period_out
    for r in range(P):
        d = (r * S) // L
        ph, par = (r * S) % L, d & 1
        ref = np.zeros(((par + T2 - 1) >> 1) + T1)
        for k2 in range(T2):
            q2 = par + k2
            ref[(q2 >> 1):(q2 >> 1) + T1] += a[ph, k2] * c[q2 & 1]
        assert offs[r] == d >> 1
        np.testing.assert_allclose(rows[r, :len(ref)], ref, rtol=0, atol=1e-15 * np.abs(ref).max())
        assert np.all(rows[r, len(ref):] == 0)


def test_fused_geometry_bench_config(gar):
    # BASELINE cfg2: 44.1k->48k QualityHigh on the New path = engine(48000, 48000*r, Quality24Bit)
    g, _ = gar.design_engine(48000.0, 48000.0 * (48000 / 44100), gar.Engine24Bit)
    assert g.fused and (g.dft_taps, g.poly_phases, g.poly_taps, g.poly_step >> 16) == (200, 80, 100, 147)
    assert (g.fir_period_out, g.fir_period_in, g.fir_taps_max) == (160, 147, 250)
    assert abs(g.useful_macs_per_output - 249.5) < 1e-9
    assert g.mfma_macs_per_output / g.useful_macs_per_output < 1.1   # banded-GEMM padding < 10 %
