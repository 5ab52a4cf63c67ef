"""32-channel blocks of the balanced streaming kernel (gar_hxt.hpp FMT 5, round 6).

f32 row streams whose channel count is a multiple of 32 (the north-star 256-channel stream among them)
run hxt_kernel on blocks of 32 channels: every load and store instruction covers whole 128-B lines, two
16-column tiles per compute wave over one 8-quad ring.  Each output keeps its A fragments, B values and
MFMA chain, so the outputs must equal the 16-channel blocks' bit for bit (knob GAR_HXT_WIDE=0, read per
launch), loud and non-finite samples included (two exact fixups per block), and the reference's within
the float32 bar (dft_stage.go:156-349 + polyphase_stage.go:186-352 through the oracle)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import F32_RMS_TOL, oracle_new, rms, signal

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device_run(gar, torch, x, ir, orr, preset, chunk=None):
    """One New stream on the device API: [frames, C] float32 rows in, Process (one call or `chunk`-frame
    calls) + Flush out, as a float32 numpy array."""
    ch = x.shape[1]
    r = gar.New(gar.Config(ir, orr, ch, preset, ComputeDtype=gar.F32))
    xd = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()
    parts = []
    step = chunk or x.shape[0]
    for s in range(0, x.shape[0], step):
        parts.append(r.process_device(xd[s:s + step]).clone())
    parts.append(r.flush_device().clone())
    torch.cuda.synchronize()
    return torch.cat(parts).cpu().numpy()


def _both(gar, torch, x, ir, orr, preset, chunk=None):
    out = {}
    for w in ("1", "0"):
        os.environ["GAR_HXT_WIDE"] = w
        try:
            out[w] = _device_run(gar, torch, x, ir, orr, preset, chunk)
        finally:
            os.environ.pop("GAR_HXT_WIDE", None)
    return out["1"], out["0"]


def _same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("ch,ir,orr,preset", [(32, 44100, 48000, 3), (64, 44100, 48000, 3), (96, 22050, 48000, 3),
                                              (64, 88200, 44100, 3)])
def test_wide_blocks_bit_identical_and_vs_oracle(gar, O, cuda, ch, ir, orr, preset):
    """Long one-shot streams (big launches: hxt_kernel) of 32 / 64 / 96 channels, with loud runs in two
    channels of different 32-channel blocks: 32-channel blocks == 16-channel blocks bit for bit, one-shot
    == 7000-frame calls bit for bit, and within the float32 bar of the oracle."""
    torch = cuda
    frames = int(2.0 * ir)
    x = signal(frames, ch, ir, seed=ch).astype(np.float32).astype(np.float64)
    x[5000:5040, 1] *= 1e4       # loud: staged as zero, the outputs recomputed exactly (tile 0)
    x[20011, ch - 3] = 40.0      # loud spike in the last tile
    wide, narrow = _both(gar, torch, x, ir, orr, preset)
    assert _same_bits(wide, narrow)
    chunked = _both(gar, torch, x, ir, orr, preset, chunk=7000)[0]
    assert _same_bits(wide, chunked)
    want = oracle_new(O, ir, orr, x, O.P_HIGH)
    for c in range(ch):
        w = np.asarray(want[c])
        assert wide.shape[0] == len(w)
        assert rms(wide[:, c], w) <= F32_RMS_TOL * max(1.0, float(np.abs(x[:, c]).max())), c


@pytest.mark.parametrize("ch", [32, 64])
def test_wide_blocks_history_seam_big_calls(gar, cuda, ch):
    """Calls large enough for hxt_kernel after the first one (44.1k -> 48k, 2.5 s in calls of 0.9 s + a
    ragged tail): each later call's first windows cross the history seam, which 32-channel blocks gather
    through hxtGatherLoad over eight quads -- the bits equal the one-shot stream's and the 16-channel blocks'."""
    torch = cuda
    ir, orr = 44100, 48000
    x = signal(int(2.5 * ir), ch, ir, seed=100 + ch).astype(np.float32).astype(np.float64)
    x[int(1.2 * ir), ch // 2] = 25.0  # a loud sample right after the second call's seam
    one = _device_run(gar, torch, x, ir, orr, 3)
    wide, narrow = _both(gar, torch, x, ir, orr, 3, chunk=int(0.9 * ir) + 17)
    assert _same_bits(wide, narrow)
    assert _same_bits(wide, one)


@pytest.mark.parametrize("ch,seconds", [(32, 0.3), (160, 0.5), (224, 0.4), (96, 1.1)])
def test_wide_blocks_odd_geometries(gar, cuda, ch, seconds):
    """Channel counts whose block count is not a multiple of 8 (160, 224: the chunk-major slot order
    is off) and streams short enough that few periods fall to each chunk (0.3 s of 32 channels: the
    group-size fallback to 16-channel blocks): the bits equal the 16-channel blocks' either way."""
    torch = cuda
    ir, orr = 44100, 48000
    x = signal(int(seconds * ir), ch, ir, seed=ch + 1).astype(np.float32).astype(np.float64)
    wide, narrow = _both(gar, torch, x, ir, orr, 3)
    assert _same_bits(wide, narrow)


def test_wide_blocks_nonfinite_input(gar, O, cuda):
    """+Inf, -Inf and NaN samples in three channels of a 64-channel stream: the NaN / +Inf / -Inf class of
    every output equals the oracle's, and 32-channel blocks give the 16-channel blocks' bits."""
    torch = cuda
    ch, ir, orr = 64, 44100, 48000
    frames = 60000
    x = signal(frames, ch, ir, seed=7).astype(np.float32).astype(np.float64)
    x[11111, 0] = np.inf
    x[22222, 33] = -np.inf
    x[33333, 63] = np.nan
    wide, narrow = _both(gar, torch, x, ir, orr, 3)
    assert _same_bits(wide, narrow)
    want = oracle_new(O, ir, orr, x, O.P_HIGH)
    for c in range(ch):
        w = np.asarray(want[c])
        g = wide[:, c].astype(np.float64)
        assert np.array_equal(np.isnan(g), np.isnan(w)), c
        assert np.array_equal(np.isposinf(g), np.isposinf(w)), c
        assert np.array_equal(np.isneginf(g), np.isneginf(w)), c
        fin = np.isfinite(w)
        assert rms(g[fin], w[fin]) <= F32_RMS_TOL, c


def test_wide_blocks_are_taken(cuda):
    """The launch geometry trace (GAR_HX_TRACE) of a 64-channel f32 row stream names fmt=5 by default and
    fmt=2 with GAR_HXT_WIDE=0 (a child process: the trace switch is read once per process)."""
    code = ("import sys, torch; sys.path.insert(0, %r); import gar; "
            "r = gar.New(gar.Config(44100, 48000, 64, gar.QualityHigh, ComputeDtype=gar.F32)); "
            "x = torch.rand((88200, 64), device='cuda') - 0.5; r.process_device(x); torch.cuda.synchronize()"
            % os.path.join(ROOT, "go-audio-resampler_amd"))
    fmts = {}
    for w in ("1", "0"):
        env = dict(os.environ, GAR_HX_TRACE="1", GAR_HXT_WIDE=w)
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        fmts[w] = [ln for ln in p.stderr.splitlines() if ln.startswith("hxt:")]
    assert any("fmt=5" in ln for ln in fmts["1"]), fmts["1"]
    assert fmts["0"] and not any("fmt=5" in ln for ln in fmts["0"]), fmts["0"]
