"""GPU: input/output memory layouts of the device entry points (gar_process_device takes any
frame/channel strides).  Channel-major (planar) and padded-row inputs, planar outputs, and a
sliced (offset, non-16-B-aligned) input must give the same bits as the interleaved layout the
fast loads are written for (planar inputs go through the gathered loads with 64-bit
addressing, never through 32-bit buffer offsets)."""
import numpy as np
import pytest

from helpers import signal

pytestmark = pytest.mark.gpu


def run(gar, torch, xd, ch, out=None, compute=None, bits=None):
    r = gar.New(gar.Config(44100, 48000, ch, gar.QualityHigh, ComputeDtype=compute or gar.F32))
    a = r.process_device(xd, pcm_bits=bits).clone()
    b = r.flush_device(dtype=xd.dtype, pcm_bits=bits).clone()
    torch.cuda.synchronize()
    return torch.cat([a, b]).cpu().numpy()


@pytest.mark.parametrize("ch", [2, 16])
def test_planar_input_equals_interleaved(gar, cuda, ch):
    torch = cuda
    n = 44100 + 321
    x = signal(n, ch, seed=5).astype(np.float32)
    inter = torch.from_numpy(x).cuda()                        # [frames][ch]
    planar = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()  # strides (1, frames)
    assert planar.stride() == (1, n)
    want = run(gar, torch, inter, ch)
    got = run(gar, torch, planar, ch)
    assert np.array_equal(got, want)


def test_padded_rows_and_offset_input(gar, cuda):
    """Rows padded to 3 floats (frame stride 3) and an input view starting one element into its
    buffer (4-B aligned only): the gathered path, same bits."""
    torch = cuda
    n, ch = 30000, 2
    x = signal(n, ch, seed=9).astype(np.float32)
    want = run(gar, torch, torch.from_numpy(x).cuda(), ch)
    pad = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
    pad[:, :2] = torch.from_numpy(x).cuda()
    assert np.array_equal(run(gar, torch, pad[:, :2], ch), want)
    flat = torch.zeros(1 + n * ch, dtype=torch.float32, device="cuda")
    flat[1:] = torch.from_numpy(x.reshape(-1)).cuda()
    assert np.array_equal(run(gar, torch, flat[1:].view(n, ch), ch), want)


def test_planar_pcm16(gar, cuda):
    torch = cuda
    n, ch = 44100, 2
    pcm = np.round(signal(n, ch, seed=2) * 32000).astype(np.int16)
    want = run(gar, torch, torch.from_numpy(pcm).cuda(), ch, bits=16)
    planar = torch.from_numpy(np.ascontiguousarray(pcm.T)).cuda().t()
    assert np.array_equal(run(gar, torch, planar, ch, bits=16), want)


def run_chunked(gar, torch, views, ch, chunk):
    """Feed the frames of `views(s, e)` (a device view of frames [s, e)) in `chunk`-frame calls."""
    r = gar.New(gar.Config(44100, 48000, ch, gar.QualityHigh, ComputeDtype=gar.F32))
    n = views.n
    parts = []
    for s in range(0, n, chunk):
        parts.append(r.process_device(views(s, min(n, s + chunk))).clone().float())
    parts.append(r.flush_device(dtype=torch.float32).clone())
    torch.cuda.synchronize()
    return torch.cat(parts).cpu().numpy()


@pytest.mark.parametrize("chunk", [4096, 999])
@pytest.mark.parametrize("layout", ["interleaved", "planar", "padded", "offset", "f64", "mono"])
def test_small_calls_every_layout_equal_one_shot(gar, cuda, layout, chunk):
    """Short calls (small launches: hxq_kernel's STEREO / ROW16 / per-column loads, history seam
    from the history buffer, loud samples fixed up per row-block group) in every input layout give
    the bits of one interleaved one-shot call."""
    torch = cuda
    ch = 1 if layout == "mono" else 2
    n = 30000
    x = signal(n, ch, seed=31).astype(np.float32)
    x[7000, 0] = 300.0      # loud: exact recompute inside a small launch
    x[12345, ch - 1] = -40.0
    want = run(gar, torch, torch.from_numpy(x).cuda(), ch)
    xd = torch.from_numpy(x).cuda()
    if layout == "planar":
        base = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
    elif layout == "padded":
        base = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
        base[:, :ch] = xd
        base = base[:, :ch]
    elif layout == "offset":
        flat = torch.zeros(1 + n * ch, dtype=torch.float32, device="cuda")
        flat[1:] = xd.reshape(-1)
        base = flat[1:].view(n, ch)
    elif layout == "f64":
        base = xd.double()
    else:
        base = xd

    class V:
        def __call__(self, s, e):
            return base[s:e]
    v = V()
    v.n = n
    got = run_chunked(gar, torch, v, ch, chunk)
    assert got.shape == want.shape
    assert np.array_equal(got, want)
