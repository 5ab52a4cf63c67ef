"""gar -- Python mirror of go-audio-resampler's public API over the MI355X engine.

Names, argument meaning and error behaviour follow the Go package `resampler`
(/root/reference resample.go, constant.go, convenience.go) so the parity tests
read like the reference's own tests.  Every sample operation runs in
libgar.so's HIP kernels; there is no CPU fallback -- importing this module
without the built library raises immediately.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GAR_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "libgar.so")  # override: A/B builds

# resampler.QualityPreset (resample.go:104-131)
QualityQuick, QualityLow, QualityMedium, QualityHigh, QualityVeryHigh, QualityCustom = range(6)
# engine.Quality (internal/engine/filter_params.go:16-41)
(EngineQuick, EngineLow, EngineMedium, EngineHigh, EngineVeryHigh,
 Engine16Bit, Engine20Bit, Engine24Bit, Engine28Bit, Engine32Bit) = range(10)
F64, F32, F32_EXACT = 0, 1, 2

GAR_OK, INVALID_CONFIG, BUFFER_TOO_SMALL, NOT_SUPPORTED, CHANNEL_MISMATCH, DEVICE, INTERNAL, INVALID_ARGUMENT = range(8)


class ResamplerError(Exception):
    code = -1


class ErrInvalidConfig(ResamplerError):   # resample.go:158
    code = INVALID_CONFIG


class ErrBufferTooSmall(ResamplerError):  # resample.go:161
    code = BUFFER_TOO_SMALL


class ErrNotSupported(ResamplerError):    # resample.go:164
    code = NOT_SUPPORTED


class ErrChannelMismatch(ResamplerError):
    code = CHANNEL_MISMATCH


class ErrDevice(ResamplerError):
    code = DEVICE


class ErrInternal(ResamplerError):
    code = INTERNAL


_ERRS = {c.code: c for c in (ErrInvalidConfig, ErrBufferTooSmall, ErrNotSupported, ErrChannelMismatch,
                             ErrDevice, ErrInternal)}


class QualitySpec(C.Structure):
    _fields_ = [("Preset", C.c_int32), ("Precision", C.c_int32), ("PhaseResponse", C.c_double),
                ("PassbandEnd", C.c_double), ("StopbandBegin", C.c_double), ("Flags", C.c_uint32)]


class _Config(C.Structure):
    _fields_ = [("InputRate", C.c_double), ("OutputRate", C.c_double), ("Channels", C.c_int32),
                ("Quality", QualitySpec), ("MaxInputSize", C.c_int64), ("EnableSIMD", C.c_int32),
                ("EnableParallel", C.c_int32), ("ComputeDtype", C.c_int32), ("Device", C.c_int32),
                ("DryRun", C.c_int32)]


class Info(C.Structure):
    _fields_ = [("Algorithm", C.c_char * 32), ("FilterLength", C.c_int32), ("Phases", C.c_int32),
                ("Latency", C.c_int32), ("MemoryUsage", C.c_int64), ("SIMDEnabled", C.c_int32),
                ("SIMDType", C.c_char * 48)]


class EngineGeometry(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dft_factor", C.c_int32), ("dft_taps", C.c_int32),
                ("poly_phases", C.c_int32), ("poly_taps", C.c_int32), ("poly_step", C.c_int64),
                ("decim_factor", C.c_int32), ("decim_taps", C.c_int32), ("fused", C.c_int32),
                ("fir_period_out", C.c_int32), ("fir_period_in", C.c_int32), ("fir_taps_max", C.c_int32),
                ("useful_macs_per_output", C.c_double), ("mfma_macs_per_output", C.c_double)]


EXPORTED = [
    "gar_config_validate", "gar_preset_spec", "gar_new", "gar_new_batch", "gar_new_engine", "gar_new_engine_quality", "gar_new_engine_dry", "gar_free",
    "gar_estimate_output", "gar_output_size", "gar_flush_size", "gar_process_f64", "gar_process_f32",
    "gar_process_into_f64", "gar_process_into_f32", "gar_process_multi_f64", "gar_flush_f64", "gar_flush_f32",
    "gar_flush_multi_f64", "gar_process_device", "gar_flush_device", "gar_device_output_size",
    "gar_device_flush_size", "gar_reset", "gar_get_ratio", "gar_get_latency", "gar_get_info", "gar_channels",
    "gar_status_string", "gar_last_error", "gar_design_engine", "gar_design_composite", "gar_profile_enable",
    "gar_profile_read", "gar_stage_state", "gar_num_stages", "gar_stage_geometry", "gar_get_statistics",
    "gar_synchronize", "gar_profile_launch_stats", "gar_profile_kinds",
]

_lib = None


def lib():
    """Load libgar.so (raises if the HIP library was not built -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libgar.so not built ({LIB_PATH}); run __graft_entry__.build()")
    # One HIP runtime per process: libgar.so and torch both depend on the
    # soname libamdhip64.so.7, and whichever is loaded first serves both.  Load
    # torch's first (it carries its own libhsa-runtime64) so the two stay in
    # step; the standalone C ABI (cgo) simply uses the system ROCm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, d, dp = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.POINTER(C.c_double)
    sig = {
        "gar_config_validate": (i32, [C.POINTER(_Config)]),
        "gar_preset_spec": (QualitySpec, [i32]),
        "gar_new": (i32, [C.POINTER(_Config), C.POINTER(vp)]),
        "gar_new_batch": (i32, [C.POINTER(_Config), i32, C.POINTER(vp)]),
        "gar_new_engine": (i32, [d, d, i32, i32, C.POINTER(vp)]),
        "gar_new_engine_quality": (i32, [d, d, i32, i32, C.POINTER(vp)]),
        "gar_new_engine_dry": (i32, [d, d, i32, i32, C.POINTER(vp)]),
        "gar_free": (None, [vp]),
        "gar_estimate_output": (i64, [vp, i64]),
        "gar_output_size": (i64, [vp, i32, i64]),
        "gar_flush_size": (i64, [vp, i32]),
        "gar_process_f64": (i32, [vp, vp, i64, vp, i64, C.POINTER(i64)]),
        "gar_process_f32": (i32, [vp, vp, i64, vp, i64, C.POINTER(i64)]),
        "gar_process_into_f64": (i32, [vp, vp, i64, vp, i64, C.POINTER(i64)]),
        "gar_process_into_f32": (i32, [vp, vp, i64, vp, i64, C.POINTER(i64)]),
        "gar_process_multi_f64": (i32, [vp, vp, i32, i64, vp, i64, vp]),
        "gar_flush_f64": (i32, [vp, vp, i64, C.POINTER(i64)]),
        "gar_flush_f32": (i32, [vp, vp, i64, C.POINTER(i64)]),
        "gar_flush_multi_f64": (i32, [vp, vp, i32, i64, vp]),
        "gar_process_device": (i32, [vp, vp, i32, i64, i64, i64, i32, vp, i32, i64, i64, i64, C.POINTER(i64), vp]),
        "gar_flush_device": (i32, [vp, i32, vp, i32, i64, i64, i64, C.POINTER(i64), vp]),
        "gar_device_output_size": (i64, [vp, i64]),
        "gar_device_flush_size": (i64, [vp]),
        "gar_reset": (None, [vp]),
        "gar_get_ratio": (d, [vp]),
        "gar_get_latency": (i32, [vp]),
        "gar_get_info": (i32, [vp, C.POINTER(Info)]),
        "gar_channels": (i32, [vp]),
        "gar_status_string": (C.c_char_p, [i32]),
        "gar_last_error": (C.c_char_p, []),
        "gar_design_engine": (i32, [d, d, i32, C.POINTER(EngineGeometry), vp, vp, vp, vp, vp, vp]),
        "gar_design_composite": (i32, [d, d, i32, vp, vp]),
        "gar_profile_enable": (None, [vp, i32]),
        "gar_profile_read": (i32, [vp, i32, C.POINTER(d), C.POINTER(i64)]),
        "gar_stage_state": (i32, [vp, i32, C.POINTER(i32), C.POINTER(i32)]),
        "gar_num_stages": (i32, [vp]),
        "gar_stage_geometry": (i32, [vp, i32, C.POINTER(d), C.POINTER(EngineGeometry)]),
        "gar_get_statistics": (i32, [vp, i32, C.POINTER(i64), C.POINTER(i64)]),
        "gar_synchronize": (i32, [vp]),
        "gar_profile_kinds": (None, [vp, C.c_uint32]),
        "gar_profile_launch_stats": (i32, [vp, i32, C.POINTER(d), C.POINTER(d), C.POINTER(d)]),
    }
    ab = os.environ.get("GAR_LIB_PATH") is not None
    for name, (res, args) in sig.items():
        if ab and not hasattr(L, name):  # development A/B against an older build: entry points it lacks are no-ops
            setattr(L, name, lambda *a, _r=res: None if _r is None else 0)
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc):
    if rc != GAR_OK:
        msg = lib().gar_last_error().decode(errors="replace")
        raise _ERRS.get(rc, ResamplerError)(msg or lib().gar_status_string(rc).decode())


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else C.c_void_p(0)


def Config(InputRate, OutputRate, Channels=1, Quality=None, MaxInputSize=0, EnableSIMD=True,
           EnableParallel=False, ComputeDtype=F64, Device=0, DryRun=False):
    """resampler.Config (resample.go:46-73) plus engine extensions."""
    c = _Config()
    c.InputRate, c.OutputRate, c.Channels = float(InputRate), float(OutputRate), int(Channels)
    if Quality is None:
        Quality = QualitySpec(Preset=QualityHigh)
    elif isinstance(Quality, int):
        Quality = QualitySpec(Preset=Quality)
    c.Quality = Quality
    c.MaxInputSize, c.EnableSIMD, c.EnableParallel = int(MaxInputSize), int(EnableSIMD), int(EnableParallel)
    c.ComputeDtype, c.Device, c.DryRun = int(ComputeDtype), int(Device), int(bool(DryRun))
    return c


def GetPresetSpec(preset):
    return lib().gar_preset_spec(preset)


class Resampler:
    """resampler.Resampler (resample.go:14-43) + ProcessInto/EstimateOutput/FlushMulti."""

    def __init__(self, handle, f32_io=False):
        self._h = C.c_void_p(handle)
        self._f32_io = f32_io
        # bound now: at interpreter exit the module globals (lib) may already be torn down
        self._free = lib().gar_free

    def __del__(self):
        h = getattr(self, "_h", None)
        free = getattr(self, "_free", None)
        if h is not None and h.value and free is not None:
            free(h)
            self._h = None

    # -- streaming, channel 0 --
    def Process(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        n = lib().gar_output_size(self._h, 0, len(x))
        out = np.empty(max(n, 1))
        got = C.c_int64(0)
        _check(lib().gar_process_f64(self._h, _p(x), len(x), _p(out), len(out), C.byref(got)))
        return out[: got.value].copy()

    def ProcessFloat32(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = lib().gar_output_size(self._h, 0, len(x))
        out = np.empty(max(n, 1), dtype=np.float32)
        got = C.c_int64(0)
        _check(lib().gar_process_f32(self._h, _p(x), len(x), _p(out), len(out), C.byref(got)))
        return out[: got.value].copy()

    def ProcessInto(self, x, out):
        x = np.ascontiguousarray(x, dtype=np.float64)
        assert out.dtype == np.float64 and out.flags.c_contiguous
        got = C.c_int64(0)
        _check(lib().gar_process_into_f64(self._h, _p(x), len(x), _p(out), len(out), C.byref(got)))
        return got.value

    def ProcessFloat32Into(self, x, out):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous
        got = C.c_int64(0)
        _check(lib().gar_process_into_f32(self._h, _p(x), len(x), _p(out), len(out), C.byref(got)))
        return got.value

    def EstimateOutput(self, n):
        return lib().gar_estimate_output(self._h, n)

    def OutputSize(self, n, channel=0):
        return lib().gar_output_size(self._h, channel, n)

    def FlushSize(self, channel=0):
        return lib().gar_flush_size(self._h, channel)

    def ProcessMulti(self, xs):
        nch = len(xs)
        n = len(xs[0]) if nch else 0
        arrs = [np.ascontiguousarray(x, dtype=np.float64) for x in xs]
        if any(len(a) != n for a in arrs):
            raise ValueError("ProcessMulti requires equal channel lengths")
        cap = max([lib().gar_output_size(self._h, c, n) for c in range(self.Channels)] + [1]) if nch == self.Channels else 1
        outs = [np.empty(cap) for _ in range(nch)]
        inp = (C.c_void_p * max(nch, 1))(*[_p(a) for a in arrs])
        outp = (C.c_void_p * max(nch, 1))(*[_p(o) for o in outs])
        counts = np.zeros(max(nch, 1), dtype=np.int64)
        _check(lib().gar_process_multi_f64(self._h, inp, nch, n, outp, cap, _p(counts)))
        return [o[: counts[c]].copy() for c, o in enumerate(outs)]

    def Flush(self):
        n = lib().gar_flush_size(self._h, 0)
        out = np.empty(max(n, 1), dtype=np.float32 if self._f32_io else np.float64)
        got = C.c_int64(0)
        fn = lib().gar_flush_f32 if self._f32_io else lib().gar_flush_f64
        _check(fn(self._h, _p(out), len(out), C.byref(got)))
        return out[: got.value].copy()

    def FlushMulti(self):
        nch = self.Channels
        cap = max([lib().gar_flush_size(self._h, c) for c in range(nch)] + [1])
        outs = [np.empty(cap) for _ in range(nch)]
        outp = (C.c_void_p * nch)(*[_p(o) for o in outs])
        counts = np.zeros(nch, dtype=np.int64)
        _check(lib().gar_flush_multi_f64(self._h, outp, nch, cap, _p(counts)))
        return [o[: counts[c]].copy() for c, o in enumerate(outs)]

    def Reset(self):
        lib().gar_reset(self._h)

    def GetRatio(self):
        return lib().gar_get_ratio(self._h)

    def GetLatency(self):
        return lib().gar_get_latency(self._h)

    def GetStatistics(self, channel=0):
        """engine.Resampler.GetStatistics (internal/engine/resampler.go:348-353)."""
        a, b = C.c_int64(0), C.c_int64(0)
        _check(lib().gar_get_statistics(self._h, channel, C.byref(a), C.byref(b)))
        return {"samplesIn": a.value, "samplesOut": b.value}

    def GetInfo(self):
        info = Info()
        _check(lib().gar_get_info(self._h, C.byref(info)))
        return info

    def profile(self, on=True, kinds=None):
        """HIP-event timing of the FIR launches; `kinds` (iterable of kind numbers) limits it."""
        lib().gar_profile_enable(self._h, int(on))
        lib().gar_profile_kinds(self._h, 0x3F if kinds is None else sum(1 << k for k in kinds))

    def profile_read(self, kind=0):
        """(total ms, launches) of one kernel kind (0 fused FIR, 1 DFT FIR, 2 decimator FIR, 3 fused FIR
        of a flush, 4 polyphase with cubic coefficients, 5 cubic stage) since the last read."""
        ms, n = C.c_double(0), C.c_int64(0)
        _check(lib().gar_profile_read(self._h, kind, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def profile_launch_stats(self, kind=0):
        """(min, median, max) ms per launch of the launches the last profile_read(kind) summed."""
        a, b, c = C.c_double(0), C.c_double(0), C.c_double(0)
        _check(lib().gar_profile_launch_stats(self._h, kind, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def synchronize(self):
        """Wait for the handle's enqueued device work; raises ResamplerError (GAR_ERR_DEVICE) when a
        kernel reported a broken invariant (gar.h gar_synchronize)."""
        _check(lib().gar_synchronize(self._h))

    def num_stages(self):
        return lib().gar_num_stages(self._h)

    def stage_geometry(self, stage):
        """(engine ratio, EngineGeometry) of pipeline stage `stage`."""
        ratio, g = C.c_double(0), EngineGeometry()
        _check(lib().gar_stage_geometry(self._h, stage, C.byref(ratio), C.byref(g)))
        return ratio.value, g

    def stage_state(self, stage):
        """(fused_plan, fused_now) of pipeline stage `stage` (channel 0's group)."""
        a, b = C.c_int32(0), C.c_int32(0)
        _check(lib().gar_stage_state(self._h, stage, C.byref(a), C.byref(b)))
        return bool(a.value), bool(b.value)

    @property
    def Channels(self):
        return lib().gar_channels(self._h)

    # -- device-resident (torch tensors on cuda) --
    def process_device(self, x, out=None, stream=None, pcm_bits=None):
        """x: [frames, channels] device tensor (float32/float64, or integer PCM: int16 = PCM16,
        int32 = PCM24/PCM32 per pcm_bits, default 32), any strides.  Returns out[:n] (out
        allocated with x's dtype if None).  Integer PCM follows cmd/resample-wav/main.go:444-543
        (input i * (1/maxVal), output int(clamp(y, -1, 1) * maxVal)).
        x.shape[1] (and out.shape[1]) must equal Channels (ErrChannelMismatch)."""
        import torch
        assert x.is_cuda and x.dim() == 2
        if x.shape[1] != self.Channels or (out is not None and out.shape[1] != self.Channels):
            raise ErrChannelMismatch(f"expected {self.Channels} channels, got {x.shape[1]}"
                                     + ("" if out is None else f" (out {out.shape[1]})"))
        frames = x.shape[0]
        n = lib().gar_device_output_size(self._h, frames)
        if n < 0:
            raise ErrNotSupported("channels not in lockstep")
        if out is None:
            out = torch.empty((max(n, 1), x.shape[1]), dtype=x.dtype, device=x.device)
        got = C.c_int64(0)
        dt = _io_type(x.dtype, pcm_bits)
        odt = _io_type(out.dtype, pcm_bits)
        st = C.c_void_p(stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream)
        _check(lib().gar_process_device(self._h, C.c_void_p(x.data_ptr()), dt, x.stride(0), x.stride(1), frames,
                                        x.shape[1], C.c_void_p(out.data_ptr()), odt, out.stride(0), out.stride(1),
                                        out.shape[0], C.byref(got), st))
        return out[: got.value]

    def flush_device(self, out=None, dtype=None, stream=None, pcm_bits=None):
        import torch
        if out is not None and out.shape[1] != self.Channels:
            raise ErrChannelMismatch(f"expected {self.Channels} channels, got {out.shape[1]}")
        n = lib().gar_device_flush_size(self._h)
        if n < 0:
            raise ErrNotSupported("channels not in lockstep")
        if out is None:
            out = torch.empty((max(n, 1), self.Channels), dtype=dtype or torch.float32, device="cuda")
        got = C.c_int64(0)
        odt = _io_type(out.dtype, pcm_bits)
        st = C.c_void_p(stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream)
        _check(lib().gar_flush_device(self._h, out.shape[1], C.c_void_p(out.data_ptr()), odt, out.stride(0),
                                      out.stride(1), out.shape[0], C.byref(got), st))
        return out[: got.value]


PCM16, PCM24, PCM32 = 16, 24, 32


def _io_type(dtype, pcm_bits=None):
    """Device sample type code of a torch dtype (gar.h GAR_F32/GAR_F64/GAR_PCM*)."""
    import torch
    if dtype == torch.float64:
        return F64
    if dtype == torch.float32:
        return F32
    if dtype == torch.int16:
        return PCM16
    if dtype == torch.int32:
        bits = pcm_bits or PCM32
        if bits not in (PCM24, PCM32):
            raise ValueError("int32 PCM holds 24- or 32-bit samples")
        return bits
    raise TypeError(f"unsupported sample dtype {dtype}")


def New(config):
    """resampler.New (resample.go:272-292)."""
    if config is None:
        raise ErrInvalidConfig("config is nil")
    h = C.c_void_p(0)
    _check(lib().gar_new(C.byref(config), C.byref(h)))
    return Resampler(h.value)


def NewBatch(config, n_streams):
    """n_streams independent New(config) resamplers as one lockstep GPU batch."""
    h = C.c_void_p(0)
    _check(lib().gar_new_batch(C.byref(config), int(n_streams), C.byref(h)))
    return Resampler(h.value)


def NewEngine(inputRate, outputRate, quality):
    """resampler.NewEngine (convenience.go:125-135), float64."""
    h = C.c_void_p(0)
    _check(lib().gar_new_engine(float(inputRate), float(outputRate), quality, F64, C.byref(h)))
    return Resampler(h.value)


def NewEngineFloat32(inputRate, outputRate, quality):
    """resampler.NewEngineFloat32 (convenience.go:329-336)."""
    h = C.c_void_p(0)
    _check(lib().gar_new_engine(float(inputRate), float(outputRate), quality, F32, C.byref(h)))
    return Resampler(h.value, f32_io=True)


def EngineNewResampler(inputRate, outputRate, quality, dtype=F64):
    """engine.NewResampler[F](inputRate, outputRate, quality) with an engine.Quality
    (internal/engine/resampler.go:51-179; the seam cmd/resample-wav/helpers.go:77-97
    drives).  dtype F64 = Resampler[float64]; F32 / F32_EXACT = Resampler[float32]."""
    h = C.c_void_p(0)
    _check(lib().gar_new_engine_quality(float(inputRate), float(outputRate), int(quality), int(dtype), C.byref(h)))
    return Resampler(h.value, f32_io=dtype != F64)


def NewEngineDry(inputRate, outputRate, quality, dtype=F64):
    """Host-only NewEngine: exact stream lengths, no GPU work (CPU tests)."""
    h = C.c_void_p(0)
    _check(lib().gar_new_engine_dry(float(inputRate), float(outputRate), quality, dtype, C.byref(h)))
    return Resampler(h.value, f32_io=dtype == F32)


def ResampleMono(x, inputRate, outputRate, quality):
    """resampler.ResampleMono (convenience.go:204-229): Process + Flush."""
    r = NewEngine(inputRate, outputRate, quality)
    return np.concatenate([r.Process(x), r.Flush()])


def ResampleMonoFloat32(x, inputRate, outputRate, quality):
    r = NewEngineFloat32(inputRate, outputRate, quality)
    return np.concatenate([r.ProcessFloat32(x), r.Flush()])


def ResampleStereo(left, right, inputRate, outputRate, quality):
    """resampler.ResampleStereo (convenience.go:233-257): one engine reused with Reset."""
    r = NewEngine(inputRate, outputRate, quality)
    lo = np.concatenate([r.Process(left), r.Flush()])
    r.Reset()
    ro = np.concatenate([r.Process(right), r.Flush()])
    return lo, ro


def design_engine(in_rate, out_rate, engine_quality):
    """Host-only engine design introspection (no GPU): geometry + coefficient banks."""
    g = EngineGeometry()
    _check(lib().gar_design_engine(in_rate, out_rate, engine_quality, C.byref(g), None, None, None, None, None, None))
    dft = np.zeros(max(g.dft_factor * g.dft_taps, 1))
    n = g.poly_phases * g.poly_taps
    pa, pb, pc, pd = (np.zeros(max(n, 1)) for _ in range(4))
    dec = np.zeros(max(g.decim_taps, 1))
    _check(lib().gar_design_engine(in_rate, out_rate, engine_quality, C.byref(g), _p(dft), _p(pa), _p(pb), _p(pc),
                                   _p(pd), _p(dec)))
    return g, {"dft": dft[: g.dft_factor * g.dft_taps], "a": pa[:n], "b": pb[:n], "c": pc[:n], "d": pd[:n],
               "decim": dec[: g.decim_taps]}


def design_composite(in_rate, out_rate, engine_quality):
    g, _ = design_engine(in_rate, out_rate, engine_quality)
    if not g.fused:
        raise ErrNotSupported("engine has no fused composite FIR")
    rows = np.zeros((g.fir_period_out, g.fir_taps_max))
    offs = np.zeros(g.fir_period_out, dtype=np.int64)
    _check(lib().gar_design_composite(in_rate, out_rate, engine_quality, _p(rows), _p(offs)))
    return rows, offs, g
