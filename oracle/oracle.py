"""ctypes wrapper over oracle/_build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It is the parity checker (a CPU restatement of
tphakala/go-audio-resampler, see gar_oracle.c) and never part of the product.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

# engine.Quality enum (internal/engine/filter_params.go:16-41)
QUICK, LOW, MEDIUM, HIGH, VERYHIGH, Q16, Q20, Q24, Q28, Q32 = range(10)
# resampler.QualityPreset (resample.go:104-131)
P_QUICK, P_LOW, P_MEDIUM, P_HIGH, P_VERYHIGH, P_CUSTOM = range(6)


class EngineInfo(C.Structure):
    _fields_ = [("kind", C.c_int), ("dft_factor", C.c_int), ("dft_taps_per_phase", C.c_int),
                ("dft_is_halfband", C.c_int), ("poly_phases", C.c_int), ("poly_taps_per_phase", C.c_int),
                ("poly_step", C.c_int64), ("decim_factor", C.c_int), ("decim_taps", C.c_int)]


class PolyParams(C.Structure):
    _fields_ = [("num_phases", C.c_int), ("ratio", C.c_double), ("total_io_ratio", C.c_double),
                ("has_pre", C.c_int), ("attenuation", C.c_double), ("is_upsampling", C.c_int),
                ("mult", C.c_double), ("fn", C.c_double), ("fp1", C.c_double), ("fs1", C.c_double),
                ("fp_raw", C.c_double), ("fs_raw", C.c_double), ("fp", C.c_double), ("fs", C.c_double),
                ("tr_bw", C.c_double), ("fc", C.c_double), ("total_taps", C.c_int), ("taps_per_phase", C.c_int)]


def build():
    """Compile the oracle (gcc) into oracle/_build/."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        d, i, i64, vp, dp = C.c_double, C.c_int, C.c_int64, C.c_void_p, C.POINTER(C.c_double)
        sig = {
            "o_bessel_i0": (d, [d]), "o_kaiser_beta": (d, [d]), "o_estimate_filter_length": (i, [d, d]),
            "o_kaiser_window": (None, [i, d, vp]), "o_design_lowpass": (i, [i, d, d, d, vp]),
            "o_design_lowpass_auto": (i, [d, d, d, d, vp, C.POINTER(i)]),
            "o_quality_to_attenuation": (d, [i]), "o_quality_to_passband_end": (d, [i]),
            "o_find_rational_approx": (None, [d, C.POINTER(i), C.POINTER(i)]),
            "o_lsx_inv_f_resp": (d, [d, d]),
            "o_compute_poly_params": (None, [i, d, d, i, d, d, C.POINTER(PolyParams)]),
            "o_design_polyphase_filter": (i, [i, d, d, i, i, vp]), "o_is_integer_ratio": (i, [d]),
            "o_engine_new": (vp, [d, d, i, i]), "o_engine_free": (None, [vp]),
            "o_engine_process": (i64, [vp, vp, i64, vp, i64]), "o_engine_flush": (i64, [vp, vp, i64]),
            "o_engine_reset": (None, [vp]), "o_engine_ratio": (d, [vp]), "o_engine_stats": (None, [vp, vp]),
            "o_engine_get_info": (None, [vp, C.POINTER(EngineInfo)]),
            "o_engine_get_coeffs": (i64, [vp, i, i, vp]),
            "o_precision_to_engine_quality": (i, [i]), "o_preset_to_engine_quality": (i, [i]),
            "o_build_pipeline": (i, [d, i, vp, vp, i]),
            "o_new": (vp, [d, d, i, i, i]), "o_new_free": (None, [vp]),
            "o_new_process": (i64, [vp, i, vp, i64, vp, i64]), "o_new_flush": (i64, [vp, i, vp, i64]),
            "o_new_reset": (None, [vp]), "o_new_latency": (i, [vp]), "o_new_estimate_output": (i64, [vp, i64]),
            "o_new_ratio": (d, [vp]), "o_new_nstages": (i, [vp, vp, vp]),
            "o_new_stage_info": (None, [vp, i, C.POINTER(EngineInfo)]),
            "o_dot": (d, [vp, vp, i64]), "o_convolve_valid": (None, [vp, vp, i64, vp, i64]),
            "o_cubic_interp_dot": (d, [vp, vp, vp, vp, vp, d, i64]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


# ---- design-level helpers -------------------------------------------------
def bessel_i0(x):
    return lib().o_bessel_i0(float(x))


def kaiser_window(n, beta):
    w = np.zeros(n)
    lib().o_kaiser_window(n, beta, _ptr(w))
    return w


def design_lowpass(ntaps, fc, att, gain=1.0):
    out = np.zeros(max(ntaps, 1))
    rc = lib().o_design_lowpass(ntaps, fc, att, gain, _ptr(out))
    if rc != 0:
        raise ValueError("invalid filter params")
    return out


def design_lowpass_auto(fc, tbw, att, gain=1.0):
    out = np.zeros(8191)
    n = C.c_int(0)
    rc = lib().o_design_lowpass_auto(fc, tbw, att, gain, _ptr(out), C.byref(n))
    if rc != 0:
        raise ValueError("invalid filter params")
    return out[: n.value].copy()


def dot(a, b):
    a, b = np.ascontiguousarray(a, float), np.ascontiguousarray(b, float)
    return lib().o_dot(_ptr(a), _ptr(b), len(a))


def convolve_valid(sig, ker):
    sig, ker = np.ascontiguousarray(sig, float), np.ascontiguousarray(ker, float)
    dst = np.zeros(max(len(sig) - len(ker) + 1, 0))
    lib().o_convolve_valid(_ptr(dst), _ptr(sig), len(sig), _ptr(ker), len(ker))
    return dst


def cubic_interp_dot(h, a, b, c, d, x):
    arrs = [np.ascontiguousarray(v, float) for v in (h, a, b, c, d)]
    return lib().o_cubic_interp_dot(*[_ptr(v) for v in arrs], float(x), len(arrs[0]))


def find_rational_approx(ratio):
    L, s = C.c_int(0), C.c_int(0)
    lib().o_find_rational_approx(ratio, C.byref(L), C.byref(s))
    return L.value, s.value


def compute_poly_params(L, ratio, tio, has_pre, att, pbe):
    p = PolyParams()
    lib().o_compute_poly_params(L, ratio, tio, int(has_pre), att, pbe, C.byref(p))
    return p


def build_pipeline(ratio, precision):
    t = np.zeros(32, dtype=np.int32)
    r = np.zeros(32)
    n = lib().o_build_pipeline(ratio, precision, _ptr(t), _ptr(r), 32)
    if n < 0:
        raise ValueError("invalid ratio")
    return list(t[:n]), list(r[:n])


# ---- engine (internal/engine.Resampler[F]) --------------------------------
class Engine:
    """engine.NewResampler[F](inRate, outRate, quality) restated."""

    def __init__(self, in_rate, out_rate, quality, f32=False):
        self.f32 = f32
        self.dt = np.float32 if f32 else np.float64
        self.h = lib().o_engine_new(in_rate, out_rate, quality, int(f32))
        if not self.h:
            raise ValueError("engine.NewResampler failed")

    def __del__(self):
        if getattr(self, "h", None):
            lib().o_engine_free(self.h)
            self.h = None

    def _cap(self, n):
        return int(n * max(self.ratio, 1.0)) + 65536

    def process(self, x):
        x = np.ascontiguousarray(x, dtype=self.dt)
        cap = self._cap(len(x))
        out = np.empty(cap, dtype=self.dt)
        m = lib().o_engine_process(self.h, _ptr(x), len(x), _ptr(out), cap)
        assert m >= 0
        return out[:m].copy()

    def flush(self):
        cap = 1 << 20
        out = np.empty(cap, dtype=self.dt)
        m = lib().o_engine_flush(self.h, _ptr(out), cap)
        assert m >= 0
        return out[:m].copy()

    def reset(self):
        lib().o_engine_reset(self.h)

    def statistics(self):
        """GetStatistics (resampler.go:348-353)."""
        v = np.zeros(2, dtype=np.int64)
        lib().o_engine_stats(self.h, _ptr(v))
        return {"samplesIn": int(v[0]), "samplesOut": int(v[1])}

    @property
    def ratio(self):
        return lib().o_engine_ratio(self.h)

    def info(self):
        inf = EngineInfo()
        lib().o_engine_get_info(self.h, C.byref(inf))
        return inf

    def coeffs(self, which, sel=0):
        out = np.zeros(8191 * 256)
        n = lib().o_engine_get_coeffs(self.h, which, sel, _ptr(out))
        return out[:n].copy()


def resample_mono(x, in_rate, out_rate, preset):
    """resampler.ResampleMono (convenience.go:204-229): NewEngine + Process + Flush."""
    q = lib().o_preset_to_engine_quality(preset)
    e = Engine(in_rate, out_rate, q)
    return np.concatenate([e.process(x), e.flush()])


# ---- New(config) path (constantRateResampler) ------------------------------
class NewResampler:
    """resampler.New(&Config{...}) restated (constant.go)."""

    def __init__(self, in_rate, out_rate, channels=1, preset=P_HIGH, precision=0):
        self.h = lib().o_new(in_rate, out_rate, channels, preset, precision)
        if not self.h:
            raise ValueError("ErrInvalidConfig")
        self.channels = channels

    def __del__(self):
        if getattr(self, "h", None):
            lib().o_new_free(self.h)
            self.h = None

    @property
    def ratio(self):
        return lib().o_new_ratio(self.h)

    def estimate_output(self, n):
        return lib().o_new_estimate_output(self.h, n)

    def process(self, x, ch=0):
        x = np.ascontiguousarray(x, dtype=np.float64)
        cap = int(len(x) * max(self.ratio, 1.0)) + 65536
        out = np.empty(cap)
        m = lib().o_new_process(self.h, ch, _ptr(x), len(x), _ptr(out), cap)
        assert m >= 0
        return out[:m].copy()

    def process_multi(self, xs):
        return [self.process(x, c) for c, x in enumerate(xs)]

    def flush(self, ch=0):
        cap = 1 << 21
        out = np.empty(cap)
        m = lib().o_new_flush(self.h, ch, _ptr(out), cap)
        assert m >= 0
        return out[:m].copy()

    def flush_multi(self):
        return [self.flush(c) for c in range(self.channels)]

    def reset(self):
        lib().o_new_reset(self.h)

    def latency(self):
        return lib().o_new_latency(self.h)

    def stages(self):
        t = np.zeros(16, dtype=np.int32)
        r = np.zeros(16)
        n = lib().o_new_nstages(self.h, _ptr(t), _ptr(r))
        return list(t[:n]), list(r[:n])

    def stage_info(self, j):
        inf = EngineInfo()
        lib().o_new_stage_info(self.h, j, C.byref(inf))
        return inf
