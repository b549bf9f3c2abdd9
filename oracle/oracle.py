"""ctypes wrapper around the CPU restatement (oracle) of the liquid-dsp algorithms.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product (python-liquiddsp_amd/) never
imports this module.  See liquid_restate.c for citations and the
"parity unpinned" statement.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libliquid_restate.so")

# filter / band / format codes (liquid_iirdes_* enums, iirfilter.hpp:5-20)
FILTER_TYPES = {"butter": 0, "cheby1": 1, "cheby2": 2, "ellip": 3, "bessel": 4}
BAND_TYPES = {"lowpass": 0, "highpass": 1, "bandpass": 2, "bandstop": 3}
FMT_TF, FMT_SOS = 0, 1


def build() -> str:
    """Compile the restatement with its Makefile (gcc) into oracle/_build/."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    if not os.path.exists(_LIB_PATH):
        build()
    lib = C.CDLL(_LIB_PATH)
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
    vp, u, i, f, sz = C.c_void_p, C.c_uint, C.c_int, C.c_float, C.c_size_t
    u32 = C.c_uint32
    sig = {
        "ora_kaiser_beta_As": (f, [f]),
        "ora_kaiser": (f, [u, u, f]),
        "ora_besseli0f": (f, [f]),
        "ora_lngammaf": (f, [f]),
        "ora_sincf": (f, [f]),
        "ora_firdes_kaiser": (i, [u, f, f, f, f32p]),
        "ora_firdes_notch": (i, [u, f, f, f32p]),
        "ora_math_eval": (None, [i, f32p, f32p, f32p, sz]),
        "ora_firfilt_create": (vp, [f32p, u, i]),
        "ora_firfilt_create_kaiser": (vp, [u, f, f, f, i]),
        "ora_firfilt_create_dc_blocker": (vp, [u, f, i]),
        "ora_firfilt_destroy": (None, [vp]),
        "ora_firfilt_reset": (None, [vp]),
        "ora_firfilt_set_scale": (None, [vp, f]),
        "ora_firfilt_get_scale": (f, [vp]),
        "ora_firfilt_get_length": (u, [vp]),
        "ora_firfilt_get_taps": (None, [vp, f32p]),
        "ora_firfilt_freqresponse": (None, [vp, f, C.POINTER(f), C.POINTER(f)]),
        "ora_firfilt_execute_block": (None, [vp, f32p, sz, f32p]),
        "ora_resamp_create": (vp, [f, u, f, f, u, i]),
        "ora_resamp_create_default": (vp, [f, i]),
        "ora_freqdem_create": (vp, [f]),
        "ora_freqdem_destroy": (None, [vp]),
        "ora_freqdem_reset": (None, [vp]),
        "ora_freqdem_demodulate_block": (None, [vp, f32p, sz, f32p]),
        "ora_bcastam_create": (vp, [u, i]),
        "ora_bcastam_destroy": (None, [vp]),
        "ora_bcastam_reset": (None, [vp]),
        "ora_bcastam_demodulate_block": (None, [vp, f32p, sz, f32p, f32p, i]),
        "ora_fmstereo_create": (vp, [f, f]),
        "ora_fmstereo_destroy": (None, [vp]),
        "ora_fmstereo_reset": (None, [vp]),
        "ora_fmstereo_execute": (sz, [vp, f32p, sz, f32p, vp]),
        "ora_fmstereo_get_state": (None, [vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(f)]),
        "ora_fmstereo_set_state": (None, [vp, u32, u32, f]),
        "ora_resamp_destroy": (None, [vp]),
        "ora_resamp_reset": (None, [vp]),
        "ora_resamp_set_rate": (i, [vp, f]),
        "ora_resamp_get_rate": (f, [vp]),
        "ora_resamp_get_step": (u32, [vp]),
        "ora_resamp_get_phase": (u32, [vp]),
        "ora_resamp_get_npfb": (u, [vp]),
        "ora_resamp_get_taps": (u, [vp, vp]),
        "ora_resamp_execute_block": (sz, [vp, f32p, sz, f32p]),
        "ora_nco_create": (vp, [i]),
        "ora_nco_destroy": (None, [vp]),
        "ora_nco_reset": (None, [vp]),
        "ora_nco_constrain": (u32, [f]),
        "ora_nco_set_frequency": (None, [vp, f]),
        "ora_nco_adjust_frequency": (None, [vp, f]),
        "ora_nco_get_frequency": (f, [vp]),
        "ora_nco_set_phase": (None, [vp, f]),
        "ora_nco_adjust_phase": (None, [vp, f]),
        "ora_nco_get_phase": (f, [vp]),
        "ora_nco_pll_set_bandwidth": (None, [vp, f]),
        "ora_nco_pll_step": (None, [vp, f]),
        "ora_nco_get_state": (None, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "ora_nco_set_state": (None, [vp, u32, u32]),
        "ora_nco_get_table": (None, [vp, f32p]),
        "ora_nco_mix_block_up": (None, [vp, f32p, f32p, sz]),
        "ora_nco_mix_block_down": (None, [vp, f32p, f32p, sz]),
        "ora_iirdes": (i, [i, i, i, u, f, f, f, f, f32p, f32p]),
        "ora_iirdes_dzpk": (None, [i, i, u, f, f, f, f, f32p, f32p, f32p]),
        "ora_iirfilt_create_sos": (vp, [f32p, f32p, u, i]),
        "ora_iirfilt_create_tf": (vp, [f32p, u, f32p, u, i]),
        "ora_iirfilt_create_prototype": (vp, [i, i, i, u, f, f, f, f, i]),
        "ora_iirfilt_destroy": (None, [vp]),
        "ora_iirfilt_reset": (None, [vp]),
        "ora_iirfilt_get_nsos": (u, [vp]),
        "ora_iirfilt_get_sos": (None, [vp, f32p, f32p]),
        "ora_iirfilt_freqresponse": (None, [vp, f, C.POINTER(f), C.POINTER(f)]),
        "ora_iirfilt_execute_block": (None, [vp, f32p, sz, f32p]),
        "ora_iirfilt_execute_block_f64": (None, [vp, f32p, sz, f32p]),
        "ora_agc_create": (vp, []),
        "ora_agc_destroy": (None, [vp]),
        "ora_agc_reset": (None, [vp]),
        "ora_agc_set_bandwidth": (None, [vp, f]),
        "ora_agc_get_bandwidth": (f, [vp]),
        "ora_agc_lock": (None, [vp, i]),
        "ora_agc_squelch_enable": (None, [vp, i]),
        "ora_agc_squelch_set_threshold": (None, [vp, f]),
        "ora_agc_squelch_get_threshold": (f, [vp]),
        "ora_agc_squelch_set_timeout": (None, [vp, u]),
        "ora_agc_squelch_get_status": (i, [vp]),
        "ora_agc_get_gain": (f, [vp]),
        "ora_agc_set_gain": (None, [vp, f]),
        "ora_agc_get_scale": (f, [vp]),
        "ora_agc_set_scale": (None, [vp, f]),
        "ora_agc_get_signal_level": (f, [vp]),
        "ora_agc_set_signal_level": (None, [vp, f]),
        "ora_agc_get_rssi": (f, [vp]),
        "ora_agc_set_rssi": (None, [vp, f]),
        "ora_agc_get_state": (None, [vp, C.POINTER(f), C.POINTER(f), C.POINTER(i), C.POINTER(u)]),
        "ora_agc_set_state": (None, [vp, f, f, i, u]),
        "ora_agc_execute_wrapper": (None, [vp, f32p, sz, f32p, vp]),
        "ora_ampmodem_create": (vp, [f, i, i]),
        "ora_ampmodem_destroy": (None, [vp]),
        "ora_ampmodem_reset": (None, [vp]),
        "ora_ampmodem_demodulate_block": (None, [vp, f32p, sz, f32p]),
        "ora_ampmodem_get_pll_state": (None, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "ora_ampmodem_get_taps": (None, [vp, f32p, f32p]),
        "ora_ampmodem_get_hilbert_taps": (None, [vp, f32p]),
        "ora_firhilb_create": (vp, [u, f]),
        "ora_firhilb_destroy": (None, [vp]),
        "ora_firhilb_reset": (None, [vp]),
        "ora_firhilb_get_taps": (None, [vp, f32p]),
        "ora_firhilb_c2r_block": (None, [vp, f32p, sz, f32p, f32p]),
        "ora_amradio_create": (vp, [f, f, f, i]),
        "ora_amradio_destroy": (None, [vp]),
        "ora_amradio_max_out": (sz, [vp, sz]),
        "ora_amradio_execute": (sz, [vp, f32p, sz, f32p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    del u8p
    return lib


_lib = None

# Build variants of the restatement (oracle/Makefile): which libm the feedback
# loops call and which order liquid's dotprod sums in are platform choices of a
# liquid-dsp build, so "liquid's output" is a family; variants.py records how
# far apart its members are.  "default" is the variant the GPU exact mode
# reproduces bit for bit.
VARIANTS = {
    "default": "libliquid_restate.so",
    "libm": "libliquid_restate_libm.so",
    "simd": "libliquid_restate_simd.so",
    "libm_simd": "libliquid_restate_libm_simd.so",
    "asan": "libliquid_restate_asan.so",          # make -C oracle asan (tests/test_sanitizers.py)
}
_variant_mods = {}


def variant(name: str):
    """This module bound to another build variant of the restatement (a separate
    module instance with its own library; same classes and functions)."""
    if name == "default" and not globals().get("_VARIANT"):
        return sys.modules[__name__]
    if name not in _variant_mods:
        import importlib.util
        spec = importlib.util.spec_from_file_location(f"oracle_variant_{name}", os.path.abspath(__file__))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod._LIB_PATH = os.path.join(_HERE, "_build", VARIANTS[name])
        mod._VARIANT = name
        _variant_mods[name] = mod
    return _variant_mods[name]


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _f32(x) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=np.float32)


def _c64_as_f32(x) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=np.complex64).view(np.float32)


# ---------------------------------------------------------------- design
def firdes_kaiser(n, fc, As, mu=0.0):
    h = np.zeros(n, np.float32)
    if lib().ora_firdes_kaiser(n, fc, As, mu, h):
        raise ValueError("firdes_kaiser: invalid configuration")
    return h


def firdes_notch(m, f0, As):
    h = np.zeros(2 * m + 1, np.float32)
    if lib().ora_firdes_notch(m, f0, As, h):
        raise ValueError("firdes_notch: invalid configuration")
    return h


def math_eval(fn: str, a, b=None):
    code = {"exp": 0, "log": 1, "atan2": 2, "tanh": 3}[fn]
    a = _f32(a)
    b = _f32(b if b is not None else np.zeros_like(a))
    y = np.empty_like(a)
    lib().ora_math_eval(code, a, b, y, a.size)
    return y


# ---------------------------------------------------------------- objects
class _Handle:
    _destroy = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            getattr(_lib, self._destroy)(h)
            self._h = None


class FIRFilter(_Handle):
    """firfilt_rrrf (cplx=False) / firfilt_crcf (cplx=True)."""
    _destroy = "ora_firfilt_destroy"

    def __init__(self, h=None, cplx=False, *, kaiser=None, dc_blocker=None):
        L = lib()
        self.cplx = bool(cplx)
        if kaiser is not None:
            self._h = L.ora_firfilt_create_kaiser(*kaiser, int(cplx))
        elif dc_blocker is not None:
            self._h = L.ora_firfilt_create_dc_blocker(*dc_blocker, int(cplx))
        else:
            h = _f32(h)
            self._h = L.ora_firfilt_create(h, h.size, int(cplx))
        if not self._h:
            raise ValueError("firfilt: invalid configuration")

    @property
    def taps(self):
        n = lib().ora_firfilt_get_length(self._h)
        h = np.zeros(n, np.float32)
        lib().ora_firfilt_get_taps(self._h, h)
        return h

    @property
    def scale(self):
        return lib().ora_firfilt_get_scale(self._h)

    @scale.setter
    def scale(self, s):
        lib().ora_firfilt_set_scale(self._h, s)

    def reset(self):
        lib().ora_firfilt_reset(self._h)

    def freqresponse(self, f):
        re, im = C.c_float(), C.c_float()
        lib().ora_firfilt_freqresponse(self._h, f, C.byref(re), C.byref(im))
        return complex(re.value, im.value)

    def __call__(self, x):
        if self.cplx:
            xf = _c64_as_f32(x)
            y = np.empty(xf.size // 2, np.complex64)
            lib().ora_firfilt_execute_block(self._h, xf, xf.size // 2, y.view(np.float32))
        else:
            xf = _f32(x)
            y = np.empty(xf.size, np.float32)
            lib().ora_firfilt_execute_block(self._h, xf, xf.size, y)
        return y


class Resampler(_Handle):
    """resamp_rrrf (cplx=False) / resamp_cccf (cplx=True) / resamp_crcf
    (cplx=True, real_taps=True); default=True: resamp_*_create_default(rate)."""
    _destroy = "ora_resamp_destroy"

    def __init__(self, rate, m=20, fc=0.25, As=60.0, npfb=13, cplx=True, real_taps=False, default=False):
        self.cplx = bool(cplx)
        kind = (1 if real_taps else 2) if cplx else 0
        if default:
            self._h = lib().ora_resamp_create_default(rate, kind)
        else:
            self._h = lib().ora_resamp_create(rate, m, fc, As, npfb, kind)
        if not self._h:
            raise ValueError("resamp: invalid configuration")

    rate = property(lambda s: lib().ora_resamp_get_rate(s._h))
    step = property(lambda s: int(lib().ora_resamp_get_step(s._h)))
    phase = property(lambda s: int(lib().ora_resamp_get_phase(s._h)))
    npfb = property(lambda s: int(lib().ora_resamp_get_npfb(s._h)))

    def set_rate(self, r):
        if lib().ora_resamp_set_rate(self._h, r):
            raise ValueError("resamp: invalid rate")

    @property
    def prototype(self):
        n = lib().ora_resamp_get_taps(self._h, None)
        h = np.zeros(n, np.float32)
        lib().ora_resamp_get_taps(self._h, h.ctypes.data)
        return h

    def reset(self):
        lib().ora_resamp_reset(self._h)

    def __call__(self, x):
        n = len(x)
        cap = int(n * self.rate) + 8 + int(np.ceil(self.rate)) * 4
        if self.cplx:
            xf = _c64_as_f32(x)
            y = np.empty(cap, np.complex64)
            nw = lib().ora_resamp_execute_block(self._h, xf, n, y.view(np.float32))
        else:
            xf = _f32(x)
            y = np.empty(cap, np.float32)
            nw = lib().ora_resamp_execute_block(self._h, xf, n, y)
        assert nw <= cap
        return y[:nw].copy()


class NCO(_Handle):
    _destroy = "ora_nco_destroy"

    def __init__(self, type=0):
        self._h = lib().ora_nco_create(type)

    def reset(self):
        lib().ora_nco_reset(self._h)

    freq = property(lambda s: lib().ora_nco_get_frequency(s._h),
                    lambda s, v: lib().ora_nco_set_frequency(s._h, v))
    phase = property(lambda s: lib().ora_nco_get_phase(s._h),
                     lambda s, v: lib().ora_nco_set_phase(s._h, v))

    def adjust_frequency(self, df):
        lib().ora_nco_adjust_frequency(self._h, df)

    def adjust_phase(self, dp):
        lib().ora_nco_adjust_phase(self._h, dp)

    def pll_set_bandwidth(self, bw):
        lib().ora_nco_pll_set_bandwidth(self._h, bw)

    def pll_step(self, dphi):
        lib().ora_nco_pll_step(self._h, dphi)

    @property
    def state(self):
        t, d = C.c_uint32(), C.c_uint32()
        lib().ora_nco_get_state(self._h, C.byref(t), C.byref(d))
        return t.value, d.value

    @state.setter
    def state(self, td):
        lib().ora_nco_set_state(self._h, td[0], td[1])

    @property
    def table(self):
        t = np.zeros(1024, np.float32)
        lib().ora_nco_get_table(self._h, t)
        return t

    def mix_up(self, x):
        xf = _c64_as_f32(x)
        y = np.empty(xf.size // 2, np.complex64)
        lib().ora_nco_mix_block_up(self._h, xf, y.view(np.float32), xf.size // 2)
        return y

    def mix_down(self, x):
        xf = _c64_as_f32(x)
        y = np.empty(xf.size // 2, np.complex64)
        lib().ora_nco_mix_block_down(self._h, xf, y.view(np.float32), xf.size // 2)
        return y


def constrain(theta: float) -> int:
    return int(lib().ora_nco_constrain(theta))


def iirdes(ftype, btype, order, fc, f0=0.0, Ap=0.5, As=60.0, fmt=FMT_SOS):
    n = order * (2 if btype in ("bandpass", "bandstop") else 1)
    r = n % 2
    L = (n - r) // 2
    hl = 3 * (L + r) if fmt == FMT_SOS else n + 1
    B = np.zeros(hl, np.float32)
    A = np.zeros(hl, np.float32)
    rc = lib().ora_iirdes(FILTER_TYPES[ftype], BAND_TYPES[btype], fmt, order, fc, f0, Ap, As, B, A)
    if rc:
        raise ValueError(f"iirdes: invalid configuration ({rc})")
    if fmt == FMT_SOS:
        return B.reshape(-1, 3), A.reshape(-1, 3)
    return B, A


def iirdes_dzpk(ftype, btype, order, fc, f0=0.0, Ap=0.5, As=60.0):
    n = order * (2 if btype in ("bandpass", "bandstop") else 1)
    zd = np.zeros(2 * n, np.float32)
    pd = np.zeros(2 * n, np.float32)
    kd = np.zeros(2, np.float32)
    lib().ora_iirdes_dzpk(FILTER_TYPES[ftype], BAND_TYPES[btype], order, fc, f0, Ap, As, zd, pd, kd)
    return (zd.view(np.complex64).copy(), pd.view(np.complex64).copy(),
            complex(kd[0], kd[1]))


class IIRFilter(_Handle):
    _destroy = "ora_iirfilt_destroy"

    def __init__(self, *, sos=None, tf=None, prototype=None, cplx=True):
        L = lib()
        self.cplx = bool(cplx)
        if sos is not None:
            B, A = (_f32(v).reshape(-1) for v in sos)
            self._h = L.ora_iirfilt_create_sos(B, A, B.size // 3, int(cplx))
        elif tf is not None:
            b, a = (_f32(v) for v in tf)
            self._h = L.ora_iirfilt_create_tf(b, b.size, a, a.size, int(cplx))
        else:
            ft, bt, fmt, order, fc, f0, ap, As = prototype
            self._h = L.ora_iirfilt_create_prototype(FILTER_TYPES[ft], BAND_TYPES[bt], fmt, order,
                                                     fc, f0, ap, As, int(cplx))
        if not self._h:
            raise ValueError("iirfilt: invalid configuration")

    def sos(self):
        n = lib().ora_iirfilt_get_nsos(self._h)
        B = np.zeros(3 * n, np.float32)
        A = np.zeros(3 * n, np.float32)
        lib().ora_iirfilt_get_sos(self._h, B, A)
        return B.reshape(n, 3), A.reshape(n, 3)

    def reset(self):
        lib().ora_iirfilt_reset(self._h)

    def freqresponse(self, f):
        re, im = C.c_float(), C.c_float()
        lib().ora_iirfilt_freqresponse(self._h, f, C.byref(re), C.byref(im))
        return complex(re.value, im.value)

    def _run(self, x, fn):
        if self.cplx:
            xf = _c64_as_f32(x)
            y = np.empty(xf.size // 2, np.complex64)
            fn(self._h, xf, xf.size // 2, y.view(np.float32))
        else:
            xf = _f32(x)
            y = np.empty(xf.size, np.float32)
            fn(self._h, xf, xf.size, y)
        return y

    def __call__(self, x):
        return self._run(x, lib().ora_iirfilt_execute_block)

    def execute_f64(self, x):
        return self._run(x, lib().ora_iirfilt_execute_block_f64)


class AGC(_Handle):
    _destroy = "ora_agc_destroy"

    def __init__(self):
        self._h = lib().ora_agc_create()

    def reset(self):
        lib().ora_agc_reset(self._h)

    bandwidth = property(lambda s: lib().ora_agc_get_bandwidth(s._h),
                         lambda s, v: lib().ora_agc_set_bandwidth(s._h, v))
    gain = property(lambda s: lib().ora_agc_get_gain(s._h),
                    lambda s, v: lib().ora_agc_set_gain(s._h, v))
    scale = property(lambda s: lib().ora_agc_get_scale(s._h),
                     lambda s, v: lib().ora_agc_set_scale(s._h, v))
    level = property(lambda s: lib().ora_agc_get_signal_level(s._h),
                     lambda s, v: lib().ora_agc_set_signal_level(s._h, v))
    rssi = property(lambda s: lib().ora_agc_get_rssi(s._h),
                    lambda s, v: lib().ora_agc_set_rssi(s._h, v))
    threshold = property(lambda s: lib().ora_agc_squelch_get_threshold(s._h),
                         lambda s, v: lib().ora_agc_squelch_set_threshold(s._h, v))
    status = property(lambda s: lib().ora_agc_squelch_get_status(s._h))

    def lock(self, on):
        lib().ora_agc_lock(self._h, int(on))

    def squelch(self, on):
        lib().ora_agc_squelch_enable(self._h, int(on))

    def set_timeout(self, t):
        lib().ora_agc_squelch_set_timeout(self._h, t)

    @property
    def state(self):
        g, y2, m, t = C.c_float(), C.c_float(), C.c_int(), C.c_uint()
        lib().ora_agc_get_state(self._h, C.byref(g), C.byref(y2), C.byref(m), C.byref(t))
        return g.value, y2.value, m.value, t.value

    @state.setter
    def state(self, s):
        lib().ora_agc_set_state(self._h, *s)

    def __call__(self, x, return_status=False):
        xf = _c64_as_f32(x)
        n = xf.size // 2
        y = np.empty(n, np.complex64)
        st = np.zeros(max(n, 1), np.uint8)
        lib().ora_agc_execute_wrapper(self._h, xf, n, y.view(np.float32), st.ctypes.data)
        return (y, st[:n]) if return_status else y


class AmpModem(_Handle):
    _destroy = "ora_ampmodem_destroy"

    def __init__(self, mod_index=0.75, type="dsb", carrier=False):
        t = {"dsb": 0, "usb": 1, "lsb": 2}[type]
        self._h = lib().ora_ampmodem_create(mod_index, t, 0 if carrier else 1)
        if not self._h:
            raise ValueError("ampmodem: invalid configuration")

    def reset(self):
        lib().ora_ampmodem_reset(self._h)

    @property
    def pll_state(self):
        t, d = C.c_uint32(), C.c_uint32()
        lib().ora_ampmodem_get_pll_state(self._h, C.byref(t), C.byref(d))
        return t.value, d.value

    def taps(self):
        lp = np.zeros(51, np.float32)
        dc = np.zeros(51, np.float32)
        lib().ora_ampmodem_get_taps(self._h, lp, dc)
        return lp, dc

    def hilbert_taps(self):
        h = np.zeros(50, np.float32)
        lib().ora_ampmodem_get_hilbert_taps(self._h, h)
        return h

    def __call__(self, x):
        xf = _c64_as_f32(x)
        y = np.empty(xf.size // 2, np.float32)
        lib().ora_ampmodem_demodulate_block(self._h, xf, xf.size // 2, y)
        return y


class FirHilb(_Handle):
    """firhilbf, complex -> real (c2r): returns (lower sideband, upper sideband)."""
    _destroy = "ora_firhilb_destroy"

    def __init__(self, m=25, As=60.0):
        self.m = int(m)
        self._h = lib().ora_firhilb_create(self.m, As)
        if not self._h:
            raise ValueError("firhilb: invalid configuration")

    def reset(self):
        lib().ora_firhilb_reset(self._h)

    def taps(self):
        h = np.zeros(2 * self.m, np.float32)
        lib().ora_firhilb_get_taps(self._h, h)
        return h

    def c2r(self, x):
        xf = _c64_as_f32(x)
        n = xf.size // 2
        y0 = np.empty(n, np.float32)
        y1 = np.empty(n, np.float32)
        lib().ora_firhilb_c2r_block(self._h, xf, n, y0, y1)
        return y0, y1


def deemphasis_coefs(sample_rate: float):
    """DeemphasisFilter coefficients, src/iirfilter.hpp:366-372."""
    x = np.float32(np.exp(-1.0 / (75.0e-6 * float(np.float32(sample_rate)))))
    a = np.array([1.0, -x], np.float32)
    b = np.array([np.float32(1.0 - float(x))], np.float32)
    return b, a


class AMRadio(_Handle):
    """README.md:41-58 chain: IIR -> resampler -> AGC -> AmpModem -> de-emphasis."""
    _destroy = "ora_amradio_destroy"

    def __init__(self, bandwidth=15000.0, iq_rate=2000000.0, pcm_rate=48000.0, iir_f64=False):
        self._h = lib().ora_amradio_create(bandwidth, iq_rate, pcm_rate, int(iir_f64))

    def __call__(self, x):
        xf = _c64_as_f32(x)
        n = xf.size // 2
        y = np.empty(lib().ora_amradio_max_out(self._h, n), np.float32)
        nw = lib().ora_amradio_execute(self._h, xf, n, y)
        return y[:nw].copy()


class FreqDem(_Handle):
    """freqdem (FreqDem, src/demod.hpp:189-219): m = cargf(conj(r[n-1]) r[n]) / (2 pi kf)."""
    _destroy = "ora_freqdem_destroy"

    def __init__(self, kf):
        self._h = lib().ora_freqdem_create(kf)

    def reset(self):
        lib().ora_freqdem_reset(self._h)

    def __call__(self, x):
        xf = _c64_as_f32(x)
        y = np.empty(len(x), np.float32)
        lib().ora_freqdem_demodulate_block(self._h, xf, len(x), y)
        return y


class BroadcastAM(_Handle):
    """BroadcastAM (src/demod.hpp:93-153).  iir_f64: evaluate the DC-blocking
    IIR in float64 (the reference for the GPU's fast IIR mode)."""
    _destroy = "ora_bcastam_destroy"

    def __init__(self, slen=25, iir_f64=False):
        self.iir_f64 = int(iir_f64)
        self._h = lib().ora_bcastam_create(slen, self.iir_f64)

    def reset(self):
        lib().ora_bcastam_reset(self._h)

    def __call__(self, x, return_pre=False):
        xf = _c64_as_f32(x)
        pre = np.empty(len(x), np.float32)
        y = np.empty(len(x), np.float32)
        lib().ora_bcastam_demodulate_block(self._h, xf, len(x), pre, y, self.iir_f64)
        return (pre, y) if return_pre else y


class FMStereo(_Handle):
    """FMStereo (src/demod.hpp:4-85): freqdem(4) -> composite PLL mixer ->
    75 us de-emphasis -> resamp_rrrf default, (L, R) interleaved float32.
    __call__(x, debug=True) also returns per-sample [s, re(sc), pe, theta bits]."""
    _destroy = "ora_fmstereo_destroy"

    def __init__(self, iq_rate=600000.0, pcm_rate=48000.0):
        self._h = lib().ora_fmstereo_create(iq_rate, pcm_rate)

    def reset(self):
        lib().ora_fmstereo_reset(self._h)

    @property
    def state(self):
        t, d, p = C.c_uint32(), C.c_uint32(), C.c_float()
        lib().ora_fmstereo_get_state(self._h, C.byref(t), C.byref(d), C.byref(p))
        return t.value, d.value, p.value

    @state.setter
    def state(self, v):
        lib().ora_fmstereo_set_state(self._h, int(v[0]) & 0xffffffff, int(v[1]) & 0xffffffff, float(v[2]))

    def __call__(self, x, debug=False):
        xf = _c64_as_f32(x)
        y = np.empty(2 * len(x) + 2, np.float32)
        dbg = np.empty(4 * len(x) + 1, np.float32) if debug else None
        nw = lib().ora_fmstereo_execute(self._h, xf, len(x), y, dbg.ctypes.data if debug else None)
        y = y[:nw].copy()
        if debug:
            d = dbg[:4 * len(x)].reshape(-1, 4)
            return y, d
        return y


class Delay:
    """wdelay read-then-push (Delay, src/utility.hpp:5-57): liquid's wdelay of
    `nd` holds nd + 1 samples, so y[n] = x[n - nd - 1] (zero history).  Real
    and complex streams keep separate lines, as in the reference."""

    def __init__(self, nd=1):
        self.delay = nd

    @property
    def delay(self):
        return self._nd

    @delay.setter
    def delay(self, nd):
        self._nd = int(nd)
        self._hist = {np.dtype(np.complex64): np.zeros(self._nd + 1, np.complex64),
                      np.dtype(np.float32): np.zeros(self._nd + 1, np.float32)}

    def __call__(self, x):
        x = np.asarray(x)
        if x.dtype not in self._hist:
            return None
        buf = np.concatenate([self._hist[x.dtype], x])
        self._hist[x.dtype] = buf[len(buf) - (self._nd + 1):].copy()
        return buf[:len(x)].copy()


def bytes_to_iq(b):
    """bytes_to_iq (src/utility.hpp:61-69): int16 (I, Q) pairs / 32767.0f."""
    b = bytes(b)
    a = np.frombuffer(b[: (len(b) // 4) * 4], dtype=np.int16).astype(np.float32)
    y = (a / np.float32(32767.0)).astype(np.float32)
    return y.view(np.complex64)
