"""Host side of the product without a GPU (runs in the CPU suite):

  * libldsp.so loads and exports every entry point include/ldsp.h declares;
  * the host-side designs behind the C ABI (Kaiser / notch taps, resampler
    prototype and phase schedule, IIR SOS for every prototype and band, NCO
    phase words, AGC defaults) are bit-identical to the restatement;
  * every compute entry point fails loudly (LDSP_EHIP) when no GPU is present:
    there is no CPU fallback;
  * the pybind11 `liquiddsp` module exposes the reference's classes, kwargs,
    defaults and properties (src/wrapper.cpp), and its calls raise RuntimeError
    without a GPU.
"""
import ctypes as C
import os
import re
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, "python-liquiddsp_amd")
LIBPATH = os.path.join(PKG, "libldsp.so")
HEADER = os.path.join(REPO, "include", "ldsp.h")

LDSP_EINVAL, LDSP_EHIP, LDSP_ERANGE = -1, -3, -4
MEM_HOST = 0


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIBPATH):
        pytest.fail("libldsp.so not built (run __graft_entry__.build())")
    L = C.CDLL(LIBPATH)
    L.ldsp_last_error.restype = C.c_char_p
    return L


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.complex64 else np.uint32)


def declared():
    return sorted(set(re.findall(r"\b(ldsp_[a-z0-9_]+)\s*\(", open(HEADER).read())))


def test_every_declared_symbol_is_exported(lib):
    names = declared()
    assert len(names) > 60
    missing = [s for s in names if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_device_count(lib):
    assert lib.ldsp_version() >= 100
    n = C.c_int(-1)
    assert lib.ldsp_device_count(C.byref(n)) == 0
    assert n.value >= 0


@pytest.mark.parametrize("n,fc,As,mu", [(127, 0.1, 60.0, 0.0), (51, 0.01, 40.0, 0.0), (25, 0.2, 20.0, 0.3),
                                        (255, 0.05, 60.0, 0.0), (4, 0.25, 30.0, -0.2)])
def test_kaiser_taps_bitwise(lib, ora, n, fc, As, mu):
    q = C.c_void_p()
    assert lib.ldsp_firfilt_create_kaiser(n, C.c_float(fc), C.c_float(As), C.c_float(mu), 1, C.byref(q)) == 0
    h = np.zeros(n, np.float32)
    assert lib.ldsp_firfilt_get_taps(q, ptr(h)) == 0
    assert (bits(h) == bits(ora.firdes_kaiser(n, fc, As, mu))).all()
    re_, im_ = C.c_float(), C.c_float()
    assert lib.ldsp_firfilt_freqresponse(q, C.c_float(0.0), C.byref(re_), C.byref(im_)) == 0
    assert abs(re_.value - float(np.sum(h.astype(np.float64)))) < 1e-4 * max(1.0, abs(re_.value))
    assert lib.ldsp_firfilt_destroy(q) == 0


def test_dc_blocker_taps_bitwise(lib, ora):
    q = C.c_void_p()
    assert lib.ldsp_firfilt_create_dc_blocker(25, C.c_float(20.0), 0, C.byref(q)) == 0
    n = C.c_uint()
    lib.ldsp_firfilt_get_length(q, C.byref(n))
    h = np.zeros(n.value, np.float32)
    lib.ldsp_firfilt_get_taps(q, ptr(h))
    assert (bits(h) == bits(ora.FIRFilter(dc_blocker=(25, 20.0), cplx=False).taps)).all()
    lib.ldsp_firfilt_destroy(q)


@pytest.mark.parametrize("rate,m,fc,nf", [(0.024, 20, 0.024, 13), (0.5, 7, 0.2, 32), (3.3, 12, 0.2, 16)])
def test_resampler_design_and_schedule(lib, ora, rate, m, fc, nf):
    q = C.c_void_p()
    r32, f32 = np.float32(rate), np.float32(fc)
    assert lib.ldsp_resamp_create(C.c_float(r32), m, C.c_float(f32), C.c_float(60.0), nf, 1, C.byref(q)) == 0
    o = ora.Resampler(r32, m, f32, 60.0, nf, cplx=True)
    npfb, step, phase, ntaps = C.c_uint(), C.c_uint32(), C.c_uint32(), C.c_uint()
    assert lib.ldsp_resamp_get_info(q, C.byref(npfb), C.byref(step), C.byref(phase), C.byref(ntaps)) == 0
    assert step.value == o.step and phase.value == o.phase
    h = np.zeros(1 << 16, np.float32)
    nh = C.c_uint()
    assert lib.ldsp_resamp_get_taps(q, ptr(h), h.size, C.byref(nh)) == 0
    assert nh.value > 0 and np.isfinite(h[:nh.value]).all()
    # the exact output count of the next call follows the phase schedule
    for nin in (0, 1, 41, 65536, 67108864):
        nout = C.c_size_t()
        assert lib.ldsp_resamp_num_outputs(q, C.c_size_t(nin), C.byref(nout)) == 0
        if nin <= 65536:
            o2 = ora.Resampler(r32, m, f32, 60.0, nf, cplx=True)
            assert nout.value == o2(np.zeros(nin, np.complex64)).size
    if rate == 0.024:
        nout = C.c_size_t()
        lib.ldsp_resamp_num_outputs(q, C.c_size_t(64 << 20), C.byref(nout))
        assert nout.value == 1_610_613
    lib.ldsp_resamp_destroy(q)


PROTOS = [("butter", "lowpass", 4, 0.1, 0.0), ("cheby1", "lowpass", 5, 0.2, 0.0), ("cheby2", "lowpass", 8, 0.0075, 0.0),
          ("butter", "highpass", 6, 0.15, 0.0), ("cheby2", "highpass", 4, 0.05, 0.0),
          ("butter", "bandpass", 3, 0.1, 0.25), ("cheby1", "bandstop", 2, 0.05, 0.2),
          ("ellip", "lowpass", 4, 0.1, 0.0), ("ellip", "lowpass", 5, 0.2, 0.0), ("ellip", "highpass", 6, 0.05, 0.0),
          ("ellip", "bandpass", 3, 0.1, 0.25), ("bessel", "lowpass", 4, 0.1, 0.0), ("bessel", "lowpass", 7, 0.02, 0.0),
          ("bessel", "highpass", 3, 0.2, 0.0), ("bessel", "bandstop", 2, 0.05, 0.2)]
FT = {"butter": 0, "cheby1": 1, "cheby2": 2, "ellip": 3, "bessel": 4}
BT = {"lowpass": 0, "highpass": 1, "bandpass": 2, "bandstop": 3}


@pytest.mark.parametrize("ft,bt,order,fc,f0", PROTOS)
def test_iir_design_bitwise(lib, ora, ft, bt, order, fc, f0):
    q = C.c_void_p()
    rc = lib.ldsp_iirfilt_create_prototype(FT[ft], BT[bt], order, C.c_float(fc), C.c_float(f0), C.c_float(0.5),
                                           C.c_float(60.0), 1, C.byref(q))
    assert rc == 0, lib.ldsp_last_error()
    ns = C.c_uint()
    lib.ldsp_iirfilt_get_nsos(q, C.byref(ns))
    B = np.zeros(3 * ns.value, np.float32)
    A = np.zeros(3 * ns.value, np.float32)
    assert lib.ldsp_iirfilt_get_sos(q, ptr(B), ptr(A)) == 0
    Bo, Ao = ora.iirdes(ft, bt, order, fc, f0, 0.5, 60.0)
    assert (bits(B) == bits(Bo.reshape(-1))).all() and (bits(A) == bits(Ao.reshape(-1))).all()
    lib.ldsp_iirfilt_destroy(q)


def test_iir_invalid_design_is_einval(lib):
    q = C.c_void_p()
    rc = lib.ldsp_iirfilt_create_prototype(0, 0, 0, C.c_float(0.1), C.c_float(0.0), C.c_float(0.5),
                                           C.c_float(60.0), 1, C.byref(q))
    assert rc == LDSP_EINVAL and lib.ldsp_last_error()


def test_nco_phase_words(lib, ora):
    q = C.c_void_p()
    assert lib.ldsp_nco_create(0, C.byref(q)) == 0
    o = ora.NCO(0)
    for f, p in ((2 * np.pi * 0.05, 0.3), (-1.0, 3.0), (7.5, -9.0)):
        lib.ldsp_nco_set_frequency(q, C.c_float(f))
        lib.ldsp_nco_set_phase(q, C.c_float(p))
        o.freq, o.phase = np.float32(f), np.float32(p)
        th, dth = C.c_uint32(), C.c_uint32()
        lib.ldsp_nco_get_state(q, C.byref(th), C.byref(dth))
        assert (th.value, dth.value) == o.state
    lib.ldsp_nco_destroy(q)


def test_agc_defaults(lib, ora):
    q = C.c_void_p()
    assert lib.ldsp_agc_create(C.byref(q)) == 0
    o = ora.AGC()
    v = C.c_float()
    for get, ref in ((lib.ldsp_agc_get_bandwidth, o.bandwidth), (lib.ldsp_agc_get_gain, o.gain),
                     (lib.ldsp_agc_get_scale, o.scale)):
        assert get(q, C.byref(v)) == 0
        assert np.float32(v.value) == np.float32(ref)
    st = C.c_int()
    lib.ldsp_agc_squelch_get_status(q, C.byref(st))
    assert st.value == o.status
    lib.ldsp_agc_destroy(q)


def test_execute_without_gpu_fails_loudly(lib):
    n = C.c_int()
    lib.ldsp_device_count(C.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is present")
    q = C.c_void_p()
    lib.ldsp_firfilt_create_kaiser(31, C.c_float(0.1), C.c_float(60.0), C.c_float(0.0), 1, C.byref(q))
    x = np.zeros(64, np.complex64)
    y = np.zeros(64, np.complex64)
    assert lib.ldsp_firfilt_execute(q, ptr(x), C.c_size_t(64), ptr(y), MEM_HOST, None) == LDSP_EHIP
    assert b"no CPU fallback" in lib.ldsp_last_error()
    lib.ldsp_firfilt_destroy(q)
    a = C.c_void_p()
    lib.ldsp_agc_create(C.byref(a))
    assert lib.ldsp_agc_execute(a, ptr(x), C.c_size_t(64), ptr(y), None, MEM_HOST, None) == LDSP_EHIP
    lib.ldsp_agc_destroy(a)


# ------------------------------------------------------------------ pybind11 module surface
@pytest.fixture(scope="module")
def ld():
    if PKG not in sys.path:
        sys.path.insert(0, PKG)
    import liquiddsp
    return liquiddsp


REFERENCE_CLASSES = ["ComplexResampler", "RealResampler", "RealFIRFilter", "RealDCBlocker", "RealKaiserBessel",
                     "ComplexIIRFilter", "RealIIRFilter", "CIIRFilter", "RIIRFilter", "CLowpassIIR", "RLowpassIIR",
                     "CHighpassIIR", "RHighpassIIR", "CBandpassIIR", "RBandpassIIR", "CBandstopIIR", "RBandstopIIR",
                     "DeemphasisFilter", "NCO", "AGC", "AmpModem"]


def test_module_classes(ld):
    for name in REFERENCE_CLASSES + ["ComplexFIRFilter"]:
        assert hasattr(ld, name), name


def test_module_defaults_and_properties(ld, ora):
    r = ld.ComplexResampler(rate=0.024, Fc=0.024)
    assert np.float32(r.rate) == np.float32(0.024)
    r.rate = 0.5
    assert np.float32(r.rate) == np.float32(0.5)
    a = ld.AGC()
    assert np.float32(a.bandwidth) == np.float32(0.01) and a.gain == 1.0 and a.scale == 1.0
    a.scale = 0.01
    assert np.float32(a.scale) == np.float32(0.01)
    n = ld.NCO()
    n.freq = 0.25
    o = ora.NCO(0)
    o.freq = 0.25                        # round-trips through the uint32 phase step, as in liquid
    assert np.float32(n.freq) == np.float32(o.freq)
    am = ld.AmpModem()
    assert (np.float32(am.modulation), am.type, am.carrier) == (np.float32(0.75), "dsb", False)
    i = ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2e6)
    assert (i.filter_type, i.order, np.float32(i.Ap), np.float32(i.As)) == ("cheby2", 8, np.float32(0.7),
                                                                             np.float32(60.0))
    B, A = i.sos()
    assert np.asarray(B).shape == (4, 3) and np.asarray(A).shape == (4, 3)
    d = ld.DeemphasisFilter()
    assert d is not None


def test_module_calls_raise_without_gpu(ld):
    if ld.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ld.ComplexResampler(rate=0.024, Fc=0.024)(np.zeros(100, np.complex64))
    with pytest.raises(RuntimeError):
        ld.AGC()(np.zeros(10, np.complex64))


@pytest.mark.parametrize("ft", ["butter", "cheby1", "cheby2", "ellip", "bessel"])
@pytest.mark.parametrize("bt", ["lowpass", "highpass", "bandpass", "bandstop"])
def test_iir_freqresponse_all_types(lib, ft, bt):
    """ldsp_iirfilt_freqresponse (iirfilter.hpp freqresponse -> iirfilt_*_freqresponse)
    for every prototype / band type: |H| equals scipy's response of the same SOS."""
    import scipy.signal as sps
    q = C.c_void_p()
    assert lib.ldsp_iirfilt_create_prototype(FT[ft], BT[bt], 4, C.c_float(0.08), C.c_float(0.2), C.c_float(1.0),
                                             C.c_float(40.0), 1, C.byref(q)) == 0, lib.ldsp_last_error()
    ns = C.c_uint()
    lib.ldsp_iirfilt_get_nsos(q, C.byref(ns))
    B = np.zeros(3 * ns.value, np.float32)
    A = np.zeros(3 * ns.value, np.float32)
    lib.ldsp_iirfilt_get_sos(q, ptr(B), ptr(A))
    sos = np.hstack([B.reshape(-1, 3), A.reshape(-1, 3)]).astype(np.float64)
    fs = np.linspace(0.0, 0.5, 41)
    _, hr = sps.sosfreqz(sos, worN=fs, fs=1.0)
    re_, im_ = C.c_float(), C.c_float()
    got = []
    for f in fs:
        assert lib.ldsp_iirfilt_freqresponse(q, C.c_float(f), C.byref(re_), C.byref(im_)) == 0
        got.append(complex(re_.value, im_.value))
    assert np.max(np.abs(np.abs(got) - np.abs(hr))) < 1e-4
    lib.ldsp_iirfilt_destroy(q)


@pytest.mark.parametrize("fn", [0, 1])
def test_loop_fast_math_equals_general(lib, fn):
    """lm_logf_fast / lm_expf_fast (the AGC loop's fast paths) give the general
    functions' bits on a sample of every float in their ranges (host build of
    ldsp_math.hpp; scripts/analysis/check_fast_math.py runs every float)."""
    checked, bad = C.c_uint64(), C.c_uint64()
    assert lib.ldsp_debug_math_fastcheck(fn, 0, 0xFFFFFFFF, 4099, C.byref(checked), C.byref(bad)) == 0
    assert checked.value > 100_000 and bad.value == 0, (checked.value, bad.value)


@pytest.mark.parametrize("typ", ["dsb", "usb", "lsb"])
def test_ampmodem_designs_bitwise(ld, ora, typ):
    """AmpModem's designs (liquid ampmodem_create): the carrier lowpass, the DC
    blocker and the usb / lsb Hilbert transform's quadrature taps
    (firhilbf_create(25, 60)) are the restatement's, bit for bit."""
    am = ld.AmpModem(modulation=0.5, type=typ, carrier=True)
    assert am.type == typ
    lp, dc, hq = am._taps()
    o = ora.AmpModem(mod_index=0.5, type=typ, carrier=True)
    olp, odc = o.taps()
    assert (bits(lp) == bits(olp)).all() and (bits(dc) == bits(odc)).all()
    assert (bits(hq) == bits(o.hilbert_taps())).all()
    assert (bits(hq) == bits(ora.FirHilb(25, 60.0).taps())).all()


def test_ampmodem_type_setter_accepts_ssb(ld):
    """AmpModem.type = 'usb' / 'lsb' rebuilds the modem (demod.hpp:250-256); an
    unknown type string leaves it unchanged."""
    am = ld.AmpModem(modulation=0.5, type="dsb", carrier=False)
    am.type = "usb"
    assert am.type == "usb"
    am.type = "lsb"
    assert am.type == "lsb"
    am.type = "ssb?"
    assert am.type == "lsb"
    am.carrier = True
    assert (am.type, am.carrier) == ("lsb", True)


def test_iirfilt_resamp_checks_before_any_device_work(lib):
    """ldsp_iirfilt_resamp_execute (liquiddsp.filter_resample's C entry): a real
    filter with a complex resampler is LDSP_EINVAL, too small an output capacity
    LDSP_ERANGE with *nout set -- both decided on the host, before any device
    call (this container has no GPU)."""
    f, r = C.c_void_p(), C.c_void_p()
    assert lib.ldsp_iirfilt_create_prototype(2, 0, 8, C.c_float(0.0075), C.c_float(0.0), C.c_float(0.5),
                                             C.c_float(60.0), 0, C.byref(f)) == 0, lib.ldsp_last_error()
    assert lib.ldsp_resamp_create(C.c_float(0.024), 20, C.c_float(0.024), C.c_float(60.0), 13, 1, C.byref(r)) == 0
    x = np.zeros(1000, np.complex64)
    y = np.zeros(100, np.complex64)
    nout = C.c_size_t(0)
    rc = lib.ldsp_iirfilt_resamp_execute(f, r, ptr(x), C.c_size_t(x.size), ptr(y), C.c_size_t(y.size),
                                         C.byref(nout), 0, None)
    assert rc == LDSP_EINVAL and b"both be complex" in lib.ldsp_last_error()
    lib.ldsp_iirfilt_destroy(f)
    assert lib.ldsp_iirfilt_create_prototype(2, 0, 8, C.c_float(0.0075), C.c_float(0.0), C.c_float(0.5),
                                             C.c_float(60.0), 1, C.byref(f)) == 0
    expect = C.c_size_t(0)
    lib.ldsp_resamp_num_outputs(r, C.c_size_t(100_000), C.byref(expect))
    rc = lib.ldsp_iirfilt_resamp_execute(f, r, ptr(x), C.c_size_t(100_000), ptr(y), C.c_size_t(10),
                                         C.byref(nout), 0, None)
    assert rc == LDSP_ERANGE and nout.value == expect.value > 10
    lib.ldsp_iirfilt_destroy(f)
    lib.ldsp_resamp_destroy(r)


def test_host_pool_without_gpu(lib):
    """ldsp_host_alloc fails cleanly with no device (LDSP_ENOMEM, NULL; the pybind
    module then returns pageable arrays), ldsp_host_free(NULL) is a no-op and a
    pointer the pool never handed out is rejected."""
    p = C.c_void_p(1)
    assert lib.ldsp_host_alloc(C.c_size_t(1 << 20), C.byref(p)) == -2
    assert p.value is None
    assert lib.ldsp_host_free(None) == 0
    junk = np.zeros(4, np.float32)
    assert lib.ldsp_host_free(ptr(junk)) == LDSP_EINVAL
    assert b"not a block" in lib.ldsp_last_error()
