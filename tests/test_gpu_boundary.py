"""The drop-in boundary: what the pybind11 layer
does with the caller's arrays and with state-resetting setters, against the
oracle object that the reference's own code path would produce.

  * a18: AmpModem.modulation / .type / .carrier rebuild the modem
    (src/demod.hpp:250-276 `ampmodem_destroy` + `makeFromArgs`), so the output
    after a setter equals a freshly created oracle modem with the new arguments;
    a setter that cannot build the new modem leaves the old one untouched.
  * a19: array_to_ptr (src/liquiddsp.hpp:16-20) borrows the buffer of a
    `py::array_t<T>` argument, which pybind11 force-casts (lists, float64,
    complex128 are converted); this module requests c_style|forcecast, so
    strided views are made contiguous too -- every such input equals the
    oracle on the contiguous force-cast copy.
  * a16: AGC level (= 1/g) and level_dB (rssi = -20 log10 g) round-trip like
    agc_crcf_{get,set}_signal_level / _rssi (src/agc.hpp:17-107).
  * resets on another stream: reset() then a call on a different torch stream
    sees the zeroed state (the zeroing is ordered like an execute).
"""
import numpy as np
import pytest

from conftest import cgauss

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.complex64 else np.uint32)


def assert_bitwise(y, ref, what=""):
    assert y.shape == ref.shape, (what, y.shape, ref.shape)
    eq = bits(y) == bits(ref)
    assert eq.all(), f"{what}: {(~eq).sum()} of {eq.size} differ; first at {int(np.argmin(eq))}"


def _am48k(rng, n, fcar=300.0):
    t = np.arange(n) / 48000.0
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t)) / 2
    s = (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * fcar * t + 0.7))
    return (s + 0.03 * cgauss(rng, n)).astype(np.complex64)


# ------------------------------------------------------------------ a18 AmpModem setters
@pytest.mark.parametrize("n2", [3000, 60_000])         # sequential and chunk-parallel second calls
def test_ampmodem_setters_rebuild_like_reference(ld, ora, rng, n2):
    x1, x2 = _am48k(rng, 20_000), _am48k(rng, n2)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    g(x1)                                               # advance the PLL state
    g.modulation = 0.8                                  # -> makeFromArgs(0.8, dsb, carrier): fresh state
    assert g.modulation == pytest.approx(0.8)
    assert g.pll_state() == (0, 0)
    assert_bitwise(g(x2), ora.AmpModem(0.8, "dsb", carrier=True)(x2), "modulation")

    g(x1)
    g.carrier = False                                   # suppressed carrier: the Costas loop, fresh state
    assert g.carrier is False
    assert_bitwise(g(x2), ora.AmpModem(0.8, "dsb", carrier=False)(x2), "carrier")

    g(x1)
    g.type = "dsb"                                      # the same type still rebuilds (demod.hpp:250-256)
    assert g.pll_state() == (0, 0)
    assert_bitwise(g(x2), ora.AmpModem(0.8, "dsb", carrier=False)(x2), "type")


def test_ampmodem_ignored_setter_keeps_modem(ld, ora, rng):
    x = _am48k(rng, 30_000)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    o = ora.AmpModem(0.5, "dsb", carrier=True)
    y1 = g(x[:10_000])
    g.type = "fm"                                       # an unknown type is ignored (demod.hpp:250) ...
    assert g.type == "dsb" and g.carrier is True and g.modulation == pytest.approx(0.5)
    y2 = g(x[10_000:])                                  # ... and the modem continues, state intact
    assert_bitwise(np.concatenate([y1, y2]), o(x))
    assert g.pll_state() == o.pll_state


# ------------------------------------------------------------------ a19 array_to_ptr inputs
def test_complex_inputs_forcecast(ld, ora, rng):
    h = ora.firdes_kaiser(51, 0.1, 60.0)
    x = cgauss(rng, 40_002)
    cases = {
        "strided view": x[::2],
        "reversed view": x[::-1],
        "complex128": x.astype(np.complex128),
        "float64 (real)": np.real(x).astype(np.float64),
        "float32 (real)": np.imag(x).astype(np.float32),
        "int16": np.round(100 * np.real(x[:5000])).astype(np.int16),
        "python list": [complex(v) for v in x[:3001]],
    }
    for name, v in cases.items():
        ref_in = np.ascontiguousarray(np.asarray(v), dtype=np.complex64)
        g = ld.ComplexFIRFilter(h)
        g.exact = True
        assert_bitwise(g(v), ora.FIRFilter(h, cplx=True)(ref_in), "fir " + name)
        r = ld.ComplexResampler(rate=0.3, Fc=0.12)
        assert_bitwise(r(v), ora.Resampler(np.float32(0.3), 20, np.float32(0.12), 60.0, 13)(ref_in), "resamp " + name)
        a = ld.AGC()
        assert_bitwise(a(v), ora.AGC()(ref_in), "agc " + name)


def test_real_inputs_forcecast(ld, ora, rng):
    h = ora.firdes_kaiser(25, 0.2, 20.0)
    x = rng.standard_normal(30_001)
    cases = {
        "float64": x,
        "strided float32": x.astype(np.float32)[1::3],
        "python list": list(x[:2000]),
        "int32": np.round(1000 * x[:4000]).astype(np.int32),
    }
    b, a = ora.deemphasis_coefs(48000.0)
    for name, v in cases.items():
        ref_in = np.ascontiguousarray(np.asarray(v), dtype=np.float32)
        g = ld.RealFIRFilter(h)
        g.exact = True
        assert_bitwise(g(v), ora.FIRFilter(h, cplx=False)(ref_in), "fir " + name)
        assert_bitwise(ld.DeemphasisFilter(48000)(v), ora.IIRFilter(tf=(b, a), cplx=False)(ref_in), "deemph " + name)


def test_device_tensor_strided_and_dtype(ld, ora, rng):
    import torch
    h = ora.firdes_kaiser(127, 0.1, 60.0)
    x = cgauss(rng, 50_000)
    xd = torch.from_numpy(x).cuda()
    for name, v, ref_in in (("strided", xd[::2], x[::2]), ("complex128", xd.to(torch.complex128), x),
                            ("real float32", xd.real.contiguous(), np.real(x))):
        g = ld.ComplexFIRFilter(h)
        g.exact = True
        y = g(v)
        assert y.is_cuda and y.dtype == torch.complex64
        assert_bitwise(y.cpu().numpy(), ora.FIRFilter(h, cplx=True)(np.ascontiguousarray(ref_in, np.complex64)), name)


# ------------------------------------------------------------------ a16 AGC level / level_dB
def test_agc_level_roundtrip(ld, ora, rng):
    g, o = ld.AGC(), ora.AGC()
    for lv in (0.25, 3.0, 1e-3):
        g.level = lv
        o.level = np.float32(lv)
        assert np.float32(g.level) == np.float32(o.level)
        assert np.float32(g.gain) == np.float32(o.gain)
    for db in (-20.0, 6.0, 0.0):
        g.level_dB = db
        o.rssi = np.float32(db)
        assert np.float32(g.level_dB) == np.float32(o.rssi)
        assert np.float32(g.gain) == np.float32(o.gain)
    # set_signal_level / set_rssi also restart the smoothed energy (y2' = 1): the
    # next block must follow the oracle bit for bit, and the getters track the loop
    x = _am48k(rng, 40_000)
    g.level = 0.5
    o.level = np.float32(0.5)
    assert_bitwise(g(x), o(x))
    assert np.float32(g.level) == np.float32(o.level)
    assert np.float32(g.level_dB) == np.float32(o.rssi)
    with pytest.raises(ValueError):
        g.level = -1.0


# ------------------------------------------------------------------ reset on another stream
def test_reset_then_call_on_another_stream(ld, ora, rng):
    import torch
    x = cgauss(rng, 200_000)
    xd = torch.from_numpy(x).cuda()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    h = ora.firdes_kaiser(127, 0.1, 60.0)
    objs = [("fir", ld.ComplexFIRFilter(h), lambda: ora.FIRFilter(h, cplx=True)),
            ("resamp", ld.ComplexResampler(rate=0.024, Fc=0.024),
             lambda: ora.Resampler(np.float32(0.024), 20, np.float32(0.024), 60.0, 13)),
            ("iir", ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=np.float32(0.0075)),
             lambda: ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(0.0075), 0.3, 0.7, 60.0)))]
    for name, g, mk in objs:
        if hasattr(g, "exact"):
            g.exact = True
        torch.cuda.synchronize()
        with torch.cuda.stream(sa):
            g(xd)                         # long call queued on stream A
        g.reset()                         # zeroing enqueued behind it
        with torch.cuda.stream(sb):
            y = g(xd[:50_000])            # stream B must see the zeroed state
        torch.cuda.synchronize()
        assert_bitwise(y.cpu().numpy(), mk()(x[:50_000]), name)
