"""GPU parity: every hot-path class of the `liquiddsp` module (HIP kernels in
libldsp) against the CPU restatement (oracle/) on identical seeded inputs.

Bars:
  * bit-exact: resampler, NCO (table), exact-mode FIR / IIR, de-emphasis,
    AGC, AmpModem (carrier + Costas), the whole AM chain in exact mode;
  * max|y - y_ref| / max|y_ref| <= 1e-6: fast-mode FIR (FMA, different order);
  * fast-mode IIR (float64 scan): error vs the float64 evaluation must be far
    below the float32 recursion's own error (liquid-dsp's float32 recursion is
    itself ~1e-4 off for the narrow cheby2, App. B).
"""
import numpy as np
import pytest
import scipy.signal as sps

from conftest import cgauss, maxrel

pytestmark = pytest.mark.gpu

L_TAPS = [1, 2, 15, 16, 17, 51, 127, 255, 513]


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.complex64 else np.uint32)


def assert_bitwise(y, ref):
    assert y.shape == ref.shape, (y.shape, ref.shape)
    eq = bits(y) == bits(ref)
    if not eq.all():
        i = int(np.argmin(eq))
        raise AssertionError(f"{(~eq).sum()} of {eq.size} differ; first at {i}: {y[i]!r} vs {ref[i]!r}")


# ------------------------------------------------------------------ math
def test_device_math_bitwise(ld, ora, rng):
    import torch
    n = 1 << 20
    cases = {
        0: (np.float32(rng.uniform(-30, 30, n)), None),
        1: (np.float32(np.exp(rng.uniform(-80, 80, n))), None),
        2: (np.float32(rng.standard_normal(n)), np.float32(rng.standard_normal(n))),
        5: None,   # atan2 special operands (zeros, infinities, NaN, tiny/huge ratios)
        3: (np.float32(rng.uniform(-12, 12, n)), None),
    }
    names = {0: "exp", 1: "log", 2: "atan2", 3: "tanh"}
    sp = np.float32([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-38, -1e-38, 1e38, -1e38, 3e-45])
    ga, gb = np.meshgrid(sp, sp)
    cases[5] = (np.ascontiguousarray(ga.ravel()), np.ascontiguousarray(gb.ravel()))
    for key, (a, b) in cases.items():
        fn = 2 if key == 5 else key
        ta = torch.from_numpy(a).cuda()
        tb = torch.from_numpy(b if b is not None else a).cuda()
        ty = torch.empty_like(ta)
        # atan2 twice: lm_atan2f (fn 2) and its select-only form lm_atan2f_vsel
        # (fn 7, the candidate evaluations of k_pll_seqc and k_fm_pll)
        for f in ((2, 7) if fn == 2 else (fn,)):
            ld._math_eval(f, ta.data_ptr(), tb.data_ptr(), ty.data_ptr(), a.size, 0)
            torch.cuda.synchronize()
            got, ref = ty.cpu().numpy(), ora.math_eval(names[fn], a, b)
            if key == 5:                      # NaN payloads are not specified: NaN-ness only
                assert np.array_equal(np.isnan(got), np.isnan(ref))
                got, ref = got[~np.isnan(ref)], ref[~np.isnan(ref)]
            assert_bitwise(got, ref)
    # the AGC loop's fast paths (fn 5 exp, 6 log: lm_*_loop, scaling-free division
    # on the device) must give the general functions' bits everywhere, in and out
    # of their fast ranges
    loop_cases = {5: np.float32(np.concatenate([rng.uniform(-0.35, 0.35, n // 2), rng.uniform(-30, 30, n // 4),
                                                np.ldexp(rng.uniform(-1, 1, n // 4), rng.integers(-40, -20, n // 4))])),
                  6: np.float32(np.concatenate([rng.uniform(0.5, 2.0, n // 2), np.exp(rng.uniform(-80, 80, n // 4)),
                                                1.0 + np.ldexp(rng.uniform(-1, 1, n // 4), -21)]))}
    for fn, a in loop_cases.items():
        ta = torch.from_numpy(a).cuda()
        ty = torch.empty_like(ta)
        ld._math_eval(fn, ta.data_ptr(), ta.data_ptr(), ty.data_ptr(), a.size, 0)
        torch.cuda.synchronize()
        assert_bitwise(ty.cpu().numpy(), ora.math_eval("exp" if fn == 5 else "log", a, None))
    th = np.float32(rng.uniform(-20, 20, 4096))
    ta = torch.from_numpy(th).cuda()
    ty = torch.empty_like(ta)
    ld._math_eval(4, ta.data_ptr(), ta.data_ptr(), ty.data_ptr(), th.size, 0)
    torch.cuda.synchronize()
    got = ty.cpu().numpy().view(np.uint32)
    ref = np.array([ora.constrain(float(t)) for t in th], np.uint32)
    assert np.array_equal(got, ref)
    # fn 8, constrain through v_fract (k_fm_pll's chain), against fn 4 on the device:
    # random angles, and every 16th theta whose p = theta / 2 pi lies around the
    # [-2^-25, 0) range where p - floor(p) rounds to 1.0 (both signs), zeros,
    # integers of turns and their neighbours
    edge = np.arange(0xB3000000, 0xB5000000, 16, dtype=np.uint32).view(np.float32)
    turns = np.float32(2 * np.pi) * np.float32(np.arange(-40, 41))
    near = np.concatenate([np.nextafter(turns, np.float32(np.inf)), np.nextafter(turns, np.float32(-np.inf)), turns])
    th8 = np.ascontiguousarray(np.concatenate([np.float32(rng.uniform(-20, 20, 1 << 18)), edge, -edge, near,
                                               np.float32([0.0, -0.0, 1e-30, -1e-30, 3e-45, -3e-45])]))
    ta = torch.from_numpy(th8).cuda()
    y4, y8 = torch.empty_like(ta), torch.empty_like(ta)
    ld._math_eval(4, ta.data_ptr(), ta.data_ptr(), y4.data_ptr(), th8.size, 0)
    ld._math_eval(8, ta.data_ptr(), ta.data_ptr(), y8.data_ptr(), th8.size, 0)
    torch.cuda.synchronize()
    assert torch.equal(y4.view(torch.int32), y8.view(torch.int32))
    sub = th8[-4096:]
    assert np.array_equal(y8.cpu().numpy()[-4096:].view(np.uint32),
                          np.array([ora.constrain(float(t)) for t in sub], np.uint32))


# ------------------------------------------------------------------ FIR
@pytest.mark.parametrize("L", L_TAPS)
@pytest.mark.parametrize("cplx", [True, False])
@pytest.mark.parametrize("mode", ["fast", "direct"])
def test_fir_fast_within_1e6(ld, ora, rng, L, cplx, mode):
    # complex "fast" with 48 <= L <= 1025 is the overlap-save FFT kernel
    h = ora.firdes_kaiser(L, 0.1, 60.0) if L > 1 else np.float32([0.7])
    n = 70_001
    x = cgauss(rng, n) if cplx else np.float32(rng.standard_normal(n))
    g = (ld.ComplexFIRFilter if cplx else ld.RealFIRFilter)(h)
    g.mode = mode
    o = ora.FIRFilter(h, cplx=cplx)
    # ragged streaming: history carried across calls
    cuts = [0, 1, 5, 4096, 4097, 30_000, n]
    y = np.concatenate([g(x[s:e]) for s, e in zip(cuts[:-1], cuts[1:])])
    ref = o(x)
    assert y.dtype == ref.dtype and len(y) == n
    # float64 truth: the fast kernel (one FMA per tap) must be at least as close
    # to it as the float32 sequential restatement is
    truth = sps.lfilter(h.astype(np.float64), 1.0, x.astype(np.complex128 if cplx else np.float64))
    err_gpu, err_ref = maxrel(y, truth), maxrel(ref, truth)
    # float32 accumulation noise grows ~sqrt(L); beyond the north-star 127 taps the
    # two summation orders are both ~1e-6 from the float64 truth
    assert err_gpu <= max(1e-6, 1.3 * err_ref), (err_gpu, err_ref)
    if L <= 127:          # north-star configuration: within 1e-6 of the restatement itself
        assert maxrel(y, ref) <= 1e-6


@pytest.mark.parametrize("L", [1, 17, 51, 127])
@pytest.mark.parametrize("cplx", [True, False])
def test_fir_exact_bitwise(ld, ora, rng, L, cplx):
    h = ora.firdes_kaiser(L, 0.1, 60.0) if L > 1 else np.float32([0.7])
    x = cgauss(rng, 20_000) if cplx else np.float32(rng.standard_normal(20_000))
    g = (ld.ComplexFIRFilter if cplx else ld.RealFIRFilter)(h)
    g.exact = True
    o = ora.FIRFilter(h, cplx=cplx)
    y = np.concatenate([g(x[:333]), g(x[333:])])
    assert_bitwise(y, o(x))


@pytest.mark.parametrize("mode", ["fast", "direct"])
def test_fir_fast_chunking_invariant(ld, ora, rng, mode):
    # direct form: bitwise invariant to how the stream is cut into calls;
    # overlap-save FFT: the 2048-point windows move with the call boundaries,
    # so a re-cut stream agrees to float32 rounding (<= 1e-6 of max|y|)
    h = ora.firdes_kaiser(127, 0.1, 60.0)
    x = cgauss(rng, 50_000)
    a = ld.ComplexFIRFilter(h)
    a.mode = mode
    whole = a(x)
    b = ld.ComplexFIRFilter(h)
    b.mode = mode
    parts = np.concatenate([b(x[:7]), b(x[7:4100]), b(x[4100:])])
    if mode == "direct":
        assert_bitwise(parts, whole)
    else:
        assert maxrel(parts, whole) <= 1e-6
    a.reset()
    assert_bitwise(a(x), whole)


@pytest.mark.parametrize("L", [127, 255])
def test_fir_fft_north_star_size(ld, ora, rng, L):
    """BASELINE north-star size (64 Mi complex64): the FFT path against the
    direct-form kernel over the whole array (size-independent property: both
    within float32 rounding of the same convolution) and against the
    restatement on a 256 Ki-sample window taken from the middle."""
    import torch
    n = 64 << 20
    h = ora.firdes_kaiser(L, 0.1, 60.0)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    xd = torch.complex(torch.randn(n, generator=g, device="cuda"), torch.randn(n, generator=g, device="cuda"))
    f = ld.ComplexFIRFilter(h)
    d = ld.ComplexFIRFilter(h)
    d.mode = "direct"
    yf = f(xd)
    yd = d(xd)
    err = float((yf - yd).abs().max() / yd.abs().max())
    assert err <= 1e-6, err
    s0, w = n // 2 + 12345, 1 << 18
    xw = xd[s0 - (L - 1): s0 + w].cpu().numpy()
    ref = ora.FIRFilter(h, cplx=True)(xw)[L - 1:]
    assert maxrel(yf[s0: s0 + w].cpu().numpy(), ref) <= 1e-6


def test_kaiserbessel_dcblocker(ld, ora, rng):
    x = np.float32(rng.standard_normal(10_000))
    kb = ld.RealKaiserBessel(25, 0.1, 20.0, 0.0)
    o = ora.FIRFilter(kaiser=(25, 0.1, 20.0, 0.0), cplx=False)
    o.scale = np.float32(1.0 / abs(np.complex64(o.freqresponse(0.0))))
    kb.exact = True
    assert_bitwise(kb(x), o(x))
    dc = ld.RealDCBlocker(25, 20.0)
    dc.exact = True
    assert_bitwise(dc(x), ora.FIRFilter(dc_blocker=(25, 20.0), cplx=False)(x))


def test_empty_inputs(ld, ora):
    h = ora.firdes_kaiser(51, 0.1, 60.0)
    assert ld.ComplexFIRFilter(h)(np.zeros(0, np.complex64)).shape == (0,)
    r = ld.ComplexResampler(rate=0.024, Fc=0.024)
    assert r(np.zeros(0, np.complex64)).shape == (0,)
    assert ld.AGC()(np.zeros(0, np.complex64)).shape == (0,)
    assert ld.AmpModem()(np.zeros(0, np.complex64)).shape == (0,)
    assert ld.ComplexIIRFilter()(np.zeros(0, np.complex64)).shape == (0,)


# ------------------------------------------------------------------ resampler
@pytest.mark.parametrize("rate,m,fc,nf", [(0.024, 20, 0.024, 13), (0.5, 7, 0.2, 32), (1.7, 10, 0.3, 64),
                                          (0.004, 4, 0.002, 8), (3.3, 12, 0.2, 16)])
@pytest.mark.parametrize("cplx", [True, False])
def test_resampler_bitwise(ld, ora, rng, rate, m, fc, nf, cplx):
    rate32 = np.float32(rate)
    cls = ld.ComplexResampler if cplx else ld.RealResampler
    g = cls(rate=rate32, len=m, Fc=np.float32(fc), As=60.0, nfilter=nf)
    o = ora.Resampler(rate32, m, np.float32(fc), 60.0, nf, cplx=cplx)
    n = 30_011
    x = cgauss(rng, n) if cplx else np.float32(rng.standard_normal(n))
    cuts = [0, 1, 2, 41, 5000, 5001, n]
    y = np.concatenate([g(x[s:e]) for s, e in zip(cuts[:-1], cuts[1:])])
    assert_bitwise(y, o(x))


def test_resampler_rate_change_and_reset(ld, ora, rng):
    x = cgauss(rng, 20_000)
    g = ld.ComplexResampler(rate=0.5, Fc=0.2)
    o = ora.Resampler(np.float32(0.5), 20, np.float32(0.2), 60.0, 13)
    y1 = g(x[:10_000])
    r1 = o(x[:10_000])
    g.rate = 0.3
    o.set_rate(np.float32(0.3))
    assert_bitwise(np.concatenate([y1, g(x[10_000:])]), np.concatenate([r1, o(x[10_000:])]))
    g.reset()
    o.reset()
    assert_bitwise(g(x), o(x))


# ------------------------------------------------------------------ NCO
@pytest.mark.parametrize("down", [False, True])
def test_nco_mix_bitwise(ld, ora, rng, down):
    g = ld.NCO("nco")
    o = ora.NCO(0)
    g.freq = o.freq = np.float32(2 * np.pi * 0.05)
    g.phase = o.phase = np.float32(0.3)
    x = cgauss(rng, 100_003)
    f = (lambda q, v: q.mix_down(v)) if down else (lambda q, v: q.mix_up(v))
    y = np.concatenate([f(g, x[:77]), f(g, x[77:])])
    assert_bitwise(y, f(o, x))
    assert g.state() == o.state


def test_nco_call_is_mix_up_and_pll(ld, ora, rng):
    g = ld.NCO()
    o = ora.NCO(0)
    for v in (0.1, -0.2, 0.05):
        g.pll_step(v)
        o.pll_step(np.float32(v))
    g.set_pll_bandwidth(0.01)
    o.pll_set_bandwidth(0.01)
    g.pll_step(0.3)
    o.pll_step(np.float32(0.3))
    assert g.state() == o.state
    x = cgauss(rng, 1000)
    assert_bitwise(g(x), o.mix_up(x))


def test_vco_close(ld, ora, rng):
    g = ld.NCO("vco")
    o = ora.NCO(1)
    g.freq = o.freq = np.float32(0.7)
    x = cgauss(rng, 10_000)
    assert maxrel(g.mix_down(x), o.mix_down(x)) < 1e-6


# ------------------------------------------------------------------ IIR
CHAIN_IIR = dict(filter_type="cheby2", order=8, Fc=np.float32(15000 / 2e6))


def test_iir_exact_bitwise(ld, ora, rng):
    x = cgauss(rng, 50_000)
    g = ld.ComplexIIRFilter(**CHAIN_IIR)
    g.exact = True
    o = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(0.0075), 0.3, 0.7, 60.0))
    y = np.concatenate([g(x[:1000]), g(x[1000:])])
    assert_bitwise(y, o(x))


@pytest.mark.parametrize("ft,bt,order,fc,f0", [("ellip", "lowpass", 6, 0.05, 0.3), ("ellip", "bandpass", 3, 0.05, 0.2),
                                                 ("bessel", "lowpass", 5, 0.02, 0.3), ("bessel", "highpass", 4, 0.1, 0.3)])
def test_iir_ellip_bessel(ld, ora, rng, ft, bt, order, fc, f0):
    # the new prototypes through both IIR paths
    x = cgauss(rng, 200_000)
    o = ora.IIRFilter(prototype=(ft, bt, 1, order, np.float32(fc), f0, 0.7, 60.0))
    g = ld.ComplexIIRFilter(filter_type=ft, band_type=bt, order=order, Fc=fc, F0=f0, Ap=0.7, As=60.0)
    g.exact = True
    assert_bitwise(np.concatenate([g(x[:777]), g(x[777:])]), o(x))
    f = ld.ComplexIIRFilter(filter_type=ft, band_type=bt, order=order, Fc=fc, F0=f0, Ap=0.7, As=60.0)
    o.reset()
    truth = o.execute_f64(x)
    o.reset()
    # fast mode: float64 scan, or the exact speculative path for fast-decaying designs
    err_gpu, err_liquid = maxrel(f(x), truth), maxrel(o(x), truth)
    assert err_gpu <= max(err_liquid, 1e-6), (err_gpu, err_liquid)


@pytest.mark.parametrize("n", [5000, 3 * 65536 + 17, 1 << 20, 1 << 26])
def test_iir_fast_scan_accuracy(ld, ora, rng, n):
    x = cgauss(rng, n)
    g = ld.ComplexIIRFilter(**CHAIN_IIR)
    o = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(0.0075), 0.3, 0.7, 60.0))
    y = np.concatenate([g(x[: n // 3]), g(x[n // 3:])])
    truth = o.execute_f64(x)
    o.reset()
    y32 = o(x)
    err_gpu = maxrel(y, truth)
    err_liquid = maxrel(y32, truth)
    assert err_gpu <= 1e-6, err_gpu                  # float64 scan, rounded once
    assert err_gpu <= err_liquid or err_liquid < 1e-6


def test_iir_real_variants(ld, ora, rng):
    x = np.float32(rng.standard_normal(40_000))
    g = ld.RealIIRFilter(filter_type="butter", order=4, Fc=0.1)
    g.exact = True
    o = ora.IIRFilter(prototype=("butter", "lowpass", 1, 4, 0.1, 0.3, 0.7, 60.0), cplx=False)
    assert_bitwise(g(x), o(x))
    g2 = ld.RLowpassIIR("cheby1", 5, 0.2)
    o2 = ora.IIRFilter(prototype=("cheby1", "lowpass", 1, 5, 0.2, 0.1, 0.5, 20.0), cplx=False)
    assert maxrel(g2(x), o2.execute_f64(x)) < 1e-6


@pytest.mark.parametrize("cplx", [False, True])
def test_iir_blocked_scan_multiblock(ld, ora, rng, cplx):
    """Blocked float64 scan (k_iir_blk, D <= 8) across several 65 536-sample
    blocks and ragged call boundaries, SOS and raw transfer-function forms,
    against the float64 sequential evaluation."""
    n = 5 * 65536 + 333
    x = cgauss(rng, n) if cplx else np.float32(rng.standard_normal(n))
    cuts = [0, 1000, 65536 + 7, 4 * 65536, n]
    g = (ld.ComplexIIRFilter if cplx else ld.RealIIRFilter)(filter_type="cheby2", order=8, Fc=0.02)
    o = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(0.02), 0.3, 0.7, 60.0), cplx=cplx)
    y = np.concatenate([g(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    assert maxrel(y, o.execute_f64(x)) <= 1e-6
    b_, a_ = sps.butter(2, 0.002)             # slow decay (not the speculative-exact path), stable in float32
    gt = (ld.CIIRFilter if cplx else ld.RIIRFilter)(np.float32(b_), np.float32(a_))
    ot = ora.IIRFilter(tf=(np.float32(b_), np.float32(a_)), cplx=cplx)
    yt = np.concatenate([gt(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    assert maxrel(yt, ot.execute_f64(x)) <= 1e-6


def test_tf_iir_and_deemphasis_bitwise(ld, ora, rng):
    x = np.float32(rng.standard_normal(300_001))
    g = ld.DeemphasisFilter(48000)
    b, a = ora.deemphasis_coefs(48000)
    o = ora.IIRFilter(tf=(b, a), cplx=False)
    y = np.concatenate([g(x[:5]), g(x[5:200_000]), g(x[200_000:])])
    assert_bitwise(y, o(x))
    bc = np.float32([0.2, 0.3, 0.1])
    ac = np.float32([1.0, -0.5, 0.2])
    xc = cgauss(rng, 100_000)
    assert_bitwise(ld.CIIRFilter(bc, ac)(xc), ora.IIRFilter(tf=(bc, ac), cplx=True)(xc))


# ------------------------------------------------------------------ AGC
def _am(rng, n, fs, fcar, amp=0.05):
    t = np.arange(n) / fs
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
    s = amp * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * fcar * t + 0.7))
    s = s + amp * 10 ** (-1.5) * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)
    return s.astype(np.complex64)


@pytest.mark.parametrize("n", [3000, 200_000])
def test_agc_bitwise(ld, ora, rng, n):
    x = _am(rng, n, 48000.0, 300.0)
    g = ld.AGC()
    g.lock = False
    g.scale = 0.01
    o = ora.AGC()
    o.scale = np.float32(0.01)
    y = np.concatenate([g(x[: n // 2]), g(x[n // 2:])])
    assert_bitwise(y, o(x))
    assert np.float32(g.gain) == np.float32(o.gain)


def test_agc_speculative_calls_on_two_streams(ld, ora, rng):
    # Calls of >= 4 (W + Wa) samples whose predecessor left a full input history
    # run every chunk from a guess (k_agc_chunks with H > 0), overlapping the
    # previous call's back half on the other stream; chunk 0 is checked against
    # the true state.  Short calls take the sequential path but still feed the
    # history; reset() keeps the history and restarts the state.
    import torch
    x = _am(rng, 260_000, 48000.0, 300.0)
    g = ld.AGC()
    g.lock = False
    g.scale = 0.01
    o = ora.AGC()
    o.scale = np.float32(0.01)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    cuts = [0, 30_000, 60_000, 65_000, 95_000, 125_000, 155_000, 200_000, 260_000]
    outs, refs = [], []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        if i == 6:
            torch.cuda.synchronize()
            g.reset()
            o.reset()
        if i == 4:                       # new bandwidth: new warm-up lengths, the history restarts
            g.bandwidth = 0.02
            o.bandwidth = np.float32(0.02)
        with torch.cuda.stream(streams[i % 2]):
            outs.append(g(xd[a:b]))
        refs.append(o(x[a:b]))
    torch.cuda.synchronize()
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), np.concatenate(refs))
    assert np.float32(g.gain) == np.float32(o.gain)


def test_agc_squelch_and_onrise(ld, ora, rng):
    quiet = cgauss(rng, 4000, 1e-3)
    loud = cgauss(rng, 4000, 1.0)
    x = np.concatenate([loud, quiet, loud, quiet])
    g = ld.AGC()
    g.squelch = True
    g.threshold = -10.0
    rises = []
    g.onRise = lambda: rises.append(1)
    o = ora.AGC()
    o.squelch(True)
    o.threshold = np.float32(-10.0)
    y = g(x)
    ref, st = o(x, return_status=True)
    assert_bitwise(y, ref)
    assert g.status == o.status
    expect = int(np.sum((st[1:] == 2) & (st[:-1] != 2)) + (st[0] == 2))
    assert len(rises) == expect and expect >= 1


def test_agc_lock(ld, ora, rng):
    x = cgauss(rng, 50_000)
    g = ld.AGC()
    g.gain = 2.0
    g.lock = True
    o = ora.AGC()
    o.gain = np.float32(2.0)
    o.lock(True)
    assert_bitwise(g(x), o(x))


# ------------------------------------------------------------------ AmpModem
@pytest.mark.parametrize("carrier", [True, False])
def test_ampmodem_bitwise(ld, ora, rng, carrier):
    x = _am(rng, 40_000, 48000.0, 300.0, amp=1.0)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=carrier)
    o = ora.AmpModem(0.5, "dsb", carrier=carrier)
    y = np.concatenate([g(x[:1234]), g(x[1234:])])
    assert_bitwise(y, o(x))
    assert g.pll_state() == o.pll_state


def test_ampmodem_walk_stats(ld, ora, rng):
    # live walker counters of the last chunk-parallel call; zero after a short (sequential) call
    x = _am(rng, 200_000, 48000.0, 300.0, amp=1.0)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    assert_bitwise(g(x), ora.AmpModem(0.5, "dsb", carrier=True)(x))
    entries, repairs, fallbacks = g._walk_stats()
    assert 0 < repairs < entries < len(x) and fallbacks <= (entries + 63) // 64    # (all of them under LDSP_DEBUG_PLL=2)
    g(x[:1000])
    assert g._walk_stats()[0] >= 0


def test_ampmodem_folded_scan_windows(ld, ora, rng):
    """The carrier chunk scan folded into k_pll_cand (cand_scan_fold): a call of
    193 candidate workgroups (the look-back reads its predecessors 64 at a time:
    four windows), one whose last workgroup is full (chunks a multiple of 64) and
    one whose last workgroup holds a single chunk -- the same output and state as
    the restatement, bit for bit."""
    sizes = [3 * 64 * 64 * 256 + 777, 3 * 64 * 256, 64 * 256 + 1]
    x = _am(rng, sum(sizes), 48000.0, 300.0, amp=1.0)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    o = ora.AmpModem(0.5, "dsb", carrier=True)
    cuts = np.cumsum([0] + sizes)
    y = np.concatenate([g(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    assert_bitwise(y, o(x))
    assert g.pll_state() == o.pll_state


@pytest.mark.parametrize("log2_b", [18, 17])
def test_ampmodem_walk_fallbacks(ld, ora, rng, log2_b):
    # A narrower walker margin (2^19 by default) leaves gaps whose proofs fail:
    # those lane-blocks are redone sample by sample (walk_fallback) and the rest
    # of their walker block continues one lane-block at a time.  Output and final
    # state must stay bit-identical.
    x = _am(rng, 400_000, 48000.0, 300.0, amp=1.0)
    o = ora.AmpModem(0.5, "dsb", carrier=True)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    prev = ld._debug_pll_margin(log2_b)
    try:
        y = g(x)
        stats = g._walk_stats()
    finally:
        ld._debug_pll_margin(prev)
    assert_bitwise(y, o(x))
    assert g.pll_state() == o.pll_state
    entries, repairs, fallbacks = stats
    assert fallbacks > 0 and repairs > 0


@pytest.mark.parametrize("carrier", [True, False])
def test_ampmodem_parallel_calls_on_two_streams(ld, ora, rng, carrier):
    # Long calls run as candidates + walker; consecutive calls alternate torch
    # streams, so call k's candidates overlap call k-1's walk (guess state, two
    # scratch slots, three history buffers).  Short calls interleave the
    # sequential loop.  Everything must stay bit-identical to one sequential run.
    import torch
    # (carrier=False: a DSB-SC signal for the Costas loop, whose candidates start
    # from the true state and whose half-turn-flipped chunks are re-run)
    if carrier:
        x = _am(rng, 6 * 20_000 + 3000, 48000.0, 300.0, amp=1.0)
    else:
        n = 6 * 20_000 + 3000
        t = np.arange(n) / 48000.0
        m = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t)) / 2
        x = (m * np.exp(1j * (2 * np.pi * 100 * t + 0.7)) + 0.02 * cgauss(rng, n)).astype(np.complex64)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=carrier)
    o = ora.AmpModem(0.5, "dsb", carrier=carrier)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    cuts = [0, 20_000, 40_000, 41_000, 61_000, 81_000, 101_000, 121_000, len(x)]
    outs = []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        with torch.cuda.stream(streams[i % 2]):
            outs.append(g(xd[a:b]))
    torch.cuda.synchronize()
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), o(x))
    assert g.pll_state() == o.pll_state


def test_ampmodem_walk_handoff_three_streams(ld, ora, rng):
    # The carrier walker is dispatched as soon as its candidates are ready and
    # waits on the device for the previous call's state (AmpState::wepoch,
    # capi.cpp amp_pll_stage).  Three rotating streams, no host sync between
    # calls, sequential-loop calls (< 1 024 samples) between walks, and a reset
    # in the middle (the epoch is re-uploaded): bitwise to the restatement, one
    # active-time record per walk.
    import torch
    x = _am(rng, 200_000, 48000.0, 300.0, amp=1.0)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    o = ora.AmpModem(0.5, "dsb", carrier=True)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream() for _ in range(3)]
    torch.cuda.synchronize()
    t0, n0 = g._walk_active()
    assert n0 == 0 and t0 == 0
    for half, cuts in enumerate(([0, 30_000, 60_000, 61_000, 90_000, 120_000, 120_500],
                                 [120_500, 150_000, 151_000, 180_000, 200_000])):
        if half == 1:
            g.reset()
            o.reset()
        outs = []
        for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
            with torch.cuda.stream(streams[i % 3]):
                outs.append(g(xd[a:b]))
        torch.cuda.synchronize()
        ref = np.concatenate([o(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
        assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), ref)
        assert g.pll_state() == o.pll_state
    ticks, walks = g._walk_active()
    assert walks == 7                  # the calls of >= 1 024 samples
    assert ticks > 0


def test_ampmodem_walk_timeout_raises(ld, ora, rng):
    # A walker whose wait for the previous call's state times out has walked
    # from a stale state.  The object must raise (LDSP_EHIP) at its next call and
    # state read instead of returning that output silently, the epoch must not go
    # backwards when the late state arrives, and reset must recover the object
    # (ldsp_debug_ampmodem_handoff forces the timeout: a 1 ms bound and an epoch
    # skew of one launch that never comes).
    import torch
    x = _am(rng, 160_000, 48000.0, 300.0, amp=1.0)
    xd = torch.from_numpy(x).cuda()
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    g(xd[:40_000])
    torch.cuda.synchronize()
    g._handoff(100_000, 1)
    g(xd[40_000:80_000])               # dispatched early, waits for an epoch that never comes
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        g(xd[80_000:120_000])
    with pytest.raises(RuntimeError, match="timed out"):
        g.pll_state()
    with pytest.raises(RuntimeError, match="timed out"):
        g(x[80_000:120_000])           # host path too
    g._handoff(0, 0)
    g.reset()
    o = ora.AmpModem(0.5, "dsb", carrier=True)
    outs = [g(xd[a:a + 40_000]) for a in (0, 40_000, 80_000, 120_000)]
    torch.cuda.synchronize()
    ref = np.concatenate([o(x[a:a + 40_000]) for a in (0, 40_000, 80_000, 120_000)])
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), ref)
    assert g.pll_state() == o.pll_state


def test_ampmodem_walk_handoff_random_streams(ld, ora, rng):
    # 48 calls of random sizes (sequential-loop and walker calls mixed, 1 ..
    # 120 000 samples) on a random one of four streams each, two objects sharing
    # the streams, no host sync: every hand-off order the epochs allow, bitwise.
    import torch
    x = _am(rng, 2_000_000, 48000.0, 300.0, amp=1.0)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream() for _ in range(4)]
    objs = [(ld.AmpModem(modulation=0.5, type="dsb", carrier=True), ora.AmpModem(0.5, "dsb", carrier=True))
            for _ in range(2)]
    sizes = rng.choice([1, 700, 1023, 1024, 5000, 40_000, 120_000], size=48)
    cuts = [[0], [0]]
    outs = [[], []]
    torch.cuda.synchronize()
    for i, m in enumerate(sizes):
        j = i % 2
        a = cuts[j][-1]
        b = min(len(x), a + int(m))
        with torch.cuda.stream(streams[int(rng.integers(4))]):
            outs[j].append(objs[j][0](xd[a:b]))
        cuts[j].append(b)
    torch.cuda.synchronize()
    for j, (g, o) in enumerate(objs):
        ref = np.concatenate([o(x[a:b]) for a, b in zip(cuts[j][:-1], cuts[j][1:])])
        assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs[j]]), ref)
        assert g.pll_state() == o.pll_state
        assert g._walk_active()[1] == sum(1 for a, b in zip(cuts[j][:-1], cuts[j][1:]) if b - a >= 1024)


# ------------------------------------------------------------------ helpers either side of the path
def test_bytes_to_iq_bitwise(ld, ora, rng):
    import torch
    raw = rng.integers(-32768, 32767, size=2 * 300_001, dtype=np.int16)
    for b in (raw.tobytes(), raw.tobytes() + b"\x01\x02\x03", b"", b"\x05\x06"):
        assert_bitwise(ld.bytes_to_iq(b), ora.bytes_to_iq(b))
    yd = ld.bytes_to_iq(torch.from_numpy(raw).cuda())
    assert yd.is_cuda and yd.dtype == torch.complex64
    assert_bitwise(yd.cpu().numpy(), ora.bytes_to_iq(raw.tobytes()))


@pytest.mark.parametrize("nd", [0, 1, 7, 1000])
def test_delay_bitwise_streaming(ld, ora, rng, nd):
    g, o = ld.Delay(nd), ora.Delay(nd)
    assert g.delay == nd
    x = cgauss(rng, 20_000)
    r = np.float32(rng.standard_normal(9_000))
    cuts = [0, 1, 5, 600, 601, 4000, 20_000]
    for a, b in zip(cuts[:-1], cuts[1:]):
        assert_bitwise(g(x[a:b]), o(x[a:b]))
        assert_bitwise(g(r[a % 9000:a % 9000 + 300]), o(r[a % 9000:a % 9000 + 300]))
    assert g(np.zeros(3, np.int32)) is None
    g.delay = 3
    o.delay = 3
    assert_bitwise(g(x[:50]), o(x[:50]))


def test_delay_device_tensor(ld, ora, rng):
    import torch
    g, o = ld.Delay(5), ora.Delay(5)
    x = cgauss(rng, 1000)
    y = g(torch.from_numpy(x).cuda())
    assert y.is_cuda and y.dtype == torch.complex64
    assert_bitwise(y.cpu().numpy(), o(x))


@pytest.mark.parametrize("kf", [0.05, 0.3])
def test_freqdem_bitwise(ld, ora, rng, kf):
    x = cgauss(rng, 300_000)
    x[1000:1010] = 0                           # cargf(0) cases
    g, o = ld.FreqDem(kf), ora.FreqDem(kf)
    y = np.concatenate([g(x[:1]), g(x[1:77_777]), g(x[77_777:])])
    assert_bitwise(y, o(x))
    g.reset()
    o.reset()
    assert_bitwise(g(x[:5000]), o(x[:5000]))


def test_broadcast_am_exact_bitwise(ld, ora, rng):
    x = _am(rng, 200_000, 48000.0, 3.0, amp=1.0)
    g = ld.BroadcastAM(slen=25)
    g.exact = True
    o = ora.BroadcastAM(25)
    y = np.concatenate([g(x[:4321]), g(x[4321:])])
    assert_bitwise(y, o(x))
    g.reset()
    o.reset()
    assert_bitwise(g(x[:9000]), o(x[:9000]))


def test_broadcast_am_fast_close(ld, ora, rng):
    # fast mode: PLL stage bit-exact, DC blocker = float64 scan; compared with
    # the same stage evaluated in float64 on the CPU
    x = _am(rng, 1 << 20, 48000.0, 3.0, amp=1.0)
    g = ld.BroadcastAM()
    assert not g.exact
    y = g(x)
    ref = ora.BroadcastAM(25, iir_f64=True)(x)
    assert maxrel(y, ref) < 1e-5


@pytest.mark.parametrize("rate", [0.024, 0.5, 1.3])
def test_default_resamplers_bitwise(ld, ora, rng, rate):
    # RResampler = resamp_rrrf_create_default, CResampler = resamp_crcf_create_default
    x = cgauss(rng, 50_000)
    r = np.float32(rng.standard_normal(50_000))
    gc, oc = ld.CResampler(rate), ora.Resampler(rate, cplx=True, real_taps=True, default=True)
    gr, orr = ld.RResampler(rate), ora.Resampler(rate, cplx=False, default=True)
    assert_bitwise(np.concatenate([gc(x[:999]), gc(x[999:])]), oc(x))
    assert_bitwise(np.concatenate([gr(r[:12345]), gr(r[12345:])]), orr(r))


def _fm(rng, n, fs):
    t = np.arange(n) / fs
    left, right = np.sin(2 * np.pi * 1000 * t), 0.5 * np.sin(2 * np.pi * 3000 * t)
    comp = 0.45 * (left + right) + 0.45 * (left - right) * np.cos(2 * np.pi * 38000 * t) \
        + 0.1 * np.cos(2 * np.pi * 19000 * t)
    x = np.exp(2j * np.pi * (75000 / fs) * np.cumsum(comp)) + 0.01 * cgauss(rng, n)
    return x.astype(np.complex64)


@pytest.mark.parametrize("iq_rate,pcm_rate", [(600000.0, 48000.0), (240000.0, 44100.0)])
def test_fmstereo_bitwise(ld, ora, rng, iq_rate, pcm_rate):
    x = _fm(rng, 150_000, iq_rate)
    g, o = ld.FMStereo(iq_rate=iq_rate, pcm_rate=pcm_rate), ora.FMStereo(iq_rate, pcm_rate)
    y = np.concatenate([g(x[:5000]), g(x[5000:5001]), g(x[5001:])])
    assert_bitwise(y, o(x))
    assert g.state() == o.state
    g.reset()
    o.reset()
    assert_bitwise(g(x[:20_000]), o(x[:20_000]))


def test_fmstereo_noise_and_special_operands(ld, ora, rng):
    """The candidate evaluation (k_fm_pll) on inputs that
    leave the predicted window often (pure noise) and on exact zeros / repeated
    samples (the discriminator output s = 0, so atan2 sees signed zeros)."""
    x = cgauss(rng, 120_000)
    x[1000:1400] = 0                      # s == 0 over a run
    x[5000:5300] = x[5000]                # repeated sample: s == 0 again
    x[7000:7010] = np.complex64(1e-30)    # tiny magnitudes
    g, o = ld.FMStereo(), ora.FMStereo()
    y = np.concatenate([g(x[:60_001]), g(x[60_001:])])
    assert_bitwise(y, o(x))
    assert g.state() == o.state


def test_fmstereo_device_tensor(ld, ora, rng):
    import torch
    x = _fm(rng, 50_000, 600000.0)
    y = ld.FMStereo()(torch.from_numpy(x).cuda())
    assert y.is_cuda and y.dtype == torch.float32
    assert_bitwise(y.cpu().numpy(), ora.FMStereo()(x))

# ------------------------------------------------------------------ chain
def _chain(ld, exact):
    bandpass = ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    bandpass.exact = exact
    resample = ld.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    am = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    audio = ld.DeemphasisFilter(48000)
    agc = ld.AGC()
    agc.lock = False
    agc.scale = 0.01

    def run(iq):
        return audio(am(agc(resample(bandpass(iq)))))
    return run


def test_amradio_exact_bitwise(ld, ora, rng):
    x = _am(rng, 1 << 18, 2e6, 1200.0, amp=0.1)
    run = _chain(ld, exact=True)
    y = np.concatenate([run(x[i:i + 65536]) for i in range(0, len(x), 65536)])
    assert_bitwise(y, ora.AMRadio()(x))


def test_amradio_two_streams_bitwise(ld, ora, rng):
    # the bench's pipelined form: consecutive chain calls on alternating streams
    import torch
    x = _am(rng, 1 << 19, 2e6, 1200.0, amp=0.1)
    run = _chain(ld, exact=True)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    outs = []
    for i, k in enumerate(range(0, len(x), 1 << 17)):
        with torch.cuda.stream(streams[i % 2]):
            outs.append(run(xd[k:k + (1 << 17)]))
    torch.cuda.synchronize()
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), ora.AMRadio()(x))


# (the fast-mode chain gate lives in tests/test_gpu_chain.py, beside the
# benchmarked-configuration test)


def test_device_tensor_path_matches_numpy(ld, ora, rng):
    import torch
    x = cgauss(rng, 100_000)
    h = ora.firdes_kaiser(127, 0.1, 60.0)
    a, b = ld.ComplexFIRFilter(h), ld.ComplexFIRFilter(h)
    yd = a(torch.from_numpy(x).cuda())
    assert yd.is_cuda and yd.dtype == torch.complex64
    assert_bitwise(yd.cpu().numpy(), b(x))
    r1 = ld.ComplexResampler(rate=0.024, Fc=0.024)
    r2 = ld.ComplexResampler(rate=0.024, Fc=0.024)
    assert_bitwise(r1(torch.from_numpy(x).cuda()).cpu().numpy(), r2(x))


@pytest.mark.parametrize("cplx", [True, False])
@pytest.mark.parametrize("order", [1, 2, 5, 8, 16])
def test_iir_exact_pipeline_call_sizes(ld, ora, rng, cplx, order):
    """Exact mode of an SOS cascade (k_iir_sect: a wave per section, one
    workgroup per component, 512-sample tiles through 4-tile LDS rings) across
    calls of every awkward size: shorter than a 32-sample group, odd, one tile
    +- 1, a ring +- 1, several rings; bit-identical to the sequential
    restatement and its state carried across."""
    sizes = [1, 2, 3, 13, 14, 15, 31, 32, 33, 511, 512, 513, 2047, 2048, 2049, 4095, 6000, 3, 40_000]
    n = sum(sizes)
    x = cgauss(rng, n) if cplx else np.float32(rng.standard_normal(n))
    cls = ld.ComplexIIRFilter if cplx else ld.RealIIRFilter
    g = cls(filter_type="cheby2", order=order, Fc=np.float32(0.02))
    g.exact = True
    g._scan_path(1)              # never the speculative chunks: the sequential exact kernel
    o = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, order, np.float32(0.02), 0.3, 0.7, 60.0), cplx=cplx)
    out, a = [], 0
    for k in sizes:
        out.append(g(x[a:a + k]))
        a += k
    assert_bitwise(np.concatenate(out), o(x))


def test_iir_exact_chain_filter_large(ld, ora, rng):
    """The chain's cheby2 order-8 band filter in exact mode on 4 Mi IQ samples in
    one call (k_iir_sect), bit-identical to the restatement."""
    import torch
    n = 1 << 22
    x = cgauss(rng, n, 0.1)
    g = ld.ComplexIIRFilter(**CHAIN_IIR)
    g.exact = True
    o = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(0.0075), 0.3, 0.7, 60.0))
    y = g(torch.from_numpy(x).cuda()).cpu().numpy()
    assert_bitwise(y, o(x))
