"""Fused and restructured kernels at the BASELINE sizes.

  * NCO mix fused into the complex FIR (BASELINE config 3: NCO.mix_down ->
    255-tap ComplexFIRFilter; reference src/nco.hpp:74-80 then
    src/firfilter.hpp:29-35): liquiddsp.mix_down_filter / mix_up_filter give
    the same bits as the two calls on the GPU (same call boundaries, so the same
    overlap-save windows), advance both objects' state identically, and stay
    within SURVEY 8(d)'s 1e-6 of the restatement.
  * The tile resampler (span streamed into LDS) at BASELINE config 2 size:
    bit-identical to the restatement on 64 Mi samples in one call.
"""
import numpy as np
import pytest

from conftest import cgauss, maxrel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.complex64 else np.uint32)


@pytest.mark.parametrize("L", [51, 127, 255])
@pytest.mark.parametrize("down", [True, False])
def test_mix_filter_equals_two_calls(ld, ora, rng, L, down):
    h = ora.firdes_kaiser(L, 0.05, 60.0)
    x = cgauss(rng, 200_003)
    cuts = [0, 1, 700, 70_000, 70_001, len(x)]

    def pair():
        nco = ld.NCO("nco")
        nco.freq = np.float32(2 * np.pi * 0.05)
        nco.phase = np.float32(0.25)
        return nco, ld.ComplexFIRFilter(h)

    n1, f1 = pair()
    n2, f2 = pair()
    fused = ld.mix_down_filter if down else ld.mix_up_filter
    y = np.concatenate([fused(n1, f1, x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    ref = np.concatenate([f2(n2.mix_down(x[a:b]) if down else n2.mix_up(x[a:b])) for a, b in zip(cuts[:-1], cuts[1:])])
    assert np.array_equal(bits(y), bits(ref))
    assert n1.state() == n2.state()
    on = ora.NCO(0)
    on.freq = np.float32(2 * np.pi * 0.05)
    on.phase = np.float32(0.25)
    oref = ora.FIRFilter(h, cplx=True)(on.mix_down(x) if down else on.mix_up(x))
    assert maxrel(y, oref) <= 1e-6
    # the filter's history holds mixed samples: an unfused call afterwards continues the same stream
    x2 = cgauss(rng, 5000)
    assert np.array_equal(bits(f1(n1.mix_down(x2) if down else n1.mix_up(x2))),
                          bits(f2(n2.mix_down(x2) if down else n2.mix_up(x2))))


@pytest.mark.parametrize("case", ["exact", "direct", "vco"])
def test_mix_filter_unfused_paths(ld, ora, rng, case):
    h = ora.firdes_kaiser(127, 0.05, 60.0)
    x = cgauss(rng, 50_000)
    ncos, firs = [], []
    for _ in range(2):
        nco = ld.NCO("vco" if case == "vco" else "nco")
        nco.freq = np.float32(0.3)
        f = ld.ComplexFIRFilter(h)
        if case != "vco":
            f.mode = case
        ncos.append(nco)
        firs.append(f)
    y = np.concatenate([ld.mix_down_filter(ncos[0], firs[0], x[:1234]), ld.mix_down_filter(ncos[0], firs[0], x[1234:])])
    ref = np.concatenate([firs[1](ncos[1].mix_down(x[:1234])), firs[1](ncos[1].mix_down(x[1234:]))])
    assert np.array_equal(bits(y), bits(ref))
    with pytest.raises(TypeError):
        ld.mix_down_filter(ncos[0], ld.RealFIRFilter(h), x)


def test_mix_filter_config3_device(ld, ora):
    """BASELINE config 3 shape on device tensors (64 Mi here; the bench runs 256 Mi):
    fused == unfused bit for bit over a ragged two-call stream."""
    import torch
    n = 64 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    xd = torch.complex(torch.randn(n, generator=g, device="cuda"), torch.randn(n, generator=g, device="cuda"))
    h = ora.firdes_kaiser(255, 0.05, 60.0)
    out = []
    for fused in (True, False):
        nco = ld.NCO("nco")
        nco.freq = np.float32(2 * np.pi * 0.05)
        f = ld.ComplexFIRFilter(h)
        parts = [xd[:12_345_677], xd[12_345_677:]]
        ys = [ld.mix_down_filter(nco, f, p) if fused else f(nco.mix_down(p)) for p in parts]
        out.append(torch.cat(ys))
    torch.cuda.synchronize()
    assert torch.equal(out[0].view(torch.float32), out[1].view(torch.float32))


def test_resampler_config2_full_size(ld, ora):
    """BASELINE config 2: ComplexResampler(48k/2M) on 64 Mi samples in one call."""
    import torch
    n = 64 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(2)
    xd = torch.complex(torch.randn(n, generator=g, device="cuda"), torch.randn(n, generator=g, device="cuda"))
    r = ld.ComplexResampler(rate=np.float32(48000 / 2000000), Fc=np.float32(48000 / 2000000))
    y = r(xd).cpu().numpy()
    ref = ora.Resampler(np.float32(48000 / 2000000), 20, np.float32(48000 / 2000000), 60.0, 13)(xd.cpu().numpy())
    assert y.shape == ref.shape == (1610613,)
    assert np.array_equal(bits(y), bits(ref))


def test_mix_filter_config3_full_size_vs_oracle(ld, ora):
    """BASELINE config 3 at its full size: NCO.mix_down -> 255-tap ComplexFIRFilter
    on 256 Mi samples in one call (reference src/nco.hpp:74-80 then
    src/firfilter.hpp:29-35).  Fused == unfused bit for bit over the whole
    stream, and within SURVEY 8(d)'s 1e-6 of the restatement on a 1 Mi prefix
    and on a 1 Mi window at the end (the restatement's NCO advanced to the
    window's start, its FIR fed the 254 samples before it)."""
    import torch
    n, w, L = 256 << 20, 1 << 20, 255
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    xd = torch.complex(torch.randn(n, generator=g, device="cuda"), torch.randn(n, generator=g, device="cuda"))
    h = ora.firdes_kaiser(L, 0.05, 60.0)
    freq = np.float32(2 * np.pi * 0.05)
    out = []
    for fused in (True, False):
        nco = ld.NCO("nco")
        nco.freq = freq
        f = ld.ComplexFIRFilter(h)
        out.append(ld.mix_down_filter(nco, f, xd) if fused else f(nco.mix_down(xd)))
    torch.cuda.synchronize()
    assert torch.equal(out[0].view(torch.float32), out[1].view(torch.float32))
    y = out[0]
    del out[1]
    # prefix
    on = ora.NCO(0)
    on.freq = freq
    dtheta = on.state[1]
    ref = ora.FIRFilter(h, cplx=True)(on.mix_down(xd[:w].cpu().numpy()))
    assert maxrel(y[:w].cpu().numpy(), ref) <= 1e-6
    # tail window [n - w, n): restatement started L - 1 samples early
    a = n - w - (L - 1)
    on = ora.NCO(0)
    on.freq = freq
    on.state = ((a * dtheta) & 0xFFFFFFFF, dtheta)
    ref = ora.FIRFilter(h, cplx=True)(on.mix_down(xd[a:].cpu().numpy()))[L - 1:]
    assert maxrel(y[n - w:].cpu().numpy(), ref) <= 1e-6


# ------------------------------------------------------------------ IIR -> resampler
def _iir_rs(ld, cplx, exact=False, fc=15000 / 2e6, rate=48000 / 2e6):
    if cplx:
        f = ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=fc)
        r = ld.ComplexResampler(rate=rate, Fc=rate)
    else:
        f = ld.RealIIRFilter(filter_type="cheby2", order=8, Fc=fc)
        r = ld.RealResampler(rate=rate, Fc=rate)
    f.exact = exact
    return f, r


@pytest.mark.parametrize("cplx", [True, False])
@pytest.mark.parametrize("exact", [False, True])
def test_filter_resample_equals_two_calls(ld, rng, cplx, exact):
    """liquiddsp.filter_resample(iir, resampler, x) == resampler(iir(x)) bit for
    bit on ragged device calls (a unit boundary's window from the side buffer, the
    call's first window from the resampler history, calls shorter than the
    window), and both objects continue the same streams afterwards (IIR state,
    resampler phase and history).  exact: the two-call fallback."""
    import torch
    n = (1 << 20) + 12_345
    x = cgauss(rng, n) if cplx else rng.standard_normal(n).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    cuts = [0, 1, 30, 2048, 2048 + 39, 4096 + 40, 70_001, 600_000, n]
    fa, ra = _iir_rs(ld, cplx, exact)
    fb, rb = _iir_rs(ld, cplx, exact)
    ys, refs = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        ys.append(ld.filter_resample(fa, ra, xd[a:b]))
        refs.append(rb(fb(xd[a:b])))
    y, ref = torch.cat(ys).cpu().numpy(), torch.cat(refs).cpu().numpy()
    assert y.shape == ref.shape and y.size > 0.023 * n
    eq = bits(y) == bits(ref)
    assert eq.all(), f"{(~eq).sum()} of {eq.size} differ; first at {int(np.argmin(eq))}"
    x2 = torch.from_numpy(cgauss(rng, 50_000) if cplx else rng.standard_normal(50_000).astype(np.float32)).cuda()
    assert torch.equal(ra(fa(x2)).view(torch.int32), rb(fb(x2)).view(torch.int32))


def test_filter_resample_64Mi_and_host(ld, rng):
    """The bench chain's front at the BASELINE size (64 Mi in one call) and the
    numpy path: the same bits as the two calls."""
    import torch
    import bench
    n = 64 << 20
    xd = bench.synth_channel(n, 0, torch.device("cuda", 0))
    fa, ra = _iir_rs(ld, True)
    fb, rb = _iir_rs(ld, True)
    y = ld.filter_resample(fa, ra, xd)
    ref = rb(fb(xd))
    assert y.shape == ref.shape and y.numel() > 1_600_000
    assert torch.equal(y.view(torch.int32), ref.view(torch.int32))
    xh = xd[:300_001].cpu().numpy()
    yh = ld.filter_resample(fa, ra, xh)
    assert isinstance(yh, np.ndarray)
    assert np.array_equal(bits(yh), bits(rb(fb(xh))))


def test_filter_resample_rotating_streams(ld, rng):
    """Consecutive fused calls on four rotating streams with no host sync: a
    call's units start when the previous call's units end (the filter state),
    under the previous call's edges, with the units' heads / tails in two
    alternating side slots.  Seven calls (each slot reused three times, unit and
    call boundaries of every kind), bit for bit against the two calls on one
    stream, and the objects continue alike afterwards."""
    import torch
    n = 6 * 262_144 + 777
    x = cgauss(rng, n)
    xd = torch.from_numpy(x).cuda()
    cuts = [0, 262_144, 300_000, 2 * 262_144 + 5, 3 * 262_144, 1_000_001, 5 * 262_144 + 64, n]
    fa, ra = _iir_rs(ld, True)
    fb, rb = _iir_rs(ld, True)
    streams = [torch.cuda.Stream() for _ in range(4)]
    torch.cuda.synchronize()
    ys = []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        with torch.cuda.stream(streams[i % 4]):        # ordered by the objects alone
            ys.append(ld.filter_resample(fa, ra, xd[a:b]))
    torch.cuda.synchronize()
    refs = [rb(fb(xd[a:b])) for a, b in zip(cuts[:-1], cuts[1:])]
    y, ref = torch.cat(ys).cpu().numpy(), torch.cat(refs).cpu().numpy()
    assert y.shape == ref.shape and y.size > 0.023 * n
    eq = bits(y) == bits(ref)
    assert eq.all(), f"{(~eq).sum()} of {eq.size} differ; first at {int(np.argmin(eq))}"
    x2 = torch.from_numpy(cgauss(rng, 50_000)).cuda()
    assert torch.equal(ra(fa(x2)).view(torch.int32), rb(fb(x2)).view(torch.int32))


@pytest.mark.parametrize("rate,fc", [(0.5, 0.2), (1.7, 0.3)])
def test_filter_resample_other_rates(ld, rng, rate, fc):
    """Rates where a unit boundary is straddled by many resampler windows (the
    edge kernel's loop after its prefetched first output) and where a unit holds
    more than 64 outputs (the fused kernel's output loop): the same bits as the
    two calls, complex (cccf taps) and real, and the streams continue alike."""
    import torch
    n = 300_007
    for cplx in (True, False):
        x = cgauss(rng, n) if cplx else rng.standard_normal(n).astype(np.float32)
        xd = torch.from_numpy(x).cuda()
        mk = (lambda: (ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2e6),
                       ld.ComplexResampler(rate=rate, Fc=fc))) if cplx else \
             (lambda: (ld.RealIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2e6),
                       ld.RealResampler(rate=rate, Fc=fc)))
        fa, ra = mk()
        fb, rb = mk()
        for a, b in ((0, 5000), (5000, 200_001), (200_001, n)):
            y = ld.filter_resample(fa, ra, xd[a:b])
            ref = rb(fb(xd[a:b]))
            assert y.shape == ref.shape
            assert torch.equal(y.view(torch.int32), ref.view(torch.int32)), (cplx, a, b)


@pytest.mark.parametrize("exact", [False, True])
def test_filter_resample_vs_oracle_1Mi(ld, ora, exact):
    """filter_resample against the restatement directly (not only against the two
    GPU calls), on a 1 Mi prefix of the bench channel: exact mode (the two-call
    fallback) bit for bit against the float32 restatement (IIR -> resampler);
    fast mode (the fused modal scan) against the restatement's float64 IIR
    followed by its resampler, within the SURVEY 8(d) 1e-6 bound (two float64
    evaluations of one filter, each rounded once to float32)."""
    import torch
    import bench
    n = 1 << 20
    xd = bench.synth_channel(n, 0, torch.device("cuda", 0))
    x = xd.cpu().numpy()
    f = ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    r = ld.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    f.exact = exact
    y = torch.cat([ld.filter_resample(f, r, xd[:300_000]), ld.filter_resample(f, r, xd[300_000:])]).cpu().numpy()
    oi = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(15000 / 2000000), 0.3, 0.7, 60.0))
    orr = ora.Resampler(np.float32(48000 / 2000000), m=20, fc=np.float32(48000 / 2000000), npfb=13, cplx=True)
    ref = orr(oi(x) if exact else oi.execute_f64(x))
    assert y.shape == ref.shape and y.size > 25_000
    if exact:
        assert np.array_equal(bits(y), bits(ref))
    else:
        assert maxrel(y, ref) <= 1e-6, maxrel(y, ref)
