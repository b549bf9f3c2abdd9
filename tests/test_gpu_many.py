"""Batched multi-channel execution (liquiddsp.execute_many / filter_resample_many,
C ABI ldsp_*_many): C independent AMRadio chains (the
reference's per-channel SDR callback, README.md:53-58) stepped with one kernel
launch per stage for all channels.  Every channel's output must equal, bit for
bit, what its own chain produces with the ordinary per-object calls -- for 8 and
16 channels (16 needs two merged launches for the modal IIR's 432-byte
arguments) over consecutive steps -- and the exact back half (AGC -> AmpModem ->
de-emphasis) must equal the CPU restatement on each channel."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CARRIERS = [1200.0, -1200.0, 900.0, -900.0, 600.0, -600.0, 300.0, -300.0]


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def _synth(n, c):
    rng = np.random.default_rng(100 + c)
    t = np.arange(n) / 2e6
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
    s = 0.1 * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * CARRIERS[c % 8] * t + 0.3 * c))
    return (s + 0.00224 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)


class Radio:
    def __init__(self, L):
        self.iir = L.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2e6)
        self.rs = L.ComplexResampler(rate=48000 / 2e6, Fc=48000 / 2e6)
        self.agc = L.AGC()
        self.agc.lock = False
        self.agc.scale = 0.01
        self.am = L.AmpModem(modulation=0.5, type="dsb", carrier=True)
        self.de = L.DeemphasisFilter(48000)

    def __call__(self, L, x):
        return self.de(self.am(self.agc(L.filter_resample(self.iir, self.rs, x))))


def _many_step(L, radios, xs):
    a = L.filter_resample_many([r.iir for r in radios], [r.rs for r in radios], xs)
    b = L.execute_many([r.agc for r in radios], a)
    c = L.execute_many([r.am for r in radios], b)
    return L.execute_many([r.de for r in radios], c), b


@pytest.mark.parametrize("C", [8, 16])
def test_many_chain_equals_per_channel(ld, C):
    import torch
    n, steps = 1 << 21, 3
    xs = [torch.from_numpy(_synth(n * steps, c)).cuda() for c in range(C)]
    many = [Radio(ld) for _ in range(C)]
    single = [Radio(ld) for _ in range(C)]
    for k in range(steps):
        blk = [x[k * n:(k + 1) * n] for x in xs]
        got, _ = _many_step(ld, many, blk)
        ref = [single[c](ld, blk[c]) for c in range(C)]
        torch.cuda.synchronize()
        for c in range(C):
            g, r = got[c].cpu().numpy(), ref[c].cpu().numpy()
            assert g.shape == r.shape and np.array_equal(g.view(np.uint32), r.view(np.uint32)), (k, c)
    for c in range(C):          # the objects' states advanced alike
        assert many[c].am.pll_state() == single[c].am.pll_state()
        assert np.float32(many[c].agc.gain) == np.float32(single[c].agc.gain)


def test_many_back_half_vs_oracle(ld, ora):
    import torch
    C, n = 8, 60_000
    pcm = []
    for c in range(C):        # AGC inputs: resampled AM at 48 kS/s (the oracle's own front)
        r = ora.Resampler(np.float32(48000 / 2e6), m=20, fc=np.float32(48000 / 2e6), npfb=13, cplx=True)
        pcm.append(r(_synth(int(n / 0.024) + 64, c))[:n].astype(np.complex64))
    agcs, ams, des = [], [], []
    for _ in range(C):
        g = ld.AGC()
        g.lock = False
        g.scale = 0.01
        agcs.append(g)
        ams.append(ld.AmpModem(modulation=0.5, type="dsb", carrier=True))
        des.append(ld.DeemphasisFilter(48000))
    outs = []
    for a, b in ((0, 25_000), (25_000, n)):       # two calls: state carried across many-calls
        xs = [torch.from_numpy(p[a:b]).cuda() for p in pcm]
        y = ld.execute_many(des, ld.execute_many(ams, ld.execute_many(agcs, xs)))
        outs.append([t.cpu().numpy() for t in y])
    for c in range(C):
        g = ora.AGC()
        g.scale = np.float32(0.01)
        am = ora.AmpModem(0.5, "dsb", True)
        de = ora.IIRFilter(tf=ora.deemphasis_coefs(48000.0), cplx=False)
        ref = de(am(g(pcm[c])))
        got = np.concatenate([outs[0][c], outs[1][c]])
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), c


def test_many_merges_launches(ld):
    # one merged walk for all channels: the profiler sees one k_pll_walk launch per many-call
    import torch
    C, n = 8, 40_000
    ams = [ld.AmpModem(modulation=0.5, type="dsb", carrier=True) for _ in range(C)]
    xs = [torch.from_numpy((_synth(int(n / 0.024), c)[::42][:n] * 5).astype(np.complex64)).cuda() for c in range(C)]
    ld.execute_many(ams, xs)
    torch.cuda.synchronize()
    ld._profile_reset()
    ld._profile_enable(True)
    ld.execute_many(ams, xs)
    torch.cuda.synchronize()
    ld._profile_enable(False)
    rep = ld._profile_report()
    assert rep["k_pll_walk"][0] == 1 and rep["k_pll_cand"][0] == 1, rep


def test_many_rejects_bad_input(ld):
    import torch
    g = ld.AGC()
    x = torch.zeros(10_000, dtype=torch.complex64, device="cuda")
    with pytest.raises(ValueError):
        ld.execute_many([g, g], [x, x])                      # the same object twice
    with pytest.raises(ValueError):
        ld.execute_many([g, ld.AGC()], [x, x[:5000]])        # unequal lengths
    with pytest.raises(ValueError):
        ld.execute_many([g], [x.cpu().numpy()])              # host arrays


def test_many_exact_iir_merged_bitwise(ld, ora):
    # exact-mode SOS cascades (the chain's cheby2 order 8, k_iir_sect: one workgroup
    # per (object, component)) run as ONE merged launch for all channels: bitwise to
    # the per-object calls over calls of awkward sizes (state carried across), and
    # to the restatement on two channels
    import torch
    C = 8
    sizes = [100_000, 513, 31, 70_001]
    n = sum(sizes)
    xh = [_synth(n, c) for c in range(C)]
    xs = [torch.from_numpy(x).cuda() for x in xh]
    fa = [ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2e6) for _ in range(C)]
    fb = [ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2e6) for _ in range(C)]
    for f in fa + fb:
        f.exact = True
    got = [[] for _ in range(C)]
    a = 0
    for i, m in enumerate(sizes):
        blk = [x[a:a + m] for x in xs]
        if i == 1:
            ld._profile_reset()
            ld._profile_enable(True)
        outs = ld.execute_many(fa, blk)
        if i == 1:
            torch.cuda.synchronize()
            ld._profile_enable(False)
            assert ld._profile_report()["k_iir_sect"][0] == 1, ld._profile_report()
        for c in range(C):
            got[c].append(outs[c])
            ref = fb[c](blk[c])
            assert torch.equal(outs[c].view(torch.int64), ref.view(torch.int64)), (i, c)
        a += m
    for c in (0, C - 1):
        o = ora.IIRFilter(prototype=("cheby2", "lowpass", 1, 8, np.float32(15000 / 2e6), 0.3, 0.7, 60.0))
        y = torch.cat(got[c]).cpu().numpy()
        assert np.array_equal(y.view(np.uint64), o(xh[c]).view(np.uint64)), c


def test_many_unbatchable_paths_fall_back(ld):
    # exact-mode transfer-function IIR filters and single-sideband AmpModems take
    # paths without merged kernels: the many-call runs the objects one after
    # another, same bits
    import torch
    import scipy.signal as sps
    C, n = 3, 200_000
    xs = [torch.from_numpy(_synth(n, c)).cuda() for c in range(C)]
    b, a = sps.butter(4, 0.002)
    fa = [ld.CIIRFilter(np.float32(b), np.float32(a)) for _ in range(C)]
    fb = [ld.CIIRFilter(np.float32(b), np.float32(a)) for _ in range(C)]
    for f in fa + fb:
        f.exact = True
        f._scan_path(1)              # not the speculative chunks: the sequential transfer-function kernel
    got = ld.execute_many(fa, xs)
    for c in range(C):
        assert torch.equal(got[c].view(torch.int64), fb[c](xs[c]).view(torch.int64)), c
    ma = [ld.AmpModem(modulation=0.5, type="usb", carrier=True) for _ in range(C)]
    mb = [ld.AmpModem(modulation=0.5, type="usb", carrier=True) for _ in range(C)]
    got = ld.execute_many(ma, [x[:20_000] * 5 for x in xs])
    for c in range(C):
        assert torch.equal(got[c].view(torch.int32), mb[c](xs[c][:20_000] * 5).view(torch.int32)), c


def test_many_exact_chain_vs_oracle(ld, ora):
    # the exact (bit-identical) AMRadio chain for several channels at once, as
    # bench.py's exact_channels_batched steps it: the channels' exact IIRs in one
    # merged launch, the resamplers per channel, the back half batched -- every
    # channel bit for bit the restatement's AMRadio on its own input, over two calls
    import torch
    C, n = 3, 1 << 20
    xh = [_synth(2 * n, c) for c in range(C)]
    xs = [torch.from_numpy(x).cuda() for x in xh]
    rs = [Radio(ld) for _ in range(C)]
    for r in rs:
        r.iir.exact = True
    outs = [[] for _ in range(C)]
    for k in range(2):
        ys = ld.execute_many([r.iir for r in rs], [x[k * n:(k + 1) * n] for x in xs])
        zs = [r.rs(y) for r, y in zip(rs, ys)]
        got = ld.execute_many([r.de for r in rs], ld.execute_many([r.am for r in rs],
                                                                    ld.execute_many([r.agc for r in rs], zs)))
        for c in range(C):
            outs[c].append(got[c])
    torch.cuda.synchronize()
    for c in range(C):
        o = ora.AMRadio()
        ref = np.concatenate([o(xh[c][k * n:(k + 1) * n]) for k in range(2)])
        y = torch.cat(outs[c]).cpu().numpy()
        assert y.shape == ref.shape and np.array_equal(y.view(np.uint32), ref.view(np.uint32)), c
