"""Small calls (the reference README's SDR callback granularity, README.md:53-62):
65 536 IQ samples per call -> ~1 573 PCM samples through the AGC and the AmpModem.

At that size the AGC runs its chunks from the true state with the approximate
loop up to each chunk (k_agc_chunks, tsa mode) and the carrier-mode AmpModem
PLL runs the one-wave candidate-kick loop (k_pll_seqc, below 2 048 samples;
its own tests are in test_gpu_pll_seqc.py; Costas mode runs candidates + walk
from 1 280 samples); both must stay bit-identical to the sequential
restatement, including the calls whose approximate trajectory left the exact
one (a one-wave call -- up to 64 chunks -- re-runs such chunks inside
k_agc_chunks, a larger one in k_agc_runfix / k_agc_verify), and across calls
rotating over several streams.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def assert_bitwise(y, ref):
    assert y.shape == ref.shape, (y.shape, ref.shape)
    eq = np.asarray(y).view(np.uint32) == np.asarray(ref).view(np.uint32)
    assert eq.all(), f"{(~eq).sum()} of {eq.size} differ; first at {int(np.argmin(eq))}"


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def _am(rng, n, fs, fc, level=0.1):
    t = np.arange(n) / fs
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t)) / 2
    env = level * (1 + 0.5 * msg) * (1 + 0.8 * (np.sin(2 * np.pi * 0.7 * t) > 0))   # level steps
    x = env * np.exp(1j * 2 * np.pi * fc / fs * np.arange(n))
    x = x + 0.003 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    return x.astype(np.complex64)


def test_agc_small_calls_bitwise(ld, ora, rng):
    """Many calls of 320 .. 2232 samples (the tsa range) on three rotating streams."""
    import torch
    x = _am(rng, 300_000, 48000.0, 300.0)
    sizes = rng.integers(320, 2233, 200)
    cuts = np.concatenate([[0], np.cumsum(sizes)])
    cuts = cuts[cuts <= len(x)]
    g = ld.AGC()
    g.lock = False
    g.scale = 0.01
    o = ora.AGC()
    o.scale = np.float32(0.01)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream() for _ in range(3)]
    torch.cuda.synchronize()
    outs, refs = [], []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        with torch.cuda.stream(streams[i % 3]):
            outs.append(g(xd[a:b]))
        refs.append(o(x[a:b]))
    torch.cuda.synchronize()
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), np.concatenate(refs))
    assert np.float32(g.gain) == np.float32(o.gain)


def test_agc_small_calls_squelch(ld, ora, rng):
    """tsa mode carries the squelch mode / timer through the approximate run too."""
    quiet = (1e-3 * (rng.standard_normal(30_000) + 1j * rng.standard_normal(30_000))).astype(np.complex64)
    loud = _am(rng, 30_000, 48000.0, 500.0, level=1.0)
    x = np.concatenate([loud, quiet, loud, quiet])
    g = ld.AGC()
    g.squelch = True
    g.threshold = -10.0
    o = ora.AGC()
    o.squelch(True)
    o.threshold = np.float32(-10.0)
    ys, rs = [], []
    for a in range(0, len(x), 1500):
        ys.append(g(x[a:a + 1500]))
        rs.append(o(x[a:a + 1500]))
    assert_bitwise(np.concatenate(ys), np.concatenate(rs))
    assert g.status == o.status


def test_amradio_readme_blocks_rotating_streams(ld, ora):
    """The README loop on 65 536-sample blocks (exact IIR, so the whole chain is
    bit-identical), 48 blocks over 3 rotating streams vs the restatement."""
    import torch
    import bench
    blk, nblk = 65536, 48
    xd = bench.synth_channel(blk * nblk, 0, torch.device("cuda", 0))
    x = xd.cpu().numpy()
    radio = bench.AMRadio(ld)
    radio.bandpass.exact = True
    streams = [torch.cuda.Stream() for _ in range(3)]
    torch.cuda.synchronize()
    outs = []
    for i in range(nblk):
        with torch.cuda.stream(streams[i % 3]):
            outs.append(radio(xd[i * blk:(i + 1) * blk]))
    torch.cuda.synchronize()
    ref = ora.AMRadio()
    refs = [ref(x[i * blk:(i + 1) * blk]) for i in range(nblk)]
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), np.concatenate(refs))


@pytest.mark.parametrize("bw", [1e-3, 1e-4])
def test_agc_small_calls_low_bandwidth(ld, ora, rng, bw):
    """At bandwidth 1e-3 (1e-4) the chunk-parallel threshold grows to ~62 k
    (~617 k) samples, so calls up to that length run tsa mode: every chunk
    approximates from the true state over up to that many samples.  Calls at the
    top of that range stay bit-identical (a trajectory that leaves the exact one
    is re-run); scripts/agc_lowbw.py times them."""
    s = 10 if bw < 5e-4 else 1
    x = _am(rng, 200_000 * s, 48000.0, 300.0)
    g = ld.AGC()
    g.bandwidth = bw
    g.lock = False
    g.scale = 0.01
    o = ora.AGC()
    o.bandwidth = np.float32(bw)
    o.scale = np.float32(0.01)
    cuts = [c * s for c in (0, 10_000, 70_000, 130_000, 190_000, 200_000)]
    ys = [g(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    rs = [o(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    assert_bitwise(np.concatenate(ys), np.concatenate(rs))


@pytest.mark.parametrize("squelch", [False, True])
def test_agc_small_calls_inkernel_repair(ld, ora, rng, squelch):
    """One-wave small calls check and repair their chunks in the chunk kernel
    (no flag / repair / verify launches).  With every chunk's start state
    pushed 1 ulp off (test hook) each chunk is re-run there, in order, from its
    predecessor's end state: still bit-identical, squelch mode and timer
    included, and so are the unperturbed calls after it."""
    loud = _am(rng, 40_000, 48000.0, 300.0)
    quiet = (1e-3 * (rng.standard_normal(20_000) + 1j * rng.standard_normal(20_000))).astype(np.complex64)
    x = np.concatenate([loud, quiet, loud])
    g = ld.AGC()
    g.lock = False
    g.scale = 0.01
    o = ora.AGC()
    o.scale = np.float32(0.01)
    if squelch:
        g.squelch = True
        g.threshold = -10.0
        o.squelch(True)
        o.threshold = np.float32(-10.0)
    sizes = [320, 1573, 2048, 4001, 257 * 17, 6000, 1573, 999]
    cuts = np.concatenate([[0], np.cumsum(sizes * 20)])
    cuts = cuts[cuts <= len(x)]
    ys, rs = [], []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        g._tsa_perturb(i < 2 * len(sizes))
        ys.append(g(x[a:b]))
        rs.append(o(x[a:b]))
    assert_bitwise(np.concatenate(ys), np.concatenate(rs))
    assert np.float32(g.gain) == np.float32(o.gain)
    if squelch:
        assert g.status == o.status
