"""AmpModem carrier loop of short calls: k_pll_seqc (k_pll.hip), used for calls
below 1 024 PCM samples in carrier mode (from round 5; longer calls, the
README's 65 536-sample SDR block with its 1 573 included, take the candidates +
walk path, so the sizes around the threshold check both sides).  Reference: ampmodem_demodulate_block behind
/root/reference/src/demod.hpp:290-296 (AmpModem(carrier=True) ->
ampmodem_demod_dsb_pll_carrier).

One wave steps the loop; beside each batch of 4 steps its 64 lanes evaluate
the kicks and output of the next batch at 16 candidate table indices per
sample, and a batch whose index leaves its window is redone directly.  Every
test is bitwise against the sequential restatement (oracle/liquid_restate.c
ampmodem_demod), state included, and the window-miss redo path is shown to
run (AmpModem._seq_stats: batches stepped, batches redone).
"""
import numpy as np
import pytest

from conftest import cgauss

pytestmark = pytest.mark.gpu

SIZES = [1, 3, 4, 5, 1023, 1024, 1573, 2047]


def assert_bitwise(y, ref):
    y, ref = np.asarray(y), np.asarray(ref)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    eq = y.view(np.uint32) == ref.view(np.uint32)
    assert eq.all(), f"{(~eq).sum()} of {eq.size} differ; first at {int(np.argmin(eq))}"


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def _am(rng, n, fs=48000.0, fc=300.0, amp=1.0, snr_noise=0.02):
    t = np.arange(n) / fs
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t)) / 2
    x = amp * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * fc * t + 0.4))
    return (x + snr_noise * cgauss(rng, n)).astype(np.complex64)


def _run_calls(ld, ora, x, sizes, streams=1):
    """Feed x through one GPU AmpModem in calls of the given sizes (cycled) and
    through the restatement in one call; returns (gpu, ref, gpu object, oracle)."""
    import torch
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    o = ora.AmpModem(0.5, "dsb", carrier=True)
    xd = torch.from_numpy(x).cuda()
    ss = [torch.cuda.Stream() for _ in range(streams)]
    torch.cuda.synchronize()
    outs, a, i = [], 0, 0
    while a < len(x):
        b = min(len(x), a + sizes[i % len(sizes)])
        with torch.cuda.stream(ss[i % streams]):
            outs.append(g(xd[a:b]))
        a, i = b, i + 1
    torch.cuda.synchronize()
    return np.concatenate([t.cpu().numpy() for t in outs]), o(x), g, o


@pytest.mark.parametrize("n", SIZES)
def test_seqc_call_size_bitwise(ld, ora, rng, n):
    """Calls of exactly n samples (whole batches, ragged tails, a single sample),
    on a locked AM carrier; state carried across 12 calls."""
    x = _am(rng, 12 * n)
    y, ref, g, o = _run_calls(ld, ora, x, [n])
    assert_bitwise(y, ref)
    assert g.pll_state() == o.pll_state


def test_seqc_mixed_sizes_two_streams(ld, ora, rng):
    x = _am(rng, 40_000)
    sizes = [int(s) for s in rng.integers(1, 2048, 60)]
    y, ref, g, o = _run_calls(ld, ora, x, sizes, streams=2)
    assert_bitwise(y, ref)
    assert g.pll_state() == o.pll_state


def test_seqc_noise_window_misses(ld, ora, rng):
    """Pure noise: the loop never locks, the extrapolated index misses its
    16-cell window often, and those batches are redone directly."""
    x = cgauss(rng, 30_000)
    y, ref, g, o = _run_calls(ld, ora, x, [1000])
    assert_bitwise(y, ref)
    assert g.pll_state() == o.pll_state
    batches, redone = g._seq_stats()
    assert batches == sum(min(1000, len(x) - a) // 4 for a in range(0, len(x), 1000))
    assert redone > 0, "the window-miss redo path did not run"


def test_seqc_unlocked_start_large_offset(ld, ora, rng):
    """Starts unlocked, carrier 3 kHz off (outside the loop's pull-in within
    the test): the trajectory the candidates extrapolate keeps being wrong."""
    x = _am(rng, 24_000, fc=3000.0, snr_noise=0.3)
    y, ref, g, o = _run_calls(ld, ora, x, [1573, 2047, 777])
    assert_bitwise(y, ref)
    assert g.pll_state() == o.pll_state
    assert g._seq_stats()[1] > 0


def test_seqc_exact_zero_runs(ld, ora, rng):
    """Exact-zero input (atan2(+-0, +-0) operands, zero outputs) between and
    inside signal stretches, including a whole call of zeros."""
    x = _am(rng, 20_000)
    x[:700] = 0
    x[5000:9000] = 0                       # covers whole 1 573-sample calls
    x[12_345:12_350] = 0
    x[-300:] = 0
    y, ref, g, o = _run_calls(ld, ora, x, [1573])
    assert_bitwise(y, ref)
    assert g.pll_state() == o.pll_state
    assert np.any(ref[5100:8900] == 0)


def test_seqc_after_squelched_agc(ld, ora, rng):
    """The README chain's AGC with squelch on: in SIGNALLO / ENABLED the
    wrapper zeroes the AGC output (/root/reference/src/agc.hpp:124-125), and
    the AmpModem then demodulates exact zeros (src/demod.hpp:290-296).  Both
    stages on the GPU, call by call, against the restatement's two stages."""
    import torch
    quiet = (1e-4 * cgauss(rng, 6000)).astype(np.complex64)
    loud = _am(rng, 6000, amp=0.3, snr_noise=0.01)
    x = np.concatenate([quiet, loud, quiet, loud, quiet])
    ga, gm = ld.AGC(), ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    ga.squelch = True
    ga.threshold = -30.0
    ga.scale = 0.5
    oa, om = ora.AGC(), ora.AmpModem(0.5, "dsb", carrier=True)
    oa.squelch(True)
    oa.threshold = np.float32(-30.0)
    oa.scale = np.float32(0.5)
    xd = torch.from_numpy(x).cuda()
    outs, refs, zeros = [], [], 0
    for a in range(0, len(x), 1573):
        b = min(len(x), a + 1573)
        mid = ga(xd[a:b])
        outs.append(gm(mid))
        r = oa(x[a:b])
        zeros += int(np.sum(r == 0))
        refs.append(om(r))
        assert_bitwise(mid.cpu().numpy().view(np.float32), r.view(np.float32))
    torch.cuda.synchronize()
    assert zeros > 5000, "squelch never zeroed the AGC output"
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), np.concatenate(refs))
    assert gm.pll_state() == om.pll_state
