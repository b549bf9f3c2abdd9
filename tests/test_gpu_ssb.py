"""AmpModem usb / lsb on the GPU (reference src/demod.hpp:221-307 ->
liquid ampmodem_demod_ssb_pll_carrier / ampmodem_demod_ssb) against the
restatement, bit for bit: the carrier PLL (short sequential calls and
chunk-parallel candidates + walk, with the table-index output) feeding the
Hilbert c2r and the DC blocker, the suppressed-carrier Hilbert alone, calls cut
anywhere (the Hilbert history crosses calls), two streams, and the type /
carrier setters' state reset (demod.hpp:250-276).  Parity unpinned: the SSB
path is restated from the recalled liquid source (oracle/liquid_restate.c)."""
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
    return np.ascontiguousarray(a).view(np.uint32)


def assert_bitwise(y, ref):
    assert y.shape == ref.shape, (y.shape, ref.shape)
    eq = bits(y) == bits(ref)
    if not eq.all():
        i = int(np.argmin(eq))
        raise AssertionError(f"{(~eq).sum()} of {eq.size} differ; first at {i}: {y[i]!r} vs {ref[i]!r}")


def _ssb(rng, n, side, carrier, fs=48000.0, fcar=300.0):
    """An SSB signal of a three-tone message (analytic for usb, conjugate for
    lsb), optionally with a carrier offset by fcar, plus noise."""
    t = np.arange(n) / fs
    sgn = 1 if side == "usb" else -1
    msg = sum(np.exp(1j * sgn * 2 * np.pi * f * t) for f in (400.0, 1000.0, 2500.0)) / 3
    s = 0.5 * msg + (1.0 if carrier else 0.0)
    s = s * np.exp(1j * (2 * np.pi * fcar * t + 0.7))
    return (0.05 * s + 0.05 * 10 ** (-1.5) * cgauss(rng, n)).astype(np.complex64)


@pytest.mark.parametrize("side", ["usb", "lsb"])
@pytest.mark.parametrize("carrier", [True, False])
@pytest.mark.parametrize("n", [1500, 60_000])
def test_ssb_bitwise(ld, ora, rng, side, carrier, n):
    # n = 1500: the carrier PLL's short-call loop (k_pll_seqc); 60 000: candidates + walk
    x = _ssb(rng, n, side, carrier)
    g = ld.AmpModem(modulation=0.5, type=side, carrier=carrier)
    o = ora.AmpModem(0.5, side, carrier=carrier)
    cut = n // 3 + 7
    y = np.concatenate([g(x[:cut]), g(x[cut:cut + 5]), g(x[cut + 5:])])
    assert_bitwise(y, o(x))
    if carrier:
        assert g.pll_state() == o.pll_state


def test_ssb_two_streams_and_device_tensors(ld, ora, rng):
    import torch
    x = _ssb(rng, 5 * 20_000 + 777, "usb", True)
    g = ld.AmpModem(modulation=0.5, type="usb", carrier=True)
    o = ora.AmpModem(0.5, "usb", carrier=True)
    xd = torch.from_numpy(x).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    cuts = [0, 20_000, 21_000, 41_000, 61_000, 81_000, len(x)]
    outs = []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        with torch.cuda.stream(streams[i % 2]):
            outs.append(g(xd[a:b]))
    torch.cuda.synchronize()
    assert all(t.is_cuda for t in outs)
    assert_bitwise(np.concatenate([t.cpu().numpy() for t in outs]), o(x))
    assert g.pll_state() == o.pll_state


def test_ssb_setters_reset_state(ld, ora, rng):
    # demod.hpp:250-276: set_type / set_carrier / set_modulation destroy and
    # re-create the modem, so the next call starts from a fresh state
    x = _ssb(rng, 30_000, "lsb", True)
    g = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    g(x[:10_000])
    g.type = "lsb"
    assert g.type == "lsb"
    assert_bitwise(g(x), ora.AmpModem(0.5, "lsb", carrier=True)(x))
    g.carrier = False
    assert_bitwise(g(x), ora.AmpModem(0.5, "lsb", carrier=False)(x))
    g.modulation = 0.8
    assert_bitwise(g(x), ora.AmpModem(0.8, "lsb", carrier=False)(x))
    g.reset()
    assert_bitwise(g(x[:5000]), ora.AmpModem(0.8, "lsb", carrier=False)(x[:5000]))


def test_ssb_recovers_message(ld, rng):
    # the demodulated sideband carries the message; the other sideband is ~silent
    n = 48_000
    x = _ssb(rng, n, "usb", False, fcar=0.0)
    up = ld.AmpModem(modulation=0.05 * 0.5, type="usb", carrier=False)(x)
    lo = ld.AmpModem(modulation=0.05 * 0.5, type="lsb", carrier=False)(x)
    rms = lambda v: float(np.sqrt(np.mean(v[n // 2:].astype(np.float64) ** 2)))
    assert np.abs(up[n // 2:]).max() > 0.5
    assert rms(lo) < 0.15 * rms(up)          # the other sideband holds only the noise
