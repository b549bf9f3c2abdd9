"""AGC chunk-parallel calls: the repair round and the one-wave verifier
(reference src/agc.hpp:109-128 AGC::execute -> agc_crcf_execute per sample).

A chunk-parallel call runs every 1 024-sample chunk from a guessed state; the
flag pass marks the chunks whose start differs from their predecessor's end,
one repair round (the default, csrc/capi.cpp ldsp_agc_execute) re-runs each run
of marked chunks from the true state, and k_agc_verify re-runs whatever is still
marked.  On benign AM no chunk needs either.  Here the test hook
ldsp_debug_agc_perturb starts every odd chunk 1 ulp off, so both paths must
produce agc_crcf's bits: with the default round (the repair threads re-run the
odd chunks) and with no round at all (the verifier alone re-runs every one of
them, serially) -- at 200 k and 1.6 M samples, over two calls (the second one
speculative: every chunk from a guess, chunk 0 checked against the true state).
Burst / fade inputs (+-40 dB steps on chunk boundaries) run at the defaults.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C = 1024          # the library's chunk length for chunk-parallel calls


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def _bitwise(y, ref):
    assert y.shape == ref.shape, (y.shape, ref.shape)
    eq = y.view(np.uint64) == ref.view(np.uint64)
    if not eq.all():
        i = int(np.argmin(eq))
        raise AssertionError(f"{(~eq).sum()} of {eq.size} differ; first at {i}: {y[i]!r} vs {ref[i]!r}")


def _am(rng, n, amp=0.05):
    t = np.arange(n) / 48000.0
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
    s = amp * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * 300.0 * t + 0.7))
    s = s + amp * 10 ** (-1.5) * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)
    return s.astype(np.complex64)


def _pair(ld, ora):
    g = ld.AGC()
    g.lock = False
    g.scale = 0.01
    o = ora.AGC()
    o.scale = np.float32(0.01)
    return g, o


@pytest.mark.parametrize("n", [200_000, 1_610_613])
@pytest.mark.parametrize("rounds", [-1, 0])
def test_agc_perturbed_chunks_bitwise(ld, ora, rng, n, rounds):
    x = _am(rng, n)
    g, o = _pair(ld, ora)
    g._perturb(True)
    g._rounds(rounds)
    h = n // 2
    y = np.concatenate([g(x[:h]), g(x[h:])])
    _bitwise(y, o(x))
    assert np.float32(g.gain) == np.float32(o.gain)
    runfix, verify = g._reruns()
    odd = (h // C) // 2 + ((n - h) // C) // 2          # odd chunks per call, both calls
    if rounds == 0:
        # no repair round: the verifier re-ran every perturbed chunk, one by one
        assert runfix == 0 and verify >= odd, (runfix, verify, odd)
    else:
        # the default round re-ran them in parallel; the verifier found nothing left
        assert runfix >= odd, (runfix, verify, odd)


@pytest.mark.parametrize("n", [200_000, 1_610_613])
def test_agc_burst_fade_bitwise(ld, ora, rng, n):
    # +-40 dB steps landing on chunk boundaries (every 3 chunks), plus a fade
    # (a 60 dB ramp over 40 chunks) in the middle: the warm-ups see level jumps
    x = _am(rng, n, amp=1.0).astype(np.complex128)
    lvl = np.ones(n)
    for b in range(0, n, 3 * C):
        lvl[b:b + 3 * C] = [1.0, 1e-2, 1e2][(b // (3 * C)) % 3]
    a = n // 2
    f = min(40 * C, n - a)
    lvl[a:a + f] *= np.logspace(0, -3, f)
    x = (x * lvl).astype(np.complex64)
    g, o = _pair(ld, ora)
    cuts = [0, n // 3, n]
    y = np.concatenate([g(x[p:q]) for p, q in zip(cuts[:-1], cuts[1:])])
    _bitwise(y, o(x))
    assert np.float32(g.gain) == np.float32(o.gain)
    runfix, verify = g._reruns()
    print(f"n={n}: repair-round re-runs {runfix}, verifier re-runs {verify}")
