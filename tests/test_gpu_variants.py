"""GPU outputs against every build variant of the restatement
(tests/golden/variants.npz, made by tests/golden/make_variants.py).

liquid-dsp's output is itself platform-dependent (libm in the feedback loops,
SIMD dotprod order), so the restatement ships four variants.  The GPU exact
mode is bit-identical to the "default" one (test_golden.py); here every GPU
output -- exact and fast modes -- is checked against all four with SURVEY
8(d)'s tolerances:
  * FIR, resampler (linear, no feedback): <= 1e-6 relative;
  * AGC, AmpModem (feedback loops, one stage): within 1e-6, i.e. no further
    from any variant than the variants are from each other on these inputs
    (recorded in variants.json, all < 1e-6);
  * the whole AMRadio chain: within the spread the variants show among
    themselves over 4 Mi samples (variants.json "chain_variant_spread_maxrel"):
    a one-cell difference of the PLL's 10-bit phase index anywhere upstream
    changes the trajectory for good, so the chain is only defined to that spread.
"""
import json
import os

import numpy as np
import pytest

from conftest import maxrel

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden.npz"))
V = np.load(os.path.join(HERE, "golden", "variants.npz"))
META = json.load(open(os.path.join(HERE, "golden", "variants.json")))
NAMES = list(META["variants"])


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def _stage_bound(stage, v):
    rec = 0.0 if v == "default" else META["golden_inputs"][stage][v]["maxrel"]
    return max(1e-6, rec)


@pytest.mark.parametrize("v", NAMES)
def test_linear_stages_vs_variant(ld, v):
    for mode in ("exact", "fast"):
        f = ld.ComplexFIRFilter(G["fir127_h"])
        f.mode = mode
        assert maxrel(f(G["fir127_x"]), V[f"{v}__fir127_y"]) <= 1e-6, (v, mode)
    r = ld.ComplexResampler(rate=np.float32(0.024), len=20, Fc=np.float32(0.024), As=60.0, nfilter=13)
    assert maxrel(r(G["resamp_x"]), V[f"{v}__resamp_y"]) <= 1e-6, v


@pytest.mark.parametrize("v", NAMES)
def test_loop_stages_vs_variant(ld, v):
    agc = ld.AGC()
    agc.lock = False
    agc.scale = 0.01
    assert maxrel(agc(G["agc_x"]), V[f"{v}__agc_y"]) <= _stage_bound("agc_y", v)
    # each demodulator on the variant's own AGC output (so only its own stage differs)
    a_in = V[f"{v}__agc_y"]
    y = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)(a_in)
    assert maxrel(y, V[f"{v}__ampmodem_y"]) <= _stage_bound("ampmodem_y", v)
    y = ld.AmpModem(modulation=0.75, type="dsb", carrier=False)(a_in)
    assert maxrel(y, V[f"{v}__ampmodem_costas_y"]) <= _stage_bound("ampmodem_costas_y", v)


@pytest.mark.parametrize("v", NAMES)
@pytest.mark.parametrize("exact", [True, False])
def test_chain_vs_variant(ld, v, exact):
    bandpass = ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    bandpass.exact = exact
    resample = ld.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    am = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    audio = ld.DeemphasisFilter(48000)
    agc = ld.AGC()
    agc.lock = False
    agc.scale = 0.01
    y = audio(am(agc(resample(bandpass(G["chain_x"])))))
    ref = V[f"{v}__chain_y"]
    assert y.shape == ref.shape
    assert maxrel(y, ref) <= META["chain_variant_spread_maxrel"], (v, exact, maxrel(y, ref))
