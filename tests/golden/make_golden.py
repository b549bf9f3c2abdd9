"""Generate the golden vectors in tests/golden/golden.npz from the CPU
restatement (oracle/), which scipy/numpy pin in tests/test_oracle_*.py.

The reference repository (colbyAtCRI/python-liquiddsp) holds no tests,
fixtures or golden vectors, and liquid-dsp itself is absent here, so these are
"parity unpinned" with respect to a real liquid-dsp run.  They
pin the restatement against regressions and are what the GPU parity tests
compare the MI355X kernels with, without needing oracle/ on the box.

Every input is stored (not regenerated from a seed) so the fixture does not
depend on numpy's distribution algorithms.  Run from the repository root:

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402


def cgauss(rng, n, scale=1.0):
    return (scale * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)


def am_signal(n, fc=1200.0, seed=4, fs=2e6):
    """0.1 (1 + 0.5 m(t)) e^{j(2 pi fc t + 0.3)} + AWGN (30 dB SNR)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / fs
    msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
    x = 0.1 * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * fc * t + 0.3))
    sigma = 0.1 * 10 ** (-30 / 20) / np.sqrt(2)
    return (x + sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)


def main():
    g = {}
    meta = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/liquid_restate.c",
            "parity": "unpinned (no liquid-dsp available); restatement pinned by scipy/numpy tests",
            "switches": {"resampler": "fixed-point 32-bit phase, npfb -> power of two (liquid >= 1.5)",
                         "nco": "1024-entry sine table, index ((theta + 2^21) >> 22) & 1023",
                         "dotprod": "portable C order (oldest sample first), no FMA",
                         "loop_math": "fdlibm expf/logf/atan2f/tanhf (oracle/ora_math.h)",
                         "complex_division": "Smith's method (gcc 11 libgcc __divsc3/__divdc3) in the IIR designs"},
            "cases": {}}

    # C1-style FIR: firdes_kaiser(127, 0.1, 60, 0), complex Gaussian, seed 1
    rng = np.random.default_rng(1)
    h = O.firdes_kaiser(127, 0.1, 60.0, 0.0)
    x = cgauss(rng, 4096)
    f = O.FIRFilter(h, cplx=True)
    g["fir127_h"], g["fir127_x"], g["fir127_y"] = h, x, f(x)
    meta["cases"]["fir127"] = "firfilt_crcf, firdes_kaiser(127, fc=0.1, As=60, mu=0), 4096 samples"

    # real FIR (RealKaiserBessel-style taps with a scale) and DC blocker
    xr = rng.standard_normal(3000).astype(np.float32)
    fr = O.FIRFilter(kaiser=(25, 0.2, 20.0, 0.0), cplx=False)
    fr.scale = 0.75
    g["firr_h"], g["firr_x"], g["firr_y"] = fr.taps, xr, fr(xr)
    dc = O.FIRFilter(dc_blocker=(25, 20.0), cplx=False)
    g["dcblock_h"], g["dcblock_y"] = dc.taps, dc(xr)
    meta["cases"]["firr"] = "firfilt_rrrf kaiser(25, 0.2, 20, 0) scale 0.75; dc_blocker(25, 20)"

    # C2-style resampler (rate 48k/2M, m=20, fc=0.024, As=60, npfb=13)
    rate = np.float32(48000 / 2000000)
    x = cgauss(rng, 20000)
    r = O.Resampler(float(rate), m=20, fc=0.024, As=60.0, npfb=13, cplx=True)
    g["resamp_x"], g["resamp_y"] = x, r(x)
    g["resamp_step"] = np.array([r.step], np.uint32)
    rr = O.Resampler(0.37, m=7, fc=0.2, As=50.0, npfb=32, cplx=False)
    xr2 = rng.standard_normal(5000).astype(np.float32)
    g["resampr_x"], g["resampr_y"] = xr2, rr(xr2)
    meta["cases"]["resamp"] = "resamp_cccf(48k/2M, 20, 0.024, 60, 13), 20000 in; resamp_rrrf(0.37, 7, 0.2, 50, 32)"

    # C3-style NCO mix_down, freq 2 pi 0.05, and a VCO
    x = cgauss(rng, 4096)
    nco = O.NCO(0)
    nco.freq = float(2 * np.pi * 0.05)
    nco.phase = 0.4
    g["nco_x"], g["nco_y"] = x, nco.mix_down(x)
    vco = O.NCO(1)
    vco.freq = 0.3
    g["vco_y"] = vco.mix_up(x)
    meta["cases"]["nco"] = "nco_crcf LIQUID_NCO f=2 pi 0.05 phase 0.4 mix_down; LIQUID_VCO f=0.3 mix_up"

    # IIR: the chain's cheby2 order-8 lowpass, Fc = 15k/2M, SOS, float32 DF-II
    Bs, As_ = O.iirdes("cheby2", "lowpass", 8, 15000 / 2e6, 0.0, 0.1, 60.0)
    x = am_signal(8192)
    fi = O.IIRFilter(prototype=("cheby2", "lowpass", O.FMT_SOS, 8, 15000 / 2e6, 0.0, 0.1, 60.0), cplx=True)
    g["iir_B"], g["iir_A"], g["iir_x"], g["iir_y"] = Bs, As_, x, fi(x)
    fi.reset()
    g["iir_y64"] = fi.execute_f64(x)          # the same recursion in float64 (SURVEY 8(d) truth), rounded once
    meta["cases"]["iir"] = "iirfilt_crcf cheby2 lowpass order 8 fc 0.0075 Ap 0.1 As 60 (SOS)"

    # De-emphasis (DeemphasisFilter(48000)), real
    b, a = O.deemphasis_coefs(48000.0)
    fd = O.IIRFilter(tf=(b, a), cplx=False)
    xr3 = rng.standard_normal(4096).astype(np.float32)
    g["deemph_b"], g["deemph_a"], g["deemph_x"], g["deemph_y"] = b, a, xr3, fd(xr3)

    # AGC and AmpModem on the chain's own intermediate signals
    radio_in = am_signal(65536)
    g["chain_x"] = radio_in
    fi.reset()
    s1 = fi(radio_in)
    r2 = O.Resampler(float(rate), m=20, fc=float(rate), As=60.0, npfb=13, cplx=True)
    s2 = r2(s1)
    agc = O.AGC()
    agc.lock(False)
    agc.scale = 0.01
    s3 = agc(s2)
    g["agc_x"], g["agc_y"] = s2, s3
    am = O.AmpModem(0.5, "dsb", True)
    g["ampmodem_y"] = am(s3)
    amc = O.AmpModem(0.75, "dsb", False)
    g["ampmodem_costas_y"] = amc(s3)
    radio = O.AMRadio()
    g["chain_y"] = radio(radio_in)
    meta["cases"]["chain"] = ("AMRadio (README.md:41-58) on 65536 samples of SURVEY C4; agc_x/agc_y and ampmodem_* "
                              "are its intermediate stages (AGC unlocked, scale 0.01; AmpModem(0.5, dsb, carrier) and "
                              "AmpModem(0.75, dsb, costas))")

    np.savez(os.path.join(HERE, "golden.npz"), **g)
    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    size = os.path.getsize(os.path.join(HERE, "golden.npz"))
    print(f"wrote golden.npz ({size / 1e6:.2f} MB, {len(g)} arrays)")


if __name__ == "__main__":
    main()
