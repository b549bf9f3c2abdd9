"""Sanitizers on host code (the GPU pool runs none, so these are CPU
tests):

* libldsp's host side (C ABI, designers, modal analysis, host pools) built with
  ASan + UBSan (`make -C python-liquiddsp_amd asan`: each -fsanitize after
  -Xarch_host, device code untouched) and driven through every host-only entry
  point, the error paths and the no-device execute paths by
  tests/sanitize/host_driver.c, leak detection on;
* the CPU restatement (oracle/, `make -C oracle asan`, gcc ASan + UBSan,
  non-recoverable) through the chains the GPU tests check against it: the
  AMRadio chain in README blocks, resamplers up- and down-sampling, FIR, IIR
  designs of every prototype, AGC with squelch, AmpModem types, BroadcastAM,
  FMStereo, FreqDem and Delay.
Any report aborts the child; the tests require a clean exit and no report text.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "python-liquiddsp_amd")
REPORTS = ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:")


def _make(path, target):
    r = subprocess.run(["make", "-s", "-j8", "-C", path, target], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]


def test_host_library_asan_ubsan():
    _make(PKG, "asan")
    exe = os.path.join(PKG, "build", "host_driver_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert not any(k in out for k in REPORTS), out[-4000:]
    assert "all checks passed" in r.stdout


ORACLE_SCRIPT = r"""
import numpy as np
from oracle import oracle
O = oracle.variant("asan")
rng = np.random.default_rng(5)
n = 300_000
t = np.arange(n) / 2e6
x = (0.1 * (1 + 0.5 * np.sin(2 * np.pi * 1000 * t)) * np.exp(2j * np.pi * 1200 * t)
     + 0.003 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
r = O.AMRadio()
for i in range(0, n, 65536):
    r(x[i:i + 65536])
for rate in (0.024, 0.5, 1.0, 2.5, 7.3):
    for cplx in (False, True):
        rs = O.Resampler(rate, m=20, fc=0.024 if rate < 1 else 0.2, npfb=13, cplx=cplx)
        xi = x[:20000] if cplx else x[:20000].real.copy()
        rs(xi[:7]); rs(xi[7:13001]); rs(xi[13001:])
    O.Resampler(rate, default=True)(x[:5000])
f = O.FIRFilter(O.firdes_kaiser(127, 0.1, 60.0), cplx=True)
f(x[:10000]); f(x[10000:10003])
for ft in ("butter", "cheby1", "cheby2", "ellip", "bessel"):
    for bt in ("lowpass", "highpass", "bandpass", "bandstop"):
        for order in (1, 2, 5, 8):
            try:
                q = O.IIRFilter(prototype=(ft, bt, O.FMT_SOS, order, 0.1, 0.25, 0.7, 60.0), cplx=True)
            except ValueError:
                continue
            q(x[:4000])
O.IIRFilter(tf=(O.deemphasis_coefs(48000.0)), cplx=False)(x[:4000].real.copy())
g = O.AGC()
g.squelch(True)
g.threshold = np.float32(-10.0)
g(x[:50000], return_status=True)
for kind in ("dsb", "usb", "lsb"):
    for carrier in (True, False):
        try:
            am = O.AmpModem(0.5, kind, carrier)
        except TypeError:
            am = O.AmpModem(modulation=0.5, type=kind, carrier=carrier)
        am(x[:30000] * 5)
O.BroadcastAM()(x[:30000] * 5)
O.FreqDem(4.0)(x[:30000])
fm = O.FMStereo(600000.0, 48000.0)
fm(x[:60000])
d = O.Delay(25)
d(x[:1000])
print("oracle asan ok")
"""


def test_oracle_asan_ubsan():
    _make(os.path.join(REPO, "oracle"), "asan")
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not libasan or not os.path.exists(libasan):
        pytest.skip("gcc's libasan.so is not installed")
    env = dict(os.environ, LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", ORACLE_SCRIPT], capture_output=True, text=True, timeout=600,
                       env=env, cwd=REPO)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert not any(k in out for k in REPORTS), out[-4000:]
    assert "oracle asan ok" in r.stdout
