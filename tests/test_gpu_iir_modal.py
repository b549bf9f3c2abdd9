"""Fast-mode IIR: the single-pass modal scan (k_iir_modal.hip) against the
float64 truth, the blocked SOS-coordinate scan and itself.

Reference: src/iirfilter.hpp:292-298 (ComplexIIRFilter.execute_block) and :353
(RealIIRFilter), iirfilt_*_execute_block over liquid's SOS cascade.  Fast mode
is a float64 evaluation of that cascade (tolerance
policy): error vs the float64 evaluation <= 1e-6 of the output range and no
worse than liquid's own float32 recursion.  The modal scan must also
  * agree with the blocked scan (same float64 filter, different float64
    rounding, both rounded once to float32) within 2 float32 ulps of the output
    range -- a wrong look-back term or chunk start state is far above that;
  * be bit-identical whether a unit reads its predecessors' published end
    states or recomputes them from the input (the path a late predecessor
    forces; `_scan_path(3)` forces it everywhere);
  * carry the state across ragged calls (cuts inside a 32-sample chunk, at and
    around the 2048-sample look-back unit) and across switches to the blocked
    scan and the exact float32 recursion (the state changes coordinates on the
    host).
"""
import numpy as np
import pytest
import scipy.signal as sps

from conftest import cgauss, maxrel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


# (liquiddsp kwargs, oracle prototype) -- the chain filter, a wide lowpass,
# a slow-decaying narrow Butterworth (look-back 20 units), elliptic order 8
# (25 units), a bandpass with 8 modes, Bessel (a zero pole), Chebyshev-I
PROTOS = [
    (dict(filter_type="cheby2", order=8, Fc=np.float32(0.0075)), ("cheby2", "lowpass", 1, 8, np.float32(0.0075), 0.3, 0.7, 60.0)),
    (dict(filter_type="cheby2", order=8, Fc=0.02), ("cheby2", "lowpass", 1, 8, np.float32(0.02), 0.3, 0.7, 60.0)),
    (dict(filter_type="butter", order=8, Fc=0.001), ("butter", "lowpass", 1, 8, np.float32(0.001), 0.3, 0.7, 60.0)),
    (dict(filter_type="ellip", order=8, Fc=0.01, Ap=0.7, As=60.0), ("ellip", "lowpass", 1, 8, np.float32(0.01), 0.3, 0.7, 60.0)),
    (dict(filter_type="cheby2", band_type="bandpass", order=8, Fc=0.05, F0=0.2),
     ("cheby2", "bandpass", 1, 8, np.float32(0.05), 0.2, 0.7, 60.0)),
    (dict(filter_type="bessel", order=5, Fc=0.02), ("bessel", "lowpass", 1, 5, np.float32(0.02), 0.3, 0.7, 60.0)),
    (dict(filter_type="cheby1", order=5, Fc=0.02, Ap=0.5), ("cheby1", "lowpass", 1, 5, np.float32(0.02), 0.3, 0.5, 60.0)),
]
CUTS = [0, 1, 31, 33, 2047, 2048, 2049, 6000, 65_536 + 7, 200_000, 333_333]


def _run(f, x, cuts):
    return np.concatenate([f(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])


@pytest.mark.parametrize("cplx", [True, False])
@pytest.mark.parametrize("k", range(len(PROTOS)))
def test_modal_vs_f64_and_blocked(ld, ora, rng, k, cplx):
    kw, proto = PROTOS[k]
    n = CUTS[-1]
    x = cgauss(rng, n) if cplx else np.float32(rng.standard_normal(n))
    cls = ld.ComplexIIRFilter if cplx else ld.RealIIRFilter
    g = cls(**kw)
    ok, m, j, err = g._modal_info()
    assert ok and 1 <= m <= 8 and 1 <= j <= 64 and err <= 1e-10, (ok, m, j, err)
    g._scan_path(2)
    y = _run(g, x, CUTS)
    o = ora.IIRFilter(prototype=proto, cplx=cplx)
    truth = o.execute_f64(x)
    o.reset()
    err_gpu, err_liquid = maxrel(y, truth), maxrel(o(x), truth)
    assert err_gpu <= 1e-6, err_gpu
    assert err_gpu <= err_liquid or err_liquid < 1e-6, (err_gpu, err_liquid)
    b = cls(**kw)
    b._scan_path(1)
    if b._modal_info()[0] and proto[1] != "bandpass":   # the blocked scan covers state dimension <= 8
        assert maxrel(y, _run(b, x, CUTS)) <= 2.5e-7


@pytest.mark.parametrize("cplx", [True, False])
def test_modal_lookback_recompute_bitwise(ld, rng, cplx):
    n = 3 * (1 << 20) + 999
    x = cgauss(rng, n) if cplx else np.float32(rng.standard_normal(n))
    cls = ld.ComplexIIRFilter if cplx else ld.RealIIRFilter
    kw = PROTOS[0][0]
    a, b = cls(**kw), cls(**kw)
    a._scan_path(2)
    b._scan_path(3)
    cuts = [0, 5000, 1 << 20, n]
    ya, yb = _run(a, x, cuts), _run(b, x, cuts)
    assert np.array_equal(ya.view(np.uint32), yb.view(np.uint32))


def test_modal_state_across_paths(ld, ora, rng):
    """modal -> blocked -> modal -> exact -> modal: the state moves between the
    modal, float64 and float32 coordinates on the host."""
    kw, proto = PROTOS[1]
    n = 400_000
    x = cgauss(rng, n)
    g = ld.ComplexIIRFilter(**kw)
    o = ora.IIRFilter(prototype=proto, cplx=True)
    cuts = [0, 70_001, 150_000, 230_000]
    parts = []
    for (a, b), path in zip(zip(cuts[:-1], cuts[1:]), [2, 1, 2]):
        g._scan_path(path)
        parts.append(g(x[a:b]))
    truth = o.execute_f64(x[:230_000])
    assert maxrel(np.concatenate(parts), truth) <= 1e-6
    # exact segment: continue the float64 truth from the same state in float32
    g.exact = True
    ye = g(x[230_000:300_000])
    g.exact = False
    g._scan_path(2)
    yf = g(x[300_000:])
    truth_all = ora.IIRFilter(prototype=proto, cplx=True).execute_f64(x)
    assert maxrel(ye, truth_all[230_000:300_000]) <= 1e-3      # float32 recursion (SURVEY App. B sensitivity)
    assert maxrel(yf, truth_all[300_000:]) <= 1e-3


def test_modal_tf_and_reset(ld, ora, rng):
    b_, a_ = sps.butter(2, 0.002)
    x = cgauss(rng, 300_001)
    g = ld.CIIRFilter(np.float32(b_), np.float32(a_))
    assert g._modal_info()[0]
    g._scan_path(2)
    y1 = _run(g, x, [0, 2049, 100_000, 300_001])
    truth = ora.IIRFilter(tf=(np.float32(b_), np.float32(a_)), cplx=True).execute_f64(x)
    assert maxrel(y1, truth) <= 1e-6
    g.reset()
    y2 = g(x)
    assert maxrel(y2, truth) <= 1e-6


def test_modal_device_tensor_streams(ld, rng):
    """Device tensors on two rotating streams: bit-identical to one stream."""
    import torch
    n = 5 * (1 << 20) + 17
    x = torch.from_numpy(cgauss(rng, n)).cuda()
    kw = PROTOS[0][0]
    a, b = ld.ComplexIIRFilter(**kw), ld.ComplexIIRFilter(**kw)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    cuts = [0, 1 << 20, 2 << 20, 3 << 20, n]
    ya = [a(x[p:q]) for p, q in zip(cuts[:-1], cuts[1:])]
    yb = []
    for i, (p, q) in enumerate(zip(cuts[:-1], cuts[1:])):
        with torch.cuda.stream(streams[i % 2]):
            yb.append(b(x[p:q]))
    torch.cuda.synchronize()
    for u, v in zip(ya, yb):
        assert torch.equal(u.view(torch.int64), v.view(torch.int64))


@pytest.mark.parametrize("n", [65_536, 200_001])
def test_modal_small_call_one_xcd_bitwise(ld, rng, n):
    """Small calls (up to 16 J units) run every unit on one XCD and read every
    predecessor's published state: bit-identical to recomputing them all."""
    x = cgauss(rng, 3 * n)
    kw = PROTOS[0][0]
    a, b = ld.ComplexIIRFilter(**kw), ld.ComplexIIRFilter(**kw)
    a._scan_path(2)
    b._scan_path(3)
    cuts = [0, n, 2 * n, 3 * n]
    ya, yb = _run(a, x, cuts), _run(b, x, cuts)
    assert np.array_equal(ya.view(np.uint32), yb.view(np.uint32))
