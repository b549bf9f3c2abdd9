"""bytes_to_iq fused into the first chain filter.

`ComplexIIRFilter.from_bytes(raw)` (C ABI `ldsp_iirfilt_execute_iq16`) is
`filter(bytes_to_iq(raw))` in one pass: reference src/utility.hpp:61-69
((float)int16 / 32767.0f per component) followed by iirfilter.hpp:292-298.
The fast scans (modal single pass, blocked) convert on load; the checks:
  * the same bits as the two-call GPU path (bytes_to_iq, then the filter), over
    ragged calls that cut the stream mid-chunk, host and device inputs, and at
    64 Mi samples in one call (the bench size);
  * exact mode (converts first, then the sequential float32 kernel) is bitwise
    equal to the restatement's bytes_to_iq -> iirfilt;
  * a real filter refuses int16 IQ input.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHAIN_IIR = dict(filter_type="cheby2", order=8, Fc=np.float32(15000 / 2e6))


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def raw_iq(rng, n):
    r = rng.integers(-32768, 32768, size=2 * n, dtype=np.int64).astype(np.int16)
    r[:8] = [32767, -32768, 0, -1, 1, -32767, 32767, 32767]   # extremes of the wire format
    return r


@pytest.mark.parametrize("path", [2, 1])       # the modal single-pass scan, the blocked scan
@pytest.mark.parametrize("cuts", [[0, 1, 257, 70_000, 70_001, 1_000_000, 1_048_583], [0, 1_048_583]])
def test_from_bytes_equals_two_calls(ld, rng, cuts, path):
    raw = raw_iq(rng, cuts[-1])
    a = ld.ComplexIIRFilter(**CHAIN_IIR)
    b = ld.ComplexIIRFilter(**CHAIN_IIR)
    a._scan_path(path)
    b._scan_path(path)
    for lo, hi in zip(cuts, cuts[1:]):
        seg = raw[2 * lo:2 * hi]
        ya = a.from_bytes(seg.tobytes() if hi - lo < 1000 else seg)
        yb = b(ld.bytes_to_iq(seg.tobytes()))
        assert ya.dtype == np.complex64 and ya.shape == (hi - lo,)
        assert np.array_equal(bits(ya), bits(yb)), (lo, hi)


def test_from_bytes_device_full_size(ld, rng):
    import torch
    n = 64 * 1024 * 1024                       # BASELINE config 4 call size
    raw = torch.from_numpy(raw_iq(rng, n)).cuda()
    a = ld.ComplexIIRFilter(**CHAIN_IIR)
    b = ld.ComplexIIRFilter(**CHAIN_IIR)
    ya = a.from_bytes(raw)
    yb = b(ld.bytes_to_iq(raw))
    assert ya.is_cuda and ya.dtype == torch.complex64 and ya.numel() == n
    assert torch.equal(ya.view(torch.float32), yb.view(torch.float32))
    # the stream continues identically (same end state)
    ya = a.from_bytes(raw[:2 * 4097])
    yb = b(ld.bytes_to_iq(raw[:2 * 4097]))
    assert torch.equal(ya.view(torch.float32), yb.view(torch.float32))


def test_from_bytes_exact_vs_oracle(ld, ora, rng):
    raw = raw_iq(rng, 300_001)
    g = ld.ComplexIIRFilter(**CHAIN_IIR)
    g.exact = True
    B, A = g.sos()
    o = ora.IIRFilter(sos=(B, A), cplx=True)
    for lo, hi in ((0, 5), (5, 100_000), (100_000, 300_001)):
        seg = raw[2 * lo:2 * hi].tobytes()
        assert np.array_equal(bits(g.from_bytes(seg)), bits(o(ora.bytes_to_iq(seg))))


def test_from_bytes_real_filter_refused(ld):
    f = ld.RealIIRFilter(filter_type="cheby2", order=4, Fc=0.1)
    with pytest.raises(ValueError):
        f.from_bytes(np.zeros(8, np.int16))


def test_from_bytes_odd_length_rounds_down(ld, rng):
    # The reference's bytes_to_iq (utility.hpp:65) converts size / 4 whole (I, Q)
    # pairs and drops 1-3 trailing bytes; from_bytes follows the same rule, so
    # from_bytes(b) == self(bytes_to_iq(b)) for every length (host bytes and
    # uint8 device tensors).
    import torch
    raw = raw_iq(rng, 5001).tobytes()
    for extra in (b"", b"\x01", b"\x01\x02", b"\x01\x02\x03"):
        a = ld.ComplexIIRFilter(**CHAIN_IIR)
        b = ld.ComplexIIRFilter(**CHAIN_IIR)
        ya = a.from_bytes(raw + extra)
        yb = b(ld.bytes_to_iq(raw + extra))
        assert ya.shape == (5001,) and np.array_equal(bits(ya), bits(yb))
        t = torch.frombuffer(bytearray(raw + extra), dtype=torch.uint8).cuda()
        a.reset()
        b.reset()
        assert torch.equal(a.from_bytes(t).view(torch.float32), b(ld.bytes_to_iq(t)).view(torch.float32))
