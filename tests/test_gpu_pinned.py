"""Page-locked host buffers on the numpy (LDSP_MEM_HOST) path: ldsp_host_alloc /
ldsp_host_free, the direct DMA of a host call whose x or y is page-locked, and
the pybind module's numpy outputs taken from that pool (so each stage of the
README chain, README.md:41-58, DMAs its input straight out of the previous
stage's array).  Results must be bit-identical to pageable buffers, the arrays
ordinary writeable numpy arrays, and the pool's limit a fallback to pageable
memory, not an error."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBPATH = os.path.join(REPO, "python-liquiddsp_amd", "libldsp.so")
LDSP_EINVAL = -1
MEM_HOST = 0


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


@pytest.fixture(scope="module")
def lib(ld):
    L = C.CDLL(LIBPATH)
    L.ldsp_last_error.restype = C.c_char_p
    return L


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _pinned(lib, n, dtype):
    p = C.c_void_p()
    nbytes = n * np.dtype(dtype).itemsize
    assert lib.ldsp_host_alloc(C.c_size_t(nbytes), C.byref(p)) == 0, lib.ldsp_last_error()
    buf = (C.c_char * nbytes).from_address(p.value)
    return p, np.frombuffer(buf, dtype=dtype, count=n)


def test_capi_pinned_buffers_bitwise(lib):
    rng = np.random.default_rng(5)
    n = 300_001
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    h = rng.standard_normal(63).astype(np.float32)
    outs = []
    for pinned in (False, True):
        q = C.c_void_p()
        assert lib.ldsp_firfilt_create(h.ctypes.data_as(C.c_void_p), C.c_uint(h.size), 1, C.byref(q)) == 0
        if pinned:
            px, xa = _pinned(lib, n, np.complex64)
            py_, ya = _pinned(lib, n, np.complex64)
            xa[:] = x
        else:
            xa, ya = x.copy(), np.empty_like(x)
        for k in range(3):          # state carries across calls through both paths
            rc = lib.ldsp_firfilt_execute(q, xa.ctypes.data_as(C.c_void_p), C.c_size_t(n),
                                          ya.ctypes.data_as(C.c_void_p), MEM_HOST, None)
            assert rc == 0, lib.ldsp_last_error()
            outs.append(ya.copy())
        lib.ldsp_firfilt_destroy(q)
        if pinned:
            assert lib.ldsp_host_free(px) == 0 and lib.ldsp_host_free(py_) == 0
    for k in range(3):
        assert (_bits(outs[k]) == _bits(outs[3 + k])).all()


def test_capi_free_checks(lib):
    assert lib.ldsp_host_free(None) == 0
    junk = np.zeros(16, np.float32)
    assert lib.ldsp_host_free(junk.ctypes.data_as(C.c_void_p)) == LDSP_EINVAL
    p, _ = _pinned(lib, 1 << 16, np.float32)
    assert lib.ldsp_host_free(p) == 0
    assert lib.ldsp_host_free(p) == LDSP_EINVAL          # already returned


def _chain(ld):
    bp = ld.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    rs = ld.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    am = ld.AmpModem(modulation=0.5, type="dsb", carrier=True)
    de = ld.DeemphasisFilter(48000)
    agc = ld.AGC()
    agc.lock = False
    agc.scale = 0.01
    return bp, rs, agc, am, de


def test_readme_chain_numpy_pinned_vs_pageable(ld):
    rng = np.random.default_rng(11)
    n, blocks = 65536, 6
    t = np.arange(n * blocks) / 2e6
    x = (0.1 * (1 + 0.5 * np.sin(2 * np.pi * 700 * t)) * np.exp(2j * np.pi * 1200 * t)).astype(np.complex64)
    x += (0.003 * (rng.standard_normal(x.size) + 1j * rng.standard_normal(x.size))).astype(np.complex64)
    a, b = _chain(ld), _chain(ld)
    for i in range(blocks):
        blk = x[i * n:(i + 1) * n]
        v = blk
        for st in a:                 # the module's own (page-locked) arrays handed on
            v = st(v)
        w = blk
        for st in b:                 # every hand-over through a fresh pageable copy
            w = np.array(st(w), copy=True)
        assert (_bits(v) == _bits(w)).all(), i


def test_outputs_writeable_and_read_afresh(ld):
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(1 << 17) + 1j * rng.standard_normal(1 << 17)).astype(np.complex64)
    y = ld.bytes_to_iq(np.zeros(4 << 17, np.uint8).tobytes())
    assert y.flags.writeable and y.dtype == np.complex64 and y.size == x.size
    y[:] = x                          # in place: the next call must read these values
    g = ld.ComplexFIRFilter(h=np.ones(1, np.float32))
    z = g(y)
    assert (_bits(z) == _bits(x)).all()


def test_pool_limit_falls_back_to_pageable(ld):
    raw = np.random.default_rng(1).integers(0, 255, 4 << 19, dtype=np.uint8).tobytes()   # -> 4 MB complex64
    first = ld.bytes_to_iq(raw)
    held = [ld.bytes_to_iq(raw) for _ in range(300)]     # 1.2 GB > the 1 GB page-locked limit
    for y in held[::25] + held[-3:]:
        assert (_bits(y) == _bits(first)).all()
    del held
    again = ld.bytes_to_iq(raw)                            # blocks back in the pool
    assert (_bits(again) == _bits(first)).all()


def test_host_pools_bounded_under_thread_churn(ld, lib, rng):
    # the staging pools of LDSP_MEM_HOST calls are per thread; a
    # thread that exits hands its pool back (thread_local holder), so 40
    # short-lived threads making host calls one after another reuse one pool
    # instead of each leaking 2 x 16 MB of page-locked memory.
    import threading
    x = (rng.standard_normal(1 << 16) + 1j * rng.standard_normal(1 << 16)).astype(np.complex64)
    f = ld.ComplexFIRFilter(np.float32([0.5, 0.25, 0.125]))
    f.mode = "exact"
    total0, idle0 = C.c_size_t(0), C.c_size_t(0)
    assert lib.ldsp_debug_host_pools(C.byref(total0), C.byref(idle0)) == 0
    outs = []

    def work():
        outs.append(f(x))

    for _ in range(40):
        t = threading.Thread(target=work)
        t.start()
        t.join()
    total, idle = C.c_size_t(0), C.c_size_t(0)
    assert lib.ldsp_debug_host_pools(C.byref(total), C.byref(idle)) == 0
    assert len(outs) == 40
    assert total.value <= total0.value + 1, (total0.value, total.value)
    assert idle.value >= 1
    # the calls still carried the filter state across threads in order
    ref = ld.ComplexFIRFilter(np.float32([0.5, 0.25, 0.125]))
    ref.mode = "exact"
    for i in range(40):
        assert np.array_equal(_bits(outs[i]), _bits(ref(x)))
