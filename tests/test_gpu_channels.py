"""BASELINE config 5 on one GPU (the one-GPU proxy of SURVEY 8(e)): eight
independent AMRadio channels (README.md:41-58 of the reference; carriers and
seeds as bench.py's ranks), each object driving two HIP streams, all eight in
flight at once on one MI355X, as bench.py's channels_per_gpu component runs
them.  Each channel must give the same bits as the same object run alone,
call after call on one stream: the objects share nothing (state, scratch,
stream marks), so any cross-object race shows up as a bit difference.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ld():
    import liquiddsp
    assert liquiddsp.device_count() > 0
    return liquiddsp


def test_eight_channels_concurrent_equal_alone(ld):
    import torch
    import bench
    dev = torch.device("cuda", 0)
    channels, calls, n, per = 8, 3, 16 << 20, 2
    xs = [bench.synth_channel(n * calls, c, dev) for c in range(channels)]
    radios = [bench.AMRadio(ld) for _ in range(channels)]
    strm = [[torch.cuda.Stream(dev) for _ in range(per)] for _ in range(channels)]
    torch.cuda.synchronize()
    outs = [[] for _ in range(channels)]
    for k in range(calls):                        # every channel's call k in flight together
        for c in range(channels):
            with torch.cuda.stream(strm[c][k % per]):
                outs[c].append(radios[c](xs[c][k * n:(k + 1) * n]))
    torch.cuda.synchronize()
    for c in range(channels):
        alone = bench.AMRadio(ld)
        for k in range(calls):
            r = alone(xs[c][k * n:(k + 1) * n])
            torch.cuda.synchronize()
            y = outs[c][k]
            assert y.shape == r.shape and y.numel() > 300_000, (c, k, y.shape, r.shape)
            if not torch.equal(y.view(torch.int32), r.view(torch.int32)):
                nd = int((y.view(torch.int32) != r.view(torch.int32)).sum())
                raise AssertionError(f"channel {c} call {k}: {nd} of {y.numel()} PCM samples differ from the lone run")
        assert alone.am.pll_state() == radios[c].am.pll_state()
        assert np.float32(alone.agc.gain) == np.float32(radios[c].agc.gain)
