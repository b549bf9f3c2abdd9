"""Test configuration.

Markers: `gpu` = needs an MI355X (HIP device); everything else runs on CPU.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD GPU (MI355X) and the HIP library")
    config.addinivalue_line("markers", "slow: long-running test")


def _have_gpu() -> bool:
    return os.path.exists("/dev/kfd")


def pytest_collection_modifyitems(config, items):
    if _have_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU (/dev/kfd absent)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def ora():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture
def rng():
    import numpy as np
    return np.random.default_rng(1234)


def cgauss(rng, n, scale=1.0):
    import numpy as np
    return (scale * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)


def maxrel(y, ref):
    import numpy as np
    y = np.asarray(y)
    ref = np.asarray(ref)
    den = np.max(np.abs(ref)) if ref.size else 1.0
    return float(np.max(np.abs(y.astype(np.complex128) - ref.astype(np.complex128))) / (den if den else 1.0)) if ref.size else 0.0
