"""liquiddsp -- MI355X-native drop-in for python-liquiddsp's streaming DSP classes.

The classes live in the compiled extension `_liquiddsp` (pybind11) over the C
ABI of libldsp.so (HIP kernels for gfx950).  torch is imported first when it is
installed: torch ships its own copy of the HIP runtime with the same SONAME
(libamdhip64.so.7) as /opt/rocm, and loading it first makes libldsp share that
single runtime, so device pointers and streams of torch tensors are valid in
libldsp calls.
"""
try:  # noqa: SIM105
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - numpy-only use
    torch = None

from ._liquiddsp import *  # noqa: F401,F403
from ._liquiddsp import (__backend__, _debug_iir_sect_trace, _debug_pll_margin, _debug_walk_early, _math_eval, _profile_enable, _profile_only,  # noqa: F401
                         _profile_report, _profile_reset, device_count)
