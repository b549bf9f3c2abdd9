"""Inputs of the AmpModem PLL for walk_spec.c: x0 = the carrier lowpass of the
AmpModem input (am_in.c64 from gen_agc_input.py), the NCO table.  CPU only (oracle)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import oracle as O  # noqa: E402

x = np.fromfile(os.path.join(HERE, "am_in.c64"), np.complex64)
lp = O.FIRFilter(kaiser=(51, 0.01, 40.0, 0.0), cplx=True)
lp(x).tofile(os.path.join(HERE, "pll_x0.c64"))
O.NCO(0).table.tofile(os.path.join(HERE, "nco_table.f32"))
print(x.size)
