"""Deterministic transcendentals used inside the AGC / PLL feedback loops
(oracle/ora_math.h): accuracy against float64 numpy must be within ~1.5 ulp,
so pinning them costs nothing against any libm."""
import numpy as np
import pytest


def _ulp_err(y, ref):
    ref32 = ref.astype(np.float32)
    sp = np.spacing(np.abs(ref32)).astype(np.float64)
    return float(np.max(np.abs(y.astype(np.float64) - ref) / sp))


@pytest.mark.parametrize("lo,hi", [(-20, 20), (-87, 88), (-1e-3, 1e-3)])
def test_expf(ora, rng, lo, hi):
    x = np.float32(rng.uniform(lo, hi, 400_000))
    assert _ulp_err(ora.math_eval("exp", x), np.exp(x.astype(np.float64))) <= 1.0


def test_logf(ora, rng):
    x = np.float32(np.exp(rng.uniform(-85, 85, 400_000)))
    x = np.concatenate([x, np.float32([1.0, 2.0, 0.5, 1e-40, 3e-39])])
    assert _ulp_err(ora.math_eval("log", x), np.log(x.astype(np.float64))) <= 1.0


def test_atan2f(ora, rng):
    a = np.float32(rng.standard_normal(400_000))
    b = np.float32(rng.standard_normal(400_000))
    ref = np.arctan2(a.astype(np.float64), b.astype(np.float64))
    assert _ulp_err(ora.math_eval("atan2", a, b), ref) <= 1.5
    # quadrant / signed-zero special cases follow C99 Annex F
    ys = np.float32([0.0, -0.0, 0.0, -0.0, 1.0, -1.0, np.inf, -np.inf])
    xs = np.float32([1.0, 1.0, -1.0, -1.0, 0.0, 0.0, np.inf, -np.inf])
    np.testing.assert_allclose(ora.math_eval("atan2", ys, xs), np.arctan2(ys, xs), rtol=1e-7)


def test_tanhf(ora, rng):
    x = np.float32(rng.uniform(-10, 10, 400_000))
    x = np.concatenate([x, np.float32(rng.uniform(-0.7, 0.7, 100_000))])
    assert _ulp_err(ora.math_eval("tanh", x), np.tanh(x.astype(np.float64))) <= 1.5


def test_iq16_conversion_sequence_exact():
    """The fused int16 IQ load (k_iir_blk<IQ16>, iq16_to_f) replaces
    (float)v / 32767.0f (bytes_to_iq, src/utility.hpp:61-69) by a product and
    one fma residual correction; it must give the same float for every int16."""
    import runpy, io, contextlib, os
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        runpy.run_path(os.path.join(os.path.dirname(__file__), "..", "scripts", "analysis", "check_iq16_div.py"),
                       run_name="__main__")
    assert buf.getvalue().strip() == "mismatches: 0"
