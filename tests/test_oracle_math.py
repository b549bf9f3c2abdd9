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
