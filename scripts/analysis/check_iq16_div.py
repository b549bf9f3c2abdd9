"""Exhaustive check: for every int16 v, the three-operation sequence
   q0 = v * r;  e = fma(-q0, 32767, v);  q = fma(e, r, q0)   (r = fl(1/32767))
gives exactly (float)v / 32767.0f, the correctly rounded quotient bytes_to_iq
computes (src/utility.hpp:61-69).  fma is evaluated exactly with fractions and
rounded to float32 once (ties to even)."""
from fractions import Fraction
import numpy as np


def rn32(x: Fraction) -> np.float32:
    f = np.float32(float(x))
    best = None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        err = abs(Fraction(float(c)) - x)
        key = (err, int(np.float32(c).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, c)
    return np.float32(best[1])


d = np.float32(32767.0)
r = np.float32(1) / d
bad = 0
for v in range(-32768, 32768):
    fv = np.float32(v)
    ref = fv / d
    q0 = fv * r
    e = rn32(Fraction(v) - Fraction(float(q0)) * 32767)
    q = rn32(Fraction(float(e)) * Fraction(float(r)) + Fraction(float(q0)))
    if q.view(np.uint32) != ref.view(np.uint32):
        bad += 1
print("mismatches:", bad)
