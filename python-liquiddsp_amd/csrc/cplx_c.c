/* cplx_c.c -- complex division for the host-side filter design (design.cpp).
 *
 * liquid-dsp is C: its designs divide _Complex values with C's `/`, i.e. the
 * runtime routines __divsc3 / __divdc3.  Their algorithm depends on the
 * runtime version (GCC <= 11 libgcc: Smith's method; newer libgcc_s: scaled /
 * widened variants -- both exist in this image and give 1-ulp different cheby2
 * poles), so the division is pinned here explicitly to Smith's method, the
 * algorithm of the GCC 11 libgcc the restatement (oracle/) is linked with.
 * Finite operands only (designs never divide by zero or infinity). */
#include <math.h>

void ldsp_cdivf(float a, float b, float c, float d, float *out)
{
    float ratio, denom;
    if (fabsf(c) < fabsf(d)) {
        ratio = c / d;
        denom = (c * ratio) + d;
        out[0] = ((a * ratio) + b) / denom;
        out[1] = ((b * ratio) - a) / denom;
    } else {
        ratio = d / c;
        denom = (d * ratio) + c;
        out[0] = ((b * ratio) + a) / denom;
        out[1] = (b - (a * ratio)) / denom;
    }
}

void ldsp_cdivd(double a, double b, double c, double d, double *out)
{
    double ratio, denom;
    if (fabs(c) < fabs(d)) {
        ratio = c / d;
        denom = (c * ratio) + d;
        out[0] = ((a * ratio) + b) / denom;
        out[1] = ((b * ratio) - a) / denom;
    } else {
        ratio = d / c;
        denom = (d * ratio) + c;
        out[0] = ((b * ratio) + a) / denom;
        out[1] = (b - (a * ratio)) / denom;
    }
}
