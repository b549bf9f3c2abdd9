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

/* ------------------------------------------------------------------------
 * Elliptic and Bessel analog prototypes for iirdes (design.cpp dzpk, ftype 3
 * and 4).  C, so that complex products, complex-by-real operations and the
 * glibc complex functions (ccosf, csinf, csqrtf, cacosf, cpow) behave exactly
 * as in liquid-dsp's own C; complex / complex divisions use Smith's method
 * (ldsp_cdivf above).  Algorithms (liquid src/filter/src/ellip.c and iirdes.c
 * ellip_azpkf / bessel_azpkf, recalled: parity unpinned): S. J. Orfanidis,
 * "Lecture notes on elliptic filter design" (Landen transformations, 7
 * iterations) with the analog pass-band edge at 1 rad/s; Bessel poles are the
 * roots of the reverse Bessel polynomial (Durand-Kerner in double) divided by
 * the approximate 3 dB frequency sqrt((2n-1) ln 2).
 * ---------------------------------------------------------------------- */
#include <complex.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#define ELLIP_NB 7

static float complex cdiv_(float complex x, float complex y)
{
    float o[2];
    ldsp_cdivf(crealf(x), cimagf(x), crealf(y), cimagf(y), o);
    return CMPLXF(o[0], o[1]);
}

static void landenf(float _k, unsigned int _n, float *_v)
{
    unsigned int i;
    float k = _k;
    for (i = 0; i < _n; i++) {
        float kp = sqrtf(1.0f - k * k);
        k = (k / (1.0f + kp)) * (k / (1.0f + kp));
        _v[i] = k;
    }
}

static void ellipkf(float _k, unsigned int _n, float *_K, float *_Kp)
{
    const float kmin = 4e-4f;
    const float kmax = sqrtf(1.0f - kmin * kmin);
    float kp = sqrtf(1.0f - _k * _k);
    float v[ELLIP_NB], vp[ELLIP_NB];
    unsigned int i;
    float K, Kp;
    if (_k > kmax) {
        float L = -logf(0.25f * kp);
        K = L + 0.25f * (L - 1.0f) * kp * kp;
    } else {
        landenf(_k, _n, v);
        K = (float)M_PI * 0.5f;
        for (i = 0; i < _n; i++) K *= (1.0f + v[i]);
    }
    if (kp > kmax) {
        float L = -logf(0.25f * _k);
        Kp = L + 0.25f * (L - 1.0f) * _k * _k;
    } else {
        landenf(kp, _n, vp);
        Kp = (float)M_PI * 0.5f;
        for (i = 0; i < _n; i++) Kp *= (1.0f + vp[i]);
    }
    *_K = K;
    *_Kp = Kp;
}

static float ellipdegf(float _N, float _k1, unsigned int _n)
{
    float K1, K1p;
    ellipkf(_k1, _n, &K1, &K1p);
    float q1 = expf(-(float)M_PI * K1p / K1);
    float q = powf(q1, 1.0f / _N);
    float b = 0.0f, a = 0.0f;
    unsigned int m;
    for (m = 0; m <= _n; m++) b += powf(q, (float)(m * (m + 1)));
    for (m = 1; m <= _n; m++) a += powf(q, (float)(m * m));
    float g = b / (1.0f + 2.0f * a);
    return 4.0f * sqrtf(q) * g * g;
}

static float complex ellip_cdf(float complex _u, float _k, unsigned int _n)
{
    float v[ELLIP_NB];
    landenf(_k, _n, v);
    float complex w = ccosf(_u * (float)(M_PI * 0.5));
    unsigned int i;
    for (i = _n; i > 0; i--) w = cdiv_((1.0f + v[i - 1]) * w, 1.0f + v[i - 1] * w * w);
    return w;
}

static float complex ellip_snf(float complex _u, float _k, unsigned int _n)
{
    float v[ELLIP_NB];
    landenf(_k, _n, v);
    float complex w = csinf(_u * (float)(M_PI * 0.5));
    unsigned int i;
    for (i = _n; i > 0; i--) w = cdiv_((1.0f + v[i - 1]) * w, 1.0f + v[i - 1] * w * w);
    return w;
}

static float complex ellip_acdf(float complex _w, float _k, unsigned int _n)
{
    float v[ELLIP_NB];
    landenf(_k, _n, v);
    float complex w = _w;
    unsigned int i;
    for (i = 0; i < _n; i++) {
        float v1 = (i == 0) ? _k : v[i - 1];
        w = cdiv_(w, 1.0f + csqrtf(1.0f - w * w * v1 * v1)) * 2.0f / (1.0f + v[i]);
    }
    return cacosf(w) * (float)(2.0 / M_PI);
}

static float complex ellip_asnf(float complex _w, float _k, unsigned int _n)
{
    return 1.0f - ellip_acdf(_w, _k, _n);
}

/* za: 2 (n / 2) zeros, pa: n poles, interleaved (re, im) */
void ldsp_ellip_azpkf(unsigned int _n, float _ep, float _es, float *za_out, float *pa_out)
{
    float complex *_za = (float complex *)za_out, *_pa = (float complex *)pa_out;
    const unsigned int nb = ELLIP_NB;
    const float k1 = _ep / _es;
    const float k = ellipdegf((float)_n, k1, nb);
    const unsigned int r = _n % 2, L = (_n - r) / 2;
    const float complex v0 = -_Complex_I * ellip_asnf(_Complex_I / _ep, k1, nb) / (float)_n;
    unsigned int i, t = 0;
    for (i = 0; i < L; i++) {
        float ui = (2.0f * (i + 1) - 1.0f) / (float)_n;
        float complex zeta = ellip_cdf(ui, k, nb);
        _za[2 * i] = cdiv_(_Complex_I, k * zeta);
        _za[2 * i + 1] = conjf(_za[2 * i]);
        float complex pz = _Complex_I * ellip_cdf(ui - _Complex_I * v0, k, nb);
        _pa[t++] = pz;
        _pa[t++] = conjf(pz);
    }
    if (r) _pa[t++] = crealf(_Complex_I * ellip_snf(_Complex_I * v0, k, nb));
}

/* pa: n poles, interleaved (re, im); n <= 48 */
void ldsp_bessel_azpkf(unsigned int _n, float *pa_out)
{
    float complex *_pa = (float complex *)pa_out;
    double c[65];
    double complex z[64];
    unsigned int i, j, it;
    c[_n] = 1.0;
    for (i = _n; i > 0; i--)
        c[i - 1] = c[i] * (double)(2 * _n - (i - 1)) * (double)i / (2.0 * (double)(_n - (i - 1)));
    const double rad = pow(c[0], 1.0 / _n);
    for (i = 0; i < _n; i++) z[i] = rad * cpow(0.4 + 0.9 * I, (double)i);
    for (it = 0; it < 1000; it++) {
        double delta = 0.0;
        for (i = 0; i < _n; i++) {
            double complex val = 0.0, den = 1.0;
            for (j = _n + 1; j > 0; j--) val = val * z[i] + c[j - 1];
            for (j = 0; j < _n; j++)
                if (j != i) den *= (z[i] - z[j]);
            double dd[2];
            ldsp_cdivd(creal(val), cimag(val), creal(den), cimag(den), dd);
            const double complex dz = CMPLX(dd[0], dd[1]);
            z[i] -= dz;
            delta = fmax(delta, cabs(dz) / cabs(z[i]));
        }
        if (delta < 1e-16) break;
    }
    const float w3dB = sqrtf((2 * _n - 1) * logf(2.0f));
    for (i = 0; i < _n; i++) _pa[i] = (float complex)z[i] / w3dB;
}
