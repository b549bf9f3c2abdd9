/*
 * ora_math.h -- deterministic single-precision transcendentals for the oracle.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/liquid_restate.c header).
 *
 * liquid-dsp calls the platform libm (expf/logf inside agc_crcf_execute, cargf
 * inside ampmodem_demod_dsb_pll_carrier, tanhf inside the Costas demod).  libm
 * results differ by an ulp between glibc, Apple libm and ROCm's ocml, so "the"
 * liquid-dsp output of those feedback loops is platform-defined.  The
 * restatement pins them to the classic fdlibm float algorithms below, written
 * as plain IEEE single-precision operations (no FMA, compile with
 * -ffp-contract=off).  The GPU kernels (python-liquiddsp_amd/csrc/ldsp_math.hpp)
 * implement the same operation sequence independently, so a sequential loop
 * evaluated on the GPU is bit-identical to this restatement.  Accuracy of each
 * function against a double-precision libm is checked in
 * tests/test_oracle_math.py (<= 1 ulp).
 *
 * Building with -DORA_USE_LIBM=1 makes the oracle call the system libm instead
 * (documented switch; the GPU parity tests require the default).
 */
#ifndef ORA_MATH_H
#define ORA_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint32_t om_bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static inline float om_float(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }

#if ORA_USE_LIBM
static inline float om_expf(float x) { return expf(x); }
static inline float om_logf(float x) { return logf(x); }
static inline float om_atan2f(float y, float x) { return atan2f(y, x); }
static inline float om_tanhf(float x) { return tanhf(x); }
#else

/* expf: fdlibm e_expf.c argument reduction x = k ln2 + r, rational kernel. */
static inline float om_expf(float x)
{
    const float ln2hi = 6.9313812256e-01f;   /* 0x3f317180 */
    const float ln2lo = 9.0580006145e-06f;   /* 0x3717f7d1 */
    const float invln2 = 1.4426950216e+00f;  /* 0x3fb8aa3b */
    const float P1 = 1.6666667163e-01f, P2 = -2.7777778450e-03f,
                P3 = 6.6137559770e-05f, P4 = -1.6533901999e-06f,
                P5 = 4.1381369442e-08f;
    uint32_t hx = om_bits(x);
    uint32_t ix = hx & 0x7fffffffu;
    int sx = (int)(hx >> 31);
    float hi = 0.0f, lo = 0.0f, t, c, y;
    int k = 0;
    if (ix >= 0x42b17180u) {                   /* |x| >= 88.7217 or NaN */
        if (ix > 0x7f800000u) return x + x;    /* NaN */
        if (ix == 0x7f800000u) return sx ? 0.0f : x;
        if (!sx) return om_float(0x7f800000u); /* overflow */
        if (ix > 0x42cff1b5u) return 0.0f;     /* underflow */
    }
    if (ix > 0x3eb17218u) {                    /* |x| > 0.5 ln2 */
        if (ix < 0x3F851592u) {                /* |x| < 1.5 ln2 */
            hi = x - (sx ? -ln2hi : ln2hi);
            lo = sx ? -ln2lo : ln2lo;
            k = 1 - sx - sx;
        } else {
            k = (int)(invln2 * x + (sx ? -0.5f : 0.5f));
            t = (float)k;
            hi = x - t * ln2hi;
            lo = t * ln2lo;
        }
        x = hi - lo;
    } else if (ix < 0x31800000u) {             /* |x| < 2^-28 */
        return 1.0f + x;
    }
    t = x * x;
    c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0f - ((x * c) / (c - 2.0f) - x);
    y = 1.0f - ((lo - (x * c) / (2.0f - c)) - hi);
    if (k >= -125) {
        uint32_t hy = om_bits(y);
        return om_float(hy + ((uint32_t)k << 23));
    } else {
        uint32_t hy = om_bits(y);
        return om_float(hy + ((uint32_t)(k + 100) << 23)) * om_float(0x0d800000u); /* 2^-100 */
    }
}

/* logf: fdlibm e_logf.c */
static inline float om_logf(float x)
{
    const float ln2_hi = 6.9313812256e-01f;  /* 0x3f317180 */
    const float ln2_lo = 9.0580006145e-06f;  /* 0x3717f7d1 */
    const float Lg1 = 6.6666668653e-01f, Lg2 = 4.0000000596e-01f,
                Lg3 = 2.8571429849e-01f, Lg4 = 2.2222198546e-01f,
                Lg5 = 1.8183572590e-01f, Lg6 = 1.5313838422e-01f,
                Lg7 = 1.4798198640e-01f;
    float hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k, ix, i, j;
    ix = (int32_t)om_bits(x);
    k = 0;
    if (ix < 0x00800000) {                      /* x < 2^-126 */
        if ((ix & 0x7fffffff) == 0) return -om_float(0x7f800000u);  /* log(+-0) = -inf */
        if (ix < 0) return om_float(0x7fc00000u);                   /* log(-#) = NaN */
        k -= 25;
        x *= 3.355443200e+07f;                  /* 2^25: subnormal, scale up */
        ix = (int32_t)om_bits(x);
    }
    if (ix >= 0x7f800000) return x + x;
    k += (ix >> 23) - 127;
    ix &= 0x007fffff;
    i = (ix + (0x95f64 << 3)) & 0x800000;
    x = om_float((uint32_t)(ix | (i ^ 0x3f800000)));  /* normalize x or x/2 */
    k += (i >> 23);
    f = x - 1.0f;
    if ((0x007fffff & (15 + ix)) < 16) {        /* |f| < 2^-20 */
        if (f == 0.0f) {
            if (k == 0) return 0.0f;
            dk = (float)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5f - 0.33333333333333333f * f);
        if (k == 0) return f - R;
        dk = (float)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0f + f);
    dk = (float)k;
    z = s * s;
    i = ix - (0x6147a << 3);
    w = z * z;
    j = (0x6b851 << 3) - ix;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5f * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* atanf: fdlibm s_atanf.c */
static inline float om_atanf(float x)
{
    static const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f,
                                    9.8279368877e-01f, 1.5707962513e+00f};
    static const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f,
                                    3.4473217170e-08f, 7.5497894159e-08f};
    static const float aT[11] = {
        3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f,
        -1.1111110449e-01f, 9.0908870101e-02f, -7.6918758452e-02f,
        6.6610731184e-02f, -5.8335702866e-02f, 4.9768779427e-02f,
        -3.6531571299e-02f, 1.6285819933e-02f};
    float w, s1, s2, z;
    int32_t ix, hx, id;
    hx = (int32_t)om_bits(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x4c800000) {                     /* |x| >= 2^26 */
        if (ix > 0x7f800000) return x + x;      /* NaN */
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {                      /* |x| < 0.4375 */
        if (ix < 0x39800000) return x;          /* |x| < 2^-12 */
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {                  /* |x| < 1.1875 */
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else                 { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else                 { id = 3; x = -1.0f / x; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -z : z;
}

/* atan2f: fdlibm e_atan2f.c (quadrant logic), used for cargf(z) = atan2f(im, re) */
static inline float om_atan2f(float y, float x)
{
    const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    float z;
    int32_t k, m, hx, hy, ix, iy;
    hx = (int32_t)om_bits(x); ix = hx & 0x7fffffff;
    hy = (int32_t)om_bits(y); iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;   /* NaN */
    if (hx == 0x3f800000) return om_atanf(y);              /* x = 1.0 */
    m = ((hy >> 31) & 1) | ((hx >> 30) & 2);                /* 2*sign(x)+sign(y) */
    if (iy == 0) {
        switch (m) {
        case 0: case 1: return y;
        case 2: return pi;
        default: return -pi;
        }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 : pi_o_2;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4;
            case 1: return -pi_o_4;
            case 2: return 3.0f * pi_o_4;
            default: return -3.0f * pi_o_4;
            }
        } else {
            switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi;
            default: return -pi;
            }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 : pi_o_2;
    k = (iy - ix) >> 23;
    if (k > 26) z = pi_o_2 + 0.5f * pi_lo;               /* |y/x| > 2^26 */
    else if (hx < 0 && k < -26) z = 0.0f;                /* |y|/x < -2^26 */
    else z = om_atanf(fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

/* tanhf: odd minimax polynomial for |x| < 0.625, 1 - 2/(e^{2|x|}+1) above. */
static inline float om_tanhf(float x)
{
    uint32_t hx = om_bits(x);
    uint32_t ix = hx & 0x7fffffffu;
    float a = om_float(ix), r;
    if (ix > 0x7f800000u) return x + x;        /* NaN */
    if (ix >= 0x41100000u) {                   /* |x| >= 9: tanh = +-1 to float precision */
        r = 1.0f;
    } else if (ix >= 0x3f200000u) {            /* |x| >= 0.625 */
        float t = om_expf(2.0f * a);
        r = 1.0f - 2.0f / (t + 1.0f);
    } else if (ix < 0x39800000u) {             /* |x| < 2^-12 */
        return x;
    } else {
        const float T1 = -3.3333331347e-01f, T2 = 1.3333205879e-01f,
                    T3 = -5.3946767002e-02f, T4 = 2.1700724959e-02f,
                    T5 = -8.1774443388e-03f, T6 = 2.1430002525e-03f;
        float z = a * a;
        r = a + a * (z * (T1 + z * (T2 + z * (T3 + z * (T4 + z * (T5 + z * T6))))));
    }
    return (hx >> 31) ? -r : r;
}
#endif /* ORA_USE_LIBM */

#endif /* ORA_MATH_H */
