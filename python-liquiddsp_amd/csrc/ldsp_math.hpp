// ldsp_math.hpp -- deterministic single-precision transcendentals for the
// sequential feedback loops (AGC gain update, PLL phase detector, Costas).
//
// liquid-dsp calls libm expf/logf (agc.proto.c execute, via agc_crcf_execute at
// reference src/agc.hpp:115) and cargf/tanhf (ampmodem.c demod, via
// ampmodem_demodulate_block at src/demod.hpp:294).  libm differs per platform,
// so the build fixes them to the fdlibm float algorithms (oracle/ora_math.h is
// the restatement).  Every function below yields exactly the bits of that
// restatement, but is written without data-dependent branches: all candidate
// results of fdlibm's argument-range cases are computed and the right one is
// selected.  On the GPU these loops run in one or a few lanes per wave, where
// exec-mask branching costs far more than the extra arithmetic; selects also
// keep the instruction stream identical for every lane of the chunked kernels.
// The library is compiled with -ffp-contract=off, so each expression is the
// same sequence of IEEE-754 single-precision operations as in the restatement.
// tests/test_gpu_parity.py::test_device_math_bitwise checks the device results
// against the restatement bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldsp {

__host__ __device__ inline uint32_t fbits(float x) { return __builtin_bit_cast(uint32_t, x); }
__host__ __device__ inline float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }
__host__ __device__ inline float fabs_(float x) { return bitsf(fbits(x) & 0x7fffffffu); }
__host__ __device__ inline float sel(bool c, float a, float b) { return c ? a : b; }

// (float)v / 32767.0f for int16 v (bytes_to_iq, reference src/utility.hpp:61-69)
// without the IEEE division sequence: the product with fl(1/32767) corrected by
// one fma residual step.  Equal to the correctly rounded quotient for all 65 536
// inputs (scripts/analysis/check_iq16_div.py, tests/test_oracle_math.py).
__device__ __forceinline__ float iq16_to_f(short v)
{
    constexpr float d = 32767.0f, r = 1.0f / 32767.0f;
    const float f = (float)v;
    const float q0 = f * r;
    return fmaf(fmaf(-q0, d, f), r, q0);
}

// e^x (fdlibm e_expf.c): x = k ln2 + r, rational kernel for e^r
__host__ __device__ inline float lm_expf(float x)
{
    constexpr float ln2hi = 6.9313812256e-01f, ln2lo = 9.0580006145e-06f, invln2 = 1.4426950216e+00f;
    constexpr float P1 = 1.6666667163e-01f, P2 = -2.7777778450e-03f, P3 = 6.6137559770e-05f,
                    P4 = -1.6533901999e-06f, P5 = 4.1381369442e-08f;
    const uint32_t hx = fbits(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const bool neg = (hx >> 31) != 0;
    // |x| in (0.5 ln2, 1.5 ln2): k = +-1
    const float hiA = x - (neg ? -ln2hi : ln2hi);
    const float loA = neg ? -ln2lo : ln2lo;
    // |x| >= 1.5 ln2: k = (int)(x/ln2 +- 0.5) (argument clamped only to keep the conversion defined)
    const float xc = x < -104.0f ? -104.0f : (x > 89.0f ? 89.0f : x);
    const int kB = (int)(invln2 * xc + (neg ? -0.5f : 0.5f));
    const float tB = (float)kB;
    const float hiB = x - tB * ln2hi;
    const float loB = tB * ln2lo;
    const bool big = ix > 0x3eb17218u;
    const bool mid = ix < 0x3F851592u;
    const float hi = mid ? hiA : hiB;
    const float lo = mid ? loA : loB;
    const int k = big ? (mid ? (neg ? -1 : 1) : kB) : 0;
    const float xr = big ? hi - lo : x;
    const float t = xr * xr;
    const float c = xr - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    const float q = (xr * c) / (c - 2.0f);                 // (xr*c)/(2-c) == -q exactly
    const float r0 = 1.0f - (q - xr);                      // k == 0
    const float y = 1.0f - ((lo + q) - hi);                // lo - (xr*c)/(2-c) == lo + q
    const uint32_t hy = fbits(y);
    const float yk = (k >= -125) ? bitsf(hy + ((uint32_t)k << 23))
                                 : bitsf(hy + ((uint32_t)(k + 100) << 23)) * bitsf(0x0d800000u);
    float r = big ? yk : r0;
    r = (ix < 0x31800000u) ? 1.0f + x : r;                 // |x| < 2^-28
    if (ix >= 0x42b17180u) {                                // rare: overflow / underflow / NaN / inf
        if (ix > 0x7f800000u) r = x + x;
        else if (ix == 0x7f800000u) r = neg ? 0.0f : x;
        else if (!neg) r = bitsf(0x7f800000u);
        else if (ix > 0x42cff1b5u) r = 0.0f;
    }
    return r;
}

// ln x (fdlibm e_logf.c)
__host__ __device__ inline float lm_logf(float x)
{
    constexpr float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    constexpr float Lg1 = 6.6666668653e-01f, Lg2 = 4.0000000596e-01f, Lg3 = 2.8571429849e-01f,
                    Lg4 = 2.2222198546e-01f, Lg5 = 1.8183572590e-01f, Lg6 = 1.5313838422e-01f,
                    Lg7 = 1.4798198640e-01f;
    const int32_t ix0 = (int32_t)fbits(x);
    const bool sub = ix0 < 0x00800000;                       // subnormal, zero or negative
    const float xs = sub ? x * 3.355443200e+07f : x;
    const int32_t ixs = (int32_t)fbits(xs);
    int32_t k = (sub ? -25 : 0) + (ixs >> 23) - 127;
    const int32_t m = ixs & 0x007fffff;
    const int32_t i = (m + (0x95f64 << 3)) & 0x800000;
    const float xn = bitsf((uint32_t)(m | (i ^ 0x3f800000)));
    k += (i >> 23);
    const float f = xn - 1.0f;
    const float dk = (float)k;
    const bool k0 = (k == 0);
    // |f| < 2^-20
    const float R1 = f * f * (0.5f - 0.33333333333333333f * f);
    const float sm_zero = k0 ? 0.0f : dk * ln2_hi + dk * ln2_lo;
    const float sm_nz = k0 ? f - R1 : dk * ln2_hi - ((R1 - dk * ln2_lo) - f);
    const float small = (f == 0.0f) ? sm_zero : sm_nz;
    // general
    const float s = f / (2.0f + f);
    const float z = s * s;
    int32_t ii = m - (0x6147a << 3);
    const float w = z * z;
    const int32_t j = (0x6b851 << 3) - m;
    const float t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const float t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    ii |= j;
    const float R = t2 + t1;
    const float hfsq = 0.5f * f * f;
    const float gA = k0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    const float gB = k0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
    float r = ((0x007fffff & (15 + m)) < 16) ? small : (ii > 0 ? gA : gB);
    if (sub || ix0 >= 0x7f800000) {                          // rare: zero / negative / inf / NaN
        if (ix0 >= 0x7f800000) r = x + x;
        else if ((ix0 & 0x7fffffff) == 0) r = -bitsf(0x7f800000u);
        else if (ix0 < 0) r = bitsf(0x7fc00000u);
    }
    return r;
}

// atan(t) for t >= 0 or NaN (fdlibm s_atanf.c, one division with selected operands)
__host__ __device__ inline float lm_atanf_pos(float t)
{
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const uint32_t ix = fbits(t) & 0x7fffffffu;
    const bool idm = ix < 0x3ee00000u;                  // id = -1: no reduction
    const bool lt1875 = ix < 0x3f980000u;
    const bool lt0687 = ix < 0x3f300000u;
    const bool lt24375 = ix < 0x401c0000u;
    // id 0: (2t-1)/(2+t)  id 1: (t-1)/(t+1)  id 2: (t-1.5)/(1+1.5t)  id 3: -1/t
    // (selects, not branches: vectorised callers stay in one basic block)
    const float n0 = 2.0f * t - 1.0f, n1 = t - 1.0f, n2 = t - 1.5f;
    const float d0 = 2.0f + t, d1 = t + 1.0f, d2 = 1.0f + 1.5f * t;
    float num = lt1875 ? (lt0687 ? n0 : n1) : (lt24375 ? n2 : -1.0f);
    float den = lt1875 ? (lt0687 ? d0 : d1) : (lt24375 ? d2 : t);
    const float hi = lt1875 ? (lt0687 ? 4.6364760399e-01f : 7.8539812565e-01f)
                            : (lt24375 ? 9.8279368877e-01f : 1.5707962513e+00f);
    const float lo = lt1875 ? (lt0687 ? 5.0121582440e-09f : 3.7748947079e-08f)
                            : (lt24375 ? 3.4473217170e-08f : 7.5497894159e-08f);
    num = idm ? t : num;
    den = idm ? 1.0f : den;
    const float xr = num / den;                         // t / 1.0 == t exactly
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    float r = idm ? xr - xr * (s1 + s2) : hi - ((xr * (s1 + s2) - lo) - xr);
    r = (ix < 0x39800000u) ? t : r;                     // |t| < 2^-12
    r = (ix >= 0x4c800000u) ? 1.5707962513e+00f + 7.5497894159e-08f : r;
    r = (ix > 0x7f800000u) ? t + t : r;                 // NaN
    return r;
}

// atan2(y, x) with C99 Annex F special cases; cargf(z) == lm_atan2f(imag, real)
__host__ __device__ inline float lm_atan2f(float y, float x)
{
    constexpr float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                    pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const int32_t k = (iy - ix) >> 23;
    float z = lm_atanf_pos(fabs_(y / x));
    z = (hx < 0 && k < -26) ? 0.0f : z;
    z = (k > 26) ? pi_o_2 + 0.5f * pi_lo : z;
    const float zm = z - pi_lo;
    const float q2 = zm - pi, q1 = pi - zm;
    float r = (m & 2) ? ((m & 1) ? q2 : q1) : ((m & 1) ? -z : z);
    // special operands, as selects (no divergent branches inside vectorised callers)
    const bool spec = iy == 0 || ix == 0 || ix >= 0x7f800000 || iy >= 0x7f800000;
    const float r_pm2 = (hy < 0) ? -pi_o_2 : pi_o_2;
    const float r_y0 = m <= 1 ? y : (m == 2 ? pi : -pi);
    const float r_ii = m == 0 ? pi_o_4 : m == 1 ? -pi_o_4 : m == 2 ? 3.0f * pi_o_4 : -3.0f * pi_o_4;
    const float r_ix = m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? pi : -pi;
    float rs = ix == 0x7f800000 ? (iy == 0x7f800000 ? r_ii : r_ix) : r_pm2;
    rs = ix == 0 ? r_pm2 : rs;
    rs = iy == 0 ? r_y0 : rs;
    rs = (ix > 0x7f800000 || iy > 0x7f800000) ? x + y : rs;
    return spec ? rs : r;
}

// c ? a : b as one v_cndmask on the device (a ballot of c as the lane mask), a
// plain select on the host.  The candidate evaluations of the one-wave serial
// loops (k_pll_seqc, k_fm_pll) call atan2 through lm_atan2f_vsel below: with
// lm_atan2f's ternaries the compiler forms exec-mask regions, which end the
// basic block and keep the candidates from interleaving with the chain steps.
__host__ __device__ inline float vsel(bool c, float a, float b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    const uint64_t m = __builtin_amdgcn_ballot_w64(c);
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
#else
    return c ? a : b;
#endif
}

// lm_atan2f operation for operation (lm_atanf_pos inlined), every select a
// vsel.  The same IEEE operations in the same order, so the same bits
// (ldsp_debug_math_eval fn 7; tests/test_gpu_parity.py::test_device_math_bitwise).
__host__ __device__ inline float lm_atan2f_vsel(float y, float x)
{
    constexpr float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                    pi_lo = -8.7422776573e-08f;
    constexpr float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                    aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                    aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                    aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const int32_t k = (iy - ix) >> 23;
    // lm_atanf_pos(|y / x|)
    const float t = fabs_(y / x);
    const uint32_t it = fbits(t) & 0x7fffffffu;
    const bool idm = it < 0x3ee00000u, lt1875 = it < 0x3f980000u, lt0687 = it < 0x3f300000u,
               lt24375 = it < 0x401c0000u;
    const float n0 = 2.0f * t - 1.0f, n1 = t - 1.0f, n2 = t - 1.5f;
    const float d0 = 2.0f + t, d1 = t + 1.0f, d2 = 1.0f + 1.5f * t;
    float num = vsel(lt1875, vsel(lt0687, n0, n1), vsel(lt24375, n2, -1.0f));
    float den = vsel(lt1875, vsel(lt0687, d0, d1), vsel(lt24375, d2, t));
    const float hi = vsel(lt1875, vsel(lt0687, 4.6364760399e-01f, 7.8539812565e-01f),
                          vsel(lt24375, 9.8279368877e-01f, 1.5707962513e+00f));
    const float lo = vsel(lt1875, vsel(lt0687, 5.0121582440e-09f, 3.7748947079e-08f),
                          vsel(lt24375, 3.4473217170e-08f, 7.5497894159e-08f));
    num = vsel(idm, t, num);
    den = vsel(idm, 1.0f, den);
    const float xr = num / den;
    const float zz = xr * xr;
    const float w = zz * zz;
    const float s1 = zz * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    float z = vsel(idm, xr - xr * (s1 + s2), hi - ((xr * (s1 + s2) - lo) - xr));
    z = vsel(it < 0x39800000u, t, z);
    z = vsel(it >= 0x4c800000u, 1.5707962513e+00f + 7.5497894159e-08f, z);
    z = vsel(it > 0x7f800000u, t + t, z);
    // lm_atan2f after the atan
    z = vsel(hx < 0 && k < -26, 0.0f, z);
    z = vsel(k > 26, pi_o_2 + 0.5f * pi_lo, z);
    const float zm = z - pi_lo;
    const float q2 = zm - pi, q1 = pi - zm;
    const float r = vsel((m & 2) != 0, vsel((m & 1) != 0, q2, q1), vsel((m & 1) != 0, -z, z));
    const bool spec = iy == 0 || ix == 0 || ix >= 0x7f800000 || iy >= 0x7f800000;
    const float r_pm2 = vsel(hy < 0, -pi_o_2, pi_o_2);
    const float r_y0 = vsel(m <= 1, y, vsel(m == 2, pi, -pi));
    const float r_ii = vsel(m == 0, pi_o_4, vsel(m == 1, -pi_o_4, vsel(m == 2, 3.0f * pi_o_4, -3.0f * pi_o_4)));
    const float r_ix = vsel(m == 0, 0.0f, vsel(m == 1, -0.0f, vsel(m == 2, pi, -pi)));
    float rs = vsel(ix == 0x7f800000, vsel(iy == 0x7f800000, r_ii, r_ix), r_pm2);
    rs = vsel(ix == 0, r_pm2, rs);
    rs = vsel(iy == 0, r_y0, rs);
    rs = vsel(ix > 0x7f800000 || iy > 0x7f800000, x + y, rs);
    return vsel(spec, rs, r);
}

// tanh: odd minimax polynomial below 0.625, 1 - 2/(e^{2|x|}+1) above
__host__ __device__ inline float lm_tanhf(float x)
{
    constexpr float T1 = -3.3333331347e-01f, T2 = 1.3333205879e-01f, T3 = -5.3946767002e-02f,
                    T4 = 2.1700724959e-02f, T5 = -8.1774443388e-03f, T6 = 2.1430002525e-03f;
    const uint32_t hx = fbits(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const float a = bitsf(ix);
    const float zz = a * a;
    const float rp = a + a * (zz * (T1 + zz * (T2 + zz * (T3 + zz * (T4 + zz * (T5 + zz * T6))))));
    const float te = lm_expf(2.0f * (ix >= 0x41100000u ? 1.0f : a));
    const float re = 1.0f - 2.0f / (te + 1.0f);
    float r = (ix >= 0x3f200000u) ? re : rp;
    r = (ix >= 0x41100000u) ? 1.0f : r;
    r = (hx >> 31) ? -r : r;
    r = (ix < 0x39800000u) ? x : r;
    r = (ix > 0x7f800000u) ? x + x : r;
    return r;
}

// ---- Fast paths for the serial loops.  A wave running one dependent chain
// issues one wave64 instruction per ~4 cycles, so a loop step costs about its
// instruction count (scripts/ubench/loop_lat.hip: lm_logf 184 ns, lm_expf 144,
// lm_atan2f 299 against 7 ns for a dependent mul + add).  The functions below
// are the same operation sequences as lm_logf / lm_expf restricted to the
// common argument range, where most of fdlibm's cases (zero, subnormal,
// infinite, NaN, |f| < 2^-20, reduced exponent) cannot occur; callers test
// *_fast_ok and take the general function otherwise.  (The same treatment of
// lm_atan2f measured slower: its cases are already selects, and a range test
// plus a branch to the general code cost more than the few selects saved; a
// near-lock atan2 (|y / x| < 0.4375: no reduction, no second division) behind a
// wave-uniform test slowed the PLL candidates by 20 %: their 64 lanes run 64
// chunks, and one lane out of range sends the wave through both paths.)  Equality with the general
// functions over the whole fast range: ldsp_debug_math_fastcheck
// (tests/test_capi_host.py samples it; scripts/analysis/check_fast_math.py runs
// every float).

// n / d correctly rounded, for operands that need no range scaling (|d| in
// [1, 4), n zero or |n| in [2^-64, 4)): on the device the compiler's own IEEE
// sequence (reciprocal, one Newton step, two residual corrections) without its
// v_div_scale / v_div_fmas scaling and v_div_fixup special cases, which such
// operands never trigger -- the same bits in 8 instructions instead of 11.
__host__ __device__ inline float div_noscale(float n, float d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    float r = __builtin_amdgcn_rcpf(d);
    float e = fmaf(-d, r, 1.0f);
    r = fmaf(e, r, r);
    float q = n * r;
    e = fmaf(-d, q, n);
    q = fmaf(e, r, q);
    e = fmaf(-d, q, n);
    return fmaf(e, r, q);
#else
    return n / d;
#endif
}

// lm_logf for normal, positive, finite x with |f| >= 2^-20
__host__ __device__ inline bool lm_logf_fast_ok(float x)
{
    const int32_t ix = (int32_t)fbits(x);
    return ix >= 0x00800000 && ix < 0x7f800000 && (0x007fffff & (15 + (ix & 0x007fffff))) >= 16;
}
__host__ __device__ inline float lm_logf_fast(float x)
{
    constexpr float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    constexpr float Lg1 = 6.6666668653e-01f, Lg2 = 4.0000000596e-01f, Lg3 = 2.8571429849e-01f,
                    Lg4 = 2.2222198546e-01f, Lg5 = 1.8183572590e-01f, Lg6 = 1.5313838422e-01f,
                    Lg7 = 1.4798198640e-01f;
    const int32_t ix = (int32_t)fbits(x);
    const int32_t m = ix & 0x007fffff;
    const int32_t i = (m + (0x95f64 << 3)) & 0x800000;
    const int32_t k = (ix >> 23) - 127 + (i >> 23);
    const float f = bitsf((uint32_t)(m | (i ^ 0x3f800000))) - 1.0f;
    const float s = div_noscale(f, 2.0f + f);            // f in (-0.293, 0.415], f == 0 or |f| >= 2^-23
    const float dk = (float)k;
    const float z = s * s;
    const float w = z * z;
    const float t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const float t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const float R = t2 + t1;
    const bool ii = ((m - (0x6147a << 3)) | ((0x6b851 << 3) - m)) > 0;
    const float hfsq = 0.5f * f * f;
    if (k == 0) return ii ? f - (hfsq - s * (hfsq + R)) : f - s * (f - R);
    return ii ? dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f)
              : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// lm_expf for 2^-28 <= |x| <= 0.5 ln2 (no argument reduction: k = 0)
__host__ __device__ inline bool lm_expf_fast_ok(float x)
{
    const uint32_t ix = fbits(x) & 0x7fffffffu;
    return ix >= 0x31800000u && ix <= 0x3eb17218u;
}
__host__ __device__ inline float lm_expf_fast(float x)
{
    constexpr float P1 = 1.6666667163e-01f, P2 = -2.7777778450e-03f, P3 = 6.6137559770e-05f,
                    P4 = -1.6533901999e-06f, P5 = 4.1381369442e-08f;
    const float t = x * x;
    const float c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    return 1.0f - (div_noscale(x * c, c - 2.0f) - x);    // c - 2 ~ -2, |x c| in [2^-57, 0.25]
}

// The general function, through the fast path when x is in its range (a
// branch, not a select: a wave whose lanes are all in range skips the general
// code).
__host__ __device__ inline float lm_logf_loop(float x)
{
    if (__builtin_expect(lm_logf_fast_ok(x), 1)) return lm_logf_fast(x);
    return lm_logf(x);
}
__host__ __device__ inline float lm_expf_loop(float x)
{
    if (__builtin_expect(lm_expf_fast_ok(x), 1)) return lm_expf_fast(x);
    return lm_expf(x);
}
// NCO(_constrain) (liquid nco.proto.c): radians -> 32-bit fixed-point phase.
// p is formed in double (1/2pi literal is double), the fraction in float
// ((float)(long)p == truncf(p)), the negative wrap in double, and the
// float->uint32 conversion goes through int64 as x86-64 gcc lowers it
// (fpart*2^32 == 2^32 wraps to 0).
__host__ __device__ inline uint32_t lm_constrain(float theta)
{
    const float p = (float)((double)theta * 0.159154943091895);
    float fpart = p - truncf(p);
    const float fneg = (float)((double)fpart + 1.0);
    fpart = fpart < 0.0f ? fneg : fpart;
    const float v = fpart * 4294967296.0f;
    return v >= 4294967296.0f ? 0u : (uint32_t)v;
}

// lm_constrain with the fraction from v_fract (p - floor(p), which the hardware
// keeps below 1): for p >= 0 that is p - trunc(p); for p < 0 it is the exact
// p - trunc(p) + 1 rounded once, as the reference's double add then float
// rounding gives, except where that rounds to 1.0 -- p in [-2^-25, 0), where
// the reference's fpart * 2^32 = 2^32 wraps to 0 and v_fract gives 1 - 2^-24:
// those p return 0 explicitly.  Bitwise to lm_constrain (ldsp_debug_math_eval
// fn 8 vs 4 in tests/test_gpu_parity.py), four operations shorter.  (The host
// form states v_fract's definition; only the device one is used.)
__host__ __device__ inline uint32_t lm_constrain_fr(float theta)
{
    const float p = (float)((double)theta * 0.159154943091895);
#if defined(__HIP_DEVICE_COMPILE__)
    const float fr = __builtin_amdgcn_fractf(p);
#else
    const float fr = fminf(p - floorf(p), 0x1.fffffep-1f);
#endif
    const uint32_t v = (uint32_t)(fr * 4294967296.0f);
    uint32_t pb;
    __builtin_memcpy(&pb, &p, 4);
    return pb - 0x80000001u <= 0x32FFFFFFu ? 0u : v;
}

} // namespace ldsp
