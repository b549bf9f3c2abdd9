/* FMStereo phase error from a per-index interval (CPU model, analysis only).
 *
 * For x != 0 the mixer's atan2 argument is (fl(-x sn), fl(x cs)) with (sn, cs)
 * the table entry of the current index, so atan2 sees the quotient
 * q' = fl(|x sn| (1+d1) / (|x cs| (1+d2))), |d1|, |d2| <= 2^-24: a handful of
 * floats around fl(|sn / cs|), whichever x is.  Enumerating them per index gives
 * the exact range [r_lo, r_hi] of the atan2 result for x > 0 and for x < 0.  The
 * phase-error update pe' = (float)(0.999 pe + 0.001 r) is monotone in r, so
 * where pe'(r_lo) == pe'(r_hi) the table gives the exact pe' without atan2.
 * This counts how often the two differ (the step then needs the real atan2)
 * and checks that the true pe' always lies between them.
 *   gcc -O2 -ffp-contract=off -o fm_interval fm_interval.c -lm && ./fm_interval fm_s.f32
 */
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
#include "../../oracle/ora_math.h"

static float tab[1024];
static float rlo[2][1024], rhi[2][1024];
static int valid[1024];

static uint32_t C_(float th)
{
    float p = th * 0.159154943091895;
    float fp = p - ((long)p);
    if (fp < 0.) fp += 1.;
    return (uint32_t)(int64_t)(fp * 0xffffffff);
}
static inline uint32_t idxof(uint32_t th) { return ((th + (1u << 21)) >> 22) & 0x3ff; }

static float quad(int m, float z)
{
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const float zm = z - pi_lo;
    return (m & 2) ? ((m & 1) ? zm - pi : pi - zm) : ((m & 1) ? -z : z);
}

int main(int argc, char** argv)
{
    const float al = 0.1f, be = sqrtf(al);
    for (int i = 0; i < 1024; i++) tab[i] = sinf(2.0f * M_PI * (float)(i) / 1024.0f);
    int nval = 0, maxw = 0;
    for (int i = 0; i < 1024; i++) {
        const float sn = tab[i], cs = tab[(i + 256) & 1023];
        valid[i] = fabsf(sn) >= 0x1p-20f && fabsf(cs) >= 0x1p-20f && fabsf(sn / cs) < 0x1p20f && fabsf(sn / cs) > 0x1p-20f;
        if (!valid[i]) continue;
        nval++;
        const double qe = fabs((double)sn / (double)cs);
        const double e = 0x1p-24;
        const float qlo = nextafterf((float)(qe * (1 - e) / (1 + e)), 0.0f);
        const float qhi = nextafterf((float)(qe * (1 + e) / (1 - e)), INFINITY);
        for (int sg = 0; sg < 2; sg++) {           /* sg 0: x > 0, 1: x < 0 */
            const float xs = sg ? -1.0f : 1.0f;
            const float y = xs * (-sn), x = xs * cs;
            const int m = (signbit(y) ? 1 : 0) | (signbit(x) ? 2 : 0);
            float lo = INFINITY, hi = -INFINITY;
            int w = 0;
            for (float q = qlo; q <= qhi; q = nextafterf(q, INFINITY), w++) {
                const float r = quad(m, om_atanf(q));
                lo = fminf(lo, r);
                hi = fmaxf(hi, r);
            }
            if (w > maxw) maxw = w;
            rlo[sg][i] = lo;
            rhi[sg][i] = hi;
        }
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    fseek(f, 0, SEEK_END);
    long n = ftell(f) / 4;
    fseek(f, 0, SEEK_SET);
    float* s = malloc(n * 4);
    if (fread(s, 4, n, f) != (size_t)n) return 1;
    fclose(f);
    uint32_t th = 0, d = 0;
    float pe = 0;
    long strad = 0, inval = 0, bad = 0, zmis = 0;
    for (long k = 0; k < n; k++) {
        const uint32_t i = idxof(th);
        const float sn = tab[i], c = tab[(i + 256) & 1023], x = s[k];
        const float r1 = x * c - 0.0f * (-sn), i1 = x * (-sn) + 0.0f * c;
        const float a = om_atan2f(i1, r1);
        const float pt = 0.999 * pe + 0.001 * a;
        if (!valid[i] || !(fabsf(x) >= 0x1p-40f && fabsf(x) <= 0x1p40f)) {
            inval++;
        } else {
            const int sg = x < 0;
            const float plo = 0.999 * pe + 0.001 * rlo[sg][i], phi = 0.999 * pe + 0.001 * rhi[sg][i];
            if (!(a >= rlo[sg][i] && a <= rhi[sg][i])) zmis++;
            if (om_bits(plo) != om_bits(phi)) strad++;
            else if (om_bits(plo) != om_bits(pt)) bad++;
        }
        pe = pt;
        d += C_(pe * al);
        th += C_(pe * be);
        th += d;
    }
    printf("n=%ld valid idx %d, max q' candidates %d: straddle %.4g%% invalid %.4g%% atan2 outside %ld, pe wrong %ld\n", n,
           nval, maxw, 100.0 * strad / n, 100.0 * inval / n, zmis, bad);
    return 0;
}
