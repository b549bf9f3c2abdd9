/*
 * liquid_restate.c -- CPU restatement ("oracle") of the liquid-dsp algorithms
 * behind python-liquiddsp's streaming receive path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library; the product library
 * (python-liquiddsp_amd/) never links or calls it.
 *
 * Where the algorithm lives: the reference (colbyAtCRI/python-liquiddsp,
 * /root/reference) is a pybind11 wrapper whose arithmetic is all in the
 * third-party C library liquid-dsp (jgaeddert/liquid-dsp, MIT).  liquid-dsp is
 * NOT vendored and its version is NOT pinned (reference CMakeLists.txt:4-10
 * `find_library(LIQUID libliquid.so)`, README.md:8 "brew install").  The API
 * used (3-argument ampmodem_create, src/demod.hpp:305) implies liquid-dsp
 * >= 1.4; this restatement follows the liquid-dsp 1.6-era sources
 * (src/filter/src/{firdes,firfilt,firpfb,resamp,iirdes,iirfilt,iirfiltsos},
 * src/nco/src/nco.proto.c, src/agc/src/agc.proto.c, src/modem/src/ampmodem.c,
 * src/buffer/src/wdelay.proto.c, src/math/src/{math,math.bessel,math.gamma}.c,
 * src/filter/src/window.c) as recalled; they are not available offline.
 *
 * PARITY UNPINNED: the reference repository holds no tests, fixtures or golden
 * vectors, and libliquid is absent from this container and the GPU image, so
 * nothing pins these outputs to a real liquid-dsp run.  They are pinned
 * instead against independent formulations (scipy.signal lfilter / sosfilt /
 * cheby2 / butter, explicit numpy polyphase sums, exact integer phase
 * schedules) in tests/test_oracle_*.py, and committed as fixtures under
 * tests/golden/.
 *
 * Version-dependent choices (switches recorded here and in DESIGN.md):
 *  - resampler: fixed-point 32-bit phase, npfb rounded up to a power of two
 *    (liquid >= 1.5 "Variant F");
 *  - NCO: 1024-entry sine table, index ((theta + 2^21) >> 22) & 1023;
 *  - dot products: the portable C dotprod (sequential accumulation from the
 *    oldest sample, no FMA); SIMD builds of liquid sum in another order,
 *    modelled by -DORA_DOTPROD_LANES=8 (a bounding variant, oracle/variants.py);
 *  - transcendentals inside feedback loops: ora_math.h (fdlibm algorithms);
 *    -DORA_USE_LIBM=1 calls the system libm (glibc) instead (variant);
 *  - complex division in the filter designs: C's `/` on _Complex operands,
 *    i.e. libgcc __divsc3 / __divdc3.  This library is linked by gcc 11, whose
 *    static libgcc implements Smith's method; newer libgcc_s (also present in
 *    the image) uses a scaled variant that moves some cheby2 poles by 1 ulp.
 *    The product pins Smith's method explicitly (csrc/cplx_c.c).
 *
 * Build flags: -ffp-contract=off (liquid's x86-64 baseline build has no FMA),
 * no -ffast-math.
 */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdbool.h>
#include <stdio.h>
#include "liquid_restate.h"
#include "ora_math.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ===================================================================== */
/* math helpers: liquid src/math/src/math.c, math.gamma.c, math.bessel.c */
/* ===================================================================== */

/* liquid math.gamma.c: liquid_lngammaf (recursion below 10, Stirling above) */
float ora_lngammaf(float _z)
{
    float g;
    if (_z < 0) {
        return 0.0f;
    } else if (_z < 10.0f) {
        return ora_lngammaf(_z + 1.0f) - logf(_z);
    } else {
        g = 0.5 * (logf(2 * M_PI) - log(_z));
        g += _z * (logf(_z + (1 / (12.0f * _z - 0.1f / _z))) - 1);
    }
    return g;
}

/* liquid math.bessel.c: liquid_besseli0f, 32-term series via lngammaf */
float ora_besseli0f(float _z)
{
    if (_z == 0.0f)
        return 1.0f;
    unsigned int k;
    float t, y = 0.0f;
    for (k = 0; k < 32; k++) {
        t = k * logf(0.5f * _z) - ora_lngammaf((float)k + 1.0f);
        y += expf(2 * t);
    }
    return y;
}

/* liquid math.c: sincf */
float ora_sincf(float _x)
{
    if (fabsf(_x) < 0.01f)
        return cosf(M_PI * _x / 2.0f) * cosf(M_PI * _x / 4.0f) * cosf(M_PI * _x / 8.0f);
    return sinf(M_PI * _x) / (M_PI * _x);
}

/* liquid firdes.c: kaiser_beta_As */
float ora_kaiser_beta_As(float _as)
{
    _as = fabsf(_as);
    float beta;
    if (_as > 50.0f)
        beta = 0.1102f * (_as - 8.7f);
    else if (_as > 21.0f)
        beta = 0.5842 * powf(_as - 21, 0.4f) + 0.07886f * (_as - 21);
    else
        beta = 0.0f;
    return beta;
}

/* liquid window.c: liquid_kaiser */
float ora_kaiser(unsigned int _i, unsigned int _wlen, float _beta)
{
    if (_i > _wlen || _beta < 0)
        return 0.0f;
    float t = (float)_i - (float)(_wlen - 1) / 2;
    float r = 2.0f * t / (float)(_wlen);
    float a = ora_besseli0f(_beta * sqrtf(1 - r * r));
    float b = ora_besseli0f(_beta);
    return a / b;
}

/* liquid firdes.c: liquid_firdes_kaiser (windowed sinc, unnormalised) */
int ora_firdes_kaiser(unsigned int _n, float _fc, float _as, float _mu, float *_h)
{
    if (_mu < -0.5f || _mu > 0.5f) return -1;
    if (_fc < 0.0f || _fc > 0.5f) return -1;
    if (_n == 0) return -1;
    float beta = ora_kaiser_beta_As(_as);
    float t, h1, h2;
    unsigned int i;
    for (i = 0; i < _n; i++) {
        t = (float)i - (float)(_n - 1) / 2 + _mu;
        h1 = ora_sincf(2.0f * _fc * t);
        h2 = ora_kaiser(i, _n, beta);
        _h[i] = h1 * h2;
    }
    return 0;
}

/* liquid firdes.c: liquid_firdes_notch (used by firfilt_*_create_dc_blocker) */
int ora_firdes_notch(unsigned int _m, float _f0, float _as, float *_h)
{
    if (_m < 1 || _m > 1000) return -1;
    if (_f0 < -0.5f || _f0 > 0.5f) return -1;
    if (_as <= 0.0f) return -1;
    float beta = ora_kaiser_beta_As(_as);
    unsigned int h_len = 2 * _m + 1;
    unsigned int i;
    float scale = 0.0f;
    for (i = 0; i < h_len; i++) {
        float p = -cosf(2.0f * M_PI * _f0 * ((float)i - (float)_m));
        float w = ora_kaiser(i, h_len, beta);
        _h[i] = p * w;
        scale += _h[i] * p;
    }
    for (i = 0; i < h_len; i++)
        _h[i] /= scale;
    _h[_m] += 1.0f;
    return 0;
}

void ora_math_eval(int fn, const float *a, const float *b, float *y, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) {
        switch (fn) {
        case 0: y[i] = om_expf(a[i]); break;
        case 1: y[i] = om_logf(a[i]); break;
        case 2: y[i] = om_atan2f(a[i], b[i]); break;
        case 3: y[i] = om_tanhf(a[i]); break;
        default: y[i] = 0.0f;
        }
    }
}

/* ===================================================================== */
/* sample window: liquid src/buffer/src/window.proto.c (oldest..newest)   */
/* ===================================================================== */
typedef struct {
    unsigned int len;    /* window length (samples) */
    unsigned int ncomp;  /* floats per sample: 1 (real) or 2 (complex) */
    unsigned int cap;    /* buffer capacity in samples */
    unsigned int pos;    /* index of oldest sample of current window */
    float *buf;
} ora_window;

static void win_init(ora_window *w, unsigned int len, unsigned int ncomp)
{
    w->len = len;
    w->ncomp = ncomp;
    w->cap = len + 4096;
    w->pos = 0;
    w->buf = (float *)calloc((size_t)w->cap * ncomp, sizeof(float));
}
static void win_free(ora_window *w) { free(w->buf); w->buf = NULL; }
static void win_reset(ora_window *w)
{
    w->pos = 0;
    memset(w->buf, 0, (size_t)w->cap * w->ncomp * sizeof(float));
}
static inline void win_push(ora_window *w, const float *v)
{
    if (w->pos + w->len == w->cap) {
        memmove(w->buf, w->buf + (size_t)(w->pos + 1) * w->ncomp,
                (size_t)(w->len - 1) * w->ncomp * sizeof(float));
        w->pos = 0;
    } else {
        w->pos++;
    }
    float *dst = w->buf + (size_t)(w->pos + w->len - 1) * w->ncomp;
    dst[0] = v[0];
    if (w->ncomp == 2) dst[1] = v[1];
}
static inline const float *win_read(const ora_window *w)
{
    return w->buf + (size_t)w->pos * w->ncomp;
}

#ifndef ORA_DOTPROD_LANES
#define ORA_DOTPROD_LANES 0
#endif
#if ORA_DOTPROD_LANES == 0
/* liquid dotprod (portable C, dotprod_*.proto.c run/run4): sequential sum
 * r = 0; r += h[i]*x[i], i = 0..n-1 (x oldest first), real taps. */
static inline float dot_rr(const float *h, const float *x, unsigned int n)
{
    float r = 0.0f;
    unsigned int i;
    for (i = 0; i < n; i++) r += h[i] * x[i];
    return r;
}
static inline void dot_cr(const float *h, const float *x, unsigned int n, float *y)
{
    float rr = 0.0f, ri = 0.0f;
    unsigned int i;
    for (i = 0; i < n; i++) {
        rr += h[i] * x[2 * i];
        ri += h[i] * x[2 * i + 1];
    }
    y[0] = rr;
    y[1] = ri;
}
/* complex taps (cccf): C99 complex product (ac - bd) + (ad + bc)j */
static inline void dot_cc(const float *h, const float *x, unsigned int n, float *y)
{
    float rr = 0.0f, ri = 0.0f;
    unsigned int i;
    for (i = 0; i < n; i++) {
        float a = h[2 * i], b = h[2 * i + 1], c = x[2 * i], d = x[2 * i + 1];
        rr += a * c - b * d;
        ri += a * d + b * c;
    }
    y[0] = rr;
    y[1] = ri;
}
#else
/* SIMD-order model of liquid's x86 dotprod (dotprod_*.sse.c / .avx.c): the
 * float stream is multiplied and accumulated ORA_DOTPROD_LANES floats at a time
 * into one vector register of partial sums (lane j holds the terms j, j + W,
 * j + 2W, ...), the register is reduced pairwise ((s0 + s1) + (s2 + s3)) ...
 * as hadd does, and the tail of n mod W floats is added sequentially.  For
 * complex data the stream is the interleaved (re, im) floats, so the even
 * lanes carry the real part and the odd lanes the imaginary part.  A bounding
 * variant (oracle/variants.py): which SIMD kernel a given liquid build uses
 * is a configure-time choice. */
#define ORA_W ORA_DOTPROD_LANES
static inline float ora_hsum(const float *a, unsigned int w, unsigned int stride)
{
    /* pairwise tree over lanes 0, stride, 2 stride, ... (w / stride of them) */
    float t[16];
    unsigned int m = w / stride, i;
    for (i = 0; i < m; i++) t[i] = a[i * stride];
    while (m > 1) {
        for (i = 0; i < m / 2; i++) t[i] = t[2 * i] + t[2 * i + 1];
        m /= 2;
    }
    return t[0];
}
static inline float dot_rr(const float *h, const float *x, unsigned int n)
{
    float acc[ORA_W];
    unsigned int i, j, t = n - n % ORA_W;
    for (j = 0; j < ORA_W; j++) acc[j] = 0.0f;
    for (i = 0; i < t; i += ORA_W)
        for (j = 0; j < ORA_W; j++) acc[j] += h[i + j] * x[i + j];
    float r = ora_hsum(acc, ORA_W, 1);
    for (; i < n; i++) r += h[i] * x[i];
    return r;
}
static inline void dot_cr(const float *h, const float *x, unsigned int n, float *y)
{
    /* taps duplicated [h0 h0 h1 h1 ...] against [x0r x0i x1r x1i ...] */
    float acc[ORA_W];
    unsigned int nf = 2 * n, i, j, t = nf - nf % ORA_W;
    for (j = 0; j < ORA_W; j++) acc[j] = 0.0f;
    for (i = 0; i < t; i += ORA_W)
        for (j = 0; j < ORA_W; j++) acc[j] += h[(i + j) / 2] * x[i + j];
    float rr = ora_hsum(acc, ORA_W, 2), ri = ora_hsum(acc + 1, ORA_W, 2);
    for (; i < nf; i += 2) {
        rr += h[i / 2] * x[i];
        ri += h[i / 2] * x[i + 1];
    }
    y[0] = rr;
    y[1] = ri;
}
static inline void dot_cc(const float *h, const float *x, unsigned int n, float *y)
{
    /* (re, im) pairs: real lanes accumulate ac - bd, imaginary lanes ad + bc */
    float acc[ORA_W];
    unsigned int nf = 2 * n, i, j, t = nf - nf % ORA_W;
    for (j = 0; j < ORA_W; j++) acc[j] = 0.0f;
    for (i = 0; i < t; i += ORA_W)
        for (j = 0; j < ORA_W; j += 2) {
            float a = h[i + j], b = h[i + j + 1], c = x[i + j], d = x[i + j + 1];
            acc[j] += a * c - b * d;
            acc[j + 1] += a * d + b * c;
        }
    float rr = ora_hsum(acc, ORA_W, 2), ri = ora_hsum(acc + 1, ORA_W, 2);
    for (; i < nf; i += 2) {
        float a = h[i], b = h[i + 1], c = x[i], d = x[i + 1];
        rr += a * c - b * d;
        ri += a * d + b * c;
    }
    y[0] = rr;
    y[1] = ri;
}
#endif

/* ===================================================================== */
/* firfilt: liquid src/filter/src/firfilt.proto.c                         */
/* reference: src/firfilter.hpp:13-35, demod.hpp:105,135                  */
/* ===================================================================== */
struct ora_firfilt_s {
    unsigned int n;
    int cplx;
    float *h;      /* taps as given */
    float *hrev;   /* reversed taps (liquid stores them reversed) */
    float scale;
    ora_window w;
};

ora_firfilt ora_firfilt_create(const float *h, unsigned int n, int cplx)
{
    if (n == 0) return NULL;
    ora_firfilt q = (ora_firfilt)calloc(1, sizeof(*q));
    q->n = n;
    q->cplx = cplx;
    q->h = (float *)malloc(n * sizeof(float));
    q->hrev = (float *)malloc(n * sizeof(float));
    unsigned int i;
    for (i = 0; i < n; i++) {
        q->h[i] = h[i];
        q->hrev[n - 1 - i] = h[i];
    }
    q->scale = 1.0f;
    win_init(&q->w, n, cplx ? 2 : 1);
    return q;
}

ora_firfilt ora_firfilt_create_kaiser(unsigned int n, float fc, float as, float mu, int cplx)
{
    float *h = (float *)malloc(n * sizeof(float));
    if (ora_firdes_kaiser(n, fc, as, mu, h)) { free(h); return NULL; }
    ora_firfilt q = ora_firfilt_create(h, n, cplx);
    free(h);
    return q;
}

ora_firfilt ora_firfilt_create_dc_blocker(unsigned int m, float as, int cplx)
{
    unsigned int n = 2 * m + 1;
    float *h = (float *)malloc(n * sizeof(float));
    if (ora_firdes_notch(m, 0.0f, as, h)) { free(h); return NULL; }
    ora_firfilt q = ora_firfilt_create(h, n, cplx);
    free(h);
    return q;
}

void ora_firfilt_destroy(ora_firfilt q)
{
    if (!q) return;
    win_free(&q->w);
    free(q->h);
    free(q->hrev);
    free(q);
}
void ora_firfilt_reset(ora_firfilt q) { win_reset(&q->w); }
void ora_firfilt_set_scale(ora_firfilt q, float s) { q->scale = s; }
float ora_firfilt_get_scale(ora_firfilt q) { return q->scale; }
unsigned int ora_firfilt_get_length(ora_firfilt q) { return q->n; }
void ora_firfilt_get_taps(ora_firfilt q, float *h) { memcpy(h, q->h, q->n * sizeof(float)); }

/* liquid firfilt_freqresponse: H = scale * sum_i hrev[i] exp(+j 2 pi f i) */
void ora_firfilt_freqresponse(ora_firfilt q, float f, float *re, float *im)
{
    float complex H = 0.0f;
    unsigned int i;
    for (i = 0; i < q->n; i++)
        H += q->hrev[i] * cexpf(_Complex_I * 2 * M_PI * f * i);
    H *= q->scale;
    *re = crealf(H);
    *im = cimagf(H);
}

static inline void firfilt_push_exec(ora_firfilt q, const float *x, float *y)
{
    win_push(&q->w, x);
    const float *r = win_read(&q->w);
    if (q->cplx) {
        float t[2];
        dot_cr(q->hrev, r, q->n, t);
        y[0] = t[0] * q->scale;
        y[1] = t[1] * q->scale;
    } else {
        y[0] = dot_rr(q->hrev, r, q->n) * q->scale;
    }
}

void ora_firfilt_execute_block(ora_firfilt q, const float *x, size_t n, float *y)
{
    size_t i;
    unsigned int c = q->cplx ? 2 : 1;
    for (i = 0; i < n; i++)
        firfilt_push_exec(q, x + i * c, y + i * c);
}

/* ===================================================================== */
/* resamp: liquid src/filter/src/resamp.proto.c + firpfb.proto.c          */
/* reference: src/resampler.hpp:72-173 (resamp_rrrf / resamp_cccf)        */
/* ===================================================================== */
struct ora_resamp_s {
    int kind;                 /* 0 rrrf, 1 crcf, 2 cccf */
    unsigned int m, npfb, bits_index, sub_len;
    float fc, as, rate;
    uint32_t step, phase;
    float *hproto;            /* n = 2 m npfb + 1 prototype taps (after gain) */
    float *sub;               /* [npfb][sub_len] reversed branch taps (cccf: interleaved re,im) */
    ora_window w;
};

static unsigned int nextpow2(unsigned int x)
{
    /* liquid_nextpow2: ceil(log2(x)) */
    unsigned int b = 0;
    x--;
    while (x > 0) { x >>= 1; b++; }
    return b;
}

int ora_resamp_set_rate(ora_resamp q, float rate)
{
    if (rate <= 0) return -1;
    if (rate < 0.004f || rate > 250.0f) return -1;
    q->rate = rate;
    q->step = (uint32_t)round((1 << 24) / q->rate);
    return 0;
}

ora_resamp ora_resamp_create(float rate, unsigned int m, float fc, float as,
                             unsigned int npfb, int kind)
{
    if (rate <= 0 || m == 0 || fc <= 0.0f || fc >= 0.5f || as <= 0.0f || npfb == 0)
        return NULL;
    ora_resamp q = (ora_resamp)calloc(1, sizeof(*q));
    q->kind = kind;
    if (ora_resamp_set_rate(q, rate)) { free(q); return NULL; }
    q->m = m;
    q->fc = fc;
    q->as = as;
    unsigned int nb = nextpow2(npfb);
    q->npfb = 1u << nb;
    q->bits_index = 24 - nb;
    /* design: n = 2 m npfb + 1 Kaiser taps at fc/npfb, gain normalised to npfb */
    unsigned int n = 2 * q->m * q->npfb + 1;
    float *hf = (float *)malloc(n * sizeof(float));
    ora_firdes_kaiser(n, q->fc / ((float)(q->npfb)), q->as, 0.0f, hf);
    unsigned int i, k;
    float gain = 0.0f;
    for (i = 0; i < n; i++) gain += hf[i];
    gain = (q->npfb) / (gain);
    q->hproto = (float *)malloc(n * sizeof(float));
    for (i = 0; i < n; i++) q->hproto[i] = hf[i] * gain;
    free(hf);
    /* firpfb_create(npfb, h, n-1): branch b taps h[b + k npfb], stored reversed */
    q->sub_len = (n - 1) / q->npfb;
    unsigned int c = (kind == 2) ? 2 : 1;
    q->sub = (float *)calloc((size_t)q->npfb * q->sub_len * c, sizeof(float));
    for (i = 0; i < q->npfb; i++) {
        for (k = 0; k < q->sub_len; k++) {
            float v = q->hproto[i + k * q->npfb];
            size_t idx = (size_t)i * q->sub_len + (q->sub_len - k - 1);
            q->sub[idx * c] = v;   /* imaginary part 0 for cccf */
        }
    }
    win_init(&q->w, q->sub_len, (kind == 0) ? 1 : 2);
    q->phase = 0;
    return q;
}

/* resamp_*_create_default (liquid resamp.proto.c, recalled): m = 7, fc = 0.25,
 * As = 60, npfb = 256.  Reference: RResampler / CResampler, src/resampler.hpp:10-13,46-49. */
ora_resamp ora_resamp_create_default(float rate, int kind)
{
    return ora_resamp_create(rate, 7, 0.25f, 60.0f, 256, kind);
}

void ora_resamp_destroy(ora_resamp q)
{
    if (!q) return;
    win_free(&q->w);
    free(q->hproto);
    free(q->sub);
    free(q);
}
void ora_resamp_reset(ora_resamp q) { win_reset(&q->w); q->phase = 0; }
float ora_resamp_get_rate(ora_resamp q) { return q->rate; }
uint32_t ora_resamp_get_step(ora_resamp q) { return q->step; }
uint32_t ora_resamp_get_phase(ora_resamp q) { return q->phase; }
unsigned int ora_resamp_get_npfb(ora_resamp q) { return q->npfb; }
unsigned int ora_resamp_get_taps(ora_resamp q, float *h)
{
    unsigned int n = 2 * q->m * q->npfb + 1;
    if (h) memcpy(h, q->hproto, n * sizeof(float));
    return n;
}

/* resamp_execute: push x; while (phase <= 0xffffff) { y = branch[phase >> bits_index]; phase += step; } phase -= 2^24 */
size_t ora_resamp_execute_block(ora_resamp q, const float *x, size_t n, float *y)
{
    size_t i, nw = 0;
    unsigned int cin = (q->kind == 0) ? 1 : 2;
    for (i = 0; i < n; i++) {
        win_push(&q->w, x + i * cin);
        const float *r = win_read(&q->w);
        while (q->phase <= 0x00ffffffu) {
            unsigned int index = q->phase >> q->bits_index;
            if (q->kind == 0) {
                y[nw] = dot_rr(q->sub + (size_t)index * q->sub_len, r, q->sub_len);
            } else if (q->kind == 1) {
                dot_cr(q->sub + (size_t)index * q->sub_len, r, q->sub_len, y + 2 * nw);
            } else {
                dot_cc(q->sub + (size_t)index * q->sub_len * 2, r, q->sub_len, y + 2 * nw);
            }
            nw++;
            q->phase += q->step;
        }
        q->phase -= (1u << 24);
    }
    return nw;
}

/* ===================================================================== */
/* nco: liquid src/nco/src/nco.proto.c (fixed-point phase, 1024 table)    */
/* reference: src/nco.hpp:4-81                                            */
/* ===================================================================== */
struct ora_nco_s {
    int type;
    float sintab[1024];
    uint32_t theta, d_theta;
    float alpha, beta;
};

/* NCO(_constrain): radians -> 32-bit fixed-point phase */
uint32_t ora_nco_constrain(float _theta)
{
    float p = _theta * 0.159154943091895;   /* 1/(2 pi) in double */
    float fpart = p - ((long)p);            /* in (-1,1) */
    if (fpart < 0.) fpart += 1.;
    /* (uint32_t)(fpart * 0xffffffff): x86-64 gcc converts through int64 */
    return (uint32_t)(int64_t)(fpart * 0xffffffff);
}

void ora_nco_reset(ora_nco q) { q->theta = 0; q->d_theta = 0; }

void ora_nco_pll_set_bandwidth(ora_nco q, float bw)
{
    if (bw < 0.0f) return;
    q->alpha = bw;
    q->beta = sqrtf(q->alpha);
}

ora_nco ora_nco_create(int type)
{
    ora_nco q = (ora_nco)calloc(1, sizeof(*q));
    q->type = type;
    unsigned int i;
    for (i = 0; i < 1024; i++)
        q->sintab[i] = sinf(2.0f * M_PI * (float)(i) / 1024.0f);
    ora_nco_reset(q);
    ora_nco_pll_set_bandwidth(q, 0.1f);
    return q;
}
void ora_nco_destroy(ora_nco q) { free(q); }
void ora_nco_set_frequency(ora_nco q, float dtheta) { q->d_theta = ora_nco_constrain(dtheta); }
void ora_nco_adjust_frequency(ora_nco q, float df) { q->d_theta += ora_nco_constrain(df); }
void ora_nco_set_phase(ora_nco q, float phi) { q->theta = ora_nco_constrain(phi); }
void ora_nco_adjust_phase(ora_nco q, float dphi) { q->theta += ora_nco_constrain(dphi); }
float ora_nco_get_frequency(ora_nco q)
{
    float d_theta = 2.0f * M_PI * (float)q->d_theta / (float)(1LLU << 32);
    return d_theta > M_PI ? d_theta - 2 * M_PI : d_theta;
}
float ora_nco_get_phase(ora_nco q)
{
    float theta = 2.0f * M_PI * (float)q->theta / (float)(1LLU << 32);
    return theta > M_PI ? theta - 2 * M_PI : theta;
}
/* NCO(_pll_step): frequency += C(alpha*dphi); phase += C(beta*dphi) */
void ora_nco_pll_step(ora_nco q, float dphi)
{
    ora_nco_adjust_frequency(q, dphi * q->alpha);
    ora_nco_adjust_phase(q, dphi * q->beta);
}
void ora_nco_get_state(ora_nco q, uint32_t *theta, uint32_t *dtheta)
{
    *theta = q->theta;
    *dtheta = q->d_theta;
}
void ora_nco_set_state(ora_nco q, uint32_t theta, uint32_t dtheta)
{
    q->theta = theta;
    q->d_theta = dtheta;
}
void ora_nco_get_table(ora_nco q, float *tab) { memcpy(tab, q->sintab, sizeof(q->sintab)); }

/* sin/cos of the current phase */
static inline void nco_sincos(const ora_nco q, float *s, float *c)
{
    if (q->type == 0) {
        uint32_t index = ((q->theta + (1u << 21)) >> 22) & 0x3ff;
        *s = q->sintab[index];
        *c = q->sintab[(index + 256) & 0x3ff];
    } else {
        /* LIQUID_VCO: direct evaluation (unpinned: liquid 1.6 interpolates a finer table) */
        float th = 2.0f * M_PI * (float)q->theta / (float)(1LLU << 32);
        *s = sinf(th);
        *c = cosf(th);
    }
}

/* y = x * conj(v) (down) / x * v (up), v = c + j s; C99 complex product, no FMA */
static inline void cmul_down(float a, float b, float c, float s, float *yr, float *yi)
{
    /* (a + jb)(c - js): re = a*c - b*(-s), im = a*(-s) + b*c */
    *yr = a * c - b * (-s);
    *yi = a * (-s) + b * c;
}
static inline void cmul_up(float a, float b, float c, float s, float *yr, float *yi)
{
    *yr = a * c - b * s;
    *yi = a * s + b * c;
}

void ora_nco_mix_block_up(ora_nco q, const float *x, float *y, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) {
        float s, c;
        nco_sincos(q, &s, &c);
        cmul_up(x[2 * i], x[2 * i + 1], c, s, &y[2 * i], &y[2 * i + 1]);
        q->theta += q->d_theta;
    }
}
void ora_nco_mix_block_down(ora_nco q, const float *x, float *y, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) {
        float s, c;
        nco_sincos(q, &s, &c);
        cmul_down(x[2 * i], x[2 * i + 1], c, s, &y[2 * i], &y[2 * i + 1]);
        q->theta += q->d_theta;
    }
}

/* ===================================================================== */
/* iirdes: liquid src/filter/src/iirdes.c (+ iirdes.pll.c not used)       */
/* reference call sites: src/iirfilter.hpp:70,88,106,124,180-234,275,332   */
/* ===================================================================== */
enum { FT_BUTTER = 0, FT_CHEBY1, FT_CHEBY2, FT_ELLIP, FT_BESSEL };
enum { BT_LOWPASS = 0, BT_HIGHPASS, BT_BANDPASS, BT_BANDSTOP };
enum { FMT_TF = 0, FMT_SOS = 1 };

/* butter_azpkf */
static void butter_azpkf(unsigned int _n, float complex *_za, float complex *_pa, float complex *_ka)
{
    unsigned int r = _n % 2;
    unsigned int L = (_n - r) / 2;
    unsigned int i, k = 0;
    (void)_za;
    for (i = 0; i < L; i++) {
        float theta = (float)(2 * (i + 1) + _n - 1) * M_PI / (float)(2 * _n);
        _pa[k++] = cexpf(_Complex_I * theta);
        _pa[k++] = cexpf(-_Complex_I * theta);
    }
    if (r) _pa[k++] = -1.0f;
    *_ka = 1.0;
}

/* cheby1_azpkf */
static void cheby1_azpkf(unsigned int _n, float _ep, float complex *_za, float complex *_pa,
                         float complex *_ka)
{
    float t0 = sqrt(1.0 + 1.0 / (_ep * _ep));
    float tp = powf(t0 + 1.0 / _ep, 1.0 / (float)(_n));
    float tm = powf(t0 - 1.0 / _ep, 1.0 / (float)(_n));
    float b = 0.5 * (tp + tm);
    float a = 0.5 * (tp - tm);
    unsigned int r = _n % 2;
    unsigned int L = (_n - r) / 2;
    unsigned int i, k = 0;
    (void)_za;
    for (i = 0; i < L; i++) {
        float theta = (float)(2 * (i + 1) + _n - 1) * M_PI / (float)(2 * _n);
        _pa[k++] = a * cosf(theta) - _Complex_I * b * sinf(theta);
        _pa[k++] = a * cosf(theta) + _Complex_I * b * sinf(theta);
    }
    if (r) _pa[k++] = -a;
    *_ka = r ? 1.0f : 1.0f / sqrtf(1.0f + _ep * _ep);
    for (i = 0; i < _n; i++) *_ka *= _pa[i];
}

/* cheby2_azpkf */
static void cheby2_azpkf(unsigned int _n, float _es, float complex *_za, float complex *_pa,
                         float complex *_ka)
{
    float t0 = sqrt(1.0 + 1.0 / (_es * _es));
    float tp = powf(t0 + 1.0 / _es, 1.0 / (float)(_n));
    float tm = powf(t0 - 1.0 / _es, 1.0 / (float)(_n));
    float b = 0.5 * (tp + tm);
    float a = 0.5 * (tp - tm);
    unsigned int r = _n % 2;
    unsigned int L = (_n - r) / 2;
    unsigned int i, k = 0;
    for (i = 0; i < L; i++) {
        float theta = (float)(2 * (i + 1) + _n - 1) * M_PI / (float)(2 * _n);
        _pa[k++] = 1.0f / (a * cosf(theta) - _Complex_I * b * sinf(theta));
        _pa[k++] = 1.0f / (a * cosf(theta) + _Complex_I * b * sinf(theta));
    }
    if (r) _pa[k++] = -1.0f / a;
    k = 0;
    for (i = 0; i < L; i++) {
        float theta = (float)(0.5f * M_PI * (2 * (i + 1) - 1) / (float)(_n));
        _za[k++] = -1.0f / (_Complex_I * cosf(theta));
        _za[k++] = 1.0f / (_Complex_I * cosf(theta));
    }
    *_ka = 1.0f;
    for (i = 0; i < _n; i++) *_ka *= _pa[i];
    for (i = 0; i < 2 * L; i++) *_ka /= _za[i];
}

/* ---- elliptic prototype: liquid src/filter/src/ellip.c + iirdes.c ellip_azpkf,
 * which follow S. J. Orfanidis, "Lecture notes on elliptic filter design"
 * (Landen transformations; recalled, parity unpinned).  Analog pass-band
 * edge 1 rad/s (fp = 1/2pi); the stop-band edge follows from the order. */
#define ELLIP_NB 7
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
/* cd(u K, k) and sn(u K, k) by descending Landen recursion */
static float complex ellip_cdf(float complex _u, float _k, unsigned int _n)
{
    float v[ELLIP_NB];
    landenf(_k, _n, v);
    float complex w = ccosf(_u * (float)(M_PI * 0.5));
    unsigned int i;
    for (i = _n; i > 0; i--) w = (1.0f + v[i - 1]) * w / (1.0f + v[i - 1] * w * w);
    return w;
}
static float complex ellip_snf(float complex _u, float _k, unsigned int _n)
{
    float v[ELLIP_NB];
    landenf(_k, _n, v);
    float complex w = csinf(_u * (float)(M_PI * 0.5));
    unsigned int i;
    for (i = _n; i > 0; i--) w = (1.0f + v[i - 1]) * w / (1.0f + v[i - 1] * w * w);
    return w;
}
/* inverse cd / sn by ascending Landen recursion */
static float complex ellip_acdf(float complex _w, float _k, unsigned int _n)
{
    float v[ELLIP_NB];
    landenf(_k, _n, v);
    float complex w = _w;
    unsigned int i;
    for (i = 0; i < _n; i++) {
        float v1 = (i == 0) ? _k : v[i - 1];
        w = w / (1.0f + csqrtf(1.0f - w * w * v1 * v1)) * 2.0f / (1.0f + v[i]);
    }
    return cacosf(w) * (float)(2.0 / M_PI);
}
static float complex ellip_asnf(float complex _w, float _k, unsigned int _n)
{
    return 1.0f - ellip_acdf(_w, _k, _n);
}
static void ellip_azpkf(unsigned int _n, float _ep, float _es, float complex *_za, float complex *_pa)
{
    const unsigned int nb = ELLIP_NB;
    const float k1 = _ep / _es;
    const float k = ellipdegf((float)_n, k1, nb);
    const unsigned int r = _n % 2, L = (_n - r) / 2;
    /* v0 = -j asn(j / ep, k1) / n (real) */
    const float complex v0 = -_Complex_I * ellip_asnf(_Complex_I / _ep, k1, nb) / (float)_n;
    unsigned int i, t = 0;
    for (i = 0; i < L; i++) {
        float ui = (2.0f * (i + 1) - 1.0f) / (float)_n;
        float complex zeta = ellip_cdf(ui, k, nb);
        _za[2 * i] = _Complex_I / (k * zeta);
        _za[2 * i + 1] = conjf(_za[2 * i]);
        float complex pz = _Complex_I * ellip_cdf(ui - _Complex_I * v0, k, nb);
        _pa[t++] = pz;
        _pa[t++] = conjf(pz);
    }
    if (r) _pa[t++] = crealf(_Complex_I * ellip_snf(_Complex_I * v0, k, nb));
}

/* ---- Bessel prototype: liquid iirdes.c bessel_azpkf (recalled, parity
 * unpinned): poles = roots of the reverse Bessel polynomial
 * theta_n(s) = sum_k (2n-k)! / (2^(n-k) k! (n-k)!) s^k (monic), here by
 * Durand-Kerner in double precision, then divided by the approximate 3 dB
 * frequency sqrt((2n-1) ln 2) [Bianchi 2007 (1.67)]. */
static void bessel_azpkf(unsigned int _n, float complex *_pa)
{
    double c[65];
    double complex z[64];
    unsigned int i, j, it;
    c[_n] = 1.0;                                  /* a_k / a_{k+1} = (2n-k)(k+1) / (2(n-k)) */
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
            const double complex dz = val / den;
            z[i] -= dz;
            delta = fmax(delta, cabs(dz) / cabs(z[i]));
        }
        if (delta < 1e-16) break;
    }
    const float w3dB = sqrtf((2 * _n - 1) * logf(2.0f));
    for (i = 0; i < _n; i++) _pa[i] = (float complex)z[i] / w3dB;
}

/* iirdes_freqprewarp */
static float iirdes_freqprewarp(int _btype, float _fc, float _f0)
{
    float m = 0.0f;
    if (_btype == BT_LOWPASS) {
        m = tanf(M_PI * _fc);
    } else if (_btype == BT_HIGHPASS) {
        m = -cosf(M_PI * _fc) / sinf(M_PI * _fc);
    } else if (_btype == BT_BANDPASS) {
        m = (cosf(2 * M_PI * _fc) - cosf(2 * M_PI * _f0)) / sinf(2 * M_PI * _fc);
    } else if (_btype == BT_BANDSTOP) {
        m = sinf(2 * M_PI * _fc) / (cosf(2 * M_PI * _fc) - cosf(2 * M_PI * _f0));
    }
    m = fabsf(m);
    return m;
}

/* bilinear_zpkf: kd = k0 * prod (1 - pd)/(1 - zd) */
static void bilinear_zpkf(const float complex *_za, unsigned int _nza, const float complex *_pa,
                          unsigned int _npa, float complex _ka, float _m, float complex *_zd,
                          float complex *_pd, float complex *_kd)
{
    unsigned int n = _npa;
    unsigned int i;
    float complex G = _ka;
    for (i = 0; i < n; i++) {
        if (i < _nza) {
            float complex zm = _za[i] * _m;
            _zd[i] = (1.0 + zm) / (1.0 - zm);
        } else {
            _zd[i] = -1.0;
        }
        float complex pm = _pa[i] * _m;
        _pd[i] = (1.0 + pm) / (1.0 - pm);
        G *= (1.0 - _pd[i]) / (1.0 - _zd[i]);
    }
    *_kd = G;
}

/* iirdes_dzpk_lp2bp */
static void iirdes_dzpk_lp2bp(const float complex *_zd, const float complex *_pd, unsigned int _n,
                              float _f0, float complex *_zdt, float complex *_pdt)
{
    float c0 = cosf(2 * M_PI * _f0);
    unsigned int i;
    float complex t0;
    for (i = 0; i < _n; i++) {
        t0 = 1 + _zd[i];
        _zdt[2 * i + 0] = 0.5f * (c0 * t0 + csqrtf(c0 * c0 * t0 * t0 - 4 * _zd[i]));
        _zdt[2 * i + 1] = 0.5f * (c0 * t0 - csqrtf(c0 * c0 * t0 * t0 - 4 * _zd[i]));
        t0 = 1 + _pd[i];
        _pdt[2 * i + 0] = 0.5f * (c0 * t0 + csqrtf(c0 * c0 * t0 * t0 - 4 * _pd[i]));
        _pdt[2 * i + 1] = 0.5f * (c0 * t0 - csqrtf(c0 * c0 * t0 * t0 - 4 * _pd[i]));
    }
}

/* liquid_cplxpair_cleanup */
static void cplxpair_cleanup(float complex *_p, unsigned int _n, unsigned int _num_pairs)
{
    unsigned int i, j;
    float complex tmp;
    for (i = 0; i < _num_pairs; i++) {
        _p[2 * i + 0] = cimagf(_p[2 * i]) < 0 ? _p[2 * i] : conjf(_p[2 * i]);
        _p[2 * i + 1] = conjf(_p[2 * i + 0]);
    }
    for (i = 0; i < _num_pairs; i++) {
        for (j = _num_pairs - 1; j > i; j--) {
            if (crealf(_p[2 * (j - 1)]) > crealf(_p[2 * j])) {
                tmp = _p[2 * (j - 1) + 0]; _p[2 * (j - 1) + 0] = _p[2 * j + 0]; _p[2 * j + 0] = tmp;
                tmp = _p[2 * (j - 1) + 1]; _p[2 * (j - 1) + 1] = _p[2 * j + 1]; _p[2 * j + 1] = tmp;
            }
        }
    }
    for (i = 2 * _num_pairs; i < _n; i++) {
        for (j = _n - 1; j > i; j--) {
            if (crealf(_p[j - 1]) > crealf(_p[j])) {
                tmp = _p[j - 1]; _p[j - 1] = _p[j]; _p[j] = tmp;
            }
        }
    }
}

/* liquid_cplxpair */
static int cplxpair(const float complex *_z, unsigned int _n, float _tol, float complex *_p)
{
    bool paired[_n > 0 ? _n : 1];
    memset(paired, 0, sizeof(paired));
    unsigned int num_pairs = 0;
    unsigned int i, j, k = 0;
    for (i = 0; i < _n; i++) {
        if (paired[i] || fabsf(cimagf(_z[i])) < _tol) continue;
        for (j = 0; j < _n; j++) {
            if (j == i || paired[j] || fabsf(cimagf(_z[j])) < _tol) continue;
            if (fabsf(cimagf(_z[i]) + cimagf(_z[j])) < _tol &&
                fabsf(crealf(_z[i]) - crealf(_z[j])) < _tol) {
                _p[k++] = _z[i];
                _p[k++] = _z[j];
                paired[i] = true;
                paired[j] = true;
                num_pairs++;
                break;
            }
        }
    }
    if (k > _n) return -1;
    for (i = 0; i < _n; i++)
        if (!paired[i]) _p[k++] = _z[i];
    cplxpair_cleanup(_p, _n, num_pairs);
    return 0;
}

/* iirdes_dzpk2sosf */
static int dzpk2sosf(const float complex *_zd, const float complex *_pd, unsigned int _n,
                     float complex _kd, float *_B, float *_A)
{
    unsigned int i;
    float tol = 1e-6f;
    float complex zp[_n], pp[_n];
    if (cplxpair(_zd, _n, tol, zp)) return -1;
    if (cplxpair(_pd, _n, tol, pp)) return -1;
    unsigned int r = _n % 2;
    unsigned int L = (_n - r) / 2;
    float complex z0, z1, p0, p1;
    for (i = 0; i < L; i++) {
        p0 = -pp[2 * i + 0];
        p1 = -pp[2 * i + 1];
        z0 = -zp[2 * i + 0];
        z1 = -zp[2 * i + 1];
        _A[3 * i + 0] = 1.0;
        _A[3 * i + 1] = crealf(p0 + p1);
        _A[3 * i + 2] = crealf(p0 * p1);
        _B[3 * i + 0] = 1.0;
        _B[3 * i + 1] = crealf(z0 + z1);
        _B[3 * i + 2] = crealf(z0 * z1);
    }
    if (r) {
        p0 = -pp[_n - 1];
        z0 = -zp[_n - 1];
        _A[3 * i + 0] = 1.0;
        _A[3 * i + 1] = crealf(p0);
        _A[3 * i + 2] = 0.0;
        _B[3 * i + 0] = 1.0;
        _B[3 * i + 1] = crealf(z0);
        _B[3 * i + 2] = 0.0;
    }
    float k = powf(crealf(_kd), 1.0f / (float)(L + r));
    for (i = 0; i < L + r; i++) {
        _B[3 * i + 0] *= k;
        _B[3 * i + 1] *= k;
        _B[3 * i + 2] *= k;
    }
    return 0;
}

/* iirdes_dzpk2tff: expand zeros/poles into polynomials (TF form) */
static void poly_expandroots(const float complex *r, unsigned int n, float complex *c)
{
    /* c = prod (x - r_i), ascending powers, c has n+1 entries */
    /* liquid polycf_expandroots */
    unsigned int i, j;
    if (n == 0) { c[0] = 0.; return; }
    for (i = 0; i <= n; i++) c[i] = (i == 0) ? 1 : 0;
    for (i = 0; i < n; i++) {
        for (j = i + 1; j > 0; j--) c[j] = -r[i] * c[j] + c[j - 1];
        c[0] *= -r[i];
    }
}
static void dzpk2tff(const float complex *_zd, const float complex *_pd, unsigned int _n,
                     float complex _kd, float *_b, float *_a)
{
    unsigned int i;
    float complex q[_n + 1];
    poly_expandroots(_pd, _n, q);
    for (i = 0; i <= _n; i++) _a[i] = crealf(q[_n - i]);
    poly_expandroots(_zd, _n, q);
    for (i = 0; i <= _n; i++) _b[i] = crealf(q[_n - i] * _kd);
}

static int iirdes_dzpk_core(int _ftype, int _btype, unsigned int _n, float _fc, float _f0,
                            float _ap, float _as, float complex *zd, float complex *pd,
                            float complex *kd_out, unsigned int *n_out)
{
    if (_fc <= 0 || _fc >= 0.5) return -1;
    if (_f0 < 0 || _f0 > 0.5) return -1;
    if (_ap <= 0 || _as <= 0 || _n == 0) return -1;
    unsigned int npa = _n, nza = 0;
    float complex pa[_n], za[_n], ka, k0 = 1.0f;
    unsigned int r = _n % 2;
    unsigned int L = (_n - r) / 2;
    unsigned int i;
    float epsilon;
    switch (_ftype) {
    case FT_BUTTER:
        nza = 0; k0 = 1.0f;
        butter_azpkf(_n, za, pa, &ka);
        break;
    case FT_CHEBY1:
        nza = 0;
        epsilon = sqrtf(powf(10.0f, _ap / 10.0f) - 1.0f);
        k0 = r ? 1.0f : 1.0f / sqrtf(1.0f + epsilon * epsilon);
        cheby1_azpkf(_n, epsilon, za, pa, &ka);
        break;
    case FT_CHEBY2:
        nza = 2 * L;
        epsilon = powf(10.0f, -_as / 20.0f);
        k0 = 1.0f;
        cheby2_azpkf(_n, epsilon, za, pa, &ka);
        break;
    case FT_ELLIP: {
        nza = 2 * L;
        float Gp = powf(10.0f, -_ap / 20.0f);
        float Gs = powf(10.0f, -_as / 20.0f);
        float ep = sqrtf(1.0f / (Gp * Gp) - 1.0f);
        float es = sqrtf(1.0f / (Gs * Gs) - 1.0f);
        k0 = r ? 1.0f : 1.0f / sqrtf(1.0f + ep * ep);
        ellip_azpkf(_n, ep, es, za, pa);
        (void)ka;
        break;
    }
    case FT_BESSEL:
        if (_n > 48) return -1;
        nza = 0;
        k0 = 1.0f;
        bessel_azpkf(_n, pa);
        break;
    default:
        return -1;
    }
    float complex kd;
    float m = iirdes_freqprewarp(_btype, _fc, _f0);
    bilinear_zpkf(za, nza, pa, npa, k0, m, zd, pd, &kd);
    if (_btype == BT_HIGHPASS || _btype == BT_BANDSTOP) {
        for (i = 0; i < _n; i++) {
            zd[i] = -zd[i];
            pd[i] = -pd[i];
        }
    }
    if (_btype == BT_BANDPASS || _btype == BT_BANDSTOP) {
        float complex zd1[2 * _n], pd1[2 * _n];
        iirdes_dzpk_lp2bp(zd, pd, _n, _f0, zd1, pd1);
        memmove(zd, zd1, 2 * _n * sizeof(float complex));
        memmove(pd, pd1, 2 * _n * sizeof(float complex));
        _n = 2 * _n;
    }
    *kd_out = kd;
    *n_out = _n;
    return 0;
}

int ora_iirdes(int ftype, int btype, int format, unsigned int n, float fc, float f0,
               float ap, float as, float *B, float *A)
{
    if (n == 0) return -1;
    float complex zd[2 * n], pd[2 * n], kd;
    unsigned int nn;
    int rc = iirdes_dzpk_core(ftype, btype, n, fc, f0, ap, as, zd, pd, &kd, &nn);
    if (rc) return rc;
    if (format == FMT_TF) {
        dzpk2tff(zd, pd, nn, kd, B, A);
        return 0;
    }
    return dzpk2sosf(zd, pd, nn, kd, B, A);
}

void ora_iirdes_dzpk(int ftype, int btype, unsigned int n, float fc, float f0, float ap,
                     float as, float *zdo, float *pdo, float *kdo)
{
    float complex zd[2 * n], pd[2 * n], kd;
    unsigned int nn, i;
    if (iirdes_dzpk_core(ftype, btype, n, fc, f0, ap, as, zd, pd, &kd, &nn)) return;
    for (i = 0; i < nn; i++) {
        zdo[2 * i] = crealf(zd[i]); zdo[2 * i + 1] = cimagf(zd[i]);
        pdo[2 * i] = crealf(pd[i]); pdo[2 * i + 1] = cimagf(pd[i]);
    }
    kdo[0] = crealf(kd);
    kdo[1] = cimagf(kd);
}

/* ===================================================================== */
/* iirfilt: liquid src/filter/src/iirfilt.proto.c + iirfiltsos.proto.c    */
/* reference: src/iirfilter.hpp:22-392                                     */
/* ===================================================================== */
struct ora_iirfilt_s {
    int sos;            /* 1: cascade of second-order sections, 0: TF (norm) */
    int cplx;
    unsigned int nsos;
    float *b, *a;       /* SOS: [nsos][3] normalised by a0; TF: nb / na */
    unsigned int nb, na, nv;
    float *v;           /* state: SOS [nsos][3][c]; TF [nv][c] */
    double *vd;         /* float64 state for the _f64 variant */
};

ora_iirfilt ora_iirfilt_create_sos(const float *B, const float *A, unsigned int nsos, int cplx)
{
    if (nsos == 0) return NULL;
    ora_iirfilt q = (ora_iirfilt)calloc(1, sizeof(*q));
    q->sos = 1;
    q->cplx = cplx;
    q->nsos = nsos;
    q->b = (float *)malloc(3 * nsos * sizeof(float));
    q->a = (float *)malloc(3 * nsos * sizeof(float));
    unsigned int i, k;
    for (i = 0; i < nsos; i++) {
        /* iirfiltsos_set_coefficients: normalise by a0 */
        float a0 = A[3 * i];
        for (k = 0; k < 3; k++) {
            q->b[3 * i + k] = B[3 * i + k] / a0;
            q->a[3 * i + k] = A[3 * i + k] / a0;
        }
    }
    q->v = (float *)calloc(3 * nsos * 2, sizeof(float));
    q->vd = (double *)calloc(3 * nsos * 2, sizeof(double));
    return q;
}

ora_iirfilt ora_iirfilt_create_tf(const float *b, unsigned int nb, const float *a,
                                  unsigned int na, int cplx)
{
    if (nb == 0 || na == 0) return NULL;
    ora_iirfilt q = (ora_iirfilt)calloc(1, sizeof(*q));
    q->sos = 0;
    q->cplx = cplx;
    q->nb = nb;
    q->na = na;
    q->nv = nb > na ? nb : na;
    q->b = (float *)malloc(nb * sizeof(float));
    q->a = (float *)malloc(na * sizeof(float));
    float a0 = a[0];
    unsigned int i;
    for (i = 0; i < nb; i++) q->b[i] = b[i] / a0;
    for (i = 0; i < na; i++) q->a[i] = a[i] / a0;
    q->v = (float *)calloc(q->nv * 2, sizeof(float));
    q->vd = (double *)calloc(q->nv * 2, sizeof(double));
    return q;
}

ora_iirfilt ora_iirfilt_create_prototype(int ftype, int btype, int format, unsigned int order,
                                         float fc, float f0, float ap, float as, int cplx)
{
    unsigned int N = order;
    if (btype == BT_BANDPASS || btype == BT_BANDSTOP) N *= 2;
    unsigned int r = N % 2;
    unsigned int L = (N - r) / 2;
    unsigned int h_len = (format == FMT_SOS) ? 3 * (L + r) : N + 1;
    float B[h_len], A[h_len];
    if (ora_iirdes(ftype, btype, format, order, fc, f0, ap, as, B, A)) return NULL;
    if (format == FMT_SOS) return ora_iirfilt_create_sos(B, A, L + r, cplx);
    return ora_iirfilt_create_tf(B, N + 1, A, N + 1, cplx);
}

void ora_iirfilt_destroy(ora_iirfilt q)
{
    if (!q) return;
    free(q->b); free(q->a); free(q->v); free(q->vd); free(q);
}
void ora_iirfilt_reset(ora_iirfilt q)
{
    if (q->sos) {
        memset(q->v, 0, 3 * q->nsos * 2 * sizeof(float));
        memset(q->vd, 0, 3 * q->nsos * 2 * sizeof(double));
    } else {
        memset(q->v, 0, q->nv * 2 * sizeof(float));
        memset(q->vd, 0, q->nv * 2 * sizeof(double));
    }
}
unsigned int ora_iirfilt_get_nsos(ora_iirfilt q) { return q->sos ? q->nsos : 0; }
void ora_iirfilt_get_sos(ora_iirfilt q, float *B, float *A)
{
    memcpy(B, q->b, 3 * q->nsos * sizeof(float));
    memcpy(A, q->a, 3 * q->nsos * sizeof(float));
}

/* iirfilt_freqresponse (liquid evaluates with exp(+j 2 pi f k), see TODO there) */
void ora_iirfilt_freqresponse(ora_iirfilt q, float f, float *re, float *im)
{
    unsigned int i;
    float complex H;
    if (!q->sos) {
        float complex Ha = 0.0f, Hb = 0.0f;
        for (i = 0; i < q->nb; i++) Hb += q->b[i] * cexpf(_Complex_I * 2 * M_PI * f * i);
        for (i = 0; i < q->na; i++) Ha += q->a[i] * cexpf(_Complex_I * 2 * M_PI * f * i);
        H = Hb / Ha;
    } else {
        H = 1.0f;
        for (i = 0; i < q->nsos; i++) {
            float complex Hb = q->b[3 * i + 0] * cexpf(_Complex_I * 2 * M_PI * f * 0) +
                               q->b[3 * i + 1] * cexpf(_Complex_I * 2 * M_PI * f * 1) +
                               q->b[3 * i + 2] * cexpf(_Complex_I * 2 * M_PI * f * 2);
            float complex Ha = q->a[3 * i + 0] * cexpf(_Complex_I * 2 * M_PI * f * 0) +
                               q->a[3 * i + 1] * cexpf(_Complex_I * 2 * M_PI * f * 1) +
                               q->a[3 * i + 2] * cexpf(_Complex_I * 2 * M_PI * f * 2);
            H *= Hb / Ha;
        }
    }
    *re = crealf(H);
    *im = cimagf(H);
}

/* iirfiltsos_execute_df2, one real component (component stride cs in v) */
static inline float sos_df2(const float *b, const float *a, float *v, float x)
{
    v[2] = v[1];
    v[1] = v[0];
    v[0] = x - a[1] * v[1] - a[2] * v[2];
    return b[0] * v[0] + b[1] * v[1] + b[2] * v[2];
}
static inline double sos_df2_d(const float *b, const float *a, double *v, double x)
{
    v[2] = v[1];
    v[1] = v[0];
    v[0] = x - (double)a[1] * v[1] - (double)a[2] * v[2];
    return (double)b[0] * v[0] + (double)b[1] * v[1] + (double)b[2] * v[2];
}

/* iirfilt_execute_norm (TF): shift v; v0 = x - dot(a[1:], v[1:]); y = dot(b, v) */
static inline float tf_norm(const float *b, unsigned int nb, const float *a, unsigned int na,
                            float *v, unsigned int nv, float x)
{
    unsigned int i;
    for (i = nv - 1; i > 0; i--) v[i] = v[i - 1];
    float v0 = dot_rr(a + 1, v + 1, na - 1);
    v0 = x - v0;
    v[0] = v0;
    return dot_rr(b, v, nb);
}
static inline double tf_norm_d(const float *b, unsigned int nb, const float *a, unsigned int na,
                               double *v, unsigned int nv, double x)
{
    unsigned int i;
    for (i = nv - 1; i > 0; i--) v[i] = v[i - 1];
    double v0 = 0.0;
    for (i = 1; i < na; i++) v0 += (double)a[i] * v[i];
    v0 = x - v0;
    v[0] = v0;
    double y = 0.0;
    for (i = 0; i < nb; i++) y += (double)b[i] * v[i];
    return y;
}

void ora_iirfilt_execute_block(ora_iirfilt q, const float *x, size_t n, float *y)
{
    size_t i;
    unsigned int c, s, nc = q->cplx ? 2 : 1;
    for (i = 0; i < n; i++) {
        for (c = 0; c < nc; c++) {
            float t = x[i * nc + c];
            if (q->sos) {
                for (s = 0; s < q->nsos; s++)
                    t = sos_df2(q->b + 3 * s, q->a + 3 * s, q->v + (s * 2 + c) * 3, t);
            } else {
                t = tf_norm(q->b, q->nb, q->a, q->na, q->v + c * q->nv, q->nv, t);
            }
            y[i * nc + c] = t;
        }
    }
}

void ora_iirfilt_execute_block_f64(ora_iirfilt q, const float *x, size_t n, float *y)
{
    size_t i;
    unsigned int c, s, nc = q->cplx ? 2 : 1;
    for (i = 0; i < n; i++) {
        for (c = 0; c < nc; c++) {
            double t = x[i * nc + c];
            if (q->sos) {
                for (s = 0; s < q->nsos; s++)
                    t = sos_df2_d(q->b + 3 * s, q->a + 3 * s, q->vd + (s * 2 + c) * 3, t);
            } else {
                t = tf_norm_d(q->b, q->nb, q->a, q->na, q->vd + c * q->nv, q->nv, t);
            }
            y[i * nc + c] = (float)t;
        }
    }
}

/* ===================================================================== */
/* agc_crcf: liquid src/agc/src/agc.proto.c                               */
/* reference: src/agc.hpp:4-149, docs src/agc_docs.cpp:53-72              */
/* ===================================================================== */
enum {
    SQ_UNKNOWN = 0, SQ_ENABLED, SQ_RISE, SQ_SIGNALHI, SQ_FALL, SQ_SIGNALLO, SQ_TIMEOUT, SQ_DISABLED
};
struct ora_agc_s {
    float g, scale, bandwidth, alpha, y2_prime;
    int is_locked;
    int squelch_mode;
    float squelch_threshold;
    unsigned int squelch_timeout, squelch_timer;
};

void ora_agc_set_bandwidth(ora_agc q, float bt)
{
    if (bt < 0 || bt > 1.0f) return;
    q->bandwidth = bt;
    q->alpha = q->bandwidth;
}
float ora_agc_get_bandwidth(ora_agc q) { return q->bandwidth; }
void ora_agc_reset(ora_agc q)
{
    q->g = 1.0f;
    q->y2_prime = 1.0f;
    q->is_locked = 0;
    q->squelch_mode = (q->squelch_mode == SQ_DISABLED) ? SQ_DISABLED : SQ_ENABLED;
}
ora_agc ora_agc_create(void)
{
    ora_agc q = (ora_agc)calloc(1, sizeof(*q));
    ora_agc_set_bandwidth(q, 0.01f);
    ora_agc_reset(q);
    q->squelch_mode = SQ_DISABLED;
    q->squelch_threshold = 0.0f;
    q->squelch_timeout = 100;
    q->scale = 1;
    return q;
}
void ora_agc_destroy(ora_agc q) { free(q); }
void ora_agc_lock(ora_agc q, int on) { q->is_locked = on ? 1 : 0; }
void ora_agc_squelch_enable(ora_agc q, int on) { q->squelch_mode = on ? SQ_ENABLED : SQ_DISABLED; }
void ora_agc_squelch_set_threshold(ora_agc q, float t) { q->squelch_threshold = t; }
float ora_agc_squelch_get_threshold(ora_agc q) { return q->squelch_threshold; }
void ora_agc_squelch_set_timeout(ora_agc q, unsigned int t) { q->squelch_timeout = t; }
int ora_agc_squelch_get_status(ora_agc q) { return q->squelch_mode; }
float ora_agc_get_gain(ora_agc q) { return q->g; }
void ora_agc_set_gain(ora_agc q, float g) { if (g > 0) q->g = g; }
float ora_agc_get_scale(ora_agc q) { return q->scale; }
void ora_agc_set_scale(ora_agc q, float s) { if (s > 0) q->scale = s; }
float ora_agc_get_signal_level(ora_agc q) { return 1.0 / q->g; }
void ora_agc_set_signal_level(ora_agc q, float x)
{
    if (x <= 0) return;
    q->g = 1.0 / x;
    q->y2_prime = 1.0;
}
float ora_agc_get_rssi(ora_agc q) { return -20 * log10(q->g); }
void ora_agc_set_rssi(ora_agc q, float rssi)
{
    q->g = powf(10.0f, -rssi / 20.0f);
    if (q->g < 1e-16f) q->g = 1e-16f;
    q->y2_prime = 1.0f;
}
void ora_agc_get_state(ora_agc q, float *g, float *y2p, int *mode, unsigned int *timer)
{
    *g = q->g; *y2p = q->y2_prime; *mode = q->squelch_mode; *timer = q->squelch_timer;
}
void ora_agc_set_state(ora_agc q, float g, float y2p, int mode, unsigned int timer)
{
    q->g = g; q->y2_prime = y2p; q->squelch_mode = mode; q->squelch_timer = timer;
}

/* AGC(_squelch_update_mode) */
static void agc_squelch_update_mode(ora_agc q)
{
    int threshold_exceeded = (ora_agc_get_rssi(q) > q->squelch_threshold);
    switch (q->squelch_mode) {
    case SQ_ENABLED:
        q->squelch_mode = threshold_exceeded ? SQ_RISE : SQ_ENABLED;
        break;
    case SQ_RISE:
        q->squelch_mode = threshold_exceeded ? SQ_SIGNALHI : SQ_FALL;
        break;
    case SQ_SIGNALHI:
        q->squelch_mode = threshold_exceeded ? SQ_SIGNALHI : SQ_FALL;
        break;
    case SQ_FALL:
        q->squelch_mode = threshold_exceeded ? SQ_SIGNALHI : SQ_SIGNALLO;
        q->squelch_timer = q->squelch_timeout;
        break;
    case SQ_SIGNALLO:
        q->squelch_timer--;
        if (q->squelch_timer == 0)
            q->squelch_mode = SQ_TIMEOUT;
        else if (threshold_exceeded)
            q->squelch_mode = SQ_SIGNALHI;
        break;
    case SQ_TIMEOUT:
        q->squelch_mode = SQ_ENABLED;
        break;
    default:
        break;
    }
}

/* AGC(_execute) */
static inline void agc_execute(ora_agc q, float xr, float xi, float *yr, float *yi)
{
    /* y = x * g */
    float a = xr * q->g, b = xi * q->g;
    /* y2 = real(y * conj(y)) = a*a - b*(-b) */
    float y2 = a * a - b * (-b);
    /* single-pole smoothing, evaluated in double (1.0 literal), stored as float */
    q->y2_prime = (1.0 - q->alpha) * q->y2_prime + q->alpha * y2;
    if (q->is_locked) { *yr = a; *yi = b; return; }
    if (q->y2_prime > 1e-6f)
        q->g *= om_expf(-0.5f * q->alpha * om_logf(q->y2_prime));
    q->g = (q->g > 1e6f) ? 1e6f : q->g;
    agc_squelch_update_mode(q);
    *yr = a * q->scale;
    *yi = b * q->scale;
}

/* python-liquiddsp AGC::execute (src/agc.hpp:109-128) */
void ora_agc_execute_wrapper(ora_agc q, const float *x, size_t n, float *y, uint8_t *status)
{
    size_t i;
    for (i = 0; i < n; i++) {
        agc_execute(q, x[2 * i], x[2 * i + 1], &y[2 * i], &y[2 * i + 1]);
        int state = q->squelch_mode;
        if (status) status[i] = (uint8_t)state;
        if (state == SQ_SIGNALLO || state == SQ_ENABLED) {
            y[2 * i] *= 0.0f;
            y[2 * i + 1] *= 0.0f;
        }
    }
}

/* ===================================================================== */
/* firhilbf (complex -> real): liquid src/filter/src/firhilb.proto.c      */
/* (liquid >= 1.4, as recalled; parity unpinned)                          */
/*   h = firdes_kaiser(4m+1, 0.25, As, 0);  h[i] = imag(h[i] e^{j pi t/2}) */
/*   with t = i - 2m (non-zero at odd t only: a unit-gain Hilbert          */
/*   transformer, the half-band prototype's passband gain being 2);        */
/*   hq[j] = h[4m - 1 - 2j], j < 2m (the odd taps, reversed).  liquid runs */
/*   c2r on polyphase windows (even / odd samples, toggled per call); in    */
/*   full-rate terms every output is                                        */
/*     yi = re x[n - 2m],  yq = sum_j hq[j] im x[n - 4m + 1 + 2j]           */
/*     (dotprod order, oldest first),  y0 = yi + yq (LSB),  y1 = yi - yq    */
/*   (USB), with zero history after create / reset.                          */
/* ===================================================================== */
struct ora_firhilb_s {
    unsigned int m;
    float *hq;                 /* 2m quadrature taps */
    ora_window w;              /* last 4m complex inputs */
};
typedef struct ora_firhilb_s *ora_firhilb;

ora_firhilb ora_firhilb_create(unsigned int m, float as)
{
    if (m < 2) return NULL;
    ora_firhilb q = (ora_firhilb)calloc(1, sizeof(*q));
    q->m = m;
    unsigned int h_len = 4 * m + 1, i, j = 0;
    float *h = (float *)malloc(h_len * sizeof(float));
    ora_firdes_kaiser(h_len, 0.25f, fabsf(as), 0.0f, h);
    for (i = 0; i < h_len; i++) {
        float t = (float)i - (float)(h_len - 1) / 2.0f;
        float complex hc = h[i] * cexpf(_Complex_I * 0.5f * M_PI * t);
        h[i] = cimagf(hc);
    }
    q->hq = (float *)malloc(2 * m * sizeof(float));
    for (i = 1; i < h_len; i += 2) q->hq[j++] = h[h_len - i - 1];
    free(h);
    win_init(&q->w, 4 * m, 2);
    return q;
}
void ora_firhilb_destroy(ora_firhilb q)
{
    if (!q) return;
    win_free(&q->w);
    free(q->hq);
    free(q);
}
void ora_firhilb_reset(ora_firhilb q) { win_reset(&q->w); }
void ora_firhilb_get_taps(ora_firhilb q, float *hq) { memcpy(hq, q->hq, 2 * q->m * sizeof(float)); }

/* firhilbf_c2r_execute(q, x, &y0 (lower sideband), &y1 (upper sideband)) */
static inline void firhilb_c2r(ora_firhilb q, const float *x, float *y0, float *y1)
{
    win_push(&q->w, x);
    const float *r = win_read(&q->w);          /* r[k] = x[n - 4m + 1 + k] */
    const unsigned int m = q->m;
    float xi[512], yq;
    unsigned int j;
    for (j = 0; j < 2 * m; j++) xi[j] = r[2 * (2 * j) + 1];
    yq = dot_rr(q->hq, xi, 2 * m);
    float yi = r[2 * (2 * m - 1)];
    *y0 = yi + yq;
    *y1 = yi - yq;
}

void ora_firhilb_c2r_block(ora_firhilb q, const float *x, size_t n, float *y0, float *y1)
{
    size_t i;
    for (i = 0; i < n; i++) firhilb_c2r(q, x + 2 * i, y0 + i, y1 + i);
}

/* ===================================================================== */
/* ampmodem: liquid src/modem/src/ampmodem.c (liquid >= 1.4)              */
/* reference: src/demod.hpp:221-307; structure mirrored at demod.hpp:133  */
/* demod per type (ampmodem_create's function pointer, as recalled):      */
/*   dsb, carrier    ampmodem_demod_dsb_pll_carrier                       */
/*   dsb, suppressed ampmodem_demod_dsb_pll_costas                        */
/*   usb/lsb, carrier    ampmodem_demod_ssb_pll_carrier: the DSB carrier  */
/*       PLL, then firhilbf_c2r(v1) -> (m_lsb, m_usb),                     */
/*       m = 0.5f * m_sideband / mod_index, DC block                      */
/*   usb/lsb, suppressed ampmodem_demod_ssb: firhilbf_c2r(x),             */
/*       y = 0.5f * m_sideband / mod_index (no PLL, no DC block)          */
/* SSB parity unpinned (recalled source, no liquid run to check against). */
/* ===================================================================== */
struct ora_ampmodem_s {
    float mod_index;
    int type;                  /* 0 dsb, 1 usb, 2 lsb */
    int suppressed_carrier;
    unsigned int m;
    ora_nco mixer;
    ora_firfilt dcblock;       /* firfilt_rrrf_create_dc_blocker(m, 20) */
    ora_firhilb hilbert;       /* firhilbf_create(m, 60) */
    ora_firfilt lowpass;       /* firfilt_crcf_create_kaiser(2m+1, 0.01, 40, 0) */
    float *delay;              /* wdelaycf(m): ring of m+1 samples */
    unsigned int dpos;
};

ora_ampmodem ora_ampmodem_create(float mod_index, int type, int suppressed_carrier)
{
    if (type < 0 || type > 2) return NULL;
    ora_ampmodem q = (ora_ampmodem)calloc(1, sizeof(*q));
    q->type = type;
    q->mod_index = mod_index;
    q->suppressed_carrier = (suppressed_carrier != 0);
    q->m = 25;
    q->mixer = ora_nco_create(0);
    ora_nco_pll_set_bandwidth(q->mixer, 0.001f);
    q->dcblock = ora_firfilt_create_dc_blocker(q->m, 20.0f, 0);
    q->hilbert = ora_firhilb_create(q->m, 60.0f);
    q->lowpass = ora_firfilt_create_kaiser(2 * q->m + 1, 0.01f, 40.0f, 0.0f, 1);
    q->delay = (float *)calloc(2 * (q->m + 1), sizeof(float));
    ora_ampmodem_reset(q);
    return q;
}
void ora_ampmodem_destroy(ora_ampmodem q)
{
    if (!q) return;
    ora_nco_destroy(q->mixer);
    ora_firfilt_destroy(q->dcblock);
    ora_firhilb_destroy(q->hilbert);
    ora_firfilt_destroy(q->lowpass);
    free(q->delay);
    free(q);
}
void ora_ampmodem_reset(ora_ampmodem q)
{
    ora_nco_reset(q->mixer);
    ora_firfilt_reset(q->dcblock);
    ora_firhilb_reset(q->hilbert);
    ora_firfilt_reset(q->lowpass);
    memset(q->delay, 0, 2 * (q->m + 1) * sizeof(float));
    q->dpos = 0;
}
void ora_ampmodem_get_hilbert_taps(ora_ampmodem q, float *hq) { ora_firhilb_get_taps(q->hilbert, hq); }
void ora_ampmodem_get_pll_state(ora_ampmodem q, uint32_t *theta, uint32_t *dtheta)
{
    ora_nco_get_state(q->mixer, theta, dtheta);
}
void ora_ampmodem_get_taps(ora_ampmodem q, float *lowpass, float *dcblock)
{
    ora_firfilt_get_taps(q->lowpass, lowpass);
    ora_firfilt_get_taps(q->dcblock, dcblock);
}

/* wdelaycf push-then-read: returns the sample pushed m samples earlier */
static inline void wdelay_push_read(ora_ampmodem q, const float *x, float *out)
{
    unsigned int len = q->m + 1;
    q->delay[2 * q->dpos] = x[0];
    q->delay[2 * q->dpos + 1] = x[1];
    q->dpos = (q->dpos + 1) % len;
    out[0] = q->delay[2 * q->dpos];
    out[1] = q->delay[2 * q->dpos + 1];
}

void ora_ampmodem_demodulate_block(ora_ampmodem q, const float *x, size_t n, float *y)
{
    size_t i;
    if (q->type != 0 && q->suppressed_carrier) {
        /* ampmodem_demod_ssb */
        for (i = 0; i < n; i++) {
            float lsb, usb;
            firhilb_c2r(q->hilbert, x + 2 * i, &lsb, &usb);
            y[i] = 0.5f * (q->type == 1 ? usb : lsb) / q->mod_index;
        }
        return;
    }
    for (i = 0; i < n; i++) {
        float x0[2], x1[2], v0r, v0i, v1r, v1i, s, c;
        firfilt_push_exec(q->lowpass, x + 2 * i, x0);
        wdelay_push_read(q, x + 2 * i, x1);
        nco_sincos(q->mixer, &s, &c);
        cmul_down(x0[0], x0[1], c, s, &v0r, &v0i);
        cmul_down(x1[0], x1[1], c, s, &v1r, &v1i);
        if (q->type != 0) {
            /* ampmodem_demod_ssb_pll_carrier */
            float phase_error = om_atan2f(v0i, v0r);           /* cargf(v0) */
            ora_nco_pll_step(q->mixer, phase_error);
            q->mixer->theta += q->mixer->d_theta;
            float v1[2] = {v1r, v1i}, lsb, usb;
            firhilb_c2r(q->hilbert, v1, &lsb, &usb);
            float m = 0.5f * (q->type == 1 ? usb : lsb) / q->mod_index;
            firfilt_push_exec(q->dcblock, &m, &y[i]);
        } else if (!q->suppressed_carrier) {
            /* ampmodem_demod_dsb_pll_carrier */
            float phase_error = om_atan2f(v0i, v0r);           /* cargf(v0) */
            ora_nco_pll_step(q->mixer, phase_error);
            q->mixer->theta += q->mixer->d_theta;               /* nco_crcf_step */
            float m = v1r / q->mod_index;
            firfilt_push_exec(q->dcblock, &m, &y[i]);
        } else {
            /* ampmodem_demod_dsb_pll_costas */
            float phase_error = om_tanhf(v0r) * v0i;
            ora_nco_pll_step(q->mixer, phase_error);
            q->mixer->theta += q->mixer->d_theta;
            y[i] = v1r / q->mod_index;
        }
    }
}

/* ===================================================================== */
/* AMRadio chain (README.md:41-58): IIR -> resampler -> AGC -> AmpModem   */
/* -> de-emphasis (src/iirfilter.hpp:366-372)                             */
/* ===================================================================== */
struct ora_amradio_s {
    ora_iirfilt bandpass;
    ora_resamp resample;
    ora_agc agc;
    ora_ampmodem am;
    ora_iirfilt deemph;
    int iir_f64;
    float *buf0, *buf1, *buf2;
    size_t cap;
};

ora_amradio ora_amradio_create(float bandwidth, float iq_rate, float pcm_rate, int iir_f64)
{
    ora_amradio q = (ora_amradio)calloc(1, sizeof(*q));
    /* ComplexIIRFilter(filter_type='cheby2', order=8, Fc=bandwidth/iq_rate), defaults
     * band_type='lowpass', F0=0.3, Ap=0.7, As=60 (wrapper.cpp:134-142) */
    float fc = (float)((double)bandwidth / (double)iq_rate);
    q->bandpass = ora_iirfilt_create_prototype(FT_CHEBY2, BT_LOWPASS, FMT_SOS, 8, fc, 0.3f, 0.7f,
                                               60.0f, 1);
    /* ComplexResampler(rate=pcm/iq, Fc=pcm/iq), len=20, As=60, nfilter=13 */
    float r = (float)((double)pcm_rate / (double)iq_rate);
    q->resample = ora_resamp_create(r, 20, r, 60.0f, 13, 2);
    q->agc = ora_agc_create();
    ora_agc_lock(q->agc, 0);
    ora_agc_set_scale(q->agc, 0.01f);
    q->am = ora_ampmodem_create(0.5f, 0, 0);   /* carrier=True -> suppressed 0 */
    /* DeemphasisFilter(pcm_rate) */
    float x = exp(-1.0 / (75.0E-6 * pcm_rate));
    float mA[2], mB[1];
    mA[0] = 1.0;
    mA[1] = -x;
    mB[0] = 1.0 - x;
    q->deemph = ora_iirfilt_create_tf(mB, 1, mA, 2, 0);
    q->iir_f64 = iir_f64;
    return q;
}

void ora_amradio_destroy(ora_amradio q)
{
    if (!q) return;
    ora_iirfilt_destroy(q->bandpass);
    ora_resamp_destroy(q->resample);
    ora_agc_destroy(q->agc);
    ora_ampmodem_destroy(q->am);
    ora_iirfilt_destroy(q->deemph);
    free(q->buf0); free(q->buf1); free(q->buf2);
    free(q);
}

size_t ora_amradio_max_out(ora_amradio q, size_t n)
{
    (void)q;
    return (size_t)((double)n * 0.03) + 64 + n / 16;
}

size_t ora_amradio_execute(ora_amradio q, const float *x, size_t n, float *y)
{
    if (n > q->cap) {
        free(q->buf0); free(q->buf1); free(q->buf2);
        q->cap = n;
        q->buf0 = (float *)malloc(2 * n * sizeof(float));
        q->buf1 = (float *)malloc(2 * n * sizeof(float) + 64);
        q->buf2 = (float *)malloc(2 * n * sizeof(float) + 64);
    }
    if (q->iir_f64)
        ora_iirfilt_execute_block_f64(q->bandpass, x, n, q->buf0);
    else
        ora_iirfilt_execute_block(q->bandpass, x, n, q->buf0);
    size_t nr = ora_resamp_execute_block(q->resample, q->buf0, n, q->buf1);
    ora_agc_execute_wrapper(q->agc, q->buf1, nr, q->buf2, NULL);
    ora_ampmodem_demodulate_block(q->am, q->buf2, nr, q->buf0);
    ora_iirfilt_execute_block(q->deemph, q->buf0, nr, y);
    return nr;
}

/* ===================================================================== */
/* freqdem: liquid src/modem/src/freqdem.c (liquid >= 1.3)              */
/* reference: FreqDem src/demod.hpp:189-219, wrapper.cpp:183-187          */
/*   ref = 1 / (2 pi kf);  m[n] = cargf(conjf(r[n-1]) * r[n]) * ref      */
/* ===================================================================== */
struct ora_freqdem_s {
    float kf, ref;
    float rp[2];
};
ora_freqdem ora_freqdem_create(float kf)
{
    ora_freqdem q = (ora_freqdem)calloc(1, sizeof(*q));
    q->kf = kf;
    q->ref = 1.0f / (2 * M_PI * q->kf);
    return q;
}
void ora_freqdem_destroy(ora_freqdem q) { free(q); }
void ora_freqdem_reset(ora_freqdem q) { q->rp[0] = q->rp[1] = 0.0f; }
void ora_freqdem_demodulate_block(ora_freqdem q, const float *x, size_t n, float *y)
{
    size_t i;
    for (i = 0; i < n; i++) {
        /* conjf(r') * r with C99 float complex multiply: (a + jb')(c + jd), b' = -b */
        const float a = q->rp[0], bq = -q->rp[1], c = x[2 * i], d = x[2 * i + 1];
        const float re = a * c - bq * d;
        const float im = a * d + bq * c;
        y[i] = om_atan2f(im, re) * q->ref;
        q->rp[0] = c;
        q->rp[1] = d;
    }
}

/* ===================================================================== */
/* BroadcastAM: reference src/demod.hpp:93-153 (python-liquiddsp's own   */
/* demodulator): Kaiser lowpass 2m+1 (fc 0.01, As 40) + wdelaycf(m) +    */
/* NCO PLL (bw 0.001) on cargf(v0), output through an SOS cheby2         */
/* highpass DC blocker (order 3, fc 20/48000, Ap 0.5, As 20) on re(v1).   */
/* ===================================================================== */
struct ora_bcastam_s {
    unsigned int m;
    ora_nco mixer;
    ora_firfilt lowpass;
    ora_iirfilt dcblock;
    float *delay;
    unsigned int dpos;
};
ora_bcastam ora_bcastam_create(unsigned int m, int iir_f64)
{
    ora_bcastam q = (ora_bcastam)calloc(1, sizeof(*q));
    q->m = m;
    q->mixer = ora_nco_create(0);
    ora_nco_pll_set_bandwidth(q->mixer, 0.001f);
    q->lowpass = ora_firfilt_create_kaiser(2 * m + 1, 0.01f, 40.0f, 0.0f, 1);
    q->dcblock = ora_iirfilt_create_prototype(2, 1, 1, 3, 20.0f / 48000.0f, 0.0f, 0.5f, 20.0f, 0);
    (void)iir_f64;
    q->delay = (float *)calloc(2 * (m + 1), sizeof(float));
    return q;
}
void ora_bcastam_destroy(ora_bcastam q)
{
    if (!q) return;
    ora_nco_destroy(q->mixer);
    ora_firfilt_destroy(q->lowpass);
    ora_iirfilt_destroy(q->dcblock);
    free(q->delay);
    free(q);
}
void ora_bcastam_reset(ora_bcastam q)
{
    ora_nco_reset(q->mixer);
    ora_firfilt_reset(q->lowpass);
    ora_iirfilt_reset(q->dcblock);
    memset(q->delay, 0, 2 * (q->m + 1) * sizeof(float));
    q->dpos = 0;
}
/* y: the PLL output re(v1) before the DC blocker (pre) and after it (y) */
void ora_bcastam_demodulate_block(ora_bcastam q, const float *x, size_t n, float *pre, float *y, int iir_f64)
{
    size_t i;
    for (i = 0; i < n; i++) {
        float x0[2], x1[2], v0r, v0i, v1r, v1i, s, c;
        firfilt_push_exec(q->lowpass, x + 2 * i, x0);
        /* wdelaycf push then read: the sample pushed m samples earlier */
        unsigned int len = q->m + 1;
        q->delay[2 * q->dpos] = x[2 * i];
        q->delay[2 * q->dpos + 1] = x[2 * i + 1];
        q->dpos = (q->dpos + 1) % len;
        x1[0] = q->delay[2 * q->dpos];
        x1[1] = q->delay[2 * q->dpos + 1];
        nco_sincos(q->mixer, &s, &c);
        cmul_down(x0[0], x0[1], c, s, &v0r, &v0i);
        cmul_down(x1[0], x1[1], c, s, &v1r, &v1i);
        float phase_error = om_atan2f(v0i, v0r);
        ora_nco_pll_step(q->mixer, phase_error);
        q->mixer->theta += q->mixer->d_theta;
        pre[i] = v1r;
    }
    if (iir_f64) ora_iirfilt_execute_block_f64(q->dcblock, pre, n, y);
    else ora_iirfilt_execute_block(q->dcblock, pre, n, y);
}

/* ===================================================================== */
/* FMStereo: reference src/demod.hpp:4-85 (python-liquiddsp's own loop)   */
/*   s = freqdem(x) (kf 4);  sc = s e^{-j theta};                         */
/*   pe = 0.999 pe + 0.001 carg(sc)   (double arithmetic, stored float);  */
/*   sc = sc e^{-j theta}; nco_pll_step(pe) (bandwidth 0.1); theta += d;  */
/*   L/R = de-emphasis(s +- re(sc)) -> resamp_rrrf_create_default(pcm/iq) */
/* An (L, R) pair is appended only when each resampler produced exactly   */
/* one output (demod_one returns nl + nr == 2, demod.hpp:45-47).          */
/* reset() resets only the two resamplers (demod.hpp:34-37); phase_error */
/* is uninitialised in the reference and starts at 0 here.               */
/* ===================================================================== */
struct ora_fmstereo_s {
    ora_nco mixer;
    ora_freqdem dem;
    ora_iirfilt emph_l, emph_r;
    ora_resamp aud_l, aud_r;
    float pe;
};
ora_fmstereo ora_fmstereo_create(float iq_rate, float pcm_rate)
{
    ora_fmstereo q = (ora_fmstereo)calloc(1, sizeof(*q));
    float b[1], a[2];
    a[0] = 1.0;
    a[1] = -exp(-1.0 / (75.0E-6 * iq_rate));
    b[0] = 1.0 + a[1];
    q->mixer = ora_nco_create(0);
    q->dem = ora_freqdem_create(4.0f);
    q->emph_l = ora_iirfilt_create_tf(b, 1, a, 2, 0);
    q->emph_r = ora_iirfilt_create_tf(b, 1, a, 2, 0);
    q->aud_l = ora_resamp_create_default(pcm_rate / iq_rate, 0);
    q->aud_r = ora_resamp_create_default(pcm_rate / iq_rate, 0);
    q->pe = 0.0f;
    return q;
}
void ora_fmstereo_destroy(ora_fmstereo q)
{
    if (!q) return;
    ora_nco_destroy(q->mixer);
    ora_freqdem_destroy(q->dem);
    ora_iirfilt_destroy(q->emph_l);
    ora_iirfilt_destroy(q->emph_r);
    ora_resamp_destroy(q->aud_l);
    ora_resamp_destroy(q->aud_r);
    free(q);
}
void ora_fmstereo_reset(ora_fmstereo q)
{
    ora_resamp_reset(q->aud_l);
    ora_resamp_reset(q->aud_r);
}
void ora_fmstereo_get_state(ora_fmstereo q, uint32_t *theta, uint32_t *dtheta, float *pe)
{
    *theta = q->mixer->theta;
    *dtheta = q->mixer->d_theta;
    *pe = q->pe;
}
void ora_fmstereo_set_state(ora_fmstereo q, uint32_t theta, uint32_t dtheta, float pe)
{
    q->mixer->theta = theta;
    q->mixer->d_theta = dtheta;
    q->pe = pe;
}
size_t ora_fmstereo_execute(ora_fmstereo q, const float *x, size_t n, float *y, float *dbg)
{
    size_t i, nw = 0;
    for (i = 0; i < n; i++) {
        float s, c, sn, r1, i1, r2, i2, l, r, lo[8], ro[8];
        ora_freqdem_demodulate_block(q->dem, x + 2 * i, 1, &s);
        nco_sincos(q->mixer, &sn, &c);
        cmul_down(s, 0.0f, c, sn, &r1, &i1);                  /* mix_down of (s + 0j) */
        q->pe = 0.999 * q->pe + 0.001 * om_atan2f(i1, r1);    /* double, stored float */
        cmul_down(r1, i1, c, sn, &r2, &i2);                   /* same phase: down again */
        ora_nco_pll_step(q->mixer, q->pe);
        q->mixer->theta += q->mixer->d_theta;                 /* nco_crcf_step */
        if (dbg) {
            dbg[4 * i] = s;
            dbg[4 * i + 1] = r2;
            dbg[4 * i + 2] = q->pe;
            uint32_t th = q->mixer->theta;
            memcpy(&dbg[4 * i + 3], &th, 4);
        }
        l = s + r2;
        r = s - r2;
        ora_iirfilt_execute_block(q->emph_l, &l, 1, &l);
        ora_iirfilt_execute_block(q->emph_r, &r, 1, &r);
        size_t nl = ora_resamp_execute_block(q->aud_l, &l, 1, lo);
        size_t nr = ora_resamp_execute_block(q->aud_r, &r, 1, ro);
        if (nl + nr == 2) {
            y[nw] = lo[0];
            y[nw + 1] = ro[0];
            nw += 2;
        }
    }
    return nw;
}
