// design.cpp -- host-side filter design for libldsp (see design.hpp).
//
// The arithmetic mirrors liquid-dsp's C sources expression by expression,
// including C's float -> double promotions (a double literal such as M_PI or
// 1.0 promotes the whole expression; complex arithmetic with a double operand
// is carried out in double complex and rounded back).  In C++ those promotions
// are spelled out explicitly.  tests/test_product_host.py checks the taps and
// second-order sections produced here against oracle/liquid_restate.c bit for
// bit.
#include "design.hpp"

#include <math.h>

#include <algorithm>
#include <complex>
#include <cstring>
#include <vector>

#include "ldsp_common.hpp"

namespace ldsp {
namespace design {

using cf = std::complex<float>;
using cd = std::complex<double>;
static constexpr double kPi = 3.14159265358979323846;

// Complex division exactly as C's `/` on _Complex operands (cplx_c.c, compiled
// as C): C++ compilers lower std::complex division with another algorithm
// (1-ulp differences in the cheby2 poles / zeros).
extern "C" void ldsp_cdivf(float ar, float ai, float br, float bi, float* out);
extern "C" void ldsp_cdivd(double ar, double ai, double br, double bi, double* out);
extern "C" void ldsp_ellip_azpkf(unsigned int n, float ep, float es, float* za, float* pa);
extern "C" void ldsp_bessel_azpkf(unsigned int n, float* pa);
static inline cf cdiv(cf x, cf y)
{
    float r[2];
    ldsp_cdivf(x.real(), x.imag(), y.real(), y.imag(), r);
    return cf(r[0], r[1]);
}
static inline cd cdiv(cd x, cd y)
{
    double r[2];
    ldsp_cdivd(x.real(), x.imag(), y.real(), y.imag(), r);
    return cd(r[0], r[1]);
}

// liquid math.gamma.c liquid_lngammaf
static float lngammaf_(float z)
{
    if (z < 0) return 0.0f;
    if (z < 10.0f) return lngammaf_(z + 1.0f) - logf(z);
    float g = (float)(0.5 * ((double)logf((float)(2 * kPi)) - log((double)z)));
    g += z * (logf(z + (1 / (12.0f * z - 0.1f / z))) - 1);
    return g;
}

// liquid math.bessel.c liquid_besseli0f
static float besseli0f_(float z)
{
    if (z == 0.0f) return 1.0f;
    float y = 0.0f;
    for (unsigned int k = 0; k < 32; k++) {
        const float t = (float)k * logf(0.5f * z) - lngammaf_((float)k + 1.0f);
        y += expf(2 * t);
    }
    return y;
}

// liquid math.c sincf
static float sincf_(float x)
{
    if (fabsf(x) < 0.01f)
        return cosf((float)(kPi * x / 2.0f)) * cosf((float)(kPi * x / 4.0f)) *
               cosf((float)(kPi * x / 8.0f));
    return (float)((double)sinf((float)(kPi * x)) / (kPi * x));
}

float kaiser_beta_As(float as)
{
    as = fabsf(as);
    if (as > 50.0f) return 0.1102f * (as - 8.7f);
    if (as > 21.0f) return (float)(0.5842 * (double)powf(as - 21, 0.4f) + (double)(0.07886f * (as - 21)));
    return 0.0f;
}

float kaiser(unsigned int i, unsigned int wlen, float beta)
{
    if (i > wlen || beta < 0) return 0.0f;
    const float t = (float)i - (float)(wlen - 1) / 2;
    const float r = 2.0f * t / (float)wlen;
    const float a = besseli0f_(beta * sqrtf(1 - r * r));
    const float b = besseli0f_(beta);
    return a / b;
}

std::vector<float> firdes_kaiser(unsigned int n, float fc, float as, float mu)
{
    LDSP_REQUIRE(mu >= -0.5f && mu <= 0.5f, "firdes_kaiser: offset must be in [-0.5, 0.5]");
    LDSP_REQUIRE(fc >= 0.0f && fc <= 0.5f, "firdes_kaiser: cutoff must be in [0, 0.5]");
    LDSP_REQUIRE(n > 0, "firdes_kaiser: filter length must be > 0");
    const float beta = kaiser_beta_As(as);
    std::vector<float> h(n);
    for (unsigned int i = 0; i < n; i++) {
        const float t = (float)i - (float)(n - 1) / 2 + mu;
        h[i] = sincf_(2.0f * fc * t) * kaiser(i, n, beta);
    }
    return h;
}

std::vector<float> firdes_notch(unsigned int m, float f0, float as)
{
    LDSP_REQUIRE(m >= 1 && m <= 1000, "firdes_notch: semi-length must be in [1, 1000]");
    LDSP_REQUIRE(f0 >= -0.5f && f0 <= 0.5f, "firdes_notch: notch frequency out of range");
    LDSP_REQUIRE(as > 0.0f, "firdes_notch: stop-band attenuation must be > 0");
    const float beta = kaiser_beta_As(as);
    const unsigned int len = 2 * m + 1;
    std::vector<float> h(len);
    float scale = 0.0f;
    for (unsigned int i = 0; i < len; i++) {
        const float p = -cosf((float)(2.0f * kPi * f0 * ((float)i - (float)m)));
        const float w = kaiser(i, len, beta);
        h[i] = p * w;
        scale += h[i] * p;
    }
    for (auto& v : h) v /= scale;
    h[m] += 1.0f;
    return h;
}

// firhilbf_create(m, As) (liquid firhilb.proto.c, as recalled): the 4m+1-tap
// half-band kaiser prototype h turned into a Hilbert transformer,
// h[i] = imag(h[i] e^{j pi t / 2}), t = i - 2m; C evaluates
// cexpf(_Complex_I * 0.5f * M_PI * t) at the float (float)(0.5 pi t) and the
// real * complex product's imaginary part is h[i] sinf(.), so the same here.
// Returns the 2m odd taps, reversed: hq[j] = h[4m - 1 - 2j].
std::vector<float> firhilb_taps(unsigned int m, float as)
{
    LDSP_REQUIRE(m >= 2, "firhilb: filter semi-length must be at least 2");
    const unsigned int len = 4 * m + 1;
    std::vector<float> h = firdes_kaiser(len, 0.25f, fabsf(as), 0.0f);
    for (unsigned int i = 0; i < len; i++) {
        const float t = (float)i - (float)(len - 1) / 2.0f;
        h[i] = h[i] * sinf((float)(0.5 * kPi * (double)t));
    }
    std::vector<float> hq;
    for (unsigned int i = 1; i < len; i += 2) hq.push_back(h[len - i - 1]);
    return hq;
}

// ---------------------------------------------------------------- iirdes
namespace {

float theta_pole(unsigned int i, unsigned int n)
{
    return (float)((double)(float)(2 * (i + 1) + n - 1) * kPi / (double)(float)(2 * n));
}

void butter_azpk(unsigned int n, std::vector<cf>& pa)
{
    const unsigned int r = n % 2, L = (n - r) / 2;
    for (unsigned int i = 0; i < L; i++) {
        const float th = theta_pole(i, n);
        pa.push_back(std::exp(cf(0.0f, th)));
        pa.push_back(std::exp(cf(-0.0f, -th)));
    }
    if (r) pa.push_back(cf(-1.0f, 0.0f));
}

// (a*cos(th)) -+ j*b*sin(th) exactly as C forms `real -+ _Complex_I*b*s`
cf ellipse_point(float a, float b, float th, bool plus)
{
    const float re = a * cosf(th);
    const float s = sinf(th);
    const cf jb = cf(0.0f * b, 1.0f * b) * s;         // (_Complex_I*b)*sinf(theta)
    return plus ? cf(re + jb.real(), jb.imag()) : cf(re - jb.real(), -jb.imag());
}

void cheby_axes(float ep, unsigned int n, float& a, float& b)
{
    const float t0 = (float)sqrt(1.0 + 1.0 / (double)(ep * ep));
    const float tp = powf((float)((double)t0 + 1.0 / (double)ep), (float)(1.0 / (double)(float)n));
    const float tm = powf((float)((double)t0 - 1.0 / (double)ep), (float)(1.0 / (double)(float)n));
    b = (float)(0.5 * (double)(tp + tm));
    a = (float)(0.5 * (double)(tp - tm));
}

void cheby1_azpk(unsigned int n, float ep, std::vector<cf>& pa)
{
    float a, b;
    cheby_axes(ep, n, a, b);
    const unsigned int r = n % 2, L = (n - r) / 2;
    for (unsigned int i = 0; i < L; i++) {
        const float th = theta_pole(i, n);
        pa.push_back(ellipse_point(a, b, th, false));
        pa.push_back(ellipse_point(a, b, th, true));
    }
    if (r) pa.push_back(cf(-a, 0.0f));
}

void cheby2_azpk(unsigned int n, float es, std::vector<cf>& za, std::vector<cf>& pa)
{
    float a, b;
    cheby_axes(es, n, a, b);
    const unsigned int r = n % 2, L = (n - r) / 2;
    for (unsigned int i = 0; i < L; i++) {
        const float th = theta_pole(i, n);
        pa.push_back(cdiv(cf(1.0f, 0.0f), ellipse_point(a, b, th, false)));
        pa.push_back(cdiv(cf(1.0f, 0.0f), ellipse_point(a, b, th, true)));
    }
    if (r) pa.push_back(cf(-1.0f / a, 0.0f));
    for (unsigned int i = 0; i < L; i++) {
        const float th = (float)(0.5 * kPi * (double)(2 * (i + 1) - 1) / (double)(float)n);
        const float c = cosf(th);
        const cf jc(0.0f * c, 1.0f * c);               // _Complex_I*cosf(theta)
        za.push_back(cdiv(cf(-1.0f, 0.0f), jc));
        za.push_back(cdiv(cf(1.0f, 0.0f), jc));
    }
}

float freqprewarp(int btype, float fc, float f0)
{
    float m = 0.0f;
    if (btype == 0) m = tanf((float)(kPi * fc));
    else if (btype == 1) m = -cosf((float)(kPi * fc)) / sinf((float)(kPi * fc));
    else if (btype == 2)
        m = (cosf((float)(2 * kPi * fc)) - cosf((float)(2 * kPi * f0))) / sinf((float)(2 * kPi * fc));
    else if (btype == 3)
        m = sinf((float)(2 * kPi * fc)) / (cosf((float)(2 * kPi * fc)) - cosf((float)(2 * kPi * f0)));
    return fabsf(m);
}

// (1.0 + z) / (1.0 - z) with C's real+complex rules, evaluated in double complex
cf bilin(cf z)
{
    const cd num(1.0 + (double)z.real(), (double)z.imag());
    const cd den(1.0 - (double)z.real(), -(double)z.imag());
    const cd q = cdiv(num, den);
    return cf((float)q.real(), (float)q.imag());
}

void bilinear(const std::vector<cf>& za, const std::vector<cf>& pa, cf ka, float m, std::vector<cf>& zd,
              std::vector<cf>& pd, cf& kd)
{
    const size_t n = pa.size();
    cf G = ka;
    zd.assign(n, cf());
    pd.assign(n, cf());
    for (size_t i = 0; i < n; i++) {
        zd[i] = (i < za.size()) ? bilin(za[i] * m) : cf(-1.0f, 0.0f);
        pd[i] = bilin(pa[i] * m);
        const cd a(1.0 - (double)pd[i].real(), -(double)pd[i].imag());
        const cd b(1.0 - (double)zd[i].real(), -(double)zd[i].imag());
        const cd g = cd((double)G.real(), (double)G.imag()) * cdiv(a, b);
        G = cf((float)g.real(), (float)g.imag());
    }
    kd = G;
}

void lp2bp(std::vector<cf>& zd, std::vector<cf>& pd, float f0)
{
    const float c0 = cosf((float)(2 * kPi * f0));
    auto xf = [&](const std::vector<cf>& in) {
        std::vector<cf> out(2 * in.size());
        for (size_t i = 0; i < in.size(); i++) {
            const cf t0 = 1.0f + in[i];                     // C: 1 + z (real + complex)
            const cf d = std::sqrt(c0 * c0 * t0 * t0 - 4.0f * in[i]);
            out[2 * i + 0] = 0.5f * (c0 * t0 + d);
            out[2 * i + 1] = 0.5f * (c0 * t0 - d);
        }
        return out;
    };
    zd = xf(zd);
    pd = xf(pd);
}

// liquid_cplxpair + liquid_cplxpair_cleanup
std::vector<cf> cplxpair(const std::vector<cf>& z, float tol)
{
    const size_t n = z.size();
    std::vector<char> paired(n, 0);
    std::vector<cf> p;
    p.reserve(n);
    size_t num_pairs = 0;
    for (size_t i = 0; i < n; i++) {
        if (paired[i] || fabsf(z[i].imag()) < tol) continue;
        for (size_t j = 0; j < n; j++) {
            if (j == i || paired[j] || fabsf(z[j].imag()) < tol) continue;
            if (fabsf(z[i].imag() + z[j].imag()) < tol && fabsf(z[i].real() - z[j].real()) < tol) {
                p.push_back(z[i]);
                p.push_back(z[j]);
                paired[i] = paired[j] = 1;
                num_pairs++;
                break;
            }
        }
    }
    for (size_t i = 0; i < n; i++)
        if (!paired[i]) p.push_back(z[i]);
    for (size_t i = 0; i < num_pairs; i++) {
        p[2 * i] = p[2 * i].imag() < 0 ? p[2 * i] : std::conj(p[2 * i]);
        p[2 * i + 1] = std::conj(p[2 * i]);
    }
    for (size_t i = 0; i < num_pairs; i++)
        for (size_t j = num_pairs - 1; j > i; j--)
            if (p[2 * (j - 1)].real() > p[2 * j].real()) {
                std::swap(p[2 * (j - 1)], p[2 * j]);
                std::swap(p[2 * (j - 1) + 1], p[2 * j + 1]);
            }
    for (size_t i = 2 * num_pairs; i < n; i++)
        for (size_t j = n - 1; j > i; j--)
            if (p[j - 1].real() > p[j].real()) std::swap(p[j - 1], p[j]);
    return p;
}

void dzpk(int ftype, int btype, unsigned int n, float fc, float f0, float ap, float as, std::vector<cf>& zd,
          std::vector<cf>& pd, cf& kd)
{
    LDSP_REQUIRE(fc > 0 && fc < 0.5f, "iirdes: cutoff frequency out of range (0, 0.5)");
    LDSP_REQUIRE(f0 >= 0 && f0 <= 0.5f, "iirdes: center frequency out of range [0, 0.5]");
    LDSP_REQUIRE(ap > 0, "iirdes: pass-band ripple must be > 0");
    LDSP_REQUIRE(as > 0, "iirdes: stop-band attenuation must be > 0");
    LDSP_REQUIRE(n > 0, "iirdes: filter order must be > 0");
    std::vector<cf> za, pa;
    cf k0(1.0f, 0.0f);
    const unsigned int r = n % 2;
    switch (ftype) {
    case 0:
        butter_azpk(n, pa);
        break;
    case 1: {
        const float ep = sqrtf(powf(10.0f, ap / 10.0f) - 1.0f);
        k0 = cf(r ? 1.0f : 1.0f / sqrtf(1.0f + ep * ep), 0.0f);
        cheby1_azpk(n, ep, pa);
        break;
    }
    case 2: {
        const float es = powf(10.0f, -as / 20.0f);
        cheby2_azpk(n, es, za, pa);
        break;
    }
    case 3: {   // elliptic (cplx_c.c)
        const float Gp = powf(10.0f, -ap / 20.0f), Gs = powf(10.0f, -as / 20.0f);
        const float ep = sqrtf(1.0f / (Gp * Gp) - 1.0f), es = sqrtf(1.0f / (Gs * Gs) - 1.0f);
        k0 = cf(r ? 1.0f : 1.0f / sqrtf(1.0f + ep * ep), 0.0f);
        za.assign(n - r, cf());
        pa.assign(n, cf());
        ldsp_ellip_azpkf(n, ep, es, reinterpret_cast<float*>(za.data()), reinterpret_cast<float*>(pa.data()));
        break;
    }
    case 4:     // Bessel (cplx_c.c)
        LDSP_REQUIRE(n <= 48, "iirdes: Bessel order must be <= 48");
        pa.assign(n, cf());
        ldsp_bessel_azpkf(n, reinterpret_cast<float*>(pa.data()));
        break;
    default:
        throw Error(LDSP_EINVAL, "iirdes: unknown filter type");
    }
    bilinear(za, pa, k0, freqprewarp(btype, fc, f0), zd, pd, kd);
    if (btype == 1 || btype == 3) {
        for (auto& z : zd) z = -z;
        for (auto& p : pd) p = -p;
    }
    if (btype == 2 || btype == 3) lp2bp(zd, pd, f0);
}

} // namespace

SOS iirdes_sos(int ftype, int btype, unsigned int order, float fc, float f0, float ap, float as)
{
    std::vector<cf> zd, pd;
    cf kd;
    dzpk(ftype, btype, order, fc, f0, ap, as, zd, pd, kd);
    const unsigned int n = (unsigned int)pd.size();
    const std::vector<cf> zp = cplxpair(zd, 1e-6f), pp = cplxpair(pd, 1e-6f);
    const unsigned int r = n % 2, L = (n - r) / 2;
    SOS s;
    s.nsos = L + r;
    s.B.assign(3 * s.nsos, 0.0f);
    s.A.assign(3 * s.nsos, 0.0f);
    unsigned int i;
    for (i = 0; i < L; i++) {
        const cf p0 = -pp[2 * i], p1 = -pp[2 * i + 1], z0 = -zp[2 * i], z1 = -zp[2 * i + 1];
        s.A[3 * i + 0] = 1.0f;
        s.A[3 * i + 1] = (p0 + p1).real();
        s.A[3 * i + 2] = (p0 * p1).real();
        s.B[3 * i + 0] = 1.0f;
        s.B[3 * i + 1] = (z0 + z1).real();
        s.B[3 * i + 2] = (z0 * z1).real();
    }
    if (r) {
        s.A[3 * i + 0] = 1.0f;
        s.A[3 * i + 1] = (-pp[n - 1]).real();
        s.A[3 * i + 2] = 0.0f;
        s.B[3 * i + 0] = 1.0f;
        s.B[3 * i + 1] = (-zp[n - 1]).real();
        s.B[3 * i + 2] = 0.0f;
    }
    const float k = powf(kd.real(), 1.0f / (float)(L + r));
    for (auto& b : s.B) b *= k;
    return s;
}

TF iirdes_tf(int ftype, int btype, unsigned int order, float fc, float f0, float ap, float as)
{
    std::vector<cf> zd, pd;
    cf kd;
    dzpk(ftype, btype, order, fc, f0, ap, as, zd, pd, kd);
    const unsigned int n = (unsigned int)pd.size();
    // liquid polycf_expandroots
    auto expand = [n](const std::vector<cf>& rt) {
        std::vector<cf> c(n + 1, cf(0.0f, 0.0f));
        c[0] = cf(1.0f, 0.0f);
        for (unsigned int i = 0; i < n; i++) {
            for (unsigned int j = i + 1; j > 0; j--) c[j] = -rt[i] * c[j] + c[j - 1];
            c[0] *= -rt[i];
        }
        return c;
    };
    TF t;
    t.a.resize(n + 1);
    t.b.resize(n + 1);
    std::vector<cf> q = expand(pd);
    for (unsigned int i = 0; i <= n; i++) t.a[i] = q[n - i].real();
    q = expand(zd);
    for (unsigned int i = 0; i <= n; i++) t.b[i] = (q[n - i] * kd).real();
    return t;
}

} // namespace design
} // namespace ldsp
