// modal.cpp -- host construction and check of an IIR filter's modal form
// (modal.hpp), in long double.
//
// For the recursion s' = A s + B u, y = C s + Dd u with D distinct poles
// lambda_k (eigenvalues of A): eigenvectors w_k by inverse iteration, beta =
// W^-1 B, V = W diag(beta) (so V^-1 B = 1), g = C V.  With z = V^-1 s:
//     z_k' = lambda_k z_k + u,    y = Dd u + sum_k g_k z_k.
// For a real filter the non-real poles come in conjugate pairs whose modes are
// conjugate for real input: one mode per pair carries weight 2 (y gets
// 2 Re(g_k z_k)), a real pole one mode of weight 1.  The kernel runs each mode
// as a real direct-form section (below: the parallel form of the filter, one
// section per pole pair).  The form is accepted only
// when it reproduces the long-double state-space recursion to 1e-10 (impulse +
// noise input, the free response of a random state, and the state round trip);
// clustered poles (narrow high-order Butterworth / Chebyshev-I designs) make V
// ill-conditioned and fail here, keeping the SOS-coordinate scan.
#include "modal.hpp"

#include <algorithm>
#include <array>
#include <cmath>

namespace ldsp {

namespace {

using ld = long double;
using cld = std::complex<long double>;

// A (n x n) X = B (n x m) by Gaussian elimination with partial pivoting; false if singular
bool csolve(std::vector<cld> A, std::vector<cld>& X, int n, int m)
{
    for (int col = 0; col < n; col++) {
        int piv = col;
        ld best = std::abs(A[col * n + col]);
        for (int r = col + 1; r < n; r++) {
            const ld v = std::abs(A[r * n + col]);
            if (v > best) {
                best = v;
                piv = r;
            }
        }
        if (!(best > 0)) return false;
        if (piv != col) {
            for (int c = 0; c < n; c++) std::swap(A[col * n + c], A[piv * n + c]);
            for (int c = 0; c < m; c++) std::swap(X[col * m + c], X[piv * m + c]);
        }
        for (int r = col + 1; r < n; r++) {
            const cld f = A[r * n + col] / A[col * n + col];
            if (f == cld(0)) continue;
            for (int c = col; c < n; c++) A[r * n + c] -= f * A[col * n + c];
            for (int c = 0; c < m; c++) X[r * m + c] -= f * X[col * m + c];
        }
    }
    for (int row = n - 1; row >= 0; row--)
        for (int c = 0; c < m; c++) {
            cld s = X[row * m + c];
            for (int k = row + 1; k < n; k++) s -= A[row * n + k] * X[k * m + c];
            X[row * m + c] = s / A[row * n + row];
        }
    return true;
}

cld cpow_u(cld z, unsigned long long e)
{
    cld r(1);
    while (e) {
        if (e & 1) r *= z;
        z *= z;
        e >>= 1;
    }
    return r;
}

// deterministic input for the host check: uniform in [-1, 1)
struct Lcg {
    uint64_t s = 0x9e3779b97f4a7c15ull;
    double next()
    {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (double)(s >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    }
};

} // namespace

std::vector<cld> sos_poles(const std::vector<float>& a, unsigned nsos)
{
    std::vector<cld> p;
    for (unsigned s = 0; s < nsos; s++) {
        const ld a1 = a[3 * s + 1], a2 = a[3 * s + 2];
        const ld disc = a1 * a1 - 4 * a2;
        if (disc >= 0) {   // q = -(a1 + sign(a1) sqrt(disc)) / 2: roots q and a2 / q
            const ld r = std::sqrt(disc);
            const ld q = -0.5L * (a1 + (a1 >= 0 ? r : -r));
            p.push_back(cld(q, 0));
            p.push_back(cld(q != 0 ? a2 / q : 0, 0));
        } else {
            const ld im = std::sqrt(-disc) / 2;
            p.push_back(cld(-a1 / 2, im));
            p.push_back(cld(-a1 / 2, -im));
        }
    }
    return p;
}

std::vector<cld> tf_poles(const std::vector<float>& a, int na, int D)
{
    // Durand-Kerner on z^D + c1 z^(D-1) + ... + cD, then Newton polishing
    std::vector<ld> c(D + 1, 0);
    c[0] = 1;
    for (int i = 1; i <= D; i++) c[i] = i < na ? (ld)a[i] : 0;
    auto P = [&](cld z) {
        cld v(1);
        for (int i = 1; i <= D; i++) v = v * z + c[i];
        return v;
    };
    auto dP = [&](cld z) {
        cld v(0), d(0);
        cld p(1);
        for (int i = 1; i <= D; i++) {
            d = d * z + p;
            p = p * z + c[i];
        }
        (void)v;
        return d;
    };
    ld R = 1;
    for (int i = 1; i <= D; i++) R = std::max(R, 1 + std::abs(c[i]));
    std::vector<cld> z(D);
    const cld seed(0.4L, 0.9L);
    for (int k = 0; k < D; k++) z[k] = R * cpow_u(seed, k + 1) / std::abs(cpow_u(seed, k + 1));
    for (int it = 0; it < 2000; it++) {
        ld moved = 0;
        for (int k = 0; k < D; k++) {
            cld den(1);
            for (int j = 0; j < D; j++)
                if (j != k) den *= z[k] - z[j];
            if (den == cld(0)) continue;
            const cld dz = P(z[k]) / den;
            z[k] -= dz;
            moved = std::max(moved, std::abs(dz));
        }
        if (moved < 1e-19L) break;
    }
    for (int k = 0; k < D; k++)
        for (int it = 0; it < 4; it++) {
            const cld d = dP(z[k]);
            if (d == cld(0)) break;
            z[k] -= P(z[k]) / d;
        }
    return z;
}

ModalForm modal_form(int D, const std::vector<ld>& A, const std::vector<ld>& B, const std::vector<ld>& C, ld Dd,
                     const std::vector<cld>& poles)
{
    ModalForm f;
    f.D = D;
    auto fail = [&](const char* why) {
        f.ok = false;
        f.why = why;
        return f;
    };
    if (D < 1 || D > 2 * k::kIirModalMax || (int)poles.size() != D) return fail("state dimension");
    ld lmax = 0, anorm = 0;
    for (int i = 0; i < D; i++) {
        lmax = std::max(lmax, std::abs(poles[i]));
        for (int j = i + 1; j < D; j++)
            if (std::abs(poles[i] - poles[j]) <= 1e-9L * std::max<ld>(1, std::abs(poles[i])))
                return fail("repeated pole");
        ld row = 0;
        for (int j = 0; j < D; j++) row += std::fabs(A[i * D + j]);
        anorm = std::max(anorm, row);
    }
    if (!(lmax < 1)) return fail("pole on or outside the unit circle");

    // eigenvectors (columns of W) by inverse iteration with a slightly shifted pole
    std::vector<cld> W(D * D);
    for (int k = 0; k < D; k++) {
        const ld sc = 1 + std::abs(poles[k]);
        const cld mu = poles[k] + cld(1e-12L * sc, 0.7e-12L * sc);
        std::vector<cld> x(D);
        for (int i = 0; i < D; i++) x[i] = cld(1 + 0.1L * i, 0.05L * i);
        for (int it = 0; it < 4; it++) {
            std::vector<cld> Mx(D * D);
            for (int i = 0; i < D; i++)
                for (int j = 0; j < D; j++) Mx[i * D + j] = cld(A[i * D + j]) - (i == j ? mu : cld(0));
            if (!csolve(Mx, x, D, 1)) return fail("eigenvector");
            ld nrm = 0;
            for (int i = 0; i < D; i++) nrm += std::norm(x[i]);
            nrm = std::sqrt(nrm);
            if (!(nrm > 0) || !std::isfinite((double)nrm)) return fail("eigenvector");
            for (int i = 0; i < D; i++) x[i] /= nrm;
        }
        ld res = 0;
        for (int i = 0; i < D; i++) {
            cld r = -poles[k] * x[i];
            for (int j = 0; j < D; j++) r += A[i * D + j] * x[j];
            res = std::max(res, std::abs(r));
        }
        if (res > 1e-10L * (1 + anorm)) return fail("eigenvector residual");
        for (int i = 0; i < D; i++) W[i * D + k] = x[i];
    }
    std::vector<cld> beta(D);
    for (int i = 0; i < D; i++) beta[i] = cld(B[i]);
    if (!csolve(W, beta, D, 1)) return fail("eigenvectors dependent");
    std::vector<cld> V(D * D), g(D, cld(0));
    for (int k = 0; k < D; k++) {
        if (!(std::abs(beta[k]) > 0)) return fail("mode not driven by the input");
        for (int i = 0; i < D; i++) {
            V[i * D + k] = W[i * D + k] * beta[k];
            g[k] += C[i] * V[i * D + k];
        }
    }
    std::vector<cld> Vi(D * D, cld(0));
    for (int i = 0; i < D; i++) Vi[i * D + i] = 1;
    if (!csolve(V, Vi, D, D)) return fail("modal basis singular");

    // one mode per conjugate pair (weight 2) or real pole (weight 1)
    std::vector<int> rep;
    std::vector<int> wt;
    int npair = 0, nreal = 0, nneg = 0;
    for (int k = 0; k < D; k++) {
        const ld im = poles[k].imag(), tol = 1e-12L * std::max<ld>(1, std::abs(poles[k]));
        if (std::fabs(im) <= tol) {
            rep.push_back(k);
            wt.push_back(1);
            nreal++;
        } else if (im > 0) {
            bool partner = false;
            for (int j = 0; j < D; j++)
                if (poles[j].imag() < 0 &&
                    std::abs(poles[j] - std::conj(poles[k])) <= 1e-9L * std::max<ld>(1, std::abs(poles[k])))
                    partner = true;
            if (!partner) return fail("complex pole without its conjugate");
            rep.push_back(k);
            wt.push_back(2);
            npair++;
        } else {
            nneg++;
        }
    }
    if (nneg != npair || 2 * npair + nreal != D) return fail("pole pairing");
    const int M = (int)rep.size();
    if (M > k::kIirModalMax) return fail("too many modes");
    f.M = M;

    // Each mode as a real second-order section (a real pole: first order) in
    // direct form: w_n = u_n - a1 w_{n-1} - a2 w_{n-2}, section state
    // v = (w_n, w_{n-1}), output c1 w_{n-1} + c2 w_{n-2}.  For a pair,
    // 1 / (1 - lambda z^-1) = (1 - conj(lambda) z^-1) / ((1 - lambda z^-1)(1 - conj(lambda) z^-1)),
    // so z_n = w_n - conj(lambda) w_{n-1}, and 2 Re(g z_{n-1}) = c1 w_{n-1} + c2 w_{n-2}
    // with c1 = 2 Re g, c2 = -2 Re(g conj(lambda)): 4 FMAs per section and
    // sample instead of the 6 of the complex recursion.
    f.cf = k::IirModalCoef{};
    f.cf.M = M;
    f.cf.d = (double)Dd;
    std::vector<ld> A11(M), A12(M);    // section matrix [[A11, A12], [1, 0]] = [[-a1, -a2], [1, 0]] (double-rounded)
    for (int m = 0; m < M; m++) {
        const int k = rep[m];
        const bool real = wt[m] == 1;
        const cld lam = real ? cld(poles[k].real(), 0) : poles[k];
        const cld gk = real ? cld(g[k].real(), 0) : g[k];
        f.cf.a1[m] = (double)(real ? -lam.real() : -2 * lam.real());
        f.cf.a2[m] = (double)(real ? 0 : std::norm(lam));
        f.cf.c1[m] = (double)(real ? gk.real() : 2 * gk.real());
        f.cf.c2[m] = (double)(real ? 0 : -2 * (gk.real() * lam.real() + gk.imag() * lam.imag()));
        A11[m] = -(ld)f.cf.a1[m];
        A12[m] = -(ld)f.cf.a2[m];
    }
    // state conversions: DF-II layout s (D) <-> section states v (2 M)
    f.to_v.assign((size_t)2 * M * D, 0.0);
    f.from_v.assign((size_t)D * 2 * M, 0.0);
    for (int m = 0; m < M; m++) {
        const int k = rep[m];
        const bool real = wt[m] == 1;
        const ld lr = poles[k].real(), li = real ? 0 : poles[k].imag();
        for (int i = 0; i < D; i++) {
            const cld r = Vi[k * D + i];                 // z_m = sum_i r s_i
            const cld v = V[i * D + k];                  // s_i gets wt Re(v z_m)
            if (real) {
                f.to_v[(size_t)(2 * m) * D + i] = (double)r.real();
                f.from_v[(size_t)i * 2 * M + 2 * m] = (double)v.real();
            } else {                                     // v1 = Im z / li, v0 = Re z + lr v1
                f.to_v[(size_t)(2 * m + 1) * D + i] = (double)(r.imag() / li);
                f.to_v[(size_t)(2 * m) * D + i] = (double)(r.real() + lr * r.imag() / li);
                f.from_v[(size_t)i * 2 * M + 2 * m] = (double)(2 * v.real());
                f.from_v[(size_t)i * 2 * M + 2 * m + 1] = (double)(-2 * (v.real() * lr + v.imag() * li));
            }
        }
    }

    // host check: the double-precision section recursion (the kernel's
    // formulas and summation order) against the long-double state-space recursion
    auto sec_step = [&](std::vector<double>& v, double u) {
        double y0 = f.cf.d * u, y1 = 0.0;
        for (int m = 0; m < M; m++) {
            double& y = (m & 1) ? y1 : y0;
            y = std::fma(f.cf.c1[m], v[2 * m], y);
            y = std::fma(f.cf.c2[m], v[2 * m + 1], y);
            const double w = std::fma(-f.cf.a1[m], v[2 * m], std::fma(-f.cf.a2[m], v[2 * m + 1], u));
            v[2 * m + 1] = v[2 * m];
            v[2 * m] = w;
        }
        return y0 + y1;
    };
    auto ss_step = [&](std::vector<ld>& s, ld u) {
        ld y = Dd * u;
        for (int i = 0; i < D; i++) y += C[i] * s[i];
        std::vector<ld> t(D, 0);
        for (int i = 0; i < D; i++) {
            ld v = B[i] * u;
            for (int j = 0; j < D; j++) v += A[i * D + j] * s[j];
            t[i] = v;
        }
        s = t;
        return y;
    };
    Lcg rng;
    double err = 0;
    {   // impulse + noise from rest
        std::vector<double> v(2 * M, 0.0);
        std::vector<ld> s(D, 0);
        double ymax = 0, dmax = 0;
        for (int n = 0; n < 4096; n++) {
            const double u = n == 0 ? 1.0 : rng.next();
            const ld ys = ss_step(s, u);
            const double ym = sec_step(v, u);
            ymax = std::max(ymax, (double)std::fabs(ys));
            dmax = std::max(dmax, std::fabs(ym - (double)ys));
        }
        err = std::max(err, ymax > 0 ? dmax / ymax : dmax);
    }
    {   // a random state: round trip and free response
        std::vector<ld> s(D);
        double smax = 0;
        for (int i = 0; i < D; i++) {
            s[i] = rng.next();
            smax = std::max(smax, (double)std::fabs(s[i]));
        }
        std::vector<double> v(2 * M, 0.0);
        for (int q = 0; q < 2 * M; q++)
            for (int i = 0; i < D; i++) v[q] += f.to_v[(size_t)q * D + i] * (double)s[i];
        double dmax = 0;
        for (int i = 0; i < D; i++) {
            double t = 0;
            for (int q = 0; q < 2 * M; q++) t += f.from_v[(size_t)i * 2 * M + q] * v[q];
            dmax = std::max(dmax, std::fabs(t - (double)s[i]));
        }
        err = std::max(err, dmax / smax);
        double ymax = 0;
        dmax = 0;
        for (int n = 0; n < 512; n++) {
            const ld ys = ss_step(s, 0);
            const double ym = sec_step(v, 0.0);
            ymax = std::max(ymax, (double)std::fabs(ys));
            dmax = std::max(dmax, std::fabs(ym - (double)ys));
        }
        if (ymax > 0) err = std::max(err, dmax / ymax);
    }
    f.err = err;
    if (!(err <= 1e-10)) return fail("modal form ill-conditioned");

    // look-back depth.  A unit's start state drops the end states of the units
    // J and more before it, i.e. sum_{i >= J} A^(2048 i) BL; bound that tail with
    // the norms of the actual 2 x 2 section powers (a section's powers can grow
    // ~1/sin(theta) above |lambda|^k before they decay) times the modal basis's
    // conditioning ||to_v|| ||from_v|| (the look-back runs in modal coordinates),
    // and take the smallest J whose bound is below 2^-70.  Start from the
    // spectral-radius estimate max |lambda|^(2048 J) < 2^-70.
    int J = 1;
    if (lmax > 0) {
        const ld need = 70 * std::log(2.0L) / (-(ld)k::kIirModalChunk * 64 * std::log(lmax));
        J = std::max(1, (int)std::ceil(need));
    }
    if (J > k::kIirModalJmax) return fail("decays too slowly for the look-back");
    {
        auto mat_inf = [&](const std::vector<double>& X, int rows, int cols) {
            ld r = 0;
            for (int i = 0; i < rows; i++) {
                ld s = 0;
                for (int j = 0; j < cols; j++) s += std::fabs((ld)X[(size_t)i * cols + j]);
                r = std::max(r, s);
            }
            return r;
        };
        const ld cond = std::max((ld)1, mat_inf(f.to_v, 2 * M, D) * mat_inf(f.from_v, D, 2 * M));
        // per section: P = A^2048 (squarings), then ||A^(2048 i)|| for i = 1, 2, ..
        std::vector<std::array<ld, 4>> U(M), Pw(M);
        for (int m = 0; m < M; m++) {
            std::array<ld, 4> b = {A11[m], A12[m], 1, 0};
            for (int s = 0; s < 11; s++)
                b = {b[0] * b[0] + b[1] * b[2], b[0] * b[1] + b[1] * b[3], b[2] * b[0] + b[3] * b[2],
                     b[2] * b[1] + b[3] * b[3]};
            U[m] = b;                                    // A^2048
            Pw[m] = {1, 0, 0, 1};
        }
        // tail[i] = max_m sum_{i' >= i} ||A_m^(2048 i')||, over i up to the point
        // where the terms are negligible (or kIirModalJmax + 1, where it fails)
        const int imax = k::kIirModalJmax + 64;
        std::vector<ld> term((size_t)imax + 1, 0);
        for (int m = 0; m < M; m++) {
            std::array<ld, 4> p = {1, 0, 0, 1};
            for (int i = 0; i <= imax; i++) {
                const ld nrm = std::max(std::fabs(p[0]) + std::fabs(p[1]), std::fabs(p[2]) + std::fabs(p[3]));
                term[(size_t)i] = std::max(term[(size_t)i], nrm);
                const std::array<ld, 4>& b = U[m];
                p = {p[0] * b[0] + p[1] * b[2], p[0] * b[1] + p[1] * b[3], p[2] * b[0] + p[3] * b[2],
                     p[2] * b[1] + p[3] * b[3]};
            }
        }
        std::vector<ld> tail((size_t)imax + 2, 0);
        {   // beyond imax: a geometric continuation at the last ratio (no decay: no bound)
            const ld a = term[(size_t)imax], r = term[(size_t)imax - 1] > 0 ? a / term[(size_t)imax - 1] : 0;
            tail[(size_t)imax + 1] = a == 0 ? 0 : (r < 1 ? a * r / (1 - r) : HUGE_VALL);
        }
        for (int i = imax; i >= 0; i--) tail[(size_t)i] = tail[(size_t)i + 1] + term[(size_t)i];
        const ld lim = std::ldexp((ld)1, -70);
        while (J <= k::kIirModalJmax && !(cond * tail[(size_t)J] < lim)) J++;
        if (J > k::kIirModalJmax) return fail("decays too slowly for the look-back (section power bound)");
    }
    f.J = J;

    // powers of the section matrices, [m00, m01, m10, m11] per section
    auto matpow2 = [&](int m, unsigned long long e) {
        ld r[4] = {1, 0, 0, 1}, b[4] = {A11[m], A12[m], 1, 0};
        while (e) {
            if (e & 1) {
                const ld t[4] = {r[0] * b[0] + r[1] * b[2], r[0] * b[1] + r[1] * b[3], r[2] * b[0] + r[3] * b[2],
                                 r[2] * b[1] + r[3] * b[3]};
                std::copy(t, t + 4, r);
            }
            const ld t[4] = {b[0] * b[0] + b[1] * b[2], b[0] * b[1] + b[1] * b[3], b[2] * b[0] + b[3] * b[2],
                             b[2] * b[1] + b[3] * b[3]};
            std::copy(t, t + 4, b);
            e >>= 1;
        }
        for (int q = 0; q < 4; q++) f.tables.push_back((double)r[q]);
    };
    f.tables.clear();
    for (int l = 0; l < 6; l++)
        for (int m = 0; m < M; m++) matpow2(m, (unsigned long long)k::kIirModalChunk << l);
    for (int t = 0; t < 64; t++)
        for (int m = 0; m < M; m++) matpow2(m, (unsigned long long)k::kIirModalChunk * t);
    for (int i = 0; i < J; i++)
        for (int m = 0; m < M; m++) matpow2(m, (unsigned long long)k::kIirModalChunk * 64 * i);
    f.ok = true;
    return f;
}

} // namespace ldsp
