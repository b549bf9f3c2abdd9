/* walk_spec.c -- CPU model of the AmpModem PLL walker (k_pll_walk): per
 * lane-block of G consecutive entries, the sequential repair chain (one
 * dependent step per repair) against speculate-and-verify passes: assume a
 * repair set M, give every entry the offset all repairs of M before it imply
 * (two prefix sums over the lanes), recompute the event mask; equal -> M is the
 * sequential loop's repair set; else keep M up to the first differing lane p,
 * take the new mask from p on, and pass again (each pass fixes lane p for good).
 *
 * Inputs (gen_agc_input.py, gen_walk_input.py): pll_x0.c64 (carrier lowpass of
 * the AmpModem input of BASELINE C4), nco_table.f32.  The phase detector uses
 * libm atan2f (statistics only, not the product's bits).
 *   gcc -O2 -o walk_spec walk_spec.c -lm && ./walk_spec [G=64] [log2B=19]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float tab[1024];
static float alpha, beta;

static uint32_t constrain(float th)
{
    float p = th * 0.159154943091895;
    float fp = p - (long)p;
    if (fp < 0.) fp += 1.;
    return (uint32_t)(int64_t)(fp * 0xffffffff);
}
static inline uint32_t tidx(uint32_t th) { return ((th + (1u << 21)) >> 22) & 0x3ffu; }
static inline void kick(uint32_t i, const float* x, uint32_t* k1, uint32_t* k2)
{
    float sn = tab[i], cs = tab[(i + 256) & 1023];
    float v0r = x[0] * cs - x[1] * (-sn), v0i = x[0] * (-sn) + x[1] * cs;
    float phi = atan2f(v0i, v0r);
    *k1 = constrain(phi * alpha);
    *k2 = constrain(phi * beta);
}

int main(int argc, char** argv)
{
    const int G = argc > 1 ? atoi(argv[1]) : 64;
    const int lb = argc > 2 ? atoi(argv[2]) : 19;
    const uint32_t B = 1u << lb;
    FILE* f = fopen("nco_table.f32", "rb");
    if (!f || fread(tab, 4, 1024, f) != 1024) return 1;
    fclose(f);
    f = fopen("pll_x0.c64", "rb");
    if (!f) return 1;
    fseek(f, 0, SEEK_END);
    long n = ftell(f) / 8;
    fseek(f, 0, SEEK_SET);
    float* x = malloc(8 * n);
    if (fread(x, 8, n, f) != (size_t)n) return 1;
    fclose(f);
    alpha = 0.001f;
    beta = sqrtf(alpha);
    const long P = 200000;        /* "previous call": its end state is the candidates' guess */
    uint32_t* T = malloc(4 * (n + 1));
    uint32_t th = 0, d = 0;
    for (long s = 0; s < n; s++) {
        T[s] = th;
        uint32_t k1, k2;
        kick(tidx(th), x + 2 * s, &k1, &k2);
        d += k1;
        th += k2 + d;
    }
    /* guess: the true state at P (the real guess is the previous call's last candidate) */
    uint32_t gth = T[P], gd = 0;
    {
        uint32_t t2 = 0, d2 = 0;
        for (long s = 0; s < P; s++) {
            uint32_t k1, k2;
            kick(tidx(t2), x + 2 * s, &k1, &k2);
            d2 += k1;
            t2 += k2 + d2;
        }
        gd = d2;
    }
    const long m = n - P;
    uint32_t* C = malloc(4 * m);
    long nent = 0, nrep = 0, multi = 0, gapmiss = 0;
    long* es = malloc(sizeof(long) * m);            /* entry sample (relative to P) */
    int32_t* dk1 = malloc(4 * m), *dk2 = malloc(4 * m), *tk1 = malloc(4 * m), *tk2 = malloc(4 * m);
    uint32_t* u = malloc(4 * m);
    unsigned char* rep = malloc(m);
    for (long s0 = 0; s0 < m; s0 += 256) {
        long s1 = s0 + 256 < m ? s0 + 256 : m;
        long w0 = s0 - 1024 < 0 ? 0 : s0 - 1024;
        uint32_t ct = gth + (uint32_t)((uint64_t)w0 * gd), cd = gd;
        for (long s = w0; s < s1; s++) {
            const float* xs = x + 2 * (P + s);
            uint32_t ic = tidx(ct), k1, k2;
            kick(ic, xs, &k1, &k2);
            if (s >= s0) {
                C[s] = ct;
                uint32_t w = ct + (1u << 21);
                int risky = ((w + B) & 0x3fffffu) < 2 * B;
                uint32_t it = tidx(T[P + s]);
                if (risky || s == s0 || s == s1 - 1) {
                    es[nent] = s;
                    u[nent] = w & 0x3fffffu;
                    int up = u[nent] >= (1u << 21);
                    uint32_t n1, n2;
                    kick((ic + (up ? 1 : 1023)) & 1023, xs, &n1, &n2);
                    dk1[nent] = (int32_t)(n1 - k1);
                    dk2[nent] = (int32_t)(n2 - k2);
                    rep[nent] = it != ic;
                    if (it != ic) {
                        uint32_t t1, t2;
                        kick(it, xs, &t1, &t2);
                        tk1[nent] = (int32_t)(t1 - k1);
                        tk2[nent] = (int32_t)(t2 - k2);
                        if (it != ((ic + (up ? 1 : 1023)) & 1023)) multi++;
                        nrep++;
                    }
                    nent++;
                } else if (it != ic) {
                    gapmiss++;
                }
            }
            cd += k1;
            ct += k2 + cd;
        }
    }
    printf("PCM samples %ld (after %ld of previous call), entries %ld (%.1f %%), repairs %ld, multi-cell %ld, "
           "mismatches in gaps %ld\n", m, P, nent, 100.0 * nent / m, nrep, multi, gapmiss);
    /* lane-blocks of G entries */
    long nlb = 0, lb0 = 0, hist[70] = {0}, tot_pass = 0, bad = 0, tot_pass_j = 0, jfail = 0;
    int32_t* f0 = malloc(4 * G);
    unsigned char *M = malloc(G), *Mn = malloc(G);
    for (long e0 = 0; e0 < nent; e0 += G) {
        int g = nent - e0 < G ? (int)(nent - e0) : G;
        nlb++;
        int nr = 0;
        for (int i = 0; i < g; i++) {
            long s = es[e0 + i];
            uint32_t ft = T[P + s] - C[s];
            for (int r = 0; r < i; r++)
                if (rep[e0 + r]) ft -= (uint32_t)tk2[e0 + r] + (uint32_t)(s - es[e0 + r]) * (uint32_t)tk1[e0 + r];
            f0[i] = (int32_t)ft;
            nr += rep[e0 + i];
        }
        if (nr == 0) lb0++;
        for (int i = 0; i < g; i++) M[i] = (u[e0 + i] + (uint32_t)f0[i]) >= (1u << 22);
        int passes = 0;
        for (;;) {
            passes++;
            for (int i = 0; i < g; i++) {
                long s = es[e0 + i];
                uint32_t xv = (uint32_t)f0[i];
                for (int j = 0; j < i; j++)
                    if (M[j]) xv += (uint32_t)dk2[e0 + j] + (uint32_t)(s - es[e0 + j]) * (uint32_t)dk1[e0 + j];
                Mn[i] = (u[e0 + i] + xv) >= (1u << 22);
            }
            int p = -1;
            for (int i = 0; i < g; i++)
                if (Mn[i] != M[i]) { p = i; break; }
            if (p < 0) break;
            for (int i = p; i < g; i++) M[i] = Mn[i];
            if (passes > 70) break;
        }
        for (int i = 0; i < g; i++)
            if (M[i] != rep[e0 + i]) { bad++; break; }
        hist[passes < 69 ? passes : 69]++;
        tot_pass += passes;
        /* Jacobi variant: M <- new mask whole, up to 4 passes */
        for (int i = 0; i < g; i++) M[i] = (u[e0 + i] + (uint32_t)f0[i]) >= (1u << 22);
        int pj = 0, ok = 0;
        while (pj < 8) {
            pj++;
            int same = 1;
            for (int i = 0; i < g; i++) {
                long s = es[e0 + i];
                uint32_t xv = (uint32_t)f0[i];
                for (int j = 0; j < i; j++)
                    if (M[j]) xv += (uint32_t)dk2[e0 + j] + (uint32_t)(s - es[e0 + j]) * (uint32_t)dk1[e0 + j];
                Mn[i] = (u[e0 + i] + xv) >= (1u << 22);
                same &= Mn[i] == M[i];
            }
            if (same) { ok = 1; break; }
            memcpy(M, Mn, g);
        }
        if (!ok) jfail++;
        tot_pass_j += pj;
    }
    /* sequential repair chain: at each repair j, is the next event (first lane > j
     * with x > W) the same under the mask before this repair as after it? */
    long steps = 0, same_next = 0;
    for (long e0 = 0; e0 < nent; e0 += G) {
        int g = nent - e0 < G ? (int)(nent - e0) : G;
        uint32_t xv[4096];
        for (int i = 0; i < g; i++) {
            long s = es[e0 + i];
            uint32_t ft = T[P + s] - C[s];
            for (int r = 0; r < i; r++)
                if (rep[e0 + r]) ft -= (uint32_t)tk2[e0 + r] + (uint32_t)(s - es[e0 + r]) * (uint32_t)tk1[e0 + r];
            xv[i] = ft;
        }
        int j = -1;
        for (;;) {
            int nj = -1;
            for (int i = j + 1; i < g; i++)
                if ((u[e0 + i] + xv[i]) >= (1u << 22)) { nj = i; break; }
            if (nj < 0) break;
            /* repair at nj: the next event before / after applying it */
            int before = -1, after = -1;
            for (int i = nj + 1; i < g; i++)
                if ((u[e0 + i] + xv[i]) >= (1u << 22)) { before = i; break; }
            for (int i = nj + 1; i < g; i++)
                xv[i] += (uint32_t)dk2[e0 + nj] + (uint32_t)(es[e0 + i] - es[e0 + nj]) * (uint32_t)dk1[e0 + nj];
            for (int i = nj + 1; i < g; i++)
                if ((u[e0 + i] + xv[i]) >= (1u << 22)) { after = i; break; }
            steps++;
            same_next += before == after;
            j = nj;
        }
    }
    printf("repair steps %ld: next event unchanged by the repair in %.1f %%\n", steps, 100.0 * same_next / steps);
    /* |f| distribution over all samples (true vs candidate offset), and how many
     * lane-blocks of 64 entries would have a gap endpoint beyond a narrower margin */
    {
        long cnt[24] = {0};
        for (long s = 0; s < m; s++) {
            int32_t fv = (int32_t)(T[P + s] - C[s]);
            uint32_t a = fv < 0 ? -(uint32_t)fv : (uint32_t)fv;
            int b = 0;
            while (b < 23 && a >= (1u << (b + 1))) b++;
            cnt[b]++;
        }
        printf("|f| over samples: ");
        for (int b = 14; b < 23; b++) printf(">=2^%d: %.3f %%  ", b, 100.0 * ({long t = 0; for (int q = b; q < 24; q++) t += cnt[q]; t;}) / m);
        printf("\n");
    }
    printf("lane-blocks of %d: %ld, without repair %ld (%.1f %%), repairs per lane-block %.2f\n", G, nlb, lb0,
           100.0 * lb0 / nlb, (double)nrep / nlb);
    printf("prefix-fix passes per lane-block: mean %.3f; final set != repairs in %ld lane-blocks (multi-cell)\n",
           (double)tot_pass / nlb, bad);
    printf("  hist:");
    for (int i = 1; i < 70; i++)
        if (hist[i]) printf(" %d:%ld", i, hist[i]);
    printf("\nJacobi passes (<= 8): mean %.3f, not converged %ld\n", (double)tot_pass_j / nlb, jfail);
    return 0;
}
