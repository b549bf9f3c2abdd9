/* walk_margin.c -- CPU model of the AmpModem PLL walker's entry margin B (same
 * inputs and trajectory model as walk_spec.c): for B = 2^17.5 .. 2^19, how many
 * samples become entries (within B of a table-cell edge, plus every 256-sample
 * chunk's first and last sample) and how many 512-entry walker blocks would fail
 * their gap proof (some entry of the block with |f| > B, f = the true trajectory's
 * offset from the candidate) and need the fallback.  Statistics only (libm
 * atan2f).   gcc -O2 -o walk_margin walk_margin.c -lm && ./walk_margin */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

int main(void)
{
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
    const long P = 200000;
    uint32_t* T = malloc(4 * (n + 1));
    uint32_t th = 0, d = 0;
    for (long s = 0; s < n; s++) {
        T[s] = th;
        uint32_t k1, k2;
        kick(tidx(th), x + 2 * s, &k1, &k2);
        d += k1;
        th += k2 + d;
    }
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
    uint32_t* W = malloc(4 * m);      /* candidate w = theta + 2^21 */
    int32_t* F = malloc(4 * m);       /* f = true - candidate */
    unsigned char* edge = malloc(m);
    for (long s0 = 0; s0 < m; s0 += 256) {
        long s1 = s0 + 256 < m ? s0 + 256 : m;
        long w0 = s0 - 1024 < 0 ? 0 : s0 - 1024;
        uint32_t ct = gth + (uint32_t)((uint64_t)w0 * gd), cd = gd;
        for (long s = w0; s < s1; s++) {
            uint32_t k1, k2;
            kick(tidx(ct), x + 2 * (P + s), &k1, &k2);
            if (s >= s0) {
                W[s] = ct + (1u << 21);
                F[s] = (int32_t)(T[P + s] - ct);
                edge[s] = s == s0 || s == s1 - 1;
            }
            cd += k1;
            ct += k2 + cd;
        }
    }
    printf("%ld PCM samples\n", m);
    for (double lb = 17.5; lb <= 19.01; lb += 0.25) {
        const uint32_t B = (uint32_t)ldexp(1.0, 0) * (uint32_t)ldexp(1.0, 0) * (uint32_t)pow(2.0, lb);
        long ne = 0, nbad_e = 0, blocks = 0, bad_blocks = 0, in_blk = 0, blk_bad = 0;
        for (long s = 0; s < m; s++) {
            const int risky = ((W[s] + B) & 0x3fffffu) < 2 * B;
            if (!(risky || edge[s])) continue;
            ne++;
            const uint32_t a = F[s] < 0 ? -(uint32_t)F[s] : (uint32_t)F[s];
            const int bad = a > B;
            nbad_e += bad;
            blk_bad |= bad;
            if (++in_blk == 512) {
                blocks++;
                bad_blocks += blk_bad;
                in_blk = 0;
                blk_bad = 0;
            }
        }
        printf("B = 2^%.2f: entries %ld (%.1f %%), entries with |f| > B %ld, 512-entry blocks %ld, failing %ld (%.2f %%)\n",
               lb, ne, 100.0 * ne / m, nbad_e, blocks, bad_blocks, 100.0 * bad_blocks / blocks);
    }
    return 0;
}
