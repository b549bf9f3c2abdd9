#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include "../../oracle/ora_math.h"
static float alpha = 0.01f;
typedef struct { float g, y; } S;
static inline void ex(S* s, float xr, float xi) {
  float a = xr * s->g, b = xi * s->g; float y2 = a*a - b*(-b);
  s->y = (1.0 - alpha) * s->y + alpha * y2;
  if (s->y > 1e-6f) s->g *= om_expf(-0.5f*alpha*om_logf(s->y));
  s->g = s->g > 1e6f ? 1e6f : s->g;
}
static int amode = 0;
static inline void ap(S* s, float xr, float xi) {
  float a = xr * s->g, b = xi * s->g; float y2 = a*a - b*(-b);
  s->y = (1.0 - alpha) * s->y + alpha * y2;
  if (s->y > 1e-6f) {
    float L = amode == 0 ? log2f(s->y)*0.69314718056f : (float)log((double)s->y);
    float t = -0.5f*alpha*L;
    float F = amode == 0 ? 1.0f + t*(1.0f + t*(0.5f + t*(0.16666667f + t*0.041666668f))) : (float)exp((double)t);
    s->g *= F; }
  s->g = s->g > 1e6f ? 1e6f : s->g;
}
static int eq(S a, S b) { return om_bits(a.g) == om_bits(b.g) && om_bits(a.y) == om_bits(b.y); }
int main(int argc, char** argv) {
  int Wa = atoi(argv[1]); int W = atoi(argv[2]); amode = argc > 3 ? atoi(argv[3]) : 0; int C = 256;
  FILE* f = fopen("agc_in.c64", "rb"); fseek(f, 0, SEEK_END); long n = ftell(f) / 8; fseek(f, 0, SEEK_SET);
  float* x = malloc(n * 8); if (fread(x, 8, n, f) != (size_t)n) return 1; fclose(f);
  S* T = malloc((n + 1) * sizeof(S)); S s = {1.0f, 1.0f};
  for (long i = 0; i < n; i++) { T[i] = s; ex(&s, x[2*i], x[2*i+1]); }
  T[n] = s;
  long k0 = (Wa + W + 256 + C - 1) / C + 1, nch = n / C;
  S* st = malloc(nch * sizeof(S)); S* en = malloc(nch * sizeof(S)); char* ok = calloc(nch, 1);
  long wrong = 0;
  for (long k = k0; k < nch; k++) {
    long s0 = k * C, w0 = s0 - W, a0 = w0 - Wa;
    double pw = 0; for (long i = a0 - 256; i < a0; i++) pw += (double)x[2*i]*x[2*i] + (double)x[2*i+1]*x[2*i+1];
    pw /= 256; S r; r.g = (float)(1.0/sqrt(pw)); r.y = 1.0f;
    for (long i = a0; i < w0; i++) ap(&r, x[2*i], x[2*i+1]);
    for (long i = w0; i < s0; i++) ex(&r, x[2*i], x[2*i+1]);
    st[k] = r; ok[k] = eq(r, T[s0]); wrong += !ok[k];
    for (long i = s0; i < s0 + C; i++) ex(&r, x[2*i], x[2*i+1]);
    en[k] = r;
  }
  /* flags and one runfix round: run start = flagged with unflagged predecessor; cost = chunks rerun */
  long flagged = 0, runs = 0, maxcost = 0, tot = 0; int hist[16] = {0}; long missed = 0;
  char* fl = calloc(nch, 1);
  for (long k = k0 + 1; k < nch; k++) { fl[k] = !eq(st[k], en[k-1]); flagged += fl[k]; if (!ok[k] && !fl[k]) missed++; }
  for (long k = k0 + 1; k < nch; k++) {
    if (!fl[k] || fl[k-1]) continue;
    runs++; S r = en[k-1]; long m = k, cost = 0; int inrun = 1;
    for (; m < nch; m++) {
      if (m > k) { if (!(inrun && fl[m])) { if (fl[m]) break; inrun = 0; if (eq(st[m], r)) break; } }
      for (long i = m*C; i < m*C + C; i++) ex(&r, x[2*i], x[2*i+1]);
      cost++;
    }
    tot += cost; if (cost > maxcost) maxcost = cost; int b = 0; while ((1 << b) <= cost) b++; hist[b]++;
  }
  printf("Wa=%d W=%d amode=%d chunks=%ld wrong-start=%ld flagged=%ld undetected-by-flags=%ld runs=%ld rerun chunks=%ld max run=%ld\n",
         Wa, W, amode, nch - k0, wrong, flagged, missed, runs, tot, maxcost);
  for (int b = 0; b < 16; b++) if (hist[b]) printf("  cost<2^%d: %d\n", b, hist[b]);
}
