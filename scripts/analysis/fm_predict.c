#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
#include "../../oracle/ora_math.h"
static float tab[1024];
static uint32_t C_(float th) { float p = th * 0.159154943091895; float fp = p - ((long)p); if (fp < 0.) fp += 1.; return (uint32_t)(int64_t)(fp * 0xffffffff); }
typedef struct { uint32_t th, d; float pe; } St;
static const float al = 0.1f; static float be;
static inline uint32_t idxof(uint32_t th) { return ((th + (1u << 21)) >> 22) & 0x3ff; }
static inline void step(St* q, float s) {
  uint32_t i = idxof(q->th); float sn = tab[i], c = tab[(i + 256) & 1023];
  float r1 = s * c - 0.0f * (-sn), i1 = s * (-sn) + 0.0f * c;
  q->pe = 0.999 * q->pe + 0.001 * om_atan2f(i1, r1);
  q->d += C_(q->pe * al); q->th += C_(q->pe * be); q->th += q->d;
}
static int cd(uint32_t a, uint32_t b) { int d = (int)((a - b) & 1023); if (d >= 512) d -= 1024; return d; }
int main(int argc, char** argv) {
  be = sqrtf(al);
  for (int i = 0; i < 1024; i++) tab[i] = sinf(2.0f * M_PI * (float)(i) / 1024.0f);
  FILE* f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long n = ftell(f) / 4; fseek(f, 0, SEEK_SET);
  float* s = malloc(n * 4); if (fread(s, 4, n, f) != (size_t)n) return 1; fclose(f);
  St* T = malloc((n + 1) * sizeof(St)); St q = {0, 0, 0.0f};
  for (long i = 0; i < n; i++) { T[i] = q; step(&q, s[i]); }
  T[n] = q;
  /* one-step and k-step linear prediction from the state */
  for (int k = 1; k <= 8; k *= 2) {
    int h[32] = {0}; long far = 0;
    for (long i = 1000; i + k < n; i++) {
      uint32_t inc = T[i].d + C_(T[i].pe * al) + C_(T[i].pe * be);   /* next increment with pe as is */
      uint32_t p = T[i].th + (uint32_t)k * inc;
      int dd = cd(idxof(p), idxof(T[i + k].th)); if (dd < -15 || dd > 15) far++; else h[dd + 16]++;
    }
    printf("k=%d pred err:", k); for (int j = 0; j < 32; j++) if (h[j]) printf(" %d:%d", j - 16, h[j]); printf(" far:%ld\n", far);
  }
  /* candidates from a cold guess W samples early: idx diff over the chunk */
  int W = atoi(argv[2]);
  long hist[64] = {0}, far = 0, tot = 0;
  for (long s0 = W + 1000; s0 + 4096 < n; s0 += 4096) {
    St c = {0, T[s0 - W].d, 0.0f}; /* phase unknown, freq known */
    c.d = (uint32_t)(19000.0 / 600000.0 * 4294967296.0);
    for (long i = s0 - W; i < s0; i++) step(&c, s[i]);
    for (long i = s0; i < s0 + 4096; i++) { int dd = cd(idxof(c.th), idxof(T[i].th)); if (dd < -31 || dd > 31) far++; else hist[dd + 32]++; tot++; step(&c, s[i]); }
  }
  printf("cold W=%d:", W); for (int j = 0; j < 64; j++) if (hist[j]) printf(" %d:%ld", j - 32, hist[j]); printf(" far:%ld of %ld\n", far, tot);
}
