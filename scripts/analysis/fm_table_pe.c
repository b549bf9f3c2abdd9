#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
#include "../../oracle/ora_math.h"
static float tab[1024], Tp[1024], Tm[1024];
static uint32_t C_(float th) { float p = th * 0.159154943091895; float fp = p - ((long)p); if (fp < 0.) fp += 1.; return (uint32_t)(int64_t)(fp * 0xffffffff); }
static inline uint32_t idxof(uint32_t th) { return ((th + (1u << 21)) >> 22) & 0x3ff; }
int main(int argc, char** argv) {
  float al = 0.1f, be = sqrtf(al);
  for (int i = 0; i < 1024; i++) tab[i] = sinf(2.0f * M_PI * (float)(i) / 1024.0f);
  for (int i = 0; i < 1024; i++) { float sn = tab[i], c = tab[(i + 256) & 1023]; Tp[i] = om_atan2f(-sn, c); Tm[i] = om_atan2f(sn, -c); }
  FILE* f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long n = ftell(f) / 4; fseek(f, 0, SEEK_SET);
  float* s = malloc(n * 4); if (fread(s, 4, n, f) != (size_t)n) return 1; fclose(f);
  uint32_t th = 0, d = 0; float pe = 0; long amis = 0, pmis = 0, zero = 0;
  for (long k = 0; k < n; k++) {
    uint32_t i = idxof(th); float sn = tab[i], c = tab[(i + 256) & 1023], x = s[k];
    float r1 = x * c - 0.0f * (-sn), i1 = x * (-sn) + 0.0f * c;
    float a = om_atan2f(i1, r1);
    float t = x > 0 ? Tp[i] : (x < 0 ? Tm[i] : a); if (x == 0) zero++;
    float pe2 = 0.999 * pe + 0.001 * t;
    pe = 0.999 * pe + 0.001 * a;
    if (om_bits(a) != om_bits(t)) amis++;
    if (om_bits(pe) != om_bits(pe2)) pmis++;
    d += C_(pe * al); th += C_(pe * be); th += d;
  }
  printf("n=%ld atan2 table mismatch %.4g, pe mismatch %.4g (%ld), s==0: %ld\n", n, (double)amis / n, (double)pmis / n, pmis, zero);
}
