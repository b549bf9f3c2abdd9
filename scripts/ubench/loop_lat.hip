// Latency of the pieces of the serial loops on gfx950 (one wave, one dependent
// chain): the AGC step (exact and approximate), its logf / expf / float64
// smoothing, an IEEE float division, atan2, constrain, and the FMStereo step.
// Each variant runs N dependent iterations; ns per iteration from HIP events.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../python-liquiddsp_amd/csrc loop_lat.hip -o loop_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "ldsp_math.hpp"

using namespace ldsp;

template <int V>
__global__ void __launch_bounds__(64) k_lat(const float* __restrict__ xin, const float* __restrict__ tabg, long N,
                                            float* out)
{
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) tab[i] = tabg[i];
    __syncthreads();
    float xs[8];
#pragma unroll
    for (int j = 0; j < 8; j++) xs[j] = xin[j];
    float y = xin[8 + threadIdx.x % 4] * 0.001f + 1.0f, g = 1.3f, y2p = 1.0f;
    uint32_t th = 12345u * threadIdx.x, d = 77777u;
    float pe = 0.01f;
    const float alpha = 0.01f, beta = 0.1f;
    for (long i = 0; i < N; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float x = xs[j];
            if (V == 0) {               // AGC exact step (agc_step without squelch / outputs)
                const float a = x * g, b = x * 0.5f * g;
                const float y2 = a * a - b * (-b);
                y2p = (float)((1.0 - (double)alpha) * (double)y2p + (double)(alpha * y2));
                if (y2p > 1e-6f) g *= lm_expf(-0.5f * alpha * lm_logf(y2p));
                g = g > 1e6f ? 1e6f : g;
            } else if (V == 1) {        // AGC approximate step
                const float a = x * g, b = x * 0.5f * g;
                const float y2 = a * a - b * (-b);
                y2p = (float)((1.0 - (double)alpha) * (double)y2p + (double)(alpha * y2));
                if (y2p > 1e-6f) {
                    const float t = -0.5f * alpha * (__builtin_amdgcn_logf(y2p) * 0.69314718056f);
                    const float u = t * (1.0f + t * (0.5f + t * (0.16666667f + t * 0.041666668f)));
                    g *= 1.0f + u;
                }
                g = g > 1e6f ? 1e6f : g;
            } else if (V == 2) {        // lm_logf chain
                y = lm_logf(y) + 1.25f;
            } else if (V == 3) {        // lm_expf chain
                y = lm_expf(y * -0.01f) + 0.25f;
            } else if (V == 4) {        // the float64 smoothing
                y = (float)((1.0 - (double)alpha) * (double)y + (double)(alpha * x));
            } else if (V == 5) {        // IEEE float division
                y = y / (2.0f + y);
            } else if (V == 6) {        // lm_atan2f
                y = lm_atan2f(y, x + 1.5f);
            } else if (V == 7) {        // lm_constrain (the PLL's C())
                const uint32_t u = lm_constrain(y);
                y = (float)(u >> 12) * 2.4e-7f + 0.01f;
            } else if (V == 8) {        // baseline: one dependent mul + add
                y = y * 0.999f + 0.001f;
            } else if (V == 9) {        // FMStereo step (k_fm_pll)
                const uint32_t idx = ((th + (1u << 21)) >> 22) & 0x3ffu;
                const float sn = tab[idx], cs = tab[(idx + 256) & 0x3ffu];
                const float r1 = x * cs - 0.0f * (-sn);
                const float i1 = x * (-sn) + 0.0f * cs;
                pe = (float)(0.999 * (double)pe + 0.001 * (double)lm_atan2f(i1, r1));
                d += lm_constrain(pe * 0.1f);
                th += lm_constrain(pe * 0.31622776f);
                th += d;
            } else if (V == 11) {       // AGC exact step through the fast paths
                const float a = x * g, b = x * 0.5f * g;
                const float y2 = a * a - b * (-b);
                y2p = (float)((1.0 - (double)alpha) * (double)y2p + (double)(alpha * y2));
                if (y2p > 1e-6f) g *= lm_expf_loop(-0.5f * alpha * lm_logf_loop(y2p));
                g = g > 1e6f ? 1e6f : g;
            } else if (V == 10) {       // LDS table read chain
                const uint32_t idx = ((th + (1u << 21)) >> 22) & 0x3ffu;
                th += __float_as_uint(tab[idx]) | 1u;
            }
        }
    }
    out[threadIdx.x] = y + g + y2p + pe + (float)th;
}

int main()
{
    float hx[16], ht[1024];
    for (int i = 0; i < 16; i++) hx[i] = 0.7f + 0.05f * (float)(i % 7);
    for (int i = 0; i < 1024; i++) ht[i] = sinf(6.283185307f * i / 1024.0f);
    float *dx, *dt, *dout;
    hipMalloc(&dx, sizeof(hx));
    hipMalloc(&dt, sizeof(ht));
    hipMalloc(&dout, 64 * sizeof(float));
    hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
    hipMemcpy(dt, ht, sizeof(ht), hipMemcpyHostToDevice);
    const long N = 1 << 18;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"agc exact step", "agc approx step", "lm_logf", "lm_expf", "f64 smoothing",
                           "float division", "lm_atan2f", "lm_constrain + 3 ops", "mul + add", "fmstereo step",
                           "lds table read + add", "agc exact step (fast)"};
    void (*ks[])(const float*, const float*, long, float*) = {k_lat<0>, k_lat<1>, k_lat<2>, k_lat<3>, k_lat<4>, k_lat<5>,
                                                              k_lat<6>, k_lat<7>, k_lat<8>, k_lat<9>, k_lat<10>,
                                                              k_lat<11>};
    for (int v = 0; v < 12; v++) {
        hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, dx, dt, 1024, dout);   // warm
        hipEventRecord(e0);
        hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, dx, dt, N, dout);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-24s %8.2f ns per iteration\n", names[v], ms * 1e6 / N);
    }
    return 0;
}
