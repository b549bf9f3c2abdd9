// Microbenchmark: cycles per sample of the exact DF-II section recursion
//   v0 = (u - a1 p1) - a2 p2          (three dependent float32 ops per sample)
// run by one lane of one wave, for the section-per-wave exact IIR (round 6).
//   R1  registers only, one chain
//   R2  input from / v0 to LDS, ds_read_b128 / ds_write_b128 per 4 samples (lane 0 exec)
//   R3  two independent chains interleaved in one wave (registers)
//   R4  R2 in 4 waves of one workgroup at once (one per SIMD)
//   R5  R2 in 8 waves (two per SIMD)
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off iir_rec.hip -o iir_rec && ./iir_rec
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int T = 256;   // samples per tile

template <int V>
__global__ void __launch_bounds__(512) k_rec(const float* x, float* out, int reps, unsigned long long* clk, float a1,
                                             float a2)
{
    __shared__ __attribute__((aligned(16))) float uin[8][T];
    __shared__ __attribute__((aligned(16))) float vout[8][T];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = lane; i < T; i += 64) uin[w][i] = x[i];
    __syncthreads();
    float p1 = 0.f, p2 = 0.f, q1 = 0.f, q2 = 0.f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (V == 1 || V == 3 || V == 9 || ((V == 10 || V == 11) && (V == 10 ? lane == 0 : lane < 32))) {
        float u0 = x[lane], u1 = x[lane + 1], u2 = x[lane + 2], u3 = x[lane + 3];
        for (int r = 0; r < reps * (T / 4); r++) {
#define STEP(u) { const float v = (u - a1 * p1) - a2 * p2; p2 = p1; p1 = v; }
#define STEPQ(u) { const float v = (u - a1 * q1) - a2 * q2; q2 = q1; q1 = v; }
            STEP(u0); if (V == 3) STEPQ(u0);
            STEP(u1); if (V == 3) STEPQ(u1);
            STEP(u2); if (V == 3) STEPQ(u2);
            STEP(u3); if (V == 3) STEPQ(u3);
            asm volatile("" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3));
        }
    } else if (V >= 6) {
        if (lane == 0) {
            const float4* ip = reinterpret_cast<const float4*>(uin[w]);
            float4* op = reinterpret_cast<float4*>(vout[w]);
            for (int r = 0; r < reps; r++) {
                float4 n0 = ip[0], n1 = ip[1], n2 = ip[2], n3 = ip[3];
                for (int g = 0; g < T / 16; g++) {
                    const float4 u[4] = {n0, n1, n2, n3};
                    const int gn = ((g + 1) & (T / 16 - 1)) * 4;
                    n0 = ip[gn]; n1 = ip[gn + 1]; n2 = ip[gn + 2]; n3 = ip[gn + 3];
                    float4 v[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        v[k].x = (u[k].x - a1 * p1) - a2 * p2;
                        v[k].y = (u[k].y - a1 * v[k].x) - a2 * p1;
                        v[k].z = (u[k].z - a1 * v[k].y) - a2 * v[k].x;
                        v[k].w = (u[k].w - a1 * v[k].z) - a2 * v[k].y;
                        p2 = v[k].z;
                        p1 = v[k].w;
                    }
#pragma unroll
                    for (int k = 0; k < 4; k++) op[g * 4 + k] = v[k];
                }
            }
        }
    } else if (lane == 0) {
        if (V == 2 && w != 0) return;
        (void)0;
        for (int r = 0; r < reps; r++) {
            const float4* ip = reinterpret_cast<const float4*>(uin[w]);
            float4* op = reinterpret_cast<float4*>(vout[w]);
            float4 n = ip[0];
#pragma unroll 4
            for (int g = 0; g < T / 4; g++) {
                const float4 u = n;
                n = ip[(g + 1) & (T / 4 - 1)];
                float4 v;
                v.x = (u.x - a1 * p1) - a2 * p2;
                v.y = (u.y - a1 * v.x) - a2 * p1;
                v.z = (u.z - a1 * v.y) - a2 * v.x;
                v.w = (u.w - a1 * v.z) - a2 * v.y;
                p2 = v.z;
                p1 = v.w;
                op[g] = v;
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = p1 + p2 + q1 + q2 + vout[w][lane];
    if (lane == 0) { clk[w] = t1 - t0; clk[8 + w] = __builtin_amdgcn_s_getreg(63492); }
}

int main()
{
    float h[T + 64];
    for (int i = 0; i < T + 64; i++) h[i] = 0.001f * (i % 17) - 0.008f;
    float *din, *dout;
    unsigned long long* dclk;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 4096);
    hipMalloc(&dclk, 128);
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const int reps = 4000;
    const double n = (double)reps * T;
    auto run = [&](auto kern, const char* name, int threads) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, din, dout, reps, dclk, 1.9f, -0.93f);
            hipEventRecord(e1);
        }
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c[16] = {};
        hipMemcpy(c, dclk, 128, hipMemcpyDeviceToHost);
        printf("%-44s %6.2f clk/sample (wave0)  %6.2f clk (wave%d)  %7.1f MS/s per chain (event %.3f ms)\n", name,
               c[0] / n, c[threads / 64 - 1] / n, threads / 64 - 1, n / (ms * 1e3), ms);
        printf("    simd ids:");
        for (int i = 0; i < threads / 64; i++) printf(" w%d:simd%llu/wid%llu/cu%llu", i, (c[8 + i] >> 4) & 3, c[8 + i] & 15, (c[8 + i] >> 8) & 15);
        printf("\n");
    };
    run(k_rec<1>, "R1 registers, one chain", 64);
    run(k_rec<10>, "R10 registers, one chain, exec = lane 0", 64);
    run(k_rec<11>, "R11 registers, one chain, exec = lanes 0-31", 64);
    run(k_rec<1>, "R1 again", 64);
    run(k_rec<3>, "R3 registers, two chains interleaved", 64);
    run(k_rec<2>, "R2 LDS in/out, lane 0", 64);
    run(k_rec<4>, "R4 LDS in/out, 4 waves", 256);
    run(k_rec<5>, "R5 LDS in/out, 8 waves", 512);
    run(k_rec<6>, "R6 LDS 16-sample groups, 1 wave", 64);
    run(k_rec<7>, "R7 LDS 16-sample groups, 4 waves", 256);
    run(k_rec<8>, "R8 LDS 16-sample groups, 8 waves", 512);
    run(k_rec<9>, "R9 registers, one chain, 4 waves", 256);
    run(k_rec<6>, "R6 again", 64);
    run(k_rec<7>, "R7 again (4 waves)", 256);
    run(k_rec<7>, "R7 2 waves", 128);
    run(k_rec<9>, "R9 registers, 2 waves", 128);
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_rec<6>, dim3(4), dim3(64), 0, 0, din, dout, reps, dclk, 1.9f, -0.93f);
        hipEventRecord(e1);
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("R6 x 4 workgroups: %.3f ms (%.1f MS/s per chain)\n", ms, n / (ms * 1e3));
    }
    return 0;
}
