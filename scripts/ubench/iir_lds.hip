// Microbenchmark: what the lane-0 exact-IIR recursion loop (k_iir_sect.hip) pays for
// its LDS traffic when several waves of one workgroup (one per SIMD) run it at once.
//   M0  input ds_read_b128 + output ds_write_b128 (k_iir_sect as built)
//   M1  input ds_read_b128, output kept in registers (no stores)
//   M2  input from registers, output ds_write_b128
//   M3  input ds_read_b128, output global_store_dwordx4 (one lane)
//   M4  input ds_read_b128 + output ds_write_b128, all 64 lanes active
// clk/sample per wave (s_memtime), for 1, 2 and 4 waves.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize iir_lds.hip -o iir_lds
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int T = 512;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

#define STEP(u, v)                       \
    {                                    \
        v = ((u) - a1 * p1) - a2 * p2;   \
        p2 = p1;                         \
        p1 = v;                          \
    }

template <int M>
__global__ void __launch_bounds__(256) k_lds(const float* x, float* gout, int reps, unsigned long long* clk, float a1,
                                             float a2)
{
    __shared__ __attribute__((aligned(16))) float uin[4][T];
    __shared__ __attribute__((aligned(16))) float vout[4][T];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = lane; i < T; i += 64) uin[w][i] = x[i];
    __syncthreads();
    float p1 = 0.f, p2 = 0.f, acc = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (lane == 0 || M == 4) {
        const float* src = uin[w];
        float* vo = vout[w];
        float* go = gout + 4096 + w * T;
        float4 r0 = make_float4(x[0], x[1], x[2], x[3]), r1 = r0, r2 = r0, r3 = r0;
        auto group = [&](float4 u0, float4 u1, float4 u2, float4 u3, int i) {
            float4 w0, w1, w2, w3;
            STEP(u0.x, w0.x) STEP(u0.y, w0.y) STEP(u0.z, w0.z) STEP(u0.w, w0.w)
            STEP(u1.x, w1.x) STEP(u1.y, w1.y) STEP(u1.z, w1.z) STEP(u1.w, w1.w)
            STEP(u2.x, w2.x) STEP(u2.y, w2.y) STEP(u2.z, w2.z) STEP(u2.w, w2.w)
            STEP(u3.x, w3.x) STEP(u3.y, w3.y) STEP(u3.z, w3.z) STEP(u3.w, w3.w)
            if (M == 1) {
                acc += w0.x + w1.y + w2.z + w3.w;
            } else if (M == 3) {
                st4(go + i, w0);
                st4(go + i + 4, w1);
                st4(go + i + 8, w2);
                st4(go + i + 12, w3);
            } else {
                st4(vo + i, w0);
                st4(vo + i + 4, w1);
                st4(vo + i + 8, w2);
                st4(vo + i + 12, w3);
            }
        };
        auto rd = [&](int i, float4& a, float4& b, float4& c, float4& d) {
            if (M == 2) {
                asm volatile("" : "+v"(r0.x), "+v"(r0.y), "+v"(r0.z), "+v"(r0.w));
                asm volatile("" : "+v"(r1.x), "+v"(r1.y), "+v"(r1.z), "+v"(r1.w));
                asm volatile("" : "+v"(r2.x), "+v"(r2.y), "+v"(r2.z), "+v"(r2.w));
                asm volatile("" : "+v"(r3.x), "+v"(r3.y), "+v"(r3.z), "+v"(r3.w));
                a = r0; b = r1; c = r2; d = r3;
            } else {
                a = ld4(src + i); b = ld4(src + i + 4); c = ld4(src + i + 8); d = ld4(src + i + 12);
            }
        };
        for (int r = 0; r < reps; r++) {
            float4 a0, a1v, a2v, a3, b0, b1, b2, b3;
            rd(0, a0, a1v, a2v, a3);
            rd(16, b0, b1, b2, b3);
            __builtin_amdgcn_sched_barrier(0);
            int i = 0;
            for (int pass = 0; pass < 2; pass++) {
                const int i1 = pass == 0 ? 32 : T;
                for (; i < i1; i += 32) {
                    group(a0, a1v, a2v, a3, i);
                    rd((i + 32) & (T - 1), a0, a1v, a2v, a3);
                    __builtin_amdgcn_sched_barrier(0);
                    group(b0, b1, b2, b3, i + 16);
                    rd((i + 48) & (T - 1), b0, b1, b2, b3);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    gout[threadIdx.x] = p1 + p2 + acc + vout[w][lane];
    if (lane == 0) clk[w] = t1 - t0;
}

int main()
{
    float h[T];
    for (int i = 0; i < T; i++) h[i] = 0.001f * (i % 17) - 0.008f;
    float *din, *dout;
    unsigned long long* dclk;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 65536);
    hipMalloc(&dclk, 64);
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const int reps = 2000;
    const double n = (double)reps * T;
    auto run = [&](auto kern, const char* name) {
        for (int waves : {1, 2, 4}) {
            for (int rep = 0; rep < 2; rep++)
                hipLaunchKernelGGL(kern, dim3(1), dim3(64 * waves), 0, 0, din, dout, reps, dclk, 1.9f, -0.93f);
            hipDeviceSynchronize();
            unsigned long long c[4] = {};
            hipMemcpy(c, dclk, 32, hipMemcpyDeviceToHost);
            printf("%-52s waves %d: %6.2f clk/sample (wave0) %6.2f (last)\n", name, waves, c[0] / n, c[waves - 1] / n);
        }
    };
    run(k_lds<0>, "M0 ds_read_b128 in, ds_write_b128 out (lane 0)");
    run(k_lds<1>, "M1 ds_read_b128 in, no stores");
    run(k_lds<2>, "M2 registers in, ds_write_b128 out");
    run(k_lds<3>, "M3 ds_read_b128 in, global_store_dwordx4 out");
    run(k_lds<4>, "M4 as M0, 64 lanes active");
    run(k_lds<0>, "M0 again");
    return 0;
}
