// VALU issue rates on gfx950: wave64 v_fma_f64 / v_fma_f32 / v_pk_fma_f32 /
// v_mul_f64 throughput with 8 independent chains per lane, 8 waves per SIMD.
// Prints instructions per CU per clock-ns and the implied cycles per wave64
// instruction at the measured shader clock (s_memtime vs s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096, kChains = 8;

template <int OP>
__global__ void __launch_bounds__(256) k_rate(float* out, long long* clk, float seed)
{
    long long t0 = __builtin_amdgcn_s_memtime();
    long long r0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (OP == 0) {          // f64 fma
        double a[kChains];
        for (int i = 0; i < kChains; i++) a[i] = seed + threadIdx.x + i;
        const double b = 0.999999, c = 1e-9;
        for (int it = 0; it < kIters; it++)
#pragma unroll
            for (int i = 0; i < kChains; i++) a[i] = __builtin_fma(a[i], b, c);
        double s = 0;
        for (int i = 0; i < kChains; i++) s += a[i];
        out[blockIdx.x * 256 + threadIdx.x] = (float)s;
    } else if constexpr (OP == 1) {   // f32 fma
        float a[kChains];
        for (int i = 0; i < kChains; i++) a[i] = seed + threadIdx.x + i;
        const float b = 0.999999f, c = 1e-9f;
        for (int it = 0; it < kIters; it++)
#pragma unroll
            for (int i = 0; i < kChains; i++) a[i] = __builtin_fmaf(a[i], b, c);
        float s = 0;
        for (int i = 0; i < kChains; i++) s += a[i];
        out[blockIdx.x * 256 + threadIdx.x] = s;
    } else if constexpr (OP == 2) {   // f64 mul
        double a[kChains];
        for (int i = 0; i < kChains; i++) a[i] = seed + threadIdx.x + i;
        const double b = 0.999999;
        for (int it = 0; it < kIters; it++)
#pragma unroll
            for (int i = 0; i < kChains; i++) a[i] = a[i] * b;
        double s = 0;
        for (int i = 0; i < kChains; i++) s += a[i];
        out[blockIdx.x * 256 + threadIdx.x] = (float)s;
    } else {                          // packed f32 fma (2 per instruction)
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 a[kChains];
        for (int i = 0; i < kChains; i++) a[i] = f2{seed + threadIdx.x + i, seed - i};
        const f2 b = {0.999999f, 0.999998f}, c = {1e-9f, 2e-9f};
        for (int it = 0; it < kIters; it++)
#pragma unroll
            for (int i = 0; i < kChains; i++) a[i] = __builtin_elementwise_fma(a[i], b, c);
        float s = 0;
        for (int i = 0; i < kChains; i++) s += a[i].x + a[i].y;
        out[blockIdx.x * 256 + threadIdx.x] = s;
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int OP>
static void run(const char* name, int cus)
{
    float* out;
    long long* clk;
    const int blocks = cus * 8;           // 8 waves per SIMD: 8 x 256-thread blocks per CU
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k_rate<OP><<<blocks, 256>>>(out, clk, 1.0f);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; r++) k_rate<OP><<<blocks, 256>>>(out, clk, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c[2];
    hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] * 10.0);   // memrealtime at 100 MHz
    const double insts = (double)reps * blocks * 4 * kIters * kChains;   // wave64 instructions
    const double per_ns = insts / (ms * 1e6);
    const double per_simd_clk = per_ns / (cus * 4) / ghz;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"shader_GHz\": %.3f, \"wave_insts_per_simd_per_clk\": %.4f, "
           "\"cycles_per_wave64_inst\": %.2f}\n",
           name, ms / reps, ghz, per_simd_clk, 1.0 / per_simd_clk);
    hipFree(out);
    hipFree(clk);
}

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d}\n", p.gcnArchName, cus);
    run<0>("v_fma_f64", cus);
    run<1>("v_fma_f32", cus);
    run<2>("v_mul_f64", cus);
    run<3>("v_pk_fma_f32", cus);
    return 0;
}
