// Latency of the dependency hops in the PLL walker's repair chain on gfx950, one
// wave, shader clocks (s_memtime) per loop iteration:
//   C0  s_ff1 -> s_add (SALU -> SALU)
//   C1  s_ff1 -> v_add (SGPR operand) -> v_cmp -> s_and        (SALU -> VALU -> SALU)
//   C2  s_ff1 -> v_readlane (lane select) -> s_and             (SALU -> readlane -> SALU)
//   C3  s_ff1 -> v_readlane -> v_add (SGPR operand) -> v_cmp -> s_and
//   C4  C3 with two readlanes and the walker's mad + add
//   C5  v_add -> v_add (VALU -> VALU, dependent)
//   C6  v_cmp -> s_cmp (VALU -> SALU via SCC) -> s_cbranch
//   C7  s_ff1 -> s_lshl -> v_cndmask (SGPR mask operand) -> v_cmp -> s_and
//   hipcc --offload-arch=gfx950 -O3 chain_lat.hip -o chain_lat && ./chain_lat
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int V>
__global__ void __launch_bounds__(64) k_chain(const uint32_t* in, uint32_t* out, int iters, unsigned long long* clk)
{
    const int lane = threadIdx.x;
    uint32_t x = in[lane], w = 0, v2 = in[lane] * 3u + 1u;
    unsigned long long mask = ~0ull, above = ~0ull;
    uint32_t j = 0, s1 = 0, s2 = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if (V == 0) {
            asm volatile("s_ff1_i32_b64 %[j], %[m]\n\ts_add_u32 %[j], %[j], 1\n\ts_lshl_b64 %[m], %[m], 1\n\t"
                         "s_or_b64 %[m], %[m], 1"
                         : [j] "+s"(j), [m] "+s"(mask) : : "scc");
        } else if (V == 1) {
            asm volatile("s_ff1_i32_b64 %[j], %[m]\n\tv_add_u32 %[x], %[j], %[x]\n\tv_cmp_gt_u32_e64 %[m], %[x], %[w]\n\t"
                         "s_and_b64 %[m], %[m], %[a]"
                         : [j] "+s"(j), [m] "+s"(mask), [x] "+v"(x) : [w] "v"(w), [a] "s"(above) : "scc");
        } else if (V == 2) {
            asm volatile("s_ff1_i32_b64 %[j], %[m]\n\tv_readlane_b32 %[s1], %[v], %[j]\n\ts_and_b32 %[s1], %[s1], 63\n\t"
                         "s_lshl_b64 %[m], 1, %[s1]"
                         : [j] "+s"(j), [m] "+s"(mask), [s1] "+s"(s1) : [v] "v"(x) : "scc");
        } else if (V == 3) {
            asm volatile("s_ff1_i32_b64 %[j], %[m]\n\tv_readlane_b32 %[s1], %[v2], %[j]\n\tv_add_u32 %[x], %[s1], %[x]\n\t"
                         "v_cmp_gt_u32_e64 %[m], %[x], %[w]\n\ts_and_b64 %[m], %[m], %[a]"
                         : [j] "+s"(j), [m] "+s"(mask), [x] "+v"(x), [s1] "+s"(s1) : [w] "v"(w), [a] "s"(above), [v2] "v"(v2)
                         : "scc");
        } else if (V == 4) {
            asm volatile("s_ff1_i32_b64 %[j], %[m]\n\tv_readlane_b32 %[s1], %[v2], %[j]\n\tv_readlane_b32 %[s2], %[x0], %[j]\n\t"
                         "v_mad_i32_i24 %[x], %[v2], %[s1], %[x]\n\tv_add_u32 %[x], %[s2], %[x]\n\t"
                         "v_cmp_gt_u32_e64 %[m], %[x], %[w]\n\ts_and_b64 %[m], %[m], %[a]"
                         : [j] "+s"(j), [m] "+s"(mask), [x] "+v"(x), [s1] "+s"(s1), [s2] "+s"(s2)
                         : [w] "v"(w), [a] "s"(above), [v2] "v"(v2), [x0] "v"(v2 ^ 7u) : "scc");
        } else if (V == 5) {
            asm volatile("v_add_u32 %[x], %[x], %[v2]\n\tv_add_u32 %[x], %[x], %[v2]\n\tv_add_u32 %[x], %[x], %[v2]\n\t"
                         "v_add_u32 %[x], %[x], %[v2]"
                         : [x] "+v"(x) : [v2] "v"(v2));
        } else if (V == 6) {
            asm volatile("v_add_u32 %[x], %[x], %[v2]\n\tv_cmp_gt_u32_e64 %[m], %[x], %[w]\n\ts_cmp_eq_u64 %[m], 0\n\t"
                         "s_cbranch_scc1 1f\n\ts_add_u32 %[j], %[j], 1\n1:"
                         : [x] "+v"(x), [m] "+s"(mask), [j] "+s"(j) : [v2] "v"(v2), [w] "v"(w) : "scc");
        } else if (V == 7) {
            asm volatile("s_ff1_i32_b64 %[j], %[m]\n\ts_lshl_b64 %[b], 1, %[j]\n\tv_cndmask_b32_e64 %[x], %[x], %[v2], %[b]\n\t"
                         "v_cmp_gt_u32_e64 %[m], %[x], %[w]\n\ts_and_b64 %[m], %[m], %[a]"
                         : [j] "+s"(j), [m] "+s"(mask), [x] "+v"(x), [b] "+s"(above)
                         : [w] "v"(w), [a] "s"(~0ull), [v2] "v"(v2) : "scc");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = x + j + s1 + s2 + (uint32_t)mask;
    if (lane == 0) *clk = t1 - t0;
}

int main()
{
    uint32_t h[64];
    for (int i = 0; i < 64; i++) h[i] = 1000u + 17u * i;
    uint32_t *din, *dout;
    unsigned long long* dclk;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 256);
    hipMalloc(&dclk, 8);
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const int iters = 100000;
    auto run = [&](auto kern, const char* name, double per) {
        for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, din, dout, iters, dclk);
        hipDeviceSynchronize();
        unsigned long long c = 0;
        hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost);
        printf("%-58s %7.1f clocks per iteration (%g chained hops)\n", name, (double)c / iters, per);
    };
    run(k_chain<0>, "C0 s_ff1 -> s_add ; s_lshl -> s_or (SALU)", 4);
    run(k_chain<1>, "C1 s_ff1 -> v_add -> v_cmp -> s_and", 4);
    run(k_chain<2>, "C2 s_ff1 -> v_readlane -> s_and -> s_lshl", 4);
    run(k_chain<3>, "C3 s_ff1 -> v_readlane -> v_add -> v_cmp -> s_and", 5);
    run(k_chain<4>, "C4 s_ff1 -> 2 readlanes -> mad -> add -> cmp -> s_and", 6);
    run(k_chain<5>, "C5 4 dependent v_add", 4);
    run(k_chain<6>, "C6 v_add -> v_cmp -> s_cmp -> s_cbranch", 4);
    run(k_chain<7>, "C7 s_ff1 -> s_lshl -> v_cndmask -> v_cmp -> s_and", 5);
    return 0;
}
