// Microbenchmark of the PLL walker's repair loop on gfx950: every lane of every
// lane-block is an event (W = 0), so each lane-block runs 64 dependent repairs.
// Reports device cycles (s_memtime) per repair for loop variants.
//   hipcc --offload-arch=gfx950 -O3 walk_loop.hip -o walk_loop && ./walk_loop
// V10 is the product loop since round 4 (k_pll.hip WX_REP); V8 the round-3 one.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t rl(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }
__device__ __forceinline__ uint32_t sel_lane(uint32_t a, uint32_t b, unsigned long long bit)
{
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(bit));
    return r;
}
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t s, uint32_t v)
{
    uint32_t r;
    asm volatile("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(s), "v"(v));
    return r;
}

template <int V>
__global__ void __launch_bounds__(64) k_loop(const uint4* E, uint32_t* out, int nlb, unsigned long long* clk)
{
    const int lane = threadIdx.x;
    const uint4 e = E[lane];
    uint32_t x = e.x, W = 0, sx = e.w & 0xffff, d1 = e.y & 0xfff, d2 = e.z;
    uint32_t Kb = 0, D = 0, xpost = 0, acc = 0;
    unsigned long long PM = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < nlb; b++) {
        unsigned long long mask = __builtin_amdgcn_ballot_w64(x + b > W);
        if (V == 0) {            // the walker's loop
            do {
                const int j = __builtin_ctzll(mask);
                const uint32_t dk1 = rl(d1, j), dk2p = rl(d2, j);
                const unsigned long long bit = 1ull << j;
                PM |= bit;
                x = mad24(sx, dk1, x) + dk2p;
                xpost = sel_lane(xpost, x, bit);
                D += dk1;
                Kb += dk2p;
                mask = __builtin_amdgcn_ballot_w64(x > W) & ((~0ull << j) << 1);
            } while (mask != 0);
        } else if (V == 1) {     // minimal chain: no snapshot, no accumulators
            do {
                const int j = __builtin_ctzll(mask);
                const uint32_t dk1 = rl(d1, j), dk2p = rl(d2, j);
                x = mad24(sx, dk1, x) + dk2p;
                mask = __builtin_amdgcn_ballot_w64(x > W) & ((~0ull << j) << 1);
            } while (mask != 0);
        } else if (V == 2) {     // no readlane: scalar operands from ff1 only
            do {
                const int j = __builtin_ctzll(mask);
                x = mad24(sx, (uint32_t)j, x) + (uint32_t)j;
                mask = __builtin_amdgcn_ballot_w64(x > W) & ((~0ull << j) << 1);
            } while (mask != 0);
        } else if (V == 4) {     // readlane results copied through the SALU before the VALU uses them
            do {
                const int j = __builtin_ctzll(mask);
                uint32_t dk1, dk2p;
                asm volatile("v_readlane_b32 %0, %2, %4\n\tv_readlane_b32 %1, %3, %4\n\ts_mov_b32 %0, %0\n\ts_mov_b32 %1, %1"
                             : "=&s"(dk1), "=&s"(dk2p) : "v"(d1), "v"(d2), "s"(j));
                x = mad24(sx, dk1, x) + dk2p;
                mask = __builtin_amdgcn_ballot_w64(x > W) & ((~0ull << j) << 1);
            } while (mask != 0);
        } else if (V == 5) {     // LDS broadcast of lane j's values into VGPRs (no SGPR hop)
            __shared__ uint2 tabd[64];
            tabd[lane] = make_uint2(d1, d2);
            do {
                const int j = __builtin_ctzll(mask);
                const uint2 dd = tabd[j];
                x = x + sx * dd.x + dd.y;
                mask = __builtin_amdgcn_ballot_w64(x > W) & ((~0ull << j) << 1);
            } while (mask != 0);
        } else if (V == 6) {     // ds_bpermute broadcast of lane j's values into VGPRs
            do {
                const int j = __builtin_ctzll(mask);
                const int a = j << 2;
                const uint32_t b1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)d1);
                const uint32_t b2 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)d2);
                x = x + sx * b1 + b2;
                mask = __builtin_amdgcn_ballot_w64(x > W) & ((~0ull << j) << 1);
            } while (mask != 0);
        } else if (V == 7 || V == 8) {   // the production asm loop (k_pll.hip walk_lb24), rolled / unrolled x4
            uint32_t xn = x ^ 5u, j, dk1, dk2;
            unsigned long long bit, above;
#define WL_BODY \
    "s_ff1_i32_b64 %[j], %[mask]\n\t" \
    "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t" \
    "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t" \
    "s_lshl_b64 %[bit], 1, %[j]\n\t" \
    "s_lshl_b64 %[above], -2, %[j]\n\t" \
    "s_or_b64 %[pm], %[pm], %[bit]\n\t" \
    "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t" \
    "v_add_u32 %[x], %[dk2], %[x]\n\t" \
    "s_add_u32 %[kb], %[kb], %[dk2]\n\t" \
    "s_add_u32 %[d], %[d], %[dk1]\n\t" \
    "v_cmp_gt_u32_e64 %[mask], %[x], %[w]\n\t" \
    "v_cndmask_b32_e64 %[xp], %[xp], %[x], %[bit]\n\t" \
    "v_mad_i32_i24 %[xn], %[sx], %[dk1], %[xn]\n\t" \
    "v_add_u32 %[xn], %[dk2], %[xn]\n\t" \
    "s_and_b64 %[mask], %[mask], %[above]\n\t"
#define WL_OPS \
    : [x] "+v"(x), [xn] "+v"(xn), [xp] "+v"(xpost), [mask] "+s"(mask), [pm] "+s"(PM), [kb] "+s"(Kb), [d] "+s"(D), \
      [j] "=&s"(j), [dk1] "=&s"(dk1), [dk2] "=&s"(dk2), [bit] "=&s"(bit), [above] "=&s"(above) \
    : [e1x] "v"(d1), [e1y] "v"(d2), [sx] "v"(sx), [w] "v"(W) : "scc"
            if (V == 7)
                asm volatile("1:\n\t" WL_BODY "s_cbranch_scc1 1b" WL_OPS);
            else
                asm volatile("1:\n\t" WL_BODY "s_cbranch_scc0 2f\n\t" WL_BODY "s_cbranch_scc0 2f\n\t" WL_BODY
                             "s_cbranch_scc0 2f\n\t" WL_BODY "s_cbranch_scc1 1b\n2:" WL_OPS);
            acc += xn;
        } else if (V == 9 || V == 10) {   // exec-masked chain: the update runs only in the lanes
            // above j (s_lshl exec), so the v_cmp's VCC is already "events after j": no s_and,
            // the loop branches on VCCZ; no per-repair snapshot / PM (derived after the loop:
            // the repaired lanes are those whose x is still > W, x holding their pre-repair offset)
            uint32_t j, dk1, dk2;
#define WX_BODY \
    "s_ff1_i32_b64 %[j], vcc\n\t" \
    "s_lshl_b64 exec, -2, %[j]\n\t" \
    "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t" \
    "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t" \
    "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t" \
    "v_add_u32 %[x], %[dk2], %[x]\n\t" \
    "s_add_u32 %[kb], %[kb], %[dk2]\n\t" \
    "s_add_u32 %[d], %[d], %[dk1]\n\t" \
    "v_cmp_gt_u32_e32 vcc, %[x], %[w]\n\t"
#define WX_OPS \
    : [x] "+v"(x), [kb] "+s"(Kb), [d] "+s"(D), [j] "=&s"(j), [dk1] "=&s"(dk1), [dk2] "=&s"(dk2) \
    : [e1x] "v"(d1), [e1y] "v"(d2), [sx] "v"(sx), [w] "v"(W), [b] "s"(b) : "scc", "vcc", "exec"
            if (V == 9)
                asm volatile("v_add_u32 %[x], %[b], %[x]\n\tv_cmp_gt_u32_e32 vcc, %[x], %[w]\n\t"
                             "s_cbranch_vccz 2f\n1:\n\t" WX_BODY "s_cbranch_vccnz 1b\n2:\n\ts_mov_b64 exec, -1" WX_OPS);
            else
                asm volatile("v_add_u32 %[x], %[b], %[x]\n\tv_cmp_gt_u32_e32 vcc, %[x], %[w]\n\t"
                             "s_cbranch_vccz 2f\n1:\n\t" WX_BODY "s_cbranch_vccz 2f\n\t" WX_BODY "s_cbranch_vccz 2f\n\t"
                             WX_BODY "s_cbranch_vccz 2f\n\t" WX_BODY "s_cbranch_vccnz 1b\n2:\n\ts_mov_b64 exec, -1" WX_OPS);
            acc += x;
            x = e.x;             // every lane an event again in the next lane-block
            continue;
        } else if (V == 11) {    // exec = the events (v_cmpx): lane j's values by readfirstlane,
            // off the s_ff1; exec = the lanes above j (s_ff1 exec, s_lshl) for the update
            uint32_t j, dk1, dk2;
#define WF_BODY \
    "v_readfirstlane_b32 %[dk1], %[e1x]\n\t" \
    "v_readfirstlane_b32 %[dk2], %[e1y]\n\t" \
    "s_ff1_i32_b64 %[j], exec\n\t" \
    "s_lshl_b64 exec, -2, %[j]\n\t" \
    "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t" \
    "v_add_u32 %[x], %[dk2], %[x]\n\t" \
    "s_add_u32 %[kb], %[kb], %[dk2]\n\t" \
    "s_add_u32 %[d], %[d], %[dk1]\n\t" \
    "v_cmpx_gt_u32_e32 vcc, %[x], %[w]\n\t"
            asm volatile("v_add_u32 %[x], %[b], %[x]\n\tv_cmpx_gt_u32_e32 vcc, %[x], %[w]\n\t"
                         "s_cbranch_execz 2f\n1:\n\t" WF_BODY "s_cbranch_execz 2f\n\t" WF_BODY "s_cbranch_execz 2f\n\t"
                         WF_BODY "s_cbranch_execz 2f\n\t" WF_BODY "s_cbranch_execnz 1b\n2:\n\ts_mov_b64 exec, -1" WX_OPS);
            acc += x;
            x = e.x;
            continue;
        } else if (V == 3) {     // pure SALU loop over the mask (no ballot per step)
            do {
                const int j = __builtin_ctzll(mask);
                const uint32_t dk1 = rl(d1, j), dk2p = rl(d2, j);
                x = mad24(sx, dk1, x) + dk2p;
                mask &= mask - 1;
            } while (mask != 0);
        }
        acc += x;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc + xpost + Kb + D + (uint32_t)PM;
    if (lane == 0) *clk = t1 - t0;
}

int main()
{
    uint4 h[64];
    for (int i = 0; i < 64; i++) h[i] = make_uint4(1000u + 17u * i, 3u + i, 7u * i, i);
    uint4* dE;
    uint32_t* dout;
    unsigned long long* dclk;
    hipMalloc(&dE, sizeof(h));
    hipMalloc(&dout, 256);
    hipMalloc(&dclk, 8);
    hipMemcpy(dE, h, sizeof(h), hipMemcpyHostToDevice);
    const int nlb = 2000;
    auto run = [&](auto kern, const char* name) {
        for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dE, dout, nlb, dclk);
        hipDeviceSynchronize();
        unsigned long long c = 0;
        hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost);
        printf("%-40s %8.1f memtime ticks per repair (x %d repairs)\n", name, (double)c / (64.0 * nlb), 64 * nlb);
    };
    run(k_loop<0>, "V0 walker loop");
    run(k_loop<1>, "V1 minimal chain");
    run(k_loop<2>, "V2 no readlane");
    run(k_loop<3>, "V3 no ballot (SALU mask walk)");
    run(k_loop<4>, "V4 readlane + s_mov");
    run(k_loop<5>, "V5 LDS broadcast");
    run(k_loop<6>, "V6 ds_bpermute broadcast");
    run(k_loop<7>, "V7 production asm, rolled");
    run(k_loop<8>, "V8 production asm, unrolled x4");
    run(k_loop<9>, "V9 exec-masked, VCC branch, rolled");
    run(k_loop<10>, "V10 exec-masked, VCC branch, unrolled x4");
    uint32_t o10[64], o11[64];
    hipMemcpy(o10, dout, 256, hipMemcpyDeviceToHost);
    run(k_loop<11>, "V11 v_cmpx + readfirstlane, unrolled x4");
    hipMemcpy(o11, dout, 256, hipMemcpyDeviceToHost);
    int same = 1;
    for (int i = 0; i < 64; i++) same &= o10[i] == o11[i];
    printf("V11 results %s V10's\n", same ? "equal" : "DIFFER FROM");
    // s_memtime frequency: compare against wall clock
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_loop<8>, dim3(1), dim3(64), 0, 0, dE, dout, nlb * 10, dclk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long c = 0;
    hipMemcpy(&c, dclk, 8, hipMemcpyDeviceToHost);
    printf("V8 x10: %.3f ms wall, %llu ticks -> %.1f MHz memtime; %.2f ns per repair\n", ms, c, c / (ms * 1e3),
           ms * 1e6 / (64.0 * nlb * 10));
    return 0;
}
