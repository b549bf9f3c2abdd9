// k_iir_sect.hip -- exact (float32, bit-identical) SOS cascade for gfx950, one
// wave per second-order section: the recursion of k_iir_seq (reference
// src/iirfilter.hpp:292-298 -> iirfilt_crcf_execute_block -> iirfiltsos_execute_df2,
// oracle/liquid_restate.c sos_df2) with the same operations in the same order.
//
// Per section and component the recursion is v0[m] = (u[m] - a1 v0[m-1]) - a2 v0[m-2]
// (liquid rounds each product: no fma), a chain of three dependent VALU operations
// per sample (mul -> sub -> sub: 26 shader clocks per sample on one wave,
// scripts/ubench/iir_rec.hip R1).  Everything else is taken off the wave that
// runs that chain:
//   * one workgroup per (object, component) -- real taps keep re and im independent
//     (and in a many-call, blockIdx.y = the object);
//   * wave s < L runs section s's recursion, 4 VALU per sample (the a2 product is
//     off the chain), its input read from LDS 16 samples at a time and its v0
//     written to an LDS ring 16 at a time (one ds_write_b128 per 16 samples: every
//     lane computes the same values, lane j stores quarter j mod 4);
//   * helper wave L + s (s >= 1, on section s's SIMD: a workgroup's waves w and
//     w + 4 share a SIMD) forms section s's input u = y of section s - 1 =
//     (b0 v0 + b1 v0[-1]) + b2 v0[-2] lane-parallel from section s - 1's ring, one
//     tile ahead into a double buffer, so the recursion wave never waits for it;
//   * the I/O wave (wave L, on section 0's SIMD) stages input tiles into LDS and
//     forms / stores the last section's y lane-parallel.
// Tiles move through rings of 4 tiles with LDS progress counters (LDS operations
// of a wave are performed in issue order, so a counter written after the data it
// covers is seen after it); a section runs at most two tiles ahead of its reader,
// which also reads the last two samples of the previous tile (its y taps).
#include "batch.hpp"
#include "kernels.hpp"
#include "ldsp_common.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kSR = 4;                   // tiles per ring
constexpr int kMaxS = kIirSectMaxSos;
constexpr int kSectThreads = 2 * kMaxS * 64;

struct SectArgs {
    const float* b;       // [3 nsos] (a0-normalised, liquid iirfiltsos layout)
    const float* a;       // [3 nsos]
    int nsos;
    int ncomp;            // 2: complex64 samples, component = blockIdx.x
    const float* x;
    long n;
    float* state;         // [ncomp][3 nsos]: per section v0[-1], v0[-2], v0[-3]
    float* y;
    unsigned long long* trace;   // diagnostics (ldsp_debug_iir_sect_trace) or null: per (object, component,
                                 // section wave) shader clocks waiting / -- / in the recursion, and in all
};

// Dynamic LDS, sized for the cascade (sect_lds): the counters, then the input
// ring, the sections' v0 rings and their double-buffered input tiles.  Tiles of
// T = 1024 samples while that fits the 160 KiB of a CU (up to 6 sections),
// 512 above.
struct SectCtr {
    // per section s, side by side so that its wave polls both with one ds_read_b64:
    //   io[s].x  its input tiles ready (s = 0: the I/O wave's input ring; else its helper's tiles)
    //   io[s].y  tiles of its v0 ring read by their reader (helper s + 1, or the I/O wave)
    int2 io[kMaxS];
    int prod[kMaxS];                     // tiles of section s's ring written
    int xcons;                           // tiles of the input ring read (wave 0)
    int abort;                           // a wait ran past its bound: every later wait returns at once
    int pad[6];
};
static_assert(sizeof(SectCtr) == 128, "counter block");
template <int T>
constexpr size_t sect_lds(int L)
{
    return sizeof(SectCtr) + sizeof(float) * ((size_t)kSR * T + (size_t)L * kSR * T + (size_t)(L - 1) * 2 * T);
}

__device__ __forceinline__ int ctr_load(const int* p)
{
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// Wait (the whole wave) until *p >= target.  Bounded (2 s; a safety net -- the
// waits form a chain without cycles, so they always end): past the bound the
// workgroup is marked aborted and finishes without waiting (its output is then
// wrong, but the launch always drains).  SLEEP: waves that share their SIMD with
// a recursion wave back off between polls.
constexpr unsigned long long kSectWaitTicks = 200000000ull;    // s_memrealtime, 100 MHz
template <bool SLEEP>
__device__ __forceinline__ void ctr_wait(const int* p, int target, int* abort)
{
    if (ctr_load(p) >= target) return;
    const unsigned long long t0 = wall_clock64();
    while (ctr_load(p) < target && !ctr_load(abort)) {
        if (SLEEP) __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > kSectWaitTicks) {
            __hip_atomic_store(abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
        }
    }
    asm volatile("" ::: "memory");
}
// Lane 0 publishes v after every LDS access the wave issued before it.
__device__ __forceinline__ void ctr_publish(int* p, int v, int lane)
{
    asm volatile("" ::: "memory");
    if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// One sample of the DF-II section (iirfiltsos_execute_df2's v[0] update).
#define SECT_STEP(u, v)                                   \
    {                                                     \
        v = ((u) - a1 * p1) - a2 * p2;                    \
        p3 = p2;                                          \
        p2 = p1;                                          \
        p1 = v;                                           \
    }

template <int kST>
__device__ __forceinline__ void sect_run(const SectArgs& A)
{
    constexpr int kRing = kST * kSR;     // floats per ring
    extern __shared__ __attribute__((aligned(16))) float dsh[];
    SectCtr& sh = *reinterpret_cast<SectCtr*>(dsh);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int L = A.nsos;
    float* const xring = dsh + sizeof(SectCtr) / sizeof(float);
    float* const vring0 = xring + kRing;                 // section s: vring0 + s * kRing
    float* const uscr0 = vring0 + L * kRing;             // section s >= 1, buffer j: uscr0 + ((s - 1) * 2 + j) * kST
    const int c = blockIdx.x;
    const long n = A.n;
    const int ntiles = (int)((n + kST - 1) / kST);
    float* st = A.state + (long)c * 3 * L;
    if (tid < kMaxS) {
        sh.prod[tid] = 0;
        sh.io[tid] = make_int2(0, 0);
    }
    if (tid == 0) {
        sh.xcons = 0;
        sh.abort = 0;
    }
    float p1 = 0.0f, p2 = 0.0f, p3 = 0.0f;
    if (wave < L) {
        p1 = st[3 * wave];
        p2 = st[3 * wave + 1];
        p3 = st[3 * wave + 2];
        // v0 at -1 / -2: the tail the reader of tile 0 takes its y taps from
        if (lane == 0) {
            vring0[wave * kRing + kRing - 1] = p1;
            vring0[wave * kRing + kRing - 2] = p2;
        }
    }
    __syncthreads();
    if (wave < L) {
        // ---- section s: the recursion
        LDSP_LATENCY_CRITICAL();
        const int s = wave;
        const float a1 = A.a[3 * s + 1], a2 = A.a[3 * s + 2];
        float* const ring = vring0 + s * kRing;
        const bool tr = A.trace != nullptr;
        unsigned long long c_wait = 0, c_loop = 0, c0 = tr ? __builtin_amdgcn_s_memtime() : 0, ca = c0;
        // Every lane runs the recursion (the same values from the same LDS words:
        // reads broadcast): with only lane 0 active the LDS accesses of waves on
        // the other SIMDs slowed each other's loops 1.5-2.5x (scripts/ubench/iir_lds.hip
        // M0 / M4).  A group's 16 outputs leave in ONE store: lane j writes the 4 of
        // quarter j mod 4 (lanes of one quarter write the same 16 bytes); with four
        // stores per group the loop ran at 35 clocks per sample instead of 26.
        const int q4 = lane & 3;
        auto group = [&](const float4 u0, const float4 u1, const float4 u2, const float4 u3, float* o) {
            float4 w0, w1, w2, w3;
            SECT_STEP(u0.x, w0.x) SECT_STEP(u0.y, w0.y) SECT_STEP(u0.z, w0.z) SECT_STEP(u0.w, w0.w)
            SECT_STEP(u1.x, w1.x) SECT_STEP(u1.y, w1.y) SECT_STEP(u1.z, w1.z) SECT_STEP(u1.w, w1.w)
            SECT_STEP(u2.x, w2.x) SECT_STEP(u2.y, w2.y) SECT_STEP(u2.z, w2.z) SECT_STEP(u2.w, w2.w)
            SECT_STEP(u3.x, w3.x) SECT_STEP(u3.y, w3.y) SECT_STEP(u3.z, w3.z) SECT_STEP(u3.w, w3.w)
            const float4 lo = q4 & 1 ? w1 : w0, hi = q4 & 1 ? w3 : w2;
            st4(o + 4 * q4, q4 & 2 ? hi : lo);
        };
        for (int k = 0; k < ntiles; k++) {
            const int slot = k & (kSR - 1);
            const int cnt = (int)min((long)kST, n - (long)k * kST);
            const float* src = s == 0 ? xring + slot * kST : uscr0 + ((s - 1) * 2 + (k & 1)) * kST;
            float* vo = ring + slot * kST;
            const int c32 = cnt & ~31;
            // The tile's first 32 inputs are read right behind the poll, under its
            // round trip: one wave's LDS operations execute in order, so when the
            // poll finds the tile published its data were written before these
            // reads ran; if the poll fails they are read again after the wait.
            float4 a0, a1v, a2v, a3, b0, b1, b2, b3;
            {
                // both conditions polled with one ds_read_b64 (an LDS round trip is
                // ~100 clocks, at every tile start); a wait only when either fails
                const unsigned long long v = __hip_atomic_load(reinterpret_cast<unsigned long long*>(&sh.io[s]),
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                asm volatile("" ::: "memory");
                auto first = [&] {
                    a0 = ld4(src), a1v = ld4(src + 4), a2v = ld4(src + 8), a3 = ld4(src + 12);
                    b0 = ld4(src + 16), b1 = ld4(src + 20), b2 = ld4(src + 24), b3 = ld4(src + 28);
                };
                first();
                // (kept here: not sunk below the poll's test by the compiler)
#define SECT_PIN4(q) asm volatile("" : "+v"(q.x), "+v"(q.y), "+v"(q.z), "+v"(q.w))
                SECT_PIN4(a0); SECT_PIN4(a1v); SECT_PIN4(a2v); SECT_PIN4(a3);
                SECT_PIN4(b0); SECT_PIN4(b1); SECT_PIN4(b2); SECT_PIN4(b3);
#undef SECT_PIN4
                const int vin = __builtin_amdgcn_readfirstlane((int)(unsigned)v);
                const int vout = __builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
                if (vin < k + 1 || vout < k + 2 - kSR) {
                    ctr_wait<false>(&sh.io[s].x, k + 1, &sh.abort);
                    ctr_wait<false>(&sh.io[s].y, k + 2 - kSR, &sh.abort);
                    asm volatile("" ::: "memory");
                    first();
                }
                asm volatile("" ::: "memory");
            }
            if (tr) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                c_wait += t - ca;
                ca = t;
            }
            // 32 samples per step in two register sets (a, b): the reads of one
            // set are issued before the other set's recursion, so they have landed
            // when it is needed.  The first step is peeled so that the loop is
            // entered with the LDS operations outstanding in the same order as
            // around its back edge (the compiler's waits at the loop head then wait
            // for the reads only, not for the older writes).  Four steps per loop
            // iteration: with one, the back edge cost the loop 0.5-0.8 clocks per
            // sample above the 26-clock chain (26.6-26.8 -> 25.8-26.1 measured).
            int i = 0;
            if (c32) {
                __builtin_amdgcn_sched_barrier(0);
                auto step32 = [&](int i, bool pre) {      // pre: read the next step's inputs
                    group(a0, a1v, a2v, a3, vo + i);
                    if (pre) {
                        a0 = ld4(src + i + 32);
                        a1v = ld4(src + i + 36);
                        a2v = ld4(src + i + 40);
                        a3 = ld4(src + i + 44);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    group(b0, b1, b2, b3, vo + i + 16);
                    if (pre) {
                        b0 = ld4(src + i + 48);
                        b1 = ld4(src + i + 52);
                        b2 = ld4(src + i + 56);
                        b3 = ld4(src + i + 60);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                };
                // the peeled first step, then 128 samples per loop iteration (one back
                // edge per 128), the tile's last step without reads past it
                const int last = c32 - 32;
                if (last > 0) step32(0, true);
                i = 32;
                for (; i + 96 < last; i += 128) {
                    step32(i, true);
                    step32(i + 32, true);
                    step32(i + 64, true);
                    step32(i + 96, true);
                }
                for (; i < last; i += 32) step32(i, true);
                step32(last, false);
                i = c32;
            }
            for (; i < cnt; i++) {
                float v;
                SECT_STEP(src[i], v)
                vo[i] = v;
            }
            if (s == 0) ctr_publish(&sh.xcons, k + 1, lane);
            ctr_publish(&sh.prod[s], k + 1, lane);
            if (tr) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                c_loop += t - ca;
                ca = t;
            }
        }
        if (tr && lane == 0) {
            unsigned long long* o = A.trace + (((long)blockIdx.y * gridDim.x + blockIdx.x) * (kMaxS + 1) + s) * 4;
            o[0] = c_wait;
            o[1] = 0;
            o[2] = c_loop;
            o[3] = __builtin_amdgcn_s_memtime() - c0;
        }
        if (lane == 0) {
            st[3 * s] = p1;
            st[3 * s + 1] = p2;
            st[3 * s + 2] = p3;
        }
    } else if (wave == L) {
        // ---- I/O: input tiles into xring, the last section's y out of its ring
        const float lb0 = A.b[3 * (L - 1)], lb1 = A.b[3 * (L - 1) + 1], lb2 = A.b[3 * (L - 1) + 2];
        const int nc = A.ncomp;
        const float* r = vring0 + (L - 1) * kRing;
        int in_k = 0, out_j = 0;
        unsigned long long t_idle = 0;
        while (out_j < ntiles) {
            bool did = false;
            const bool ab = ctr_load(&sh.abort) != 0;
            if (in_k < ntiles && (ab || ctr_load(&sh.xcons) >= in_k + 1 - kSR)) {
                const long g0 = (long)in_k * kST;
                float v[kST / 64];
#pragma unroll
                for (int i = 0; i < kST / 64; i++) {
                    const long g = g0 + i * 64 + lane;
                    v[i] = g < n ? A.x[g * nc + c] : 0.0f;
                }
                float* xo = xring + (in_k & (kSR - 1)) * kST;
#pragma unroll
                for (int i = 0; i < kST / 64; i++) xo[i * 64 + lane] = v[i];
                in_k++;
                ctr_publish(&sh.io[0].x, in_k, lane);
                did = true;
            }
            if (out_j < in_k && (ab || ctr_load(&sh.prod[L - 1]) > out_j)) {
                asm volatile("" ::: "memory");
                const long g0 = (long)out_j * kST;
                const int base = (out_j & (kSR - 1)) * kST;
#pragma unroll
                for (int i = 0; i < kST / 64; i++) {
                    const int m = base + i * 64 + lane;
                    const float e0 = r[m], e1 = r[(m - 1) & (kRing - 1)], e2 = r[(m - 2) & (kRing - 1)];
                    const float yv = (lb0 * e0 + lb1 * e1) + lb2 * e2;
                    const long g = g0 + i * 64 + lane;
                    if (g < n) A.y[g * nc + c] = yv;
                }
                out_j++;
                ctr_publish(&sh.io[L - 1].y, out_j, lane);
                did = true;
            }
            if (!did) {
                __builtin_amdgcn_s_sleep(1);
                const unsigned long long t = wall_clock64();
                if (!t_idle) {
                    t_idle = t;
                } else if (t - t_idle > kSectWaitTicks) {
                    __hip_atomic_store(&sh.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else {
                t_idle = 0;
            }
        }
    } else if (wave < 2 * L) {
        // ---- helper of section s: its input tiles, one ahead, into a double buffer
        const int s = wave - L;
        const float pb0 = A.b[3 * (s - 1)], pb1 = A.b[3 * (s - 1) + 1], pb2 = A.b[3 * (s - 1) + 2];
        const float* r = vring0 + (s - 1) * kRing;
        for (int k = 0; k < ntiles; k++) {
            ctr_wait<true>(&sh.prod[s - 1], k + 1, &sh.abort);
            ctr_wait<true>(&sh.prod[s], k - 1, &sh.abort);   // section s is done with buffer k & 1 (tile k - 2)
            const int slot = k & (kSR - 1);
            float* const us0 = uscr0 + ((s - 1) * 2 + (k & 1)) * kST;
            // 8 samples per lane and pass; every pass's reads issued before the first use
            constexpr int P = kST / 512;
            float2 h[P];
            float4 q0[P], q1[P];
#pragma unroll
            for (int pp = 0; pp < P; pp++) {
                const int base = slot * kST + pp * 512 + 8 * lane;
                h[pp] = *reinterpret_cast<const float2*>(r + ((base - 2) & (kRing - 1)));
                q0[pp] = ld4(r + base);
                q1[pp] = ld4(r + base + 4);
            }
#pragma unroll
            for (int pp = 0; pp < P; pp++) {
                const float e[10] = {h[pp].x, h[pp].y, q0[pp].x, q0[pp].y, q0[pp].z, q0[pp].w,
                                     q1[pp].x, q1[pp].y, q1[pp].z, q1[pp].w};
                float u[8];
#pragma unroll
                for (int i = 0; i < 8; i++) u[i] = (pb0 * e[i + 2] + pb1 * e[i + 1]) + pb2 * e[i];
                float* us = us0 + pp * 512 + 8 * lane;
                st4(us, make_float4(u[0], u[1], u[2], u[3]));
                st4(us + 4, make_float4(u[4], u[5], u[6], u[7]));
            }
            ctr_publish(&sh.io[s - 1].y, k + 1, lane);
            ctr_publish(&sh.io[s].x, k + 1, lane);
        }
    }
}

__device__ __forceinline__ void sect_run512(const SectArgs& a) { sect_run<512>(a); }
__device__ __forceinline__ void sect_run1024(const SectArgs& a) { sect_run<1024>(a); }
LDSP_KERNEL_PAIR(k_iir_sect512, SectArgs, sect_run512, kSectThreads)
LDSP_KERNEL_PAIR(k_iir_sect1024, SectArgs, sect_run1024, kSectThreads)

unsigned long long* g_sect_trace = nullptr;

} // namespace

int iir_sect_trace(void* dev_buf)
{
    g_sect_trace = (unsigned long long*)dev_buf;
    return 0;
}

void iir_sect(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, void* y, hipStream_t s)
{
    if (n == 0) return;
    LDSP_REQUIRE(d.sos && d.nsos >= 1 && d.nsos <= kIirSectMaxSos, "iir_sect: 1..8 second-order sections");
    LDSP_REQUIRE(n < (size_t(1) << 40), "iir_sect: call too long");
    SectArgs a;
    a.b = d.b;
    a.a = d.a;
    a.nsos = d.nsos;
    a.ncomp = cplx ? 2 : 1;
    a.x = (const float*)x;
    a.n = (long)n;
    a.state = state;
    a.y = (float*)y;
    a.trace = g_sect_trace;
    constexpr size_t kLdsMax = 160 * 1024;
    const bool big = sect_lds<1024>(d.nsos) <= kLdsMax;
    const size_t lds = big ? sect_lds<1024>(d.nsos) : sect_lds<512>(d.nsos);
    auto one = big ? k_iir_sect1024 : k_iir_sect512;
    auto many = big ? k_iir_sect1024_many : k_iir_sect512_many;
    static bool attr[2] = {false, false};     // the largest dynamic LDS any launch may ask for, once per kernel pair
    if (!attr[big]) {
        const int mx = (int)kLdsMax;
        LDSP_HIP(hipFuncSetAttribute((const void*)one, hipFuncAttributeMaxDynamicSharedMemorySize, mx));
        LDSP_HIP(hipFuncSetAttribute((const void*)many, hipFuncAttributeMaxDynamicSharedMemorySize, mx));
        attr[big] = true;
    }
    // waves: L sections, the I/O wave, L - 1 helpers
    launch("k_iir_sect", one, many, dim3(a.ncomp), dim3(2 * d.nsos * 64), lds, s, a);
}

} // namespace k
} // namespace ldsp
