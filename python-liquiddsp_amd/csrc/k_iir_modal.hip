// k_iir_modal.hip -- fast-mode IIR filtering (iirfilt_crcf / iirfilt_rrrf
// execute_block, reference src/iirfilter.hpp:292-298 and :353) in ONE pass over
// HBM, in modal coordinates.
//
// The host (modal.cpp) diagonalises the filter's state-space form s' = A s +
// B u, y = C s + D u into its modes (one per pole; a conjugate pair is one
// mode for real input) and runs each mode as a real direct-form section -- the
// parallel form of the filter:
//     w_n = u_n - a1 w_{n-1} - a2 w_{n-2},   y_n = D u_n + sum_k c1 w_{n-1} + c2 w_{n-2}
// (each component of the signal is real; a real pole is a first-order section,
// a2 = c2 = 0).  The sections are independent, so every matrix of the chunked
// linear scan is block-diagonal with 2 x 2 blocks A_k = [[-a1, -a2], [1, 0]].
// A workgroup owns 2048 consecutive samples (the look-back unit); each of its
// waves owns one component (I or Q), each lane a 32-sample chunk of it:
//  * the chunk's end state from a zero start, L (the recursion, 2 FMAs per
//    section and sample);
//  * the wave's 64 chunks combine in a Kogge-Stone scan with A^(32 d);
//  * the wave publishes the unit's end state from zero, BL_w, as {32-bit half,
//    call epoch} granules, before it waits for anything; a reader takes a
//    granule only when its tag is this call's epoch (MI355X_MICROARCH.md:
//    data-tagged 8-byte granules, no release/acquire fence), so a stale line
//    can delay a reader but never feed it old data;
//  * its true start state is the look-back sum over the J units before it,
//        S_w = sum_{i<J} A^(2048 i) BL_{w-1-i}  (+ A^(2048 w) S_call if w < J),
//    exact to 2^-70 of the state (the host picks J from max |lambda|: older
//    units contribute less than that).  A predecessor whose granules do not
//    carry this call's epoch within the spin budget is recomputed from its input
//    by the waiting wave -- the same instructions, so the same bits -- so no
//    wave depends on the order in which the dispatcher starts workgroups;
//  * every chunk re-runs from E_{t-1} + A^(32 t) S_w writing its outputs
//    (4 FMAs per section and sample).
// The tile is loaded and stored coalesced through LDS (one plane per component);
// the samples stay in LDS between the two passes, so HBM sees each sample read
// once and written once (16 B per complex sample, 8 B real), against 24 B
// and a one-workgroup carry kernel for the SOS-coordinate blocked scan
// (k_iir.hip), which remains the path for filters whose modal form is
// ill-conditioned.
#include <algorithm>
#include <type_traits>

#include "batch.hpp"
#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"
#include "resamp_dev.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kC = kIirModalChunk;      // samples per lane
constexpr int kUnit = 64 * kC;          // samples per workgroup = look-back unit
constexpr int kRow = kC + 1;            // LDS plane row stride (floats): conflict-free lane reads
constexpr uint64_t kSpinTicks = 5000;   // 50 us of s_memrealtime (100 MHz) before recomputing
static_assert(kC == 32, "the tile indexing below assumes 32-sample chunks");

template <int M>
struct Modal {            // per section: (w_n, w_{n-1})
    double w0[M], w1[M];
};

typedef const double __attribute__((address_space(4)))* cdptr;   // uniform tables -> scalar loads

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double rl_f64(double v, int l)
{
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// component c of sample i of the input
template <int NC, bool IQ16>
__device__ __forceinline__ float comp_at(const void* __restrict__ xv, long i, int c)
{
    if constexpr (IQ16) return iq16_to_f(((const short*)xv)[2 * i + c]);
    else return ((const float*)xv)[NC * i + c];
}

// Raw buffer access to the unit's samples: a descriptor over exactly the
// samples of the call inside the unit (the hardware range check returns zeros
// for loads past n and drops stores past n), per-lane 32-bit offsets and the
// per-instruction step in soffset -- one address VGPR for the whole tile.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t unit_rsrc(const void* base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

template <int S, bool VEC>   // S bytes per sample; VEC: 16-byte accesses, else one sample each
struct Acc {
    static constexpr int kP = VEC ? 16 / S : 1;       // samples per access
    static constexpr int kW = kP * S / 4;             // dwords per access
    static __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so, uint32_t (&d)[kW])
    {
        if constexpr (kW == 4) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0);
            d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        } else if constexpr (kW == 2) {
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0);
            d[0] = v.x, d[1] = v.y;
        } else {
            d[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0);
        }
    }
    static __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so, const uint32_t (&d)[kW])
    {
        if constexpr (kW == 4) __builtin_amdgcn_raw_buffer_store_b128(u32x4{d[0], d[1], d[2], d[3]}, rs, vo, so, 0);
        else if constexpr (kW == 2) __builtin_amdgcn_raw_buffer_store_b64(u32x2{d[0], d[1]}, rs, vo, so, 0);
        else __builtin_amdgcn_raw_buffer_store_b32(d[0], rs, vo, so, 0);
    }
};

// The unit's samples into the LDS planes, plane c row t = chunk t of component
// c; all NC x 64 threads, consecutive samples per lane and instruction.  VEC:
// 16-byte loads (a whole unit, 16-byte aligned input), else one sample per load.
template <int NC, bool IQ16, bool VEC>
__device__ __forceinline__ void tile_load(__amdgpu_buffer_rsrc_t rs, int tid, float (*__restrict__ pl)[64 * kRow])
{
    constexpr int S = IQ16 ? 4 : 4 * NC, T = 64 * NC;
    using A = Acc<S, VEC>;
    constexpr int kQ = kUnit / (T * A::kP);
    static_assert((T * A::kP) % 32 == 0 && 32 % A::kP == 0, "whole rows per instruction");
    uint32_t r[kQ][A::kW];
#pragma unroll
    for (int q = 0; q < kQ; q++) A::load(rs, (uint32_t)tid * A::kP * S, (uint32_t)q * T * A::kP * S, r[q]);
    // sample e = (tid + T q) kP + j sits at row e / 32, column e % 32: a per-lane
    // base plus constant offsets (immediate LDS offsets, no per-sample index math)
    const int base = ((tid * A::kP) >> 5) * kRow + ((tid * A::kP) & 31);
#pragma unroll
    for (int q = 0; q < kQ; q++)
#pragma unroll
        for (int j = 0; j < A::kP; j++) {
            const int a = base + (T * A::kP / 32) * kRow * q + j;
            if constexpr (IQ16) {
                pl[0][a] = iq16_to_f((short)(r[q][j] & 0xffff));
                pl[1][a] = iq16_to_f((short)(r[q][j] >> 16));
            } else if constexpr (NC == 2) {
                pl[0][a] = __uint_as_float(r[q][2 * j]);
                pl[1][a] = __uint_as_float(r[q][2 * j + 1]);
            } else {
                pl[0][a] = __uint_as_float(r[q][j]);
            }
        }
}

// The unit's outputs from the LDS planes (complex or real float).
template <int NC, bool VEC>
__device__ __forceinline__ void tile_store(__amdgpu_buffer_rsrc_t rs, int tid, const float (*__restrict__ pl)[64 * kRow])
{
    constexpr int S = 4 * NC, T = 64 * NC;
    using A = Acc<S, VEC>;
    constexpr int kQ = kUnit / (T * A::kP);
    const int base = ((tid * A::kP) >> 5) * kRow + ((tid * A::kP) & 31);
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        uint32_t d[A::kW];
#pragma unroll
        for (int j = 0; j < A::kP; j++) {
            const int a = base + (T * A::kP / 32) * kRow * q + j;
            if constexpr (NC == 2) {
                d[2 * j] = __float_as_uint(pl[0][a]);
                d[2 * j + 1] = __float_as_uint(pl[1][a]);
            } else {
                d[j] = __float_as_uint(pl[0][a]);
            }
        }
        A::store(rs, (uint32_t)tid * A::kP * S, (uint32_t)q * T * A::kP * S, d);
    }
}

// One component of unit v into this wave's plane (the rare paths: a
// predecessor recomputed, the own input reloaded after it).
template <int NC, bool IQ16>
__device__ __forceinline__ void comp_load(const void* __restrict__ xv, long n, long v, int lane, int c,
                                          float* __restrict__ pl)
{
    const long wb = v * kUnit;
#pragma unroll 4
    for (int q = 0; q < kC; q++) {
        const int e = lane + 64 * q;
        const long gi = wb + e;
        pl[(e >> 5) * kRow + (e & 31)] = gi < n ? comp_at<NC, IQ16>(xv, gi, c) : 0.0f;
    }
    wave_lds_sync();
}

// Pass 1 + the wave's inclusive scan: E_t = sum_{j <= t} A^(32 (t - j)) L_j
// (lane 63: the unit's end state from a zero start), L = the chunk's end state
// from zero: per section w = u - a1 w1 - a2 w2, 2 FMAs per sample (a1, a2 as
// SGPR operands).  One pair of samples at a time (sched_barrier): hoisting later
// samples' conversions ran out of VGPRs.  The scan's 2 x 2 powers are uniform:
// read through the constant address space they are scalar loads.
typedef const double __attribute__((address_space(4)))* cdptr;

template <int M, typename U>
__device__ __forceinline__ void modal_scan(const IirModalCoef& cf, const double* __restrict__ PSg, const U& u,
                                           int lane, Modal<M>& E)
{
    const cdptr PS = (cdptr)PSg;
#pragma unroll
    for (int k = 0; k < M; k++) E.w0[k] = E.w1[k] = 0.0;
#pragma unroll
    for (int g = 0; g < kC / 2; g++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const double ud = (double)u[2 * g + h];
#pragma unroll
            for (int k = 0; k < M; k++) {
                const double w = fma(-cf.a1[k], E.w0[k], fma(-cf.a2[k], E.w1[k], ud));
                E.w1[k] = E.w0[k];
                E.w0[k] = w;
            }
        }
        // the states of every section materialised after each pair: keeps the
        // recursion sample-major (the compiler otherwise runs it section by section,
        // interleaved with the scan, and holds all 32 converted samples: 123 -> 89
        // VGPRs, same time, r05z)
#pragma unroll
        for (int k = 0; k < M; k++) asm volatile("" : "+v"(E.w0[k]), "+v"(E.w1[k]));
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int l = 0; l < 6; l++) {
        const int d = 1 << l;
#pragma unroll
        for (int k = 0; k < M; k++) {
            const double o0 = __shfl_up(E.w0[k], d), o1 = __shfl_up(E.w1[k], d);
            const double m00 = PS[(l * M + k) * 4], m01 = PS[(l * M + k) * 4 + 1];
            const double m10 = PS[(l * M + k) * 4 + 2], m11 = PS[(l * M + k) * 4 + 3];
            if (lane >= d) {
                E.w0[k] = fma(m00, o0, fma(m01, o1, E.w0[k]));
                E.w1[k] = fma(m10, o0, fma(m11, o1, E.w1[k]));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Pass 2: the chunk from section states z; row = this lane's samples in the
// LDS plane, overwritten by the outputs (as float).  The output sum runs in two
// chains (sections 0, 2, .. after D u; sections 1, 3, ..) so that no sample
// waits for a serial chain of 2 M + 1 FMAs.  GUARD: the call ends inside this
// unit; the state stops after sample cnt - 1.
template <int M, bool GUARD>
__device__ __forceinline__ void modal_run(const IirModalCoef& cf, Modal<M>& z, float* __restrict__ row, int cnt)
{
#pragma unroll
    for (int s = 0; s < kC; s++) {
        const bool on = !GUARD || s < cnt;
        const double ud = (double)row[s];
        double y = cf.d * ud;
#pragma unroll
        for (int k = 0; k < M; k++) {
            y = fma(cf.c1[k], z.w0[k], y);
            y = fma(cf.c2[k], z.w1[k], y);
            const double w = fma(-cf.a1[k], z.w0[k], fma(-cf.a2[k], z.w1[k], ud));
            z.w1[k] = on ? z.w0[k] : z.w1[k];
            z.w0[k] = on ? w : z.w0[k];
        }
        row[s] = (float)y;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// t += P_k a per section (P = [M][2 x 2], row-major)
template <int M>
__device__ __forceinline__ void add_mat(const double* __restrict__ P, const Modal<M>& a, Modal<M>& t)
{
#pragma unroll
    for (int k = 0; k < M; k++) {
        t.w0[k] = fma(P[4 * k], a.w0[k], fma(P[4 * k + 1], a.w1[k], t.w0[k]));
        t.w1[k] = fma(P[4 * k + 2], a.w0[k], fma(P[4 * k + 3], a.w1[k], t.w1[k]));
    }
}

#ifndef LDSP_MODAL_WPE
#define LDSP_MODAL_WPE 1
#endif
template <int NC, int M, bool IQ16, bool RS = false>
__device__ __forceinline__ void k_iir_modal_body(const IirModalCoef& cf, const void* __restrict__ xv, long n, long nw,
                                                 const IirModalPlan& p, const double* __restrict__ st_in,
                                                 double* __restrict__ st_out, float* __restrict__ yv,
                                                 const IirResampFuse& f)
{
    constexpr int kGran = M * 4;        // {half, epoch} granules per published component state
    __shared__ float pl[NC][64 * kRow];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int c = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wave's component (wave-uniform)
    // XCD-aware unit order: blocks b, b + 8, b + 16, .. share an XCD (observed
    // round-robin placement, MI355X_MICROARCH.md -- used for speed only) and take
    // one contiguous range of units each, so a unit's predecessors were published
    // into the same L2 (plain stores, read back with L2-served sc1 loads).  The
    // first J units of a range need units of another range: those recompute them.
    // A small call (p.one_xcd) runs every unit on block 0's XCD instead: its
    // ranges would be a few units long and their first units' recomputes of
    // up to J predecessors would set the call's latency.
    const long xq = blockIdx.x & 7, xi = blockIdx.x >> 3;
    if (p.one_xcd && xq != 0) return;
#ifdef LDSP_TUNING
    // bit 3: stagger the first round of workgroups, in groups of 64 consecutive units of
    // an XCD's range (so that a unit's predecessors never start later than it), by
    // (b >> 9) x (variant >> 4) x ~3.4 us
    if ((p.variant & 8) && blockIdx.x < 2048)
        for (int i = 0; i < (int)(blockIdx.x >> 9) * (p.variant >> 4); i++) __builtin_amdgcn_s_sleep(127);
#endif
    long range0 = 0;
    if (!p.one_xcd)
        for (long y = 0; y < xq; y++) range0 += (nw - y + 7) >> 3;
    const long w = range0 + xi;
    const long wb = w * kUnit;
    const bool full = wb + kUnit <= n;
    constexpr int kSin = IQ16 ? 4 : 4 * NC, kSout = 4 * NC;
    const uint32_t cnt = (uint32_t)min((long)kUnit, n - wb);   // samples of the call in this unit
    const bool vec = full && (((uintptr_t)xv | (uintptr_t)yv) & 15) == 0;
    {
        const __amdgpu_buffer_rsrc_t rx = unit_rsrc((const char*)xv + wb * kSin, cnt * kSin);
        if (vec) tile_load<NC, IQ16, true>(rx, tid, pl);
        else tile_load<NC, IQ16, false>(rx, tid, pl);
    }
    __syncthreads();
    // the unit's publication (pass 1, scan, BL_w) is what later units wait for:
    // issue it ahead of other waves' pass 2 on this SIMD
    __builtin_amdgcn_s_setprio(2);
    float* row = pl[c] + lane * kRow;  // this lane's chunk of its component: input, then output
    float u[kC];                        // pass 1 only; pass 2 reads the plane again
#pragma unroll
    for (int s = 0; s < kC; s++) u[s] = row[s];

    Modal<M> E;
#ifdef LDSP_TUNING
    if (p.variant & 4)
        for (int k = 0; k < M; k++) E.w0[k] = E.w1[k] = u[k];
    else
#endif
    modal_scan<M>(cf, p.PS, u, lane, E);

    // publish BL_w of this component = E at lane 63 (the last unit has no reader)
    if (w + 1 < nw && lane == 63) {
        uint64_t* g = p.agg + (w * NC + c) * kGran;
        const uint64_t tag = (uint64_t)p.epoch << 32;
#pragma unroll
        for (int k = 0; k < M; k++) {
            const uint64_t br = __builtin_bit_cast(uint64_t, E.w0[k]), bi = __builtin_bit_cast(uint64_t, E.w1[k]);
            g[4 * k + 0] = tag | (uint32_t)br;
            g[4 * k + 1] = tag | (uint32_t)(br >> 32);
            g[4 * k + 2] = tag | (uint32_t)bi;
            g[4 * k + 3] = tag | (uint32_t)(bi >> 32);
        }
    }

    __builtin_amdgcn_s_setprio(0);
    // look-back: lane i < jw fetches BL_{w-1-i} (S_call when i == w)
#ifdef LDSP_TUNING
    const int jw = (p.variant & 1) ? 0 : (int)min((long)p.J, w + 1);
#else
    const int jw = (int)min((long)p.J, w + 1);
#endif
    Modal<M> a;                         // lane i < jw: predecessor i's state
#pragma unroll
    for (int k = 0; k < M; k++) a.w0[k] = a.w1[k] = 0.0;
    bool need = false;
    if (lane < jw) {
        if (lane == w) {
#pragma unroll
            for (int k = 0; k < M; k++) {
                a.w0[k] = st_in[(c * M + k) * 2];
                a.w1[k] = st_in[(c * M + k) * 2 + 1];
            }
        } else if (p.recompute || w - 1 - lane < range0) {   // test hook, or a unit of another XCD's range
            need = true;
        } else {
            const uint64_t* g = p.agg + ((w - 1 - lane) * NC + c) * kGran;
            const uint64_t t0 = wall_clock64();
            bool ok;
            for (;;) {
                uint32_t bad = 0;
#pragma unroll
                for (int k = 0; k < M; k++) {
                    const uint64_t g0 = __hip_atomic_load(g + 4 * k + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t g1 = __hip_atomic_load(g + 4 * k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t g2 = __hip_atomic_load(g + 4 * k + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t g3 = __hip_atomic_load(g + 4 * k + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bad |= ((uint32_t)(g0 >> 32) ^ p.epoch) | ((uint32_t)(g1 >> 32) ^ p.epoch) |
                           ((uint32_t)(g2 >> 32) ^ p.epoch) | ((uint32_t)(g3 >> 32) ^ p.epoch);
                    a.w0[k] = __builtin_bit_cast(double, (g1 << 32) | (uint32_t)g0);
                    a.w1[k] = __builtin_bit_cast(double, (g3 << 32) | (uint32_t)g2);
                }
                ok = bad == 0;
                if (ok || wall_clock64() - t0 > kSpinTicks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            need = !ok;
        }
    }
    // predecessors not seen in time: recompute their end states here (the
    // plane is the scratch; this wave's own input is reloaded afterwards)
    uint64_t miss = __ballot(need);
    if (miss) {
        while (miss) {
            const int i = __builtin_ctzll(miss);
            miss &= miss - 1;
            comp_load<NC, IQ16>(xv, n, w - 1 - i, lane, c, pl[c]);
#pragma unroll
            for (int s = 0; s < kC; s++) u[s] = row[s];
            Modal<M> Eo;
            modal_scan<M>(cf, p.PS, u, lane, Eo);
#pragma unroll
            for (int k = 0; k < M; k++) {
                const double e0 = rl_f64(Eo.w0[k], 63), e1 = rl_f64(Eo.w1[k], 63);
                if (lane == i) {
                    a.w0[k] = e0;
                    a.w1[k] = e1;
                }
            }
        }
        comp_load<NC, IQ16>(xv, n, w, lane, c, pl[c]);
#pragma unroll
        for (int s = 0; s < kC; s++) u[s] = row[s];
        modal_scan<M>(cf, p.PS, u, lane, E);
    }
    // this lane's exclusive prefix E_{t-1}
    Modal<M> z;
#pragma unroll
    for (int k = 0; k < M; k++) {
        const double er = __shfl_up(E.w0[k], 1), ei = __shfl_up(E.w1[k], 1);
        z.w0[k] = lane == 0 ? 0.0 : er;
        z.w1[k] = lane == 0 ? 0.0 : ei;
    }
    // S_w = sum_i A^(2048 i) a_i, in order of i, on wave-uniform values (the
    // predecessors' states read lane by lane, the powers as scalar loads);
    // chunk start = E_{t-1} + A^(32 t) S_w
    const cdptr PB = (cdptr)p.PB;
    Modal<M> S;
#pragma unroll
    for (int k = 0; k < M; k++) S.w0[k] = S.w1[k] = 0.0;
    for (int i = 0; i < jw; i++)
#pragma unroll
        for (int k = 0; k < M; k++) {
            const double a0 = rl_f64(a.w0[k], i), a1 = rl_f64(a.w1[k], i);
            const int q = (i * M + k) * 4;
            S.w0[k] = fma(PB[q], a0, fma(PB[q + 1], a1, S.w0[k]));
            S.w1[k] = fma(PB[q + 2], a0, fma(PB[q + 3], a1, S.w1[k]));
        }
    add_mat<M>(p.PL + (size_t)lane * M * 4, S, z);

    const long rem = n - (wb + (long)lane * kC);
#ifdef LDSP_TUNING
    if (p.variant & 2) row[0] += (float)z.w0[0];
    else
#endif
    if (full) modal_run<M, false>(cf, z, row, kC);
    else modal_run<M, true>(cf, z, row, (int)max(0L, min((long)kC, rem)));
    if (rem > 0 && rem <= kC)            // the chunk holding sample n - 1: the call's end state
#pragma unroll
        for (int k = 0; k < M; k++) {
            st_out[(c * M + k) * 2] = z.w0[k];
            st_out[(c * M + k) * 2 + 1] = z.w1[k];
        }
    if constexpr (RS) {
        // the resampler on this unit's outputs, still in the planes (both
        // components: complex taps mix them)
        __syncthreads();
        auto at = [&](int cc, long e) { return pl[cc][(e >> 5) * kRow + (e & 31)]; };
        const int H = f.sub_len - 1;
        const int hc = min(H, (int)cnt);
        float* __restrict__ sd = f.side + (size_t)w * 2 * H * NC;
        for (int t = lane; t < hc; t += 64) {
            sd[t * NC + c] = at(c, t);                                  // head
            sd[(2 * H - hc + t) * NC + c] = at(c, (long)cnt - hc + t);  // tail, right-aligned
        }
        const uint64_t kA = resamp_kmin(f.P0, wb + H, f.step);
        const uint64_t kB = min((uint64_t)f.K, resamp_kmin(f.P0, wb + (long)cnt, f.step));
        for (uint64_t k = kA + lane; k < kB; k += 64) {
            const long j = resamp_j(f.P0, k, f.step);
            const uint64_t ph = f.P0 + k * (uint64_t)f.step - ((uint64_t)j << 24);
            const size_t b = (size_t)(ph >> f.bits_index);
            const long e0 = j - H - wb;
            float r = 0.0f;
            if (NC == 2 && f.ctaps) {       // rs_mac: r.x += h.x v.x - h.y v.y, r.y += h.x v.y + h.y v.x
                const float2* __restrict__ hb = reinterpret_cast<const float2*>(f.sub) + b * f.sub_len;
                for (int i = 0; i < f.sub_len; i++) {
                    const float2 h = hb[i];
                    const float vr = at(0, e0 + i), vi = at(NC - 1, e0 + i);
                    r = r + (c == 0 ? h.x * vr - h.y * vi : h.x * vi + h.y * vr);
                }
            } else {                        // real taps: componentwise (rs_mac_cr / rrrf)
                const float* __restrict__ hb = f.sub + b * f.sub_len;
                for (int i = 0; i < f.sub_len; i++) r = r + hb[i] * at(c, e0 + i);
            }
            f.y[k * NC + c] = r;
        }
        return;
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t ry = unit_rsrc((const char*)yv + wb * kSout, cnt * kSout);
    if (vec) tile_store<NC, true>(ry, tid, pl);
    else tile_store<NC, false>(ry, tid, pl);
}

struct IirModalArgs {
    IirModalCoef cf;
    const void* xv;
    long n, nw;
    IirModalPlan p;
    const double* st_in;
    double* st_out;
    float* yv;
    IirResampFuse f;
};
template <int NC, int M, bool IQ16, bool RS = false>
__global__ void __launch_bounds__(64 * NC, LDSP_MODAL_WPE) k_iir_modal(IirModalArgs a)
{
    k_iir_modal_body<NC, M, IQ16, RS>(a.cf, a.xv, a.n, a.nw, a.p, a.st_in, a.st_out, a.yv, a.f);
}
template <int NC, int M, bool IQ16, bool RS = false>
__global__ void __launch_bounds__(64 * NC, LDSP_MODAL_WPE) k_iir_modal_many(Many<IirModalArgs> m)
{
    const IirModalArgs& a = m.a[blockIdx.y];
    k_iir_modal_body<NC, M, IQ16, RS>(a.cf, a.xv, a.n, a.nw, a.p, a.st_in, a.st_out, a.yv, a.f);
}

// IIR -> resampler fusion, the outputs whose window straddles a unit boundary:
// one thread per unit u, for the outputs whose window ends in u's first H samples
// (their earlier samples: unit u - 1's tail, or the resampler history before the
// call's first sample), from the side buffer.  The first such output's window
// samples and branch taps (up to 64 each) are all loaded before its dot product,
// so a thread waits for one memory round trip, and the grid is only one thread per
// 2 048 input samples; any further outputs (rates above ~1.6) take the plain loop.
// Block 0 also writes the resampler's new history (the call's last H filter
// outputs).  Same arithmetic and order as the resampler kernels.
template <int NC>
__device__ __forceinline__ void k_iir_resamp_edges_body(const IirResampFuse& f, long n, long nw,
                                                        const float* __restrict__ hist, float* __restrict__ hist_out)
{
    const int H = f.sub_len - 1;
    auto sample = [&](long g, int c) -> float {
        if (g < 0) return hist[(g + H) * NC + c];
        const long u = g / kUnit, o = g - u * kUnit;
        const long cu = min((long)kUnit, n - u * kUnit);
        const float* sd = f.side + (size_t)u * 2 * H * NC;
        if (o < min((long)H, cu)) return sd[o * NC + c];
        return sd[(H + o - cu + H) * NC + c];
    };
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x == 0)                            // block 0's threads: the new history, one sample each
        for (int t = threadIdx.x; t < H; t += 256)
            for (int c = 0; c < NC; c++) hist_out[t * NC + c] = sample(n - H + t, c);
    if (u >= nw) return;
    const long wb = u * kUnit, cu = min((long)kUnit, n - wb);
    const uint64_t kA = resamp_kmin(f.P0, wb, f.step);
    const uint64_t kB = min((uint64_t)f.K, resamp_kmin(f.P0, wb + min((long)H, cu), f.step));
    const bool ct = NC == 2 && f.ctaps;
    constexpr int kPre = 64;
    uint64_t k = kA;
    if (k < kB && f.sub_len <= kPre) {
        const long j = resamp_j(f.P0, k, f.step);
        const size_t b = (size_t)((f.P0 + k * (uint64_t)f.step - ((uint64_t)j << 24)) >> f.bits_index);
        float hx[kPre], hy[kPre], v0[kPre], v1[kPre];
#pragma unroll
        for (int i = 0; i < kPre; i++) {
            const int ii = min(i, f.sub_len - 1);
            if (ct) {
                const float2 h = reinterpret_cast<const float2*>(f.sub)[b * f.sub_len + ii];
                hx[i] = h.x;
                hy[i] = h.y;
            } else {
                hx[i] = f.sub[b * f.sub_len + ii];
            }
            v0[i] = sample(j - H + ii, 0);
            v1[i] = sample(j - H + ii, NC - 1);
        }
        if (ct) {                   // rs_mac
            float rx = 0.0f, ry = 0.0f;
#pragma unroll
            for (int i = 0; i < kPre; i++)
                if (i < f.sub_len) {
                    rx = rx + (hx[i] * v0[i] - hy[i] * v1[i]);
                    ry = ry + (hx[i] * v1[i] + hy[i] * v0[i]);
                }
            f.y[k * NC] = rx;
            f.y[k * NC + NC - 1] = ry;
        } else {
            for (int c = 0; c < NC; c++) {
                float r = 0.0f;
#pragma unroll
                for (int i = 0; i < kPre; i++)
                    if (i < f.sub_len) r = r + hx[i] * (c == 0 ? v0[i] : v1[i]);
                f.y[k * NC + c] = r;
            }
        }
        k++;
    }
    for (; k < kB; k++) {
        const long j = resamp_j(f.P0, k, f.step);
        const size_t b = (size_t)((f.P0 + k * (uint64_t)f.step - ((uint64_t)j << 24)) >> f.bits_index);
        if (ct) {
            const float2* __restrict__ hb = reinterpret_cast<const float2*>(f.sub) + b * f.sub_len;
            float2 r = make_float2(0.0f, 0.0f);
            for (int i = 0; i < f.sub_len; i++) rs_mac(r, hb[i], make_float2(sample(j - H + i, 0), sample(j - H + i, NC - 1)));
            f.y[k * NC] = r.x;
            f.y[k * NC + NC - 1] = r.y;
        } else {
            const float* __restrict__ hb = f.sub + b * f.sub_len;
            for (int c = 0; c < NC; c++) {
                float r = 0.0f;
                for (int i = 0; i < f.sub_len; i++) r = r + hb[i] * sample(j - H + i, c);
                f.y[k * NC + c] = r;
            }
        }
    }
}

struct IirResampEdgesArgs {
    IirResampFuse f;
    long n, nw;
    const float* hist;
    float* hist_out;
};
template <int NC>
__global__ void __launch_bounds__(256) k_iir_resamp_edges(IirResampEdgesArgs a)
{
    k_iir_resamp_edges_body<NC>(a.f, a.n, a.nw, a.hist, a.hist_out);
}
template <int NC>
__global__ void __launch_bounds__(256) k_iir_resamp_edges_many(Many<IirResampEdgesArgs> m)
{
    const IirResampEdgesArgs& a = m.a[blockIdx.y];
    k_iir_resamp_edges_body<NC>(a.f, a.n, a.nw, a.hist, a.hist_out);
}

template <int NC, int M, bool IQ16, bool RS = false>
void launch_modal(const IirModalCoef& cf, const void* x, size_t n, const double* st_in, double* st_out,
                  const IirModalPlan& p, float* y, hipStream_t s, const IirResampFuse& f = IirResampFuse{})
{
    const long nw = iir_modal_units(n);
    // blocks b = q mod 8 share an XCD (the kernel's unit ranges): a merged launch
    // keeps that only when every object's grid is a multiple of 8 (batch.hpp)
    const IirModalArgs a{cf, x, (long)n, nw, p, st_in, st_out, y, f};
    const dim3 g((unsigned)(p.one_xcd ? 8 * nw : nw)), b(64 * NC);
    if constexpr (IQ16)
        launch<IirModalArgs>(RS ? "k_iir_modal_rs" : "k_iir_modal", k_iir_modal<NC, M, IQ16, RS>, nullptr, g, b, 0, s, a,
                             true);
    else
        launch<IirModalArgs>(RS ? "k_iir_modal_rs" : "k_iir_modal", k_iir_modal<NC, M, IQ16, RS>,
                             k_iir_modal_many<NC, M, IQ16, RS>, g, b, 0, s, a, true);
}

} // namespace

long iir_modal_units(size_t n) { return (long)((n + kUnit - 1) / kUnit); }

size_t iir_resamp_side_bytes(size_t n, int sub_len, bool cplx)
{
    return (size_t)iir_modal_units(n) * 2 * std::max(sub_len - 1, 1) * (cplx ? 2 : 1) * sizeof(float);
}

void iir_modal_resamp(bool cplx, const IirModalCoef& cf, const void* x, size_t n, const double* st_in,
                      double* st_out, const IirModalPlan& p, const IirResampFuse& f, const void* hist,
                      void* hist_out, hipStream_t s)
{
    if (n == 0) return;
    LDSP_REQUIRE(cf.M >= 1 && cf.M <= kIirModalMax, "iir: modal form with 1..8 modes");
    LDSP_REQUIRE(p.J >= 1 && p.J <= kIirModalJmax, "iir: look-back depth out of range");
    LDSP_REQUIRE(f.sub_len >= 2 && f.sub_len - 1 <= 1024, "iir_resamp: resampler window of 2 .. 1025 samples");
#define LDSP_MODAL(MM)                                                                                        \
    case MM:                                                                                                  \
        if (cplx) launch_modal<2, MM, false, true>(cf, x, n, st_in, st_out, p, nullptr, s, f);                \
        else launch_modal<1, MM, false, true>(cf, x, n, st_in, st_out, p, nullptr, s, f);                     \
        break;
    switch (cf.M) {
        LDSP_MODAL(1) LDSP_MODAL(2) LDSP_MODAL(3) LDSP_MODAL(4) LDSP_MODAL(5) LDSP_MODAL(6) LDSP_MODAL(7) LDSP_MODAL(8)
    default: throw Error(LDSP_EUNSUP, "iir: unsupported number of modes");
    }
#undef LDSP_MODAL
    const long nw = iir_modal_units(n);
    const unsigned g = (unsigned)((nw + 255) / 256);
    const IirResampEdgesArgs a{f, (long)n, nw, (const float*)hist, (float*)hist_out};
    if (cplx)
        launch("k_iir_resamp_edges", k_iir_resamp_edges<2>, k_iir_resamp_edges_many<2>, dim3(g), dim3(256), 0, s, a);
    else
        launch("k_iir_resamp_edges", k_iir_resamp_edges<1>, k_iir_resamp_edges_many<1>, dim3(g), dim3(256), 0, s, a);
}

void iir_modal(bool cplx, const IirModalCoef& cf, const void* x, size_t n, const double* st_in, double* st_out,
               const IirModalPlan& p, void* y, hipStream_t s, bool iq16)
{
    if (n == 0) return;
    LDSP_REQUIRE(cf.M >= 1 && cf.M <= kIirModalMax, "iir: modal form with 1..8 modes");
    LDSP_REQUIRE(p.J >= 1 && p.J <= kIirModalJmax, "iir: look-back depth out of range");
    LDSP_REQUIRE(!iq16 || cplx, "iir: int16 IQ input needs a complex filter");
    float* yf = (float*)y;
#define LDSP_MODAL(MM)                                                                        \
    case MM:                                                                                  \
        if (iq16) launch_modal<2, MM, true>(cf, x, n, st_in, st_out, p, yf, s);                \
        else if (cplx) launch_modal<2, MM, false>(cf, x, n, st_in, st_out, p, yf, s);          \
        else launch_modal<1, MM, false>(cf, x, n, st_in, st_out, p, yf, s);                    \
        break;
    switch (cf.M) {
        LDSP_MODAL(1) LDSP_MODAL(2) LDSP_MODAL(3) LDSP_MODAL(4) LDSP_MODAL(5) LDSP_MODAL(6) LDSP_MODAL(7) LDSP_MODAL(8)
    default: throw Error(LDSP_EUNSUP, "iir: unsupported number of modes");
    }
#undef LDSP_MODAL
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
