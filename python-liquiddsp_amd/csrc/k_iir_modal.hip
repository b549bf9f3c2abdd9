// k_iir_modal.hip -- fast-mode IIR filtering (iirfilt_crcf / iirfilt_rrrf
// execute_block, reference src/iirfilter.hpp:292-298 and :353) in ONE pass over
// HBM, in modal coordinates.
//
// The host (capi.cpp, IirObj::modal_setup) diagonalises the filter's state-space
// form s' = A s + B u, y = C s + D u: with A = V diag(lambda) V^-1 and V^-1 B = 1
// the state z = V^-1 s evolves as one first-order complex recursion per pole,
//     y_n = D u_n + sum_k Re(g_k z_k),      z_k <- lambda_k z_k + u_n
// (a conjugate pole pair is one mode whose weight 2 is folded into g_k; each
// component of the signal is real).  Every matrix of the chunked linear scan is
// then diagonal.  A workgroup owns 2048 consecutive samples (the look-back
// unit); each of its waves owns one component (I or Q), each lane a 32-sample
// chunk of it:
//  * the chunk ends, from a zero start, in L_k = sum_s lambda_k^(31 - s) u_s;
//  * the wave's 64 chunks combine in a Kogge-Stone scan with lambda^(32 d);
//  * the wave publishes the unit's end state from zero, BL_w, as {32-bit half,
//    call epoch} granules with write-through stores, before it waits for
//    anything (MI355X_MICROARCH.md: data-tagged 8-byte granules, sc1 stores and
//    loads, no release/acquire fence);
//  * its true start state is the look-back sum over the J units before it,
//        S_w = sum_{i<J} lambda^(2048 i) BL_{w-1-i}  (+ lambda^(2048 w) S_call if w < J),
//    exact to 2^-70 of the state (the host picks J from max |lambda|: older
//    units contribute less than that).  A predecessor whose granules do not
//    carry this call's epoch within the spin budget is recomputed from its input
//    by the waiting wave -- the same instructions, so the same bits -- so no
//    wave depends on the order in which the dispatcher starts workgroups;
//  * every chunk re-runs from E_{t-1} + lambda^(32 t) S_w writing its outputs.
// The tile is loaded and stored coalesced through LDS (one plane per component);
// the samples stay in LDS between the two passes, so HBM sees each sample read
// once and written once (16 B per complex sample, 8 B real), against 24 B
// and a one-workgroup carry kernel for the SOS-coordinate blocked scan
// (k_iir.hip), which remains the path for filters whose modal form is
// ill-conditioned.
#include <algorithm>
#include <type_traits>

#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kC = kIirModalChunk;      // samples per lane
constexpr int kUnit = 64 * kC;          // samples per workgroup = look-back unit
constexpr int kRow = kC + 1;            // LDS plane row stride (floats): conflict-free lane reads
constexpr uint64_t kSpinTicks = 5000;   // 50 us of s_memrealtime (100 MHz) before recomputing
static_assert(kC == 32, "the tile indexing below assumes 32-sample chunks");

template <int M>
struct Modal {
    double r[M], i[M];
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

// The unit's samples [wb, wb + 2048) into the LDS planes, plane c row t = chunk t
// of component c; all NC x 64 threads, 64 consecutive samples per wave
// instruction (zero past n).
template <int NC, bool IQ16, bool FULL>
__device__ __forceinline__ void tile_load(const void* __restrict__ xv, long n, long wb, int tid,
                                          float (*__restrict__ pl)[64 * kRow])
{
    constexpr int kQ = kUnit / (64 * NC);
    if constexpr (NC == 2) {
        using Raw = std::conditional_t<IQ16, int, float2>;
        const Raw* __restrict__ xr = (const Raw*)xv;
        Raw r[kQ];
#pragma unroll
        for (int q = 0; q < kQ; q++) {
            const long gi = wb + tid + 128 * q;
            if (FULL) r[q] = xr[gi];
            else r[q] = gi < n ? xr[gi] : Raw{};
        }
#pragma unroll
        for (int q = 0; q < kQ; q++) {
            const int e = tid + 128 * q;
            const int a = (e >> 5) * kRow + (e & 31);
            if constexpr (IQ16) {
                pl[0][a] = iq16_to_f((short)(r[q] & 0xffff));
                pl[1][a] = iq16_to_f((short)(r[q] >> 16));
            } else {
                pl[0][a] = r[q].x;
                pl[1][a] = r[q].y;
            }
        }
    } else {
        const float* __restrict__ xr = (const float*)xv;
        float r[kQ];
#pragma unroll
        for (int q = 0; q < kQ; q++) {
            const long gi = wb + tid + 64 * q;
            if (FULL) r[q] = xr[gi];
            else r[q] = gi < n ? xr[gi] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < kQ; q++) {
            const int e = tid + 64 * q;
            pl[0][(e >> 5) * kRow + (e & 31)] = r[q];
        }
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

// Pass 1 + the wave's inclusive scan: E_t = sum_{j <= t} lambda^(32 (t - j)) L_j
// (lane 63: the unit's end state from a zero start).  L = sum_s lambda^(31-s) u_s
// in pairs: Horner over the pairs with lambda^2, the pair sums u1 + lambda u0
// (SGPR operands: lambda and lambda^2 only, so pass 1 and pass 2 keep their
// coefficients in scalar registers), 3 FMAs per mode and sample.  One pair at a
// time (sched_barrier): hoisting later samples' conversions ran out of VGPRs.
// The scan powers are uniform: read through the constant address space they
// are scalar loads.


template <int M>
__device__ __forceinline__ void modal_scan(const IirModalCoef& cf, const double* __restrict__ PSg, const float (&u)[kC],
                                           int lane, Modal<M>& E)
{
    const cdptr PS = (cdptr)PSg;
#pragma unroll
    for (int k = 0; k < M; k++) E.r[k] = E.i[k] = 0.0;
#pragma unroll
    for (int g = 0; g < kC / 2; g++) {
        const double u0 = (double)u[2 * g], u1 = (double)u[2 * g + 1];
#pragma unroll
        for (int k = 0; k < M; k++) {
            const double pr = fma(cf.lr[k], u0, u1), pi = cf.li[k] * u0;     // u1 + lambda u0
            const double er = E.r[k], ei = E.i[k];                            // E = lambda^2 E + pair
            E.r[k] = fma(cf.l2r[k], er, fma(-cf.l2i[k], ei, pr));
            E.i[k] = fma(cf.l2r[k], ei, fma(cf.l2i[k], er, pi));
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int l = 0; l < 6; l++) {
        const int d = 1 << l;
        const bool take = lane >= d;
#pragma unroll
        for (int k = 0; k < M; k++) {
            const double orr = __shfl_up(E.r[k], d), oi = __shfl_up(E.i[k], d);
            const double ar = PS[(l * M + k) * 2], ai = PS[(l * M + k) * 2 + 1];
            const double nr = fma(ar, orr, fma(-ai, oi, E.r[k]));
            const double ni = fma(ar, oi, fma(ai, orr, E.i[k]));
            E.r[k] = take ? nr : E.r[k];
            E.i[k] = take ? ni : E.i[k];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Pass 2: the chunk from state z; row = this lane's samples in the LDS plane,
// overwritten by the outputs (as float).  The output sum runs in two chains
// (modes 0, 2, .. after D u; modes 1, 3, ..) so that no sample waits for a
// serial chain of 2 M + 1 FMAs.  GUARD: the call ends inside this unit; the
// state stops after sample cnt - 1.
template <int M, bool GUARD>
__device__ __forceinline__ void modal_run(const IirModalCoef& cf, Modal<M>& z, float* __restrict__ row, int cnt)
{
#pragma unroll
    for (int s = 0; s < kC; s++) {
        const bool on = !GUARD || s < cnt;
        const double ud = (double)row[s];
        double y0 = cf.d * ud, y1 = 0.0;
#pragma unroll
        for (int k = 0; k < M; k++) {
            double& y = (k & 1) ? y1 : y0;
            y = fma(cf.gr[k], z.r[k], y);
            y = fma(-cf.gi[k], z.i[k], y);
            const double nr = fma(cf.lr[k], z.r[k], fma(-cf.li[k], z.i[k], ud));
            const double ni = fma(cf.li[k], z.r[k], cf.lr[k] * z.i[k]);
            z.r[k] = on ? nr : z.r[k];
            z.i[k] = on ? ni : z.i[k];
        }
        row[s] = (float)(y0 + y1);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// t += pw (x) a per mode (complex product, pw = [M][re, im])
template <int M>
__device__ __forceinline__ void add_pow(const double* __restrict__ pw, const Modal<M>& a, Modal<M>& t)
{
#pragma unroll
    for (int k = 0; k < M; k++) {
        const double pr = pw[2 * k], pi = pw[2 * k + 1];
        t.r[k] = fma(pr, a.r[k], fma(-pi, a.i[k], t.r[k]));
        t.i[k] = fma(pr, a.i[k], fma(pi, a.r[k], t.i[k]));
    }
}

#ifndef LDSP_MODAL_WPE
#define LDSP_MODAL_WPE 1
#endif
template <int NC, int M, bool IQ16>
__global__ void __launch_bounds__(64 * NC, LDSP_MODAL_WPE) k_iir_modal(IirModalCoef cf, const void* __restrict__ xv, long n, long nw,
                                                       IirModalPlan p, const double* __restrict__ st_in,
                                                       double* __restrict__ st_out, float* __restrict__ yv)
{
    constexpr int kGran = M * 4;        // {half, epoch} granules per published component state
    __shared__ float pl[NC][64 * kRow];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int c = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wave's component (wave-uniform)
    const long w = blockIdx.x;
    const long wb = w * kUnit;
    const bool full = wb + kUnit <= n;
    if (full) tile_load<NC, IQ16, true>(xv, n, wb, tid, pl);
    else tile_load<NC, IQ16, false>(xv, n, wb, tid, pl);
    __syncthreads();
    float* row = pl[c] + lane * kRow;  // this lane's chunk of its component: input, then output
    float u[kC];                        // pass 1 only; pass 2 reads the plane again
#pragma unroll
    for (int s = 0; s < kC; s++) u[s] = row[s];

    Modal<M> E;
#ifdef LDSP_TUNING
    if (p.variant & 4)
        for (int k = 0; k < M; k++) E.r[k] = E.i[k] = u[k];
    else
#endif
    modal_scan<M>(cf, p.PS, u, lane, E);

    // publish BL_w of this component = E at lane 63 (the last unit has no reader)
    if (w + 1 < nw && lane == 63) {
        uint64_t* g = p.agg + (w * NC + c) * kGran;
        const uint64_t tag = (uint64_t)p.epoch << 32;
#pragma unroll
        for (int k = 0; k < M; k++) {
            const uint64_t br = __builtin_bit_cast(uint64_t, E.r[k]), bi = __builtin_bit_cast(uint64_t, E.i[k]);
            __hip_atomic_store(g + 4 * k + 0, tag | (uint32_t)br, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 4 * k + 1, tag | (uint32_t)(br >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 4 * k + 2, tag | (uint32_t)bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 4 * k + 3, tag | (uint32_t)(bi >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // this lane's exclusive prefix E_{t-1}
    Modal<M> z;
#pragma unroll
    for (int k = 0; k < M; k++) {
        const double er = __shfl_up(E.r[k], 1), ei = __shfl_up(E.i[k], 1);
        z.r[k] = lane == 0 ? 0.0 : er;
        z.i[k] = lane == 0 ? 0.0 : ei;
    }

    // look-back: lane i < jw holds lambda^(2048 i) x (BL_{w-1-i}, or S_call when i == w)
#ifdef LDSP_TUNING
    const int jw = (p.variant & 1) ? 0 : (int)min((long)p.J, w + 1);
#else
    const int jw = (int)min((long)p.J, w + 1);
#endif
    Modal<M> term;
#pragma unroll
    for (int k = 0; k < M; k++) term.r[k] = term.i[k] = 0.0;
    bool need = false;
    if (lane < jw) {
        Modal<M> a;
        if (lane == w) {
#pragma unroll
            for (int k = 0; k < M; k++) {
                a.r[k] = st_in[(c * M + k) * 2];
                a.i[k] = st_in[(c * M + k) * 2 + 1];
            }
        } else if (p.recompute) {
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
                    a.r[k] = __builtin_bit_cast(double, (g1 << 32) | (uint32_t)g0);
                    a.i[k] = __builtin_bit_cast(double, (g3 << 32) | (uint32_t)g2);
                }
                ok = bad == 0;
                if (ok || wall_clock64() - t0 > kSpinTicks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            need = !ok;
        }
        if (!need) add_pow<M>(p.PB + (size_t)lane * M * 2, a, term);
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
            Modal<M> a;
#pragma unroll
            for (int k = 0; k < M; k++) {
                a.r[k] = rl_f64(Eo.r[k], 63);
                a.i[k] = rl_f64(Eo.i[k], 63);
            }
            if (lane == i) add_pow<M>(p.PB + (size_t)i * M * 2, a, term);
        }
        comp_load<NC, IQ16>(xv, n, w, lane, c, pl[c]);
    }
    // S_w = sum of the terms in lane order; chunk start = E_{t-1} + lambda^(32 t) S_w
    Modal<M> S;
#pragma unroll
    for (int k = 0; k < M; k++) S.r[k] = S.i[k] = 0.0;
    for (int i = 0; i < jw; i++)
#pragma unroll
        for (int k = 0; k < M; k++) {
            S.r[k] += rl_f64(term.r[k], i);
            S.i[k] += rl_f64(term.i[k], i);
        }
    add_pow<M>(p.PL + (size_t)lane * M * 2, S, z);

    const long rem = n - (wb + (long)lane * kC);
#ifdef LDSP_TUNING
    if (p.variant & 2) row[0] += (float)z.r[0];
    else
#endif
    if (full) modal_run<M, false>(cf, z, row, kC);
    else modal_run<M, true>(cf, z, row, (int)max(0L, min((long)kC, rem)));
    if (rem > 0 && rem <= kC)            // the chunk holding sample n - 1: the call's end state
#pragma unroll
        for (int k = 0; k < M; k++) {
            st_out[(c * M + k) * 2] = z.r[k];
            st_out[(c * M + k) * 2 + 1] = z.i[k];
        }
    __syncthreads();
    constexpr int kQ = kUnit / (64 * NC);
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        const int e = tid + 64 * NC * q;
        const int a = (e >> 5) * kRow + (e & 31);
        const long gi = wb + e;
        if (full || gi < n) {
            if constexpr (NC == 2) ((float2*)yv)[gi] = make_float2(pl[0][a], pl[1][a]);
            else yv[gi] = pl[0][a];
        }
    }
}

template <int NC, int M, bool IQ16>
void launch_modal(const IirModalCoef& cf, const void* x, size_t n, const double* st_in, double* st_out,
                  const IirModalPlan& p, float* y, hipStream_t s)
{
    const long nw = iir_modal_units(n);
    LDSP_PROF(s, "k_iir_modal");
    hipLaunchKernelGGL((k_iir_modal<NC, M, IQ16>), dim3((unsigned)nw), dim3(64 * NC), 0, s, cf, x, (long)n, nw, p,
                       st_in, st_out, y);
}

} // namespace

long iir_modal_units(size_t n) { return (long)((n + kUnit - 1) / kUnit); }

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
