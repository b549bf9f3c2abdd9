// k_iir.hip -- IIR filter kernels for gfx950 (iirfilt_{rrrf,crcf}, reference
// src/iirfilter.hpp:56,166,296,353 execute_block and :389 per-sample execute).
//
// The recursion is inherently sequential, so three evaluation strategies exist:
//  iir_seq  : the float32 direct-form-II recursion exactly as liquid evaluates
//             it (one lane per real component) -- bit-identical, slow.
//  iir_scan : chunked linear scan in float64.  The cascade is a linear system
//             s' = A s + B u; chunks of C samples run from a zero state (K1),
//             a single workgroup propagates the chunk-boundary states with
//             precomputed powers of A (K2), and every chunk re-runs from its
//             true start state writing outputs (K3).  Error ~1e-12 relative,
//             i.e. more accurate than liquid's float32 recursion.
//  iir_spec : speculative exact chunks for fast-decaying filters (de-emphasis):
//             each chunk starts W samples early from a zero state; because the
//             filter forgets its state, the float32 trajectory coalesces
//             bit-for-bit with the true one; a single-wave verifier compares
//             every chunk's guessed start state with its predecessor's end state
//             and re-runs the (rare) chunks that did not coalesce.
#include <type_traits>

#include "batch.hpp"
#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kMaxSos = 8;     // sections handled by the register-resident kernels

// Loads in the verifier read words that another lane of the same wave may have
// just rewritten; non-temporal loads are served from L2 (they bypass the CU's
// vector L1), so they always see those writes.
__device__ __forceinline__ float ldnt(const float* p) { return __builtin_nontemporal_load(p); }
constexpr int kMaxTf = 17;     // TF coefficients (nv)

// --------------------------------------------------------------- float32 step
// iirfiltsos_execute_df2: v2=v1; v1=v0; v0 = x - a1 v1 - a2 v2; y = b0 v0 + b1 v1 + b2 v2
struct SosF {
    float b[kMaxSos][3], a[kMaxSos][3];
    int nsos;
};
struct TfF {
    float b[kMaxTf], a[kMaxTf];
    int nb, na, nv;
};

// Z: compile-time size class (sections / taps the loops are unrolled to; the
// runtime counts still guard every term, so the operation sequence is the same
// for any Z >= the filter's size).  Unrolled to the maximum, the guarded terms
// of a first-order filter became a chain of ~50 selects per sample.
template <int Z = kMaxTf>
__device__ __forceinline__ float sos_step(const SosF& c, float (&v)[kMaxSos][3], float x)
{
    constexpr int KS = Z < kMaxSos ? Z : kMaxSos;
    float t = x;
#pragma unroll
    for (int s = 0; s < KS; s++) {
        if (s < c.nsos) {
            v[s][2] = v[s][1];
            v[s][1] = v[s][0];
            v[s][0] = t - c.a[s][1] * v[s][1] - c.a[s][2] * v[s][2];
            t = c.b[s][0] * v[s][0] + c.b[s][1] * v[s][1] + c.b[s][2] * v[s][2];
        }
    }
    return t;
}

// iirfilt_execute_norm: shift v; v0 = x - dot(a[1:], v[1:]); y = dot(b, v) (sequential dotprod)
template <int Z = kMaxTf>
__device__ __forceinline__ float tf_step(const TfF& c, float (&v)[kMaxTf], float x)
{
    constexpr int KT = Z < kMaxTf ? Z : kMaxTf;
#pragma unroll
    for (int i = KT - 1; i > 0; i--)
        if (i < c.nv) v[i] = v[i - 1];
    float r = 0.0f;
#pragma unroll
    for (int i = 1; i < KT; i++)
        if (i < c.na) r = r + c.a[i] * v[i];
    v[0] = x - r;
    float y = 0.0f;
#pragma unroll
    for (int i = 0; i < KT; i++)
        if (i < c.nb) y = y + c.b[i] * v[i];
    return y;
}

// size class of a filter for the templates above (host side)
inline int iir_size_class(const IirDesc& d)
{
    const int m = d.sos ? d.nsos : d.nv;
    return m <= 2 ? 2 : m <= 4 ? 4 : kMaxTf;
}

__device__ void load_sos(SosF& c, const IirDesc& d)
{
    c.nsos = d.nsos;
#pragma unroll
    for (int s = 0; s < kMaxSos; s++)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            c.b[s][k] = s < d.nsos ? d.b[3 * s + k] : 0.0f;
            c.a[s][k] = s < d.nsos ? d.a[3 * s + k] : 0.0f;
        }
}
__device__ void load_tf(TfF& c, const IirDesc& d)
{
    c.nb = d.nb;
    c.na = d.na;
    c.nv = d.nv;
#pragma unroll
    for (int i = 0; i < kMaxTf; i++) {
        c.b[i] = i < d.nb ? d.b[i] : 0.0f;
        c.a[i] = i < d.na ? d.a[i] : 0.0f;
    }
}

// state layout in memory (float32): SOS [comp][nsos][3], TF [comp][nv]
__device__ __forceinline__ int fstate_size(const IirDesc& d) { return d.sos ? 3 * d.nsos : d.nv; }

// --------------------------------------------------------------- sequential
template <int Z>
__global__ void k_iir_seq(IirDesc d, const float* __restrict__ x, long n, int ncomp, float* __restrict__ state,
                          float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
    const int c = threadIdx.x;
    if (c >= ncomp) return;
    float* st = state + c * fstate_size(d);
    if (d.sos) {
        SosF cf;
        load_sos(cf, d);
        float v[kMaxSos][3];
#pragma unroll
        for (int s = 0; s < kMaxSos; s++)
#pragma unroll
            for (int k = 0; k < 3; k++) v[s][k] = s < d.nsos ? st[3 * s + k] : 0.0f;
        for (long i = 0; i < n; i++) y[i * ncomp + c] = sos_step<Z>(cf, v, x[i * ncomp + c]);
#pragma unroll
        for (int s = 0; s < kMaxSos; s++)
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (s < d.nsos) st[3 * s + k] = v[s][k];
    } else {
        TfF cf;
        load_tf(cf, d);
        float v[kMaxTf];
#pragma unroll
        for (int i = 0; i < kMaxTf; i++) v[i] = i < d.nv ? st[i] : 0.0f;
        for (long i = 0; i < n; i++) y[i * ncomp + c] = tf_step<Z>(cf, v, x[i * ncomp + c]);
#pragma unroll
        for (int i = 0; i < kMaxTf; i++)
            if (i < d.nv) st[i] = v[i];
    }
}

// x[a, b) of component c through a float32 step, loads batched 8 ahead (off the
// recurrence's dependence chain); whole batches without a per-sample bound check,
// then the tail.  WRITE stores the outputs.
template <bool WRITE, class StepF>
__device__ __forceinline__ void run_f32(StepF&& step, const float* __restrict__ x, float* __restrict__ y, long a,
                                        long b, int ncomp, int c)
{
    constexpr int kQ = 8;
    if (a >= b) return;
    const long full = a + (b - a) / kQ * kQ;
    float nx[kQ];
#pragma unroll
    for (int j = 0; j < kQ; j++) nx[j] = x[min(a + j, b - 1) * ncomp + c];
    long i = a;
    for (; i < full; i += kQ) {
        float cx[kQ];
#pragma unroll
        for (int j = 0; j < kQ; j++) cx[j] = nx[j];
#pragma unroll
        for (int j = 0; j < kQ; j++) nx[j] = x[min(i + kQ + j, b - 1) * ncomp + c];
#pragma unroll
        for (int j = 0; j < kQ; j++) {
            const float o = step(cx[j]);
            if (WRITE) y[(i + j) * ncomp + c] = o;
        }
    }
    for (; i < b; i++) {
        const float o = step(x[i * ncomp + c]);
        if (WRITE) y[i * ncomp + c] = o;
    }
}

// --------------------------------------------------------------- speculative exact
// scratch layout: [nchunks][2 (guess, end)][ncomp][fstate]  + flags
// STAGE: the workgroup first copies its chunks' input window (64 chunk-lanes x C
// samples + W of warm-up) into LDS with coalesced loads; the lanes' loops then
// read LDS.  From global memory each batch of 8 steps waited an L2 / HBM round
// trip (~150 ns a step for a first-order filter, whose step is ~10 ns).
template <int Z, bool STAGE>
__device__ __forceinline__ void k_iir_spec_chunks_body(const IirDesc& d, const float* __restrict__ xg, long n, int ncomp,
                                                       const float* __restrict__ state0, int C, int W, long nch,
                                                       float* __restrict__ sc, float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
    extern __shared__ float xs[];
    const long ch = (long)blockIdx.x * 64 + threadIdx.x;
    const float* x = xg;
    if (STAGE) {
        const long first = (long)blockIdx.x * 64 / ncomp, last = min(nch - 1, ((long)blockIdx.x * 64 + 63) / ncomp);
        const long lo = max(0L, first * C - W), hi = min(n, (last + 1) * C);
        for (long i = threadIdx.x; i < (hi - lo) * ncomp; i += 64) xs[i] = xg[lo * ncomp + i];
        __syncthreads();
        x = xs - lo * ncomp;            // x[i * ncomp + c] for lo <= i < hi
    }
    if (ch >= nch * ncomp) return;
    const long chunk = ch / ncomp;
    const int c = (int)(ch % ncomp);
    const int fs = fstate_size(d);
    const long s0 = chunk * C;
    const long s1 = min(n, s0 + C);
    long w0 = s0 - W;
    float* guess = sc + ((chunk * 2 + 0) * ncomp + c) * fs;
    float* endst = sc + ((chunk * 2 + 1) * ncomp + c) * fs;
    const bool from_true = w0 <= 0;
    if (from_true) w0 = 0;
    if (d.sos) {
        SosF cf;
        load_sos(cf, d);
        float v[kMaxSos][3];
#pragma unroll
        for (int s = 0; s < kMaxSos; s++)
#pragma unroll
            for (int k = 0; k < 3; k++) v[s][k] = (from_true && s < d.nsos) ? state0[c * fs + 3 * s + k] : 0.0f;
        run_f32<false>([&](float u) { return sos_step<Z>(cf, v, u); }, x, y, w0, s0, ncomp, c);
#pragma unroll
        for (int s = 0; s < kMaxSos; s++)
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (s < d.nsos) guess[3 * s + k] = v[s][k];
        run_f32<true>([&](float u) { return sos_step<Z>(cf, v, u); }, x, y, s0, s1, ncomp, c);
#pragma unroll
        for (int s = 0; s < kMaxSos; s++)
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (s < d.nsos) endst[3 * s + k] = v[s][k];
    } else {
        TfF cf;
        load_tf(cf, d);
        float v[kMaxTf];
#pragma unroll
        for (int i = 0; i < kMaxTf; i++) v[i] = (from_true && i < d.nv) ? state0[c * fs + i] : 0.0f;
        run_f32<false>([&](float u) { return tf_step<Z>(cf, v, u); }, x, y, w0, s0, ncomp, c);
#pragma unroll
        for (int i = 0; i < kMaxTf; i++)
            if (i < d.nv) guess[i] = v[i];
        run_f32<true>([&](float u) { return tf_step<Z>(cf, v, u); }, x, y, s0, s1, ncomp, c);
#pragma unroll
        for (int i = 0; i < kMaxTf; i++)
            if (i < d.nv) endst[i] = v[i];
    }
}
struct IirSpecChunksArgs {
    IirDesc d;
    const float* xg;
    long n;
    int ncomp;
    const float* state0;
    int C, W;
    long nch;
    float* sc;
    float* y;
};
template <int Z, bool STAGE>
__global__ void __launch_bounds__(64) k_iir_spec_chunks(IirSpecChunksArgs a)
{
    k_iir_spec_chunks_body<Z, STAGE>(a.d, a.xg, a.n, a.ncomp, a.state0, a.C, a.W, a.nch, a.sc, a.y);
}
template <int Z, bool STAGE>
__global__ void __launch_bounds__(64) k_iir_spec_chunks_many(Many<IirSpecChunksArgs> m)
{
    const IirSpecChunksArgs& a = m.a[blockIdx.y];
    k_iir_spec_chunks_body<Z, STAGE>(a.d, a.xg, a.n, a.ncomp, a.state0, a.C, a.W, a.nch, a.sc, a.y);
}


// Verifier: one wave walks the chunks in order.  Chunk k's outputs are exact
// iff its guessed start state equals chunk k-1's (exact) end state bit for bit
// (chunks whose warm-up reached the call start began from the true state).
// Parallel pre-check: bit c of flags[c / 64] = chunk c's guessed start state
// differs from chunk c-1's end state (before any re-run).
__device__ __forceinline__ void k_iir_spec_flags_body(const IirDesc& d, int ncomp, int C, int W, long nch,
                                                      const float* __restrict__ sc,
                                                      unsigned long long* __restrict__ flags)
{
    LDSP_LATENCY_CRITICAL();
    const int fs = fstate_size(d);
    const int per = ncomp * fs;
    const long kk = (long)blockIdx.x * 64 + threadIdx.x;
    bool bad = false;
    if (kk >= 1 && kk < nch && kk * C - W > 0) {
        const float* g = sc + (kk * 2 + 0) * per;
        const float* e = sc + ((kk - 1) * 2 + 1) * per;
        for (int i = 0; i < per; i++) bad |= __float_as_uint(g[i]) != __float_as_uint(e[i]);
    }
    const unsigned long long m = __ballot(bad);
    if (threadIdx.x == 0) flags[blockIdx.x] = m;
}
struct IirSpecFlagsArgs {
    IirDesc d;
    int ncomp, C, W;
    long nch;
    const float* sc;
    unsigned long long* flags;
};
__device__ __forceinline__ void k_iir_spec_flags_run(const IirSpecFlagsArgs& a)
{
    k_iir_spec_flags_body(a.d, a.ncomp, a.C, a.W, a.nch, a.sc, a.flags);
}
LDSP_KERNEL_PAIR(k_iir_spec_flags, IirSpecFlagsArgs, k_iir_spec_flags_run, 64)


__device__ __forceinline__ uint32_t rl_u32(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }

template <int Z>
__device__ __forceinline__ void k_iir_spec_verify_body(const IirDesc& d, const float* __restrict__ x, long n, int ncomp,
                                                       int C, int W, long nch, float* __restrict__ sc,
                                                       const unsigned long long* __restrict__ flags,
                                                       float* __restrict__ state, float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
    const int lane = threadIdx.x;
    const int fs = fstate_size(d);
    const int per = ncomp * fs;   // floats per (chunk, kind)
    const long nw = (nch + 63) / 64;
    long k = 1;
    bool direct = false;          // chunk k's predecessor was re-run: compare states, not its flag
    while (k < nch) {
        long kb;
        if (direct) {
            bool bad = false;
            if (k * C - W > 0 && lane < per) {
                const float* g = sc + (k * 2 + 0) * per;
                const float* e = sc + ((k - 1) * 2 + 1) * per;
                bad = __float_as_uint(ldnt(g + lane)) != __float_as_uint(ldnt(e + lane));
            }
            if (__ballot(bad) == 0) {
                direct = false;
                k++;
                continue;
            }
            kb = k;
        } else {
            // flags of 64 x 64 chunks per step (k_iir_spec_flags)
            const long wk = k >> 6;
            unsigned long long w = (wk + lane < nw) ? flags[wk + lane] : 0ull;
            if (lane == 0) w &= ~0ull << (k & 63);
            const unsigned long long bm = __ballot(w != 0ull);
            if (bm == 0) {
                k = (wk + 64) << 6;
                continue;
            }
            const int L = __builtin_ctzll(bm);
            const unsigned long long wd = ((unsigned long long)rl_u32((uint32_t)(w >> 32), L) << 32) |
                                          rl_u32((uint32_t)w, L);
            kb = ((wk + L) << 6) + __builtin_ctzll(wd);
            if (kb >= nch) break;
        }
        // re-run chunk kb from chunk kb-1's end state (lane c handles component c)
        if (lane < ncomp) {
            const int c = lane;
            const float* e = sc + ((kb - 1) * 2 + 1) * per + c * fs;
            float* en = sc + (kb * 2 + 1) * per + c * fs;
            float* gn = sc + (kb * 2 + 0) * per + c * fs;
            const long s0 = kb * C, s1 = min(n, s0 + C);
            if (d.sos) {
                SosF cf;
                load_sos(cf, d);
                float v[kMaxSos][3];
#pragma unroll
                for (int s = 0; s < kMaxSos; s++)
#pragma unroll
                    for (int q = 0; q < 3; q++) v[s][q] = s < d.nsos ? ldnt(e + 3 * s + q) : 0.0f;
                for (long i = s0; i < s1; i++) y[i * ncomp + c] = sos_step<Z>(cf, v, x[i * ncomp + c]);
#pragma unroll
                for (int s = 0; s < kMaxSos; s++)
#pragma unroll
                    for (int q = 0; q < 3; q++)
                        if (s < d.nsos) en[3 * s + q] = v[s][q];
            } else {
                TfF cf;
                load_tf(cf, d);
                float v[kMaxTf];
#pragma unroll
                for (int i = 0; i < kMaxTf; i++) v[i] = i < d.nv ? ldnt(e + i) : 0.0f;
                for (long i = s0; i < s1; i++) y[i * ncomp + c] = tf_step<Z>(cf, v, x[i * ncomp + c]);
#pragma unroll
                for (int i = 0; i < kMaxTf; i++)
                    if (i < d.nv) en[i] = v[i];
            }
            for (int i = 0; i < fs; i++) gn[i] = ldnt(e + i);   // mark the chunk as verified
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        k = kb + 1;
        direct = true;
    }
    // carried state = end state of the last chunk
    for (int i = lane; i < per; i += 64) state[i] = ldnt(sc + ((nch - 1) * 2 + 1) * per + i);
}
struct IirSpecVerifyArgs {
    IirDesc d;
    const float* x;
    long n;
    int ncomp, C, W;
    long nch;
    float* sc;
    const unsigned long long* flags;
    float* state;
    float* y;
};
template <int Z>
__global__ void __launch_bounds__(64) k_iir_spec_verify(IirSpecVerifyArgs a)
{
    k_iir_spec_verify_body<Z>(a.d, a.x, a.n, a.ncomp, a.C, a.W, a.nch, a.sc, a.flags, a.state, a.y);
}
template <int Z>
__global__ void __launch_bounds__(64) k_iir_spec_verify_many(Many<IirSpecVerifyArgs> m)
{
    const IirSpecVerifyArgs& a = m.a[blockIdx.y];
    k_iir_spec_verify_body<Z>(a.d, a.x, a.n, a.ncomp, a.C, a.W, a.nch, a.sc, a.flags, a.state, a.y);
}


// --------------------------------------------------------------- float64 scan
// double state vector per component: SOS [2s, 2s+1] = (v0, v1) of section s
// (the values that become v1, v2 at the next step); TF [i] = v[i], i < nv - 1.
constexpr int kMaxD = 16;

struct CoefD {
    double b[kMaxD + 1], a[kMaxD + 1];
};

__device__ __forceinline__ void load_coefd(CoefD& c, const IirDesc& d)
{
    const int nbv = d.sos ? 3 * d.nsos : d.nb;
    const int nav = d.sos ? 3 * d.nsos : d.na;
#pragma unroll
    for (int i = 0; i <= kMaxD; i++) {
        c.b[i] = i < nbv ? (double)d.b[i] : 0.0;
        c.a[i] = i < nav ? (double)d.a[i] : 0.0;
    }
}

// SOS coefficients for section s live at [3s..3s+2]; kMaxD/2 = 8 sections -> 24
// entries, so SOS uses a wider table.
struct SosD {
    double b[kMaxD / 2][3], a[kMaxD / 2][3];
};
__device__ __forceinline__ void load_sosd(SosD& c, const IirDesc& d)
{
#pragma unroll
    for (int s = 0; s < kMaxD / 2; s++)
#pragma unroll
        for (int q = 0; q < 3; q++) {
            c.b[s][q] = s < d.nsos ? (double)d.b[3 * s + q] : 0.0;
            c.a[s][q] = s < d.nsos ? (double)d.a[3 * s + q] : 0.0;
        }
}

__device__ __forceinline__ double sos_step_d(const SosD& c, int nsos, double (&v)[kMaxD], double x)
{
    double t = x;
#pragma unroll
    for (int s = 0; s < kMaxD / 2; s++) {
        if (s < nsos) {
            const double v1 = v[2 * s], v2 = v[2 * s + 1];
            const double v0 = fma(-c.a[s][2], v2, fma(-c.a[s][1], v1, t));
            t = fma(c.b[s][2], v2, fma(c.b[s][1], v1, c.b[s][0] * v0));
            v[2 * s + 1] = v1;
            v[2 * s] = v0;
        }
    }
    return t;
}

__device__ __forceinline__ double tf_step_d(const CoefD& c, int nb, int na, double (&v)[kMaxD], double x)
{
    double r = x;
#pragma unroll
    for (int i = 1; i <= kMaxD; i++)
        if (i < na) r = fma(-c.a[i], v[i - 1], r);
    double y = c.b[0] * r;
#pragma unroll
    for (int i = 1; i <= kMaxD; i++)
        if (i < nb) y = fma(c.b[i], v[i - 1], y);
#pragma unroll
    for (int i = kMaxD - 1; i > 0; i--) v[i] = v[i - 1];
    v[0] = r;
    return y;
}

template <bool WRITE>
__device__ __forceinline__ void run_chunk_d(const IirDesc& d, const float* __restrict__ x, long s0, long s1,
                                            int ncomp, int c, double (&v)[kMaxD], float* __restrict__ y)
{
    if (d.sos) {
        SosD cf;
        load_sosd(cf, d);
        const int ns = d.nsos;
        for (long i = s0; i < s1; i++) {
            const double o = sos_step_d(cf, ns, v, (double)x[i * ncomp + c]);
            if (WRITE) y[i * ncomp + c] = (float)o;
        }
    } else {
        CoefD cf;
        load_coefd(cf, d);
        const int nb = d.nb, na = d.na;
        for (long i = s0; i < s1; i++) {
            const double o = tf_step_d(cf, nb, na, v, (double)x[i * ncomp + c]);
            if (WRITE) y[i * ncomp + c] = (float)o;
        }
    }
}

// K1: end state of each chunk from a zero start (per component)
__global__ void __launch_bounds__(256) k_iir_scan_local(IirDesc d, const float* __restrict__ x, long n, int ncomp,
                                                        int C, long nch, double* __restrict__ Lout)
{
    const long chunk = (long)blockIdx.x * 256 + threadIdx.x;
    if (chunk >= nch) return;
    const long s0 = chunk * C, s1 = min(n, s0 + C);
    for (int c = 0; c < ncomp; c++) {
        double v[kMaxD];
#pragma unroll
        for (int i = 0; i < kMaxD; i++) v[i] = 0.0;
        run_chunk_d<false>(d, x, s0, s1, ncomp, c, v, nullptr);
        double* o = Lout + (chunk * ncomp + c) * d.D;
#pragma unroll
        for (int i = 0; i < kMaxD; i++)
            if (i < d.D) o[i] = v[i];
    }
}

// out += M in, D x D row-major, all in registers (D is a template constant)
template <int D>
__device__ __forceinline__ void matvec_acc(const double* __restrict__ M, const double (&in)[D], double (&out)[D])
{
#pragma unroll
    for (int r = 0; r < D; r++) {
        double acc = out[r];
#pragma unroll
        for (int q = 0; q < D; q++) acc = fma(M[r * D + q], in[q], acc);
        out[r] = acc;
    }
}

// K2: one workgroup of 1024 threads; thread t owns chunks [t G, (t+1) G).
// Writes carry[c] = start state of chunk c (per component).
template <int D>
__global__ void __launch_bounds__(1024) k_iir_scan_carry(int ncomp, long nch, int G, int levels,
                                                         const double* __restrict__ AC,
                                                         const double* __restrict__ AG,
                                                         const double* __restrict__ state0,
                                                         const double* __restrict__ Lc, double* __restrict__ carry)
{
    LDSP_LATENCY_CRITICAL();
    extern __shared__ __attribute__((aligned(16))) double sh[];   // [1024][D]
    const int t = threadIdx.x;
    const long c0 = (long)t * G;
    const long c1 = min(nch, c0 + G);
    for (int comp = 0; comp < ncomp; comp++) {
        double P[D], Q[D];
#pragma unroll
        for (int i = 0; i < D; i++) P[i] = 0.0;
        for (long c = c0; c < c1; c++) {
#pragma unroll
            for (int i = 0; i < D; i++) Q[i] = Lc[(c * ncomp + comp) * D + i];
            matvec_acc<D>(AC, P, Q);
#pragma unroll
            for (int i = 0; i < D; i++) P[i] = Q[i];
        }
        __syncthreads();
        if (t + 1 < 1024)
#pragma unroll
            for (int i = 0; i < D; i++) sh[(t + 1) * D + i] = P[i];
        if (t == 0)
#pragma unroll
            for (int i = 0; i < D; i++) sh[i] = state0[comp * D + i];
        __syncthreads();
        // inclusive Hillis-Steele scan: I_t = M I_{t-1} + e_t with M = A^{C G}
        for (int l = 0; l < levels; l++) {
            const int dd = 1 << l;
            double mine[D], other[D];
#pragma unroll
            for (int i = 0; i < D; i++) {
                mine[i] = sh[t * D + i];
                other[i] = t >= dd ? sh[(t - dd) * D + i] : 0.0;
            }
            __syncthreads();
            if (t >= dd) {
                matvec_acc<D>(AG + (size_t)l * D * D, other, mine);
#pragma unroll
                for (int i = 0; i < D; i++) sh[t * D + i] = mine[i];
            }
            __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < D; i++) P[i] = sh[t * D + i];
        for (long c = c0; c < c1; c++) {
#pragma unroll
            for (int i = 0; i < D; i++) {
                carry[(c * ncomp + comp) * D + i] = P[i];
                Q[i] = Lc[(c * ncomp + comp) * D + i];
            }
            matvec_acc<D>(AC, P, Q);
#pragma unroll
            for (int i = 0; i < D; i++) P[i] = Q[i];
        }
    }
}

// K3: every chunk from its true start state, outputs in float; the last chunk
// writes the carried state.
__global__ void __launch_bounds__(256) k_iir_scan_final(IirDesc d, const float* __restrict__ x, long n, int ncomp,
                                                        int C, long nch, const double* __restrict__ carry,
                                                        double* __restrict__ state64, float* __restrict__ y)
{
    const long chunk = (long)blockIdx.x * 256 + threadIdx.x;
    if (chunk >= nch) return;
    const long s0 = chunk * C, s1 = min(n, s0 + C);
    for (int c = 0; c < ncomp; c++) {
        double v[kMaxD];
        const double* in = carry + (chunk * ncomp + c) * d.D;
#pragma unroll
        for (int i = 0; i < kMaxD; i++) v[i] = i < d.D ? in[i] : 0.0;
        run_chunk_d<true>(d, x, s0, s1, ncomp, c, v, y);
        if (chunk == nch - 1)
#pragma unroll
            for (int i = 0; i < kMaxD; i++)
                if (i < d.D) state64[c * d.D + i] = v[i];
    }
}

template <int D>
void launch_carry(int ncomp, const IirScanPlan& p, const double* state64, hipStream_t s)
{
    const size_t lds = (size_t)1024 * D * sizeof(double);
    if (lds > 64 * 1024)
        LDSP_HIP(hipFuncSetAttribute((const void*)k_iir_scan_carry<D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
    {
        LDSP_PROF(s, "k_iir_scan_carry");
        hipLaunchKernelGGL(k_iir_scan_carry<D>, dim3(1), dim3(1024), lds, s, ncomp, p.nchunks, p.G, p.levels, p.AC,
                           p.AG, state64, p.local, p.carry);
    }
    LDSP_HIP(hipGetLastError());
}

// --------------------------------------------------------------- blocked float64 scan
// Replaces K1/K3 above for state dimension D <= 8 (SOS up to 4 sections, TF up
// to 9 taps).  Chunks of kBC samples, kBN chunks per block (one workgroup,
// one chunk per thread):
//   k_iir_blk<FINAL=false>: every chunk from a zero state -> local end state
//       L_j (global); in-block Hillis-Steele scan E_j = L_j + A^C E_{j-1}
//       -> block local end state BL_b.
//   k_iir_scan_carry over blocks (A^{kBC kBN}) -> block start states BS_b.
//   k_iir_blk<FINAL=true>: the same in-block scan with E_0 += A^C BS_b gives
//       every chunk's true start state; chunks re-run writing outputs.
// Input and output tiles (kBT samples x 64 chunks per wave) are staged through
// LDS so that every global access is coalesced; both components of a complex
// stream run in the same lane (two independent dependence chains).  Per
// section the recurrence is arranged so that only v0 = t - (a1 v1 + a2 v2)
// and t' = b0 v0 + (b1 v1 + b2 v2) sit on the sample-to-sample critical path.
constexpr int kBC = 256;   // samples per chunk
constexpr int kBT = 16;    // samples per staged tile
constexpr int kBN = 256;   // chunks per block = threads per workgroup

template <int D>
struct StepSos {           // D = 2 nsos; state (v[2s], v[2s+1]) = (v1, v2) of section s
    double b[D / 2][3], a[D / 2][3];
    __device__ __forceinline__ double operator()(double (&v)[D], double x) const
    {
        double t = x;
#pragma unroll
        for (int s = 0; s < D / 2; s++) {
            const double v1 = v[2 * s], v2 = v[2 * s + 1];
            const double pa = fma(a[s][2], v2, a[s][1] * v1);
            const double pb = fma(b[s][2], v2, b[s][1] * v1);
            const double v0 = t - pa;
            t = fma(b[s][0], v0, pb);
            v[2 * s + 1] = v1;
            v[2 * s] = v0;
        }
        return t;
    }
};

template <int D>
struct StepTf {            // nv = D + 1 taps; v[i] = w[n - 1 - i]
    double b[D + 1], a[D + 1];
    __device__ __forceinline__ double operator()(double (&v)[D], double x) const
    {
        double pa = 0.0, pb = 0.0;
#pragma unroll
        for (int i = D; i >= 1; i--) {
            pa = fma(a[i], v[i - 1], pa);
            pb = fma(b[i], v[i - 1], pb);
        }
        const double r = x - pa;
#pragma unroll
        for (int i = D - 1; i > 0; i--) v[i] = v[i - 1];
        v[0] = r;
        return fma(b[0], r, pb);
    }
};

template <int NC>
struct SampT {
    using T = float2;
    static __device__ __forceinline__ double get(const float2& s, int c) { return c ? (double)s.y : (double)s.x; }
    static __device__ __forceinline__ void put(float2& s, int c, float v) { if (c) s.y = v; else s.x = v; }
};
template <>
struct SampT<1> {
    using T = float;
    static __device__ __forceinline__ double get(const float& s, int) { return (double)s; }
    static __device__ __forceinline__ void put(float& s, int, float v) { s = v; }
};

__device__ __forceinline__ void iir_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// D x D matvec out += M in (M row-major in global memory, uniform across lanes)
template <int D>
__device__ __forceinline__ void mv_acc(const double* __restrict__ M, const double (&in)[D], double (&out)[D])
{
#pragma unroll
    for (int r = 0; r < D; r++) {
        double acc = out[r];
#pragma unroll
        for (int q = 0; q < D; q++) acc = fma(M[r * D + q], in[q], acc);
        out[r] = acc;
    }
}

// The staging tiles and the scan buffer share LDS (they are used in separate
// phases, fenced by __syncthreads): 35 KB per block, and at most 168 VGPRs, so
// three blocks (12 waves) fit a CU to hide the HBM latency of the tile stream.

// IQ16: the input is the SDR wire format (int16 I, Q pairs) converted on load
// exactly as bytes_to_iq (utility.hpp:61-69: (float)v / 32767.0f), so a chain
// fed raw IQ reads 4 B per sample in both passes instead of 8.
template <int NC, int D, bool FINAL, class Step, bool IQ16 = false>
__global__ void __launch_bounds__(kBN) __attribute__((amdgpu_waves_per_eu(3)))
k_iir_blk(Step step, const void* __restrict__ xf, long n, long nch, const double* __restrict__ AL,
          double* __restrict__ Lloc, const double* __restrict__ BS, double* __restrict__ BL,
          double* __restrict__ state64, float* __restrict__ yf)
{
    using S = SampT<NC>;
    using T = typename S::T;
    constexpr int kRow = kBT + 1;
    constexpr size_t kStage = sizeof(T) * (kBN / 64) * 64 * kRow, kScn = sizeof(double) * kBN * NC * D;
    __shared__ __attribute__((aligned(16))) char lds[kStage > kScn ? kStage : kScn];
    T (*stage)[64 * kRow] = reinterpret_cast<T (*)[64 * kRow]>(lds);
    double (*scn)[NC][D] = reinterpret_cast<double (*)[NC][D]>(lds);
    static_assert(!IQ16 || NC == 2, "int16 IQ input is complex");
    const T* __restrict__ x = (const T*)xf;
    const short2* __restrict__ x16 = (const short2*)xf;
    T* __restrict__ y = (T*)yf;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const long b = blockIdx.x;
    const long gc = b * kBN + t;
    const long wbase = (b * kBN + wave * 64) * (long)kBC;   // first sample of this wave's 64 chunks
    const long cbase = gc * (long)kBC;                       // first sample of this lane's chunk
    T* st = stage[wave];
    double v[NC][D];
    double E[NC][D];

    // Runs this lane's chunk over the staged tiles from state v.
    auto run = [&](auto write_tag) {
        constexpr bool WRITE = decltype(write_tag)::value;
        // raw loads stay in flight across the tile; int16 pairs are converted
        // only when staged (a conversion next to its load would wait for it)
        using Raw = std::conditional_t<IQ16, int, T>;
        Raw nxt[kBT];
        auto fetch = [&](int k) {
#pragma unroll
            for (int q = 0; q < kBT; q++) {
                const int e = lane + 64 * q;
                const long gi = wbase + (long)(e >> 4) * kBC + k * kBT + (e & 15);
                Raw z{};
                if constexpr (IQ16) nxt[q] = gi < n ? ((const int*)x16)[gi] : z;
                else nxt[q] = gi < n ? x[gi] : z;
            }
        };
        fetch(0);
        for (int k = 0; k < kBC / kBT; k++) {
#pragma unroll
            for (int q = 0; q < kBT; q++) {
                const int e = lane + 64 * q;
                if constexpr (IQ16)
                    st[(e >> 4) * kRow + (e & 15)] =
                        make_float2(iq16_to_f((short)(nxt[q] & 0xffff)), iq16_to_f((short)(nxt[q] >> 16)));
                else
                    st[(e >> 4) * kRow + (e & 15)] = nxt[q];
            }
            if (k + 1 < kBC / kBT) fetch(k + 1);
            iir_wave_sync();
            T in[kBT];
#pragma unroll
            for (int i = 0; i < kBT; i++) in[i] = st[lane * kRow + i];
            iir_wave_sync();
            const long rem = n - (cbase + k * kBT);          // samples of this tile inside the call
            if (rem >= kBT) {
#pragma unroll
                for (int i = 0; i < kBT; i++) {
                    T o{};
#pragma unroll
                    for (int c = 0; c < NC; c++) {
                        const double r = step(v[c], S::get(in[i], c));
                        if (WRITE) S::put(o, c, (float)r);
                    }
                    if (WRITE) st[lane * kRow + i] = o;
                }
            } else {                                          // the call ends inside this tile: stop the state there
#pragma unroll
                for (int i = 0; i < kBT; i++) {
                    T o{};
                    if (i < rem) {
#pragma unroll
                        for (int c = 0; c < NC; c++) {
                            const double r = step(v[c], S::get(in[i], c));
                            if (WRITE) S::put(o, c, (float)r);
                        }
                    }
                    if (WRITE) st[lane * kRow + i] = o;
                }
            }
            if (WRITE) {
                iir_wave_sync();
#pragma unroll
                for (int q = 0; q < kBT; q++) {
                    const int e = lane + 64 * q;
                    const long gi = wbase + (long)(e >> 4) * kBC + k * kBT + (e & 15);
                    if (gi < n) y[gi] = st[(e >> 4) * kRow + (e & 15)];
                }
                iir_wave_sync();
            }
        }
    };

    if (!FINAL) {
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i < D; i++) v[c][i] = 0.0;
        run(std::false_type{});
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i < D; i++) {
                E[c][i] = v[c][i];
                if (gc < nch) Lloc[(gc * NC + c) * D + i] = v[c][i];
            }
    } else {
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i < D; i++) E[c][i] = gc < nch ? Lloc[(gc * NC + c) * D + i] : 0.0;
        if (t == 0) {
#pragma unroll
            for (int c = 0; c < NC; c++) {
                double s0[D];
#pragma unroll
                for (int i = 0; i < D; i++) s0[i] = BS[(b * NC + c) * D + i];
                mv_acc<D>(AL, s0, E[c]);
            }
        }
    }
    // inclusive scan over the block's chunks: E_j = L_j + A^C E_{j-1}
    __syncthreads();                     // every wave done with the staging tiles (same LDS)
#pragma unroll
    for (int c = 0; c < NC; c++)
#pragma unroll
        for (int i = 0; i < D; i++) scn[t][c][i] = E[c][i];
    __syncthreads();
#pragma unroll 1
    for (int l = 0; (1 << l) < kBN; l++) {
        const int dd = 1 << l;
        if (t >= dd) {
#pragma unroll
            for (int c = 0; c < NC; c++) {
                double o[D];
#pragma unroll
                for (int i = 0; i < D; i++) o[i] = scn[t - dd][c][i];
                mv_acc<D>(AL + (size_t)l * D * D, o, E[c]);
            }
        }
        __syncthreads();
        if (t >= dd)
#pragma unroll
            for (int c = 0; c < NC; c++)
#pragma unroll
                for (int i = 0; i < D; i++) scn[t][c][i] = E[c][i];
        __syncthreads();
    }
    if (!FINAL) {
        if (t == kBN - 1)
#pragma unroll
            for (int c = 0; c < NC; c++)
#pragma unroll
                for (int i = 0; i < D; i++) BL[(b * NC + c) * D + i] = E[c][i];
        return;
    }
#pragma unroll
    for (int c = 0; c < NC; c++)
#pragma unroll
        for (int i = 0; i < D; i++) v[c][i] = t == 0 ? BS[(b * NC + c) * D + i] : scn[t - 1][c][i];
    __syncthreads();                     // scan buffer read: the staging tiles may reuse it
    run(std::true_type{});
    if (gc == nch - 1)
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int i = 0; i < D; i++) state64[c * D + i] = v[c][i];
}

template <int NC, int D, class Step, bool IQ16 = false>
void launch_blk(const Step& st, const IirDesc& d, const void* x, size_t n, double* state64, const IirBlkPlan& p,
                float* y, hipStream_t s)
{
    const unsigned g = (unsigned)p.nblk;
    {
        LDSP_PROF(s, "k_iir_blk_local");
        hipLaunchKernelGGL((k_iir_blk<NC, D, false, Step, IQ16>), dim3(g), dim3(kBN), 0, s, st, x, (long)n, p.nchunks,
                           p.AL, p.local, (const double*)nullptr, p.blocal, (double*)nullptr, (float*)nullptr);
    }
    LDSP_HIP(hipGetLastError());
    IirScanPlan cp;
    cp.nchunks = p.nblk;
    cp.G = p.G;
    cp.levels = 10;
    cp.AC = p.AB;
    cp.AG = p.AG;
    cp.local = p.blocal;
    cp.carry = p.bstart;
    if (p.nblk == 1) {                  // one block: its start state is the call's
        LDSP_HIP(hipMemcpyAsync(p.bstart, state64, sizeof(double) * NC * D, hipMemcpyDeviceToDevice, s));
    } else {
        launch_carry<D>(NC, cp, state64, s);
    }
    {
        LDSP_PROF(s, "k_iir_blk_final");
        hipLaunchKernelGGL((k_iir_blk<NC, D, true, Step, IQ16>), dim3(g), dim3(kBN), 0, s, st, x, (long)n, p.nchunks,
                           p.AL, p.local, (const double*)p.bstart, (double*)nullptr, state64, y);
    }
    LDSP_HIP(hipGetLastError());
}

template <int NC, int D, bool IQ16 = false>
void dispatch_blk(const IirDesc& d, const float* cb, const float* ca, const void* x, size_t n, double* state64,
                  const IirBlkPlan& p, float* y, hipStream_t s)
{
    if (d.sos) {
        if constexpr (D % 2 == 0) {
            StepSos<D> st;
            for (int q = 0; q < D / 2; q++)
                for (int k = 0; k < 3; k++) {
                    st.b[q][k] = (double)cb[3 * q + k];
                    st.a[q][k] = (double)ca[3 * q + k];
                }
            launch_blk<NC, D, StepSos<D>, IQ16>(st, d, x, n, state64, p, y, s);
        }
    } else {
        StepTf<D> st;
        for (int i = 0; i <= D; i++) {
            st.b[i] = i < d.nb ? (double)cb[i] : 0.0;
            st.a[i] = i < d.na ? (double)ca[i] : 0.0;
        }
        launch_blk<NC, D, StepTf<D>, IQ16>(st, d, x, n, state64, p, y, s);
    }
}

} // namespace

void iir_seq(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, void* y, hipStream_t s)
{
    if (n == 0) return;
    LDSP_REQUIRE(d.sos ? d.nsos <= kMaxSos : d.nv <= kMaxTf, "iir: filter order too high for the GPU kernels");
    if (d.sos && d.nsos >= 1 && d.nsos <= kIirSectMaxSos) {     // a wave per section (k_iir_sect.hip)
        iir_sect(cplx, d, x, n, state, y, s);
        return;
    }
    {
        LDSP_PROF(s, "k_iir_seq");
        const int z = iir_size_class(d);
        auto launch = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, s, d, (const float*)x, (long)n, cplx ? 2 : 1, state, (float*)y);
        };
        if (z == 2) launch(k_iir_seq<2>);
        else if (z == 4) launch(k_iir_seq<4>);
        else launch(k_iir_seq<kMaxTf>);
    }
    LDSP_HIP(hipGetLastError());
}

size_t spec_flags_offset(long nchunks, int ncomp, int fs)
{
    return ((size_t)nchunks * 2 * ncomp * fs * sizeof(float) + 255) / 256 * 256;
}

size_t spec_scratch_bytes(long nchunks, int ncomp, int fs)
{
    return spec_flags_offset(nchunks, ncomp, fs) + (size_t)((nchunks + 63) / 64 + 64) * 8;
}

void iir_spec(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, const SpecPlan& p, void* y,
              hipStream_t s)
{
    if (n == 0) return;
    const int ncomp = cplx ? 2 : 1;
    const long work = p.nchunks * ncomp;
    const int z = iir_size_class(d);
    {
        // a workgroup's window: 64 / ncomp chunks of C samples + W, ncomp floats each
        const size_t stage = (size_t)4 * (64 * (size_t)p.C + (size_t)ncomp * p.W);
        const bool st = stage <= 64 * 1024;
        const IirSpecChunksArgs a{d, (const float*)x, (long)n, ncomp, (const float*)state, p.C, p.W, p.nchunks,
                                  (float*)p.scratch, (float*)y};
        const dim3 g((unsigned)((work + 63) / 64)), b(64);
        const size_t shm = st ? stage : 0;
#define SPEC_CHUNKS(Z, S) launch("k_iir_spec_chunks", k_iir_spec_chunks<Z, S>, k_iir_spec_chunks_many<Z, S>, g, b, shm, s, a)
        if (st) {
            if (z == 2) SPEC_CHUNKS(2, true);
            else if (z == 4) SPEC_CHUNKS(4, true);
            else SPEC_CHUNKS(kMaxTf, true);
        } else {
            if (z == 2) SPEC_CHUNKS(2, false);
            else if (z == 4) SPEC_CHUNKS(4, false);
            else SPEC_CHUNKS(kMaxTf, false);
        }
#undef SPEC_CHUNKS
    }
    const int fs = d.sos ? 3 * d.nsos : d.nv;
    unsigned long long* flags = (unsigned long long*)((char*)p.scratch + spec_flags_offset(p.nchunks, ncomp, fs));
    launch("k_iir_spec_flags", k_iir_spec_flags, k_iir_spec_flags_many, dim3((unsigned)((p.nchunks + 63) / 64)),
           dim3(64), 0, s, IirSpecFlagsArgs{d, ncomp, p.C, p.W, p.nchunks, (const float*)p.scratch, flags});
    {
        const IirSpecVerifyArgs a{d, (const float*)x, (long)n, ncomp, p.C, p.W, p.nchunks, (float*)p.scratch,
                                  (const unsigned long long*)flags, state, (float*)y};
#define SPEC_VERIFY(Z) launch("k_iir_spec_verify", k_iir_spec_verify<Z>, k_iir_spec_verify_many<Z>, dim3(1), dim3(64), 0, s, a)
        if (z == 2) SPEC_VERIFY(2);
        else if (z == 4) SPEC_VERIFY(4);
        else SPEC_VERIFY(kMaxTf);
#undef SPEC_VERIFY
    }
}

void iir_scan(bool cplx, const IirDesc& d, const void* x, size_t n, double* state64, const IirScanPlan& p, void* y,
              hipStream_t s)
{
    if (n == 0) return;
    LDSP_REQUIRE(d.D >= 1 && d.D <= kMaxD, "iir: state dimension too large for the scan kernels");
    const int ncomp = cplx ? 2 : 1;
    const unsigned g = (unsigned)((p.nchunks + 255) / 256);
    {
        LDSP_PROF(s, "k_iir_scan_local");
        hipLaunchKernelGGL(k_iir_scan_local, dim3(g), dim3(256), 0, s, d, (const float*)x, (long)n, ncomp, p.C,
                           p.nchunks, p.local);
    }
    LDSP_HIP(hipGetLastError());
    switch (d.D) {
    case 1: launch_carry<1>(ncomp, p, state64, s); break;
    case 2: launch_carry<2>(ncomp, p, state64, s); break;
    case 3: launch_carry<3>(ncomp, p, state64, s); break;
    case 4: launch_carry<4>(ncomp, p, state64, s); break;
    case 5: launch_carry<5>(ncomp, p, state64, s); break;
    case 6: launch_carry<6>(ncomp, p, state64, s); break;
    case 7: launch_carry<7>(ncomp, p, state64, s); break;
    case 8: launch_carry<8>(ncomp, p, state64, s); break;
    case 10: launch_carry<10>(ncomp, p, state64, s); break;
    case 12: launch_carry<12>(ncomp, p, state64, s); break;
    case 14: launch_carry<14>(ncomp, p, state64, s); break;
    case 16: launch_carry<16>(ncomp, p, state64, s); break;
    default:
        throw Error(LDSP_EUNSUP, "iir: unsupported state dimension for the scan kernels");
    }
    {
        LDSP_PROF(s, "k_iir_scan_final");
        hipLaunchKernelGGL(k_iir_scan_final, dim3(g), dim3(256), 0, s, d, (const float*)x, (long)n, ncomp, p.C,
                           p.nchunks, p.carry, state64, (float*)y);
    }
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp

namespace ldsp {
namespace k {
void iir_blk(bool cplx, const IirDesc& d, const float* hb, const float* ha, const void* x, size_t n, double* state64,
             const IirBlkPlan& p, void* y, hipStream_t s, bool iq16)
{
    if (n == 0) return;
    LDSP_REQUIRE(d.D >= 1 && d.D <= kIirBlkMaxD, "iir: state dimension too large for the blocked scan");
    LDSP_REQUIRE(!iq16 || cplx, "iir: int16 IQ input needs a complex filter");
    float* yf = (float*)y;
#define LDSP_BLK(DD)                                                                          \
    case DD:                                                                                  \
        if (iq16) dispatch_blk<2, DD, true>(d, hb, ha, x, n, state64, p, yf, s);               \
        else if (cplx) dispatch_blk<2, DD>(d, hb, ha, x, n, state64, p, yf, s);                \
        else dispatch_blk<1, DD>(d, hb, ha, x, n, state64, p, yf, s);                          \
        break;
    switch (d.D) {
        LDSP_BLK(1) LDSP_BLK(2) LDSP_BLK(3) LDSP_BLK(4) LDSP_BLK(5) LDSP_BLK(6) LDSP_BLK(7) LDSP_BLK(8)
    default: throw Error(LDSP_EUNSUP, "iir: unsupported state dimension");
    }
#undef LDSP_BLK
}

} // namespace k
} // namespace ldsp
