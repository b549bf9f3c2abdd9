// k_fir.hip -- FIR, polyphase resampler and NCO kernels for gfx950.
//
// FIR (replaces firfilt_{rrrf,crcf}_execute_block behind reference
// src/firfilter.hpp:33 and the crcf filter of demod.hpp:135):
//   fast : 256 threads x 16 consecutive outputs per thread (4096 per block).
//          The input tile + (L-1) halo is staged once in LDS with one pad slot
//          every 16 samples, so each lane's sliding-window reads (lane stride
//          17 slots) are bank-conflict free.  Taps are wave-uniform and arrive
//          through scalar loads (SGPR operands of v_fma_f32); the window is
//          register-blocked 16 x 16 so every LDS read feeds 16 FMAs.
//   exact: one output per thread, liquid dotprod order (oldest sample first,
//          separate multiply and add) -> bit-identical to the restatement.
// Resampler (resamp_{rrrf,cccf}_execute, reference src/resampler.hpp:164-167):
//   the host computes the output count and phase schedule in closed form
//   (integer arithmetic), so each output's input index and polyphase branch
//   are computed independently on the GPU; a 64-thread block stages the input
//   span of its 64 outputs in LDS with coalesced loads.
// NCO mix (nco_crcf_mix_block_{up,down}, reference src/nco.hpp:70,78):
//   theta_i = theta_0 + i * dtheta (mod 2^32, exact), 1024-entry table in LDS.
#include "resamp_dev.hpp"
#include "batch.hpp"
#include "kernels.hpp"
#include "ldsp_common.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kR = 16;             // outputs per thread (fast FIR)
constexpr int kThreads = 256;
constexpr int kTile = kR * kThreads;

__host__ __device__ __forceinline__ int fslot(int e) { return e + (e >> 4); }

__device__ __forceinline__ float vzero(float) { return 0.0f; }
__device__ __forceinline__ float2 vzero(float2) { return make_float2(0.0f, 0.0f); }
__device__ __forceinline__ float vfma(float h, float v, float a) { return fmaf(h, v, a); }
__device__ __forceinline__ float2 vfma(float h, float2 v, float2 a)
{
    return make_float2(fmaf(h, v.x, a.x), fmaf(h, v.y, a.y));
}
__device__ __forceinline__ float vscale(float a, float s) { return a * s; }
__device__ __forceinline__ float2 vscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// exact accumulate: r = r + h*x (no contraction: library built with -ffp-contract=off)
__device__ __forceinline__ float vmac(float r, float h, float v) { return r + h * v; }
__device__ __forceinline__ float2 vmac(float2 r, float h, float2 v)
{
    return make_float2(r.x + h * v.x, r.y + h * v.y);
}

template <typename T, bool PARTIAL>
__device__ __forceinline__ void fir_kblock(T (&acc)[kR], T (&anew)[kR], const T (&bold)[kR], const T* lds,
                                           int b0, const float* __restrict__ hk, int rem)
{
#pragma unroll
    for (int i = 0; i < kR; i++)
        if (!PARTIAL || i >= kR - rem) anew[i] = lds[fslot(b0 + i - (kR - 1))];
#pragma unroll
    for (int s = 0; s < kR; s++) {
        const float hs = hk[s];      // taps are zero padded to a multiple of kR
        if (!PARTIAL || s < rem) {   // wave-uniform
#pragma unroll
            for (int r = 0; r < kR; r++) {
                const T v = (r > s) ? bold[r - s - 1] : anew[r - s + kR - 1];
                acc[r] = vfma(hs, v, acc[r]);
            }
        }
    }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) k_fir_fast(const T* __restrict__ x, const T* __restrict__ hist,
                                                       T* __restrict__ hist_out, long n,
                                                       const float* __restrict__ h, int L, float scale,
                                                       T* __restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const long tile0 = (long)blockIdx.x * kTile;
    const int halo = L - 1;
    const int span = kTile + halo;
    const int tid = threadIdx.x;
    const T z = vzero(T());
    for (int e = tid; e < span; e += kThreads) {
        const long gi = tile0 - halo + e;
        T v = z;
        if (gi >= 0) {
            if (gi < n) v = x[gi];
        } else {
            v = hist[gi + halo];
        }
        lds[fslot(e)] = v;
    }
    if (blockIdx.x == 0) {
        for (int j = tid; j < halo; j += kThreads) {
            const long gi = n - halo + j;
            hist_out[j] = gi >= 0 ? x[gi] : hist[gi + halo];
        }
    }
    __syncthreads();

    T acc[kR], A[kR], B[kR];
#pragma unroll
    for (int r = 0; r < kR; r++) acc[r] = z;
    const int base = tid * kR + halo;
#pragma unroll
    for (int j = 0; j < kR - 1; j++) B[j] = lds[fslot(base + 1 + j)];
    B[kR - 1] = z;
    const int nfull = L / kR;
    const int rem = L - nfull * kR;
    int kb = 0;
    for (; kb + 2 <= nfull; kb += 2) {
        fir_kblock<T, false>(acc, A, B, lds, base - kb * kR, h + kb * kR, 0);
        fir_kblock<T, false>(acc, B, A, lds, base - (kb + 1) * kR, h + (kb + 1) * kR, 0);
    }
    if (kb < nfull) {
        fir_kblock<T, false>(acc, A, B, lds, base - kb * kR, h + kb * kR, 0);
        kb++;
        if (rem) fir_kblock<T, true>(acc, B, A, lds, base - kb * kR, h + kb * kR, rem);
    } else if (rem) {
        fir_kblock<T, true>(acc, A, B, lds, base - kb * kR, h + kb * kR, rem);
    }

    __syncthreads();
#pragma unroll
    for (int r = 0; r < kR; r++) lds[fslot(tid * kR + r)] = vscale(acc[r], scale);
    __syncthreads();
    for (int e = tid; e < kTile; e += kThreads) {
        const long gi = tile0 + e;
        if (gi < n) y[gi] = lds[fslot(e)];
    }
}

constexpr int kExactOut = 256;

template <typename T>
__device__ __forceinline__ void k_fir_exact_body(const T* __restrict__ x, const T* __restrict__ hist,
                                                 T* __restrict__ hist_out, long n,
                                                 const float* __restrict__ hrev, int L, float scale,
                                                 T* __restrict__ y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const long tile0 = (long)blockIdx.x * kExactOut;
    const int halo = L - 1;
    const int span = kExactOut + halo;
    const int tid = threadIdx.x;
    const T z = vzero(T());
    for (int e = tid; e < span; e += kThreads) {
        const long gi = tile0 - halo + e;
        T v = z;
        if (gi >= 0) {
            if (gi < n) v = x[gi];
        } else {
            v = hist[gi + halo];
        }
        lds[e] = v;
    }
    if (blockIdx.x == 0) {
        for (int j = tid; j < halo; j += kThreads) {
            const long gi = n - halo + j;
            hist_out[j] = gi >= 0 ? x[gi] : hist[gi + halo];
        }
    }
    __syncthreads();
    const long o = tile0 + tid;
    if (o >= n) return;
    T r = z;
    for (int i = 0; i < L; i++) r = vmac(r, hrev[i], lds[tid + i]);
    y[o] = vscale(r, scale);
}

template <typename T>
struct FirExactArgs {
    const T* x;
    const T* hist;
    T* hist_out;
    long n;
    const float* hrev;
    int L;
    float scale;
    T* y;
};
template <typename T>
__global__ void __launch_bounds__(kThreads) k_fir_exact(FirExactArgs<T> a)
{
    k_fir_exact_body<T>(a.x, a.hist, a.hist_out, a.n, a.hrev, a.L, a.scale, a.y);
}
template <typename T>
__global__ void __launch_bounds__(kThreads) k_fir_exact_many(Many<FirExactArgs<T>> m)
{
    const FirExactArgs<T>& a = m.a[blockIdx.y];
    k_fir_exact_body<T>(a.x, a.hist, a.hist_out, a.n, a.hrev, a.L, a.scale, a.y);
}

template <typename T>
__global__ void k_fir_hist_only(const T* __restrict__ x, const T* __restrict__ hist, T* __restrict__ hist_out,
                                long n, int halo)
{
    for (int j = threadIdx.x; j < halo; j += blockDim.x) {
        const long gi = n - halo + j;
        hist_out[j] = gi >= 0 ? x[gi] : hist[gi + halo];
    }
}

size_t fast_lds_bytes(int L, size_t elem)
{
    const int span = kTile + L - 1;
    return (size_t)(fslot(span - 1) + 1) * elem;
}

template <typename T>
void fir_fast_t(const void* x, const void* hist, void* hist_out, size_t n, const float* taps, int L, float scale,
                void* y, hipStream_t s)
{
    const size_t lds = fast_lds_bytes(L, sizeof(T));
    if (lds > 64 * 1024)
        LDSP_HIP(hipFuncSetAttribute((const void*)k_fir_fast<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
    const unsigned grid = (unsigned)((n + kTile - 1) / kTile);
    {
        LDSP_PROF(s, "k_fir_fast");
        hipLaunchKernelGGL(k_fir_fast<T>, dim3(grid), dim3(kThreads), lds, s, (const T*)x, (const T*)hist,
                           (T*)hist_out, (long)n, taps, L, scale, (T*)y);
    }
    LDSP_HIP(hipGetLastError());
}

template <typename T>
void fir_exact_t(const void* x, const void* hist, void* hist_out, size_t n, const float* taps, int L, float scale,
                 void* y, hipStream_t s)
{
    const size_t lds = (size_t)(kExactOut + L - 1) * sizeof(T);
    if (lds > 64 * 1024)
        LDSP_HIP(hipFuncSetAttribute((const void*)k_fir_exact<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
    if (lds > 64 * 1024)
        LDSP_HIP(hipFuncSetAttribute((const void*)k_fir_exact_many<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
    const unsigned grid = (unsigned)((n + kExactOut - 1) / kExactOut);
    launch("k_fir_exact", k_fir_exact<T>, k_fir_exact_many<T>, dim3(grid), dim3(kThreads), lds, s,
           FirExactArgs<T>{(const T*)x, (const T*)hist, (T*)hist_out, (long)n, taps, L, scale, (T*)y});
}

template <typename T>
void fir_hist_t(const void* x, const void* hist, void* hist_out, size_t n, int L, hipStream_t s)
{
    {
        LDSP_PROF(s, "k_fir_hist_only");
        hipLaunchKernelGGL(k_fir_hist_only<T>, dim3(1), dim3(256), 0, s, (const T*)x, (const T*)hist, (T*)hist_out,
                           (long)n, L - 1);
    }
    LDSP_HIP(hipGetLastError());
}

} // namespace

void fir_fast(bool cplx, const void* x, const void* hist, void* hist_out, size_t n, const float* taps_pad, int L,
              float scale, void* y, hipStream_t s)
{
    if (n == 0) {
        if (L > 1) cplx ? fir_hist_t<float2>(x, hist, hist_out, n, L, s) : fir_hist_t<float>(x, hist, hist_out, n, L, s);
        return;
    }
    if (cplx) fir_fast_t<float2>(x, hist, hist_out, n, taps_pad, L, scale, y, s);
    else fir_fast_t<float>(x, hist, hist_out, n, taps_pad, L, scale, y, s);
}

void fir_exact(bool cplx, const void* x, const void* hist, void* hist_out, size_t n, const float* taps_rev, int L,
               float scale, void* y, hipStream_t s)
{
    if (n == 0) {
        if (L > 1) cplx ? fir_hist_t<float2>(x, hist, hist_out, n, L, s) : fir_hist_t<float>(x, hist, hist_out, n, L, s);
        return;
    }
    if (cplx) fir_exact_t<float2>(x, hist, hist_out, n, taps_rev, L, scale, y, s);
    else fir_exact_t<float>(x, hist, hist_out, n, taps_rev, L, scale, y, s);
}

// ====================================================================== resampler
namespace {

template <bool CPLX, bool RT = false>
__global__ void __launch_bounds__(64) k_resamp(const void* __restrict__ xv_, const void* __restrict__ hist_,
                                               void* __restrict__ hist_out_, long n, const float* __restrict__ sub,
                                               ResampPlan p, void* __restrict__ y_)
{
    using T = typename std::conditional<CPLX, float2, float>::type;
    const T* x = (const T*)xv_;
    const T* hist = (const T*)hist_;
    T* hist_out = (T*)hist_out_;
    T* y = (T*)y_;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int tid = threadIdx.x;
    const int halo = p.sub_len - 1;
    if (blockIdx.x == 0) {
        for (int j = tid; j < halo; j += 64) {
            const long gi = n - halo + j;
            hist_out[j] = gi >= 0 ? x[gi] : hist[gi + halo];
        }
    }
    const long k0 = (long)blockIdx.x * p.KB;
    const long k1 = min((long)p.K, k0 + p.KB);
    if (k0 >= k1) return;
    const long jlo = resamp_j(p.P0, k0, p.step) - halo;
    const long jhi = resamp_j(p.P0, k1 - 1, p.step);
    const int span = (int)(jhi - jlo + 1);
    for (int e = tid; e < span; e += 64) {
        const long gi = jlo + e;
        T v;
        if (gi >= 0) v = x[gi];
        else v = hist[gi + halo];
        lds[e] = v;
    }
    __syncthreads();
    const long k = k0 + tid;
    if (k >= k1) return;
    const long j = resamp_j(p.P0, k, p.step);
    const uint64_t ph = p.P0 + (uint64_t)k * p.step - ((uint64_t)j << 24);
    const int b = (int)(ph >> p.bits_index);
    const int off = (int)(j - halo - jlo);
    if constexpr (CPLX && RT) {
        const float* hb = sub + (size_t)b * p.sub_len;
        float2 r = make_float2(0.0f, 0.0f);
        for (int i = 0; i < p.sub_len; i++) rs_mac_cr(r, hb[i], lds[off + i]);
        y[k] = r;
    } else if constexpr (CPLX) {
        const float2* hb = reinterpret_cast<const float2*>(sub) + (size_t)b * p.sub_len;
        float2 r = make_float2(0.0f, 0.0f);
        for (int i = 0; i < p.sub_len; i++) rs_mac(r, hb[i], lds[off + i]);
        y[k] = r;
    } else {
        const float* hb = sub + (size_t)b * p.sub_len;
        float r = 0.0f;
        for (int i = 0; i < p.sub_len; i++) r = r + hb[i] * lds[off + i];
        y[k] = r;
    }
}

// Direct variant (used when the branch table fits in LDS): one output per
// thread, its sub_len window read straight from global memory.  Neighbouring
// outputs' windows are ~1/rate samples apart, so a wave's loads touch ~64 lines
// per instruction but every line is fetched from HBM once and re-read from L1;
// no LDS staging or workgroup barrier sits between the loads and the math.
template <bool CPLX, bool RT = false>
__global__ void __launch_bounds__(256) k_resamp_direct(const void* __restrict__ xv_, const void* __restrict__ hist_,
                                                       void* __restrict__ hist_out_, long n,
                                                       const float* __restrict__ sub, ResampPlan p,
                                                       void* __restrict__ y_)
{
    using T = typename std::conditional<CPLX, float2, float>::type;
    using TT = typename std::conditional<CPLX && !RT, float2, float>::type;   // tap type
    const T* __restrict__ x = (const T*)xv_;
    const T* __restrict__ hist = (const T*)hist_;
    T* hist_out = (T*)hist_out_;
    T* y = (T*)y_;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TT* taps = reinterpret_cast<TT*>(smem);                // [npfb][sub_len]
    const int tid = threadIdx.x;
    const int halo = p.sub_len - 1;
    if (blockIdx.x == 0) {
        for (int j = tid; j < halo; j += 256) {
            const long gi = n - halo + j;
            hist_out[j] = gi >= 0 ? x[gi] : hist[gi + halo];
        }
    }
    const TT* subT = (const TT*)sub;
    for (int i = tid; i < p.npfb * p.sub_len; i += 256) taps[i] = subT[i];
    __syncthreads();
    const long k = (long)blockIdx.x * 256 + tid;
    if (k >= (long)p.K) return;
    const long j = resamp_j(p.P0, k, p.step);
    const uint64_t ph = p.P0 + (uint64_t)k * p.step - ((uint64_t)j << 24);
    const int b = (int)(ph >> p.bits_index);
    const TT* hb = taps + (size_t)b * p.sub_len;
    const long g0 = j - halo;
    T r{};
    if (g0 >= 0) {
        const T* xb = x + g0;
        for (int i = 0; i < p.sub_len; i++) {
            if constexpr (CPLX && RT) rs_mac_cr(r, hb[i], xb[i]);
            else if constexpr (CPLX) rs_mac(r, hb[i], xb[i]);
            else r = r + hb[i] * xb[i];
        }
    } else {
        for (int i = 0; i < p.sub_len; i++) {
            const long gi = g0 + i;
            const T v = gi >= 0 ? x[gi] : hist[gi + halo];
            if constexpr (CPLX && RT) rs_mac_cr(r, hb[i], v);
            else if constexpr (CPLX) rs_mac(r, hb[i], v);
            else r = r + hb[i] * v;
        }
    }
    y[k] = r;
}

// Tile variant (the default): a workgroup of kRsThreads computes p.KB
// consecutive outputs.  Their input span [a, jhi] -- a = j(k0) - halo, moved
// down to a 16-byte boundary -- is streamed into LDS with 16-byte loads, all of
// a thread's loads issued before the first wait, so every HBM line is fetched
// once by full-width coalesced loads; then each output runs its sub_len-tap
// dot product from LDS in the restatement's order (bit-identical to
// k_resamp_direct).  Branch taps live in LDS beside the span.
constexpr int kRsThreads = 256;
typedef float rs_f4 __attribute__((ext_vector_type(4)));

template <bool CPLX, bool RT>
__global__ void __launch_bounds__(kRsThreads) k_resamp_tile(const void* __restrict__ xv_, const void* __restrict__ hist_,
                                                          void* __restrict__ hist_out_, long n,
                                                          const float* __restrict__ sub, ResampPlan p, int tap_bytes,
                                                          void* __restrict__ y_)
{
    using T = typename std::conditional<CPLX, float2, float>::type;
    using TT = typename std::conditional<CPLX && !RT, float2, float>::type;   // tap type
    constexpr int V = 16 / (int)sizeof(T);                                   // samples per 16-byte load
    const T* __restrict__ x = (const T*)xv_;
    const T* __restrict__ hist = (const T*)hist_;
    T* y = (T*)y_;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TT* taps = reinterpret_cast<TT*>(smem);                     // [npfb][sub_len]
    T* win = reinterpret_cast<T*>(smem + tap_bytes);            // the span, 16-byte aligned
    const int tid = threadIdx.x;
    const int halo = p.sub_len - 1;
    if (blockIdx.x == 0) {
        T* hist_out = (T*)hist_out_;
        for (int j = tid; j < halo; j += kRsThreads) {
            const long gi = n - halo + j;
            hist_out[j] = gi >= 0 ? x[gi] : hist[gi + halo];
        }
    }
    const TT* subT = (const TT*)sub;
    for (int i = tid; i < p.npfb * p.sub_len; i += kRsThreads) taps[i] = subT[i];
    const long k0 = (long)blockIdx.x * p.KB;
    const long k1 = min((long)p.K, k0 + p.KB);
    const long jlo = resamp_j(p.P0, k0, p.step) - halo;
    const long jhi = resamp_j(p.P0, k1 - 1, p.step);          // < n
    const long mis = (long)(((uintptr_t)x / sizeof(T)) & (V - 1));   // x's misalignment in samples
    const long a = ((jlo + mis) & ~(long)(V - 1)) - mis;      // x + a is 16-byte aligned
    const int cnt = (int)(jhi - a + 1);
    if (a >= 0) {
        const int nvec = (int)min((long)(cnt / V), (n - a) / V);
        const rs_f4* __restrict__ xv = reinterpret_cast<const rs_f4*>(x + a);
        rs_f4* wv = reinterpret_cast<rs_f4*>(win);
        constexpr int U = 8;
        for (int v0 = tid; v0 < nvec; v0 += kRsThreads * U) {
            rs_f4 r[U];
#pragma unroll
            for (int u = 0; u < U; u++)
                if (v0 + u * kRsThreads < nvec) r[u] = __builtin_nontemporal_load(xv + v0 + u * kRsThreads);
#pragma unroll
            for (int u = 0; u < U; u++)
                if (v0 + u * kRsThreads < nvec) wv[v0 + u * kRsThreads] = r[u];
        }
        for (int e = nvec * V + tid; e < cnt; e += kRsThreads) win[e] = x[a + e];
    } else {                                                  // the call's first outputs: history ++ x
        for (int e = tid; e < cnt; e += kRsThreads) {
            const long gi = a + e;
            T v{};
            if (gi >= 0) v = x[gi];
            else if (gi >= -halo) v = hist[gi + halo];
            win[e] = v;
        }
    }
    __syncthreads();
    const long k = k0 + tid;
    if (k >= k1) return;
    const long j = resamp_j(p.P0, k, p.step);
    const uint64_t ph = p.P0 + (uint64_t)k * p.step - ((uint64_t)j << 24);
    const int b = (int)(ph >> p.bits_index);
    const TT* hb = taps + (size_t)b * p.sub_len;
    const T* xb = win + (j - halo - a);
    T r{};
    for (int i = 0; i < p.sub_len; i++) {
        if constexpr (CPLX && RT) rs_mac_cr(r, hb[i], xb[i]);
        else if constexpr (CPLX) rs_mac(r, hb[i], xb[i]);
        else r = r + hb[i] * xb[i];
    }
    y[k] = r;
}

} // namespace

int resamp_tile_outputs(uint32_t step, int sub_len, int npfb, bool cplx, bool real_taps)
{
    // outputs per workgroup: as many as the threads, halved until taps + span fit 48 KiB
    const size_t elem = cplx ? 8 : 4;
    const size_t tap = ((size_t)npfb * sub_len * ((cplx && !real_taps) ? 8 : 4) + 15) / 16 * 16;
    int kb = kRsThreads;
    auto bytes = [&](int q) { return tap + (((uint64_t)(q - 1) * step >> 24) + sub_len + 4) * elem; };
    while (kb > 1 && bytes(kb) > 48 * 1024) kb >>= 1;
    return bytes(kb) <= 64 * 1024 ? kb : 0;
}

void resamp(bool cplx, bool real_taps, const void* x, const void* hist, void* hist_out, size_t n, const float* sub,
            const ResampPlan& p, void* y, hipStream_t s)
{
    const size_t elem = cplx ? 8 : 4;
    const size_t tap_lds = (size_t)p.npfb * p.sub_len * ((cplx && !real_taps) ? 8 : 4);
    if (p.KB > 0 && p.tile && p.K > 0) {
        const int tap_bytes = (int)((tap_lds + 15) / 16 * 16);
        const size_t lds = (size_t)tap_bytes + (((uint64_t)(p.KB - 1) * p.step >> 24) + p.sub_len + 4) * elem;
        const unsigned g = (unsigned)((p.K + p.KB - 1) / p.KB);
        auto go = [&](const void* fn) {
            LDSP_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        };
        LDSP_PROF(s, "k_resamp");
        if (cplx && real_taps) {
            go((const void*)k_resamp_tile<true, true>);
            hipLaunchKernelGGL((k_resamp_tile<true, true>), dim3(g), dim3(kRsThreads), lds, s, x, hist, hist_out,
                               (long)n, sub, p, tap_bytes, y);
        } else if (cplx) {
            go((const void*)k_resamp_tile<true, false>);
            hipLaunchKernelGGL((k_resamp_tile<true, false>), dim3(g), dim3(kRsThreads), lds, s, x, hist, hist_out,
                               (long)n, sub, p, tap_bytes, y);
        } else {
            go((const void*)k_resamp_tile<false, false>);
            hipLaunchKernelGGL((k_resamp_tile<false, false>), dim3(g), dim3(kRsThreads), lds, s, x, hist, hist_out,
                               (long)n, sub, p, tap_bytes, y);
        }
        LDSP_HIP(hipGetLastError());
        return;
    }
    if (tap_lds <= 64 * 1024 && p.K > 0) {
        const unsigned g = (unsigned)((p.K + 255) / 256);
        LDSP_PROF(s, "k_resamp");
        if (cplx && real_taps) {
            LDSP_HIP(hipFuncSetAttribute((const void*)k_resamp_direct<true, true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)tap_lds));
            hipLaunchKernelGGL((k_resamp_direct<true, true>), dim3(g), dim3(256), tap_lds, s, x, hist, hist_out,
                               (long)n, sub, p, y);
        } else if (cplx) {
            LDSP_HIP(hipFuncSetAttribute((const void*)k_resamp_direct<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)tap_lds));
            hipLaunchKernelGGL(k_resamp_direct<true>, dim3(g), dim3(256), tap_lds, s, x, hist, hist_out, (long)n, sub,
                               p, y);
        } else {
            LDSP_HIP(hipFuncSetAttribute((const void*)k_resamp_direct<false>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)tap_lds));
            hipLaunchKernelGGL(k_resamp_direct<false>, dim3(g), dim3(256), tap_lds, s, x, hist, hist_out, (long)n,
                               sub, p, y);
        }
        LDSP_HIP(hipGetLastError());
        return;
    }
    // very large branch tables: stage each group's input span in LDS instead
    const size_t lds = (size_t)p.span_max * elem;
    const unsigned grid = (unsigned)std::max<size_t>(1, (p.K + p.KB - 1) / p.KB);
    auto go = [&](const void* fn) {
        if (lds > 64 * 1024) LDSP_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    };
    LDSP_PROF(s, "k_resamp");
    if (cplx && real_taps) {
        go((const void*)k_resamp<true, true>);
        hipLaunchKernelGGL((k_resamp<true, true>), dim3(grid), dim3(64), lds, s, x, hist, hist_out, (long)n, sub, p, y);
    } else if (cplx) {
        go((const void*)k_resamp<true>);
        hipLaunchKernelGGL(k_resamp<true>, dim3(grid), dim3(64), lds, s, x, hist, hist_out, (long)n, sub, p, y);
    } else {
        go((const void*)k_resamp<false>);
        hipLaunchKernelGGL(k_resamp<false>, dim3(grid), dim3(64), lds, s, x, hist, hist_out, (long)n, sub, p, y);
    }
    LDSP_HIP(hipGetLastError());
}

// ====================================================================== NCO
namespace {

__global__ void __launch_bounds__(256) k_nco_mix(const float2* __restrict__ x, float2* __restrict__ y, long n,
                                                 uint32_t theta0, uint32_t dtheta, const float* __restrict__ table,
                                                 int down)
{
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) tab[i] = table[i];
    __syncthreads();
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint32_t th = theta0 + (uint32_t)((uint64_t)i * dtheta);
        const uint32_t idx = ((th + (1u << 21)) >> 22) & 0x3ffu;
        const float sn = tab[idx];
        const float cs = tab[(idx + 256) & 0x3ffu];
        const float2 v = x[i];
        float2 o;
        if (down) {   // x * conj(c + js): (a c - b (-s)) + j (a (-s) + b c)
            o.x = v.x * cs - v.y * (-sn);
            o.y = v.x * (-sn) + v.y * cs;
        } else {      // x * (c + js)
            o.x = v.x * cs - v.y * sn;
            o.y = v.x * sn + v.y * cs;
        }
        y[i] = o;
    }
}

// LIQUID_VCO: direct sin/cos of the fixed-point phase (not table based)
__global__ void __launch_bounds__(256) k_vco_mix(const float2* __restrict__ x, float2* __restrict__ y, long n,
                                                 uint32_t theta0, uint32_t dtheta, int down)
{
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint32_t th = theta0 + (uint32_t)((uint64_t)i * dtheta);
        const float a = (float)(6.283185307179586 * (double)(float)th / 4294967296.0);
        float sn, cs;
        sincosf(a, &sn, &cs);
        const float2 v = x[i];
        float2 o;
        if (down) {
            o.x = v.x * cs - v.y * (-sn);
            o.y = v.x * (-sn) + v.y * cs;
        } else {
            o.x = v.x * cs - v.y * sn;
            o.y = v.x * sn + v.y * cs;
        }
        y[i] = o;
    }
}

} // namespace

void nco_mix(const void* x, void* y, size_t n, uint32_t theta0, uint32_t dtheta, const float* table, bool down,
             int type, hipStream_t s)
{
    if (n == 0) return;
    const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    if (type == 0)
        {
            LDSP_PROF(s, "k_nco_mix");
            hipLaunchKernelGGL(k_nco_mix, dim3(grid), dim3(256), 0, s, (const float2*)x, (float2*)y, (long)n, theta0,
                               dtheta, table, (int)down);
        }
    else
        {
            LDSP_PROF(s, "k_vco_mix");
            hipLaunchKernelGGL(k_vco_mix, dim3(grid), dim3(256), 0, s, (const float2*)x, (float2*)y, (long)n, theta0,
                               dtheta, (int)down);
        }
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
