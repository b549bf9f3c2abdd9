// k_misc.hip -- small streaming kernels for the rest of the receive-path API:
//   bytes_to_iq  (reference src/utility.hpp:61-69): int16 (I, Q) -> complex64 / 32767
//   Delay        (src/utility.hpp:5-57, wdelay read-then-push): y[n] = x[n - nd - 1]
//   FreqDem      (src/demod.hpp:189-219 -> freqdem_demodulate_block):
//                y[n] = cargf(conjf(x[n-1]) x[n]) * ref, ref = 1 / (2 pi kf)
//   FMStereo     (src/demod.hpp:39-84) composite-signal mixer loop: a nonlinear
//                recurrence through (theta, dtheta, phase_error) that neither
//                coalesces nor has a linear offset structure (the phase error is
//                a rounded float filter), so it runs as one exact sequential
//                lane, with the other waves streaming its input and output.
// All are embarrassingly parallel (each output depends on a fixed window of
// inputs), HBM-bound, grid-stride loops of 16-byte-or-narrower coalesced
// accesses; streaming state (delay line, previous sample) lives in device
// buffers that the launch reads and rewrites (ping-pong on the host side).
#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

__global__ void __launch_bounds__(256) k_bytes_to_iq(const short2* __restrict__ x, float2* __restrict__ y, long n)
{
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const short2 v = x[i];
        y[i] = make_float2((float)v.x / 32767.0f, (float)v.y / 32767.0f);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) k_delay(const T* __restrict__ x, const T* __restrict__ hist,
                                               T* __restrict__ hist_out, long n, int D, T* __restrict__ y)
{
    const long stride = (long)gridDim.x * 256;
    const long i0 = (long)blockIdx.x * 256 + threadIdx.x;
    for (long i = i0; i < n; i += stride) y[i] = i < D ? hist[i] : x[i - D];
    // new line: the last D samples of hist ++ x
    for (long j = i0; j < D; j += stride) {
        const long idx = n + j;
        hist_out[j] = idx < D ? hist[idx] : x[idx - D];
    }
}

__global__ void __launch_bounds__(256) k_freqdem(const float2* __restrict__ x, const float2* __restrict__ prev,
                                                 float2* __restrict__ prev_out, long n, float ref, float* __restrict__ y)
{
    const long stride = (long)gridDim.x * 256;
    const long i0 = (long)blockIdx.x * 256 + threadIdx.x;
    for (long i = i0; i < n; i += stride) {
        const float2 rp = i > 0 ? x[i - 1] : prev[0];
        const float2 r = x[i];
        // conjf(r') * r with the C99 float complex product: (a + j b')(c + j d), b' = -b
        const float a = rp.x, bq = -rp.y;
        const float re = a * r.x - bq * r.y;
        const float im = a * r.y + bq * r.x;
        y[i] = lm_atan2f(im, re) * ref;
    }
    if (i0 == 0) prev_out[0] = n > 0 ? x[n - 1] : prev[0];
}

// ------------------------------------------------------------------ FMStereo loop
constexpr int kFmChunk = 4096;
constexpr int kFmBatch = 4;      // samples per speculation batch

// One exact mixer step (demod.hpp:61-79; nco_crcf_mix_down with the 1024-entry
// table):  (r1, i1) = (x + 0j) e^{-j theta};  pe = (float)(0.999 pe + 0.001 atan2(i1, r1));
// u = re((r1, i1) e^{-j theta});  dtheta += C(alpha pe);  theta += C(beta pe) + dtheta.
__device__ __forceinline__ float fm_step(float x, const float* tab, uint32_t& theta, uint32_t& d, float& pe,
                                         float alpha, float beta)
{
    const uint32_t idx = ((theta + (1u << 21)) >> 22) & 0x3ffu;
    const float sn = tab[idx];
    const float cs = tab[(idx + 256) & 0x3ffu];
    const float r1 = x * cs - 0.0f * (-sn);
    const float i1 = x * (-sn) + 0.0f * cs;
    pe = (float)(0.999 * (double)pe + 0.001 * (double)lm_atan2f(i1, r1));
    const float u = r1 * cs - i1 * (-sn);
    d += lm_constrain(pe * alpha);
    theta += lm_constrain(pe * beta);
    theta += d;
    return u;
}

// The chain theta -> index -> atan2 -> pe -> C() -> theta is serial and does not
// coalesce, but atan2 and the mixer output depend only on
// the input sample and the table index.  So the chain runs in batches of
// kFmBatch samples and only looks each step's index up among candidates
// evaluated ahead of it -- the same bits the direct evaluation gives:
//  * wave 0, the chain: at the start of batch g it publishes its state (theta,
//    dtheta, pe) to an LDS ring, then takes batch g's candidates (read from LDS
//    one batch ahead, into registers) and runs the 4 steps with readlane lookups;
//  * waves 1 and 2, the helpers (one half of every batch's candidates each): for
//    batch g they wait for the chain's state at batch g - 2, extrapolate the
//    trajectory with the phase error held (theta_h = theta + h (C(beta pe) + d) +
//    C(alpha pe) h (h + 1) / 2, h = 8..11 samples ahead) and evaluate atan2 and u
//    at kFmNC indices around it for each of the batch's samples, then flag their
//    half of the ring slot;
//  * wave 3 stores chunk c - 1's l / r and streams chunk c + 1 of s into the
//    LDS double buffer while the others work on chunk c.
// A batch in which some index falls outside its window (~1 % of batches on FM
// composite signals at this horizon) is redone with the direct step
// from the saved state.  The hand-offs are LDS words with the batch number as a
// tag (written after the data they guard; one wave's LDS accesses complete in
// order), so no barrier sits inside a chunk.
constexpr int kFmNC = 32;        // candidate indices per sample (the chain wave's two lane halves)
static_assert(kFmNC == 32, "the chain evaluates C(alpha pe) and C(beta pe) of every candidate in one wave");
constexpr int kFmRing = 8;       // batch slots of the hand-off rings
constexpr int kFmHor = 2;        // batches between the state a helper extrapolates from and its batch
constexpr uint64_t kFmWaitTicks = 2000;   // 20 us of s_memrealtime: a hand-off that late is given up (exactly)

struct FmBatchC {
    double w[kFmBatch];          // sample j, candidate lane & 31: 0.001 * (double) atan2
    float u[kFmBatch];           // and the mixer output
};

// candidate e = j kFmNC + k (sample j of the batch, offset k from its base)
__device__ __forceinline__ void fm_eval(const float* sp, int i0, int cnt, const float* tab, uint32_t base, int e,
                                        float& z, float& u)
{
    const int j = e / kFmNC;
    const uint32_t idx = (base + (uint32_t)(e % kFmNC)) & 0x3ffu;
    const float x = sp[min(i0 + j, cnt - 1)];
    const float sn = tab[idx];
    const float cs = tab[(idx + 256) & 0x3ffu];
    const float r1 = x * cs - 0.0f * (-sn);
    const float i1 = x * (-sn) + 0.0f * cs;
    z = lm_atan2f_vsel(i1, r1);
    u = r1 * cs - i1 * (-sn);
}

__device__ __forceinline__ uint32_t fm_base(uint32_t theta, uint32_t d, float pe, float alpha, float beta, uint32_t h)
{
    const uint32_t ca = lm_constrain(pe * alpha), cb = lm_constrain(pe * beta);
    const uint32_t pred = theta + h * (cb + d) + ca * (h * (h + 1) / 2);
    return (((pred + (1u << 21)) >> 22) - kFmNC / 2) & 0x3ffu;
}

// Tags: one wave's LDS accesses execute in issue order, so a tag stored after its
// data (or loaded before it) needs only the compiler kept from reordering them
// (cbar), not a wait.
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_ld_u32(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st_u32(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

__global__ void __launch_bounds__(256) k_fm_pll(const float* __restrict__ s, long n, FmState* st,
                                                const float* __restrict__ table, float* __restrict__ lo,
                                                float* __restrict__ ro)
{
    __shared__ float tab[1024];
    __shared__ float sb[2][kFmChunk + kFmBatch];
    __shared__ float ub[2][kFmChunk + 64];     // + 64: lanes 1..63 of wave 0 store their (identical) u here
    // per slot and sample: 0.001 (double) atan2 at candidate k in entries k and k + 32
    // (the chain's two lane halves), the mixer output at candidate k
    __shared__ double cw[kFmRing][kFmBatch][64];
    __shared__ float cu[kFmRing][kFmBatch][kFmNC];
    __shared__ uint32_t cbase[kFmRing][kFmBatch];
    __shared__ uint32_t crdy[kFmRing][2];     // per helper: batch g + 1 once its half of slot g % kFmRing holds batch g's candidates
    __shared__ uint32_t sst[kFmRing][4];      // chain state at the start of batch g: theta, dtheta, pe, g + 1
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    for (int i = tid; i < 1024; i += 256) tab[i] = table[i];
    for (int i = tid; i < kFmRing; i += 256) crdy[i][0] = crdy[i][1] = 0u, sst[i][3] = 0u;
    const long nch = (n + kFmChunk - 1) / kFmChunk;
    for (int i = tid; i < kFmChunk; i += 256) sb[0][i] = i < n ? s[i] : 0.0f;
    uint32_t theta = st->theta, d = st->dtheta;
    float pe = st->pe;
    const float alpha = st->alpha, beta = st->beta;
    constexpr int kBpc = kFmChunk / kFmBatch;        // batches per full chunk
#ifdef LDSP_TUNING
    uint32_t n_miss = 0, n_late = 0, n_spin = 0, n_hwait = 0;
#endif
    __syncthreads();
    if (wave == 0) LDSP_LATENCY_CRITICAL();
    for (long c = 0; c <= nch; c++) {
        const int cur = (int)(c & 1);
        const long base = c * kFmChunk;
        const int cnt = c < nch ? (int)min((long)kFmChunk, n - base) : 0;
        const int nb = cnt / kFmBatch;
        const uint32_t g0 = (uint32_t)(c * kBpc);     // call-wide number of the chunk's first batch
        const float* sp = sb[cur];
        if (wave == 0 && c < nch) {
            float* up = ub[cur];
            const int uoff = lane == 0 ? 0 : kFmChunk + lane;   // lane 0 stores the chain's u
            // lanes 0..31 form C(alpha pe), lanes 32..63 C(beta pe), of candidate lane & 31
            const float mco = lane < 32 ? alpha : beta;
            FmBatchC cc{}, nx{};
            uint32_t cb4 = 0, nb4 = 0, ctag = 0, ntag = 0;
            auto fetch = [&](uint32_t g, FmBatchC& v, uint32_t& b4, uint32_t& tag) {
                const int sl = (int)(g % kFmRing);
                const uint32_t t0 = lds_ld_u32(&crdy[sl][0]), t1 = lds_ld_u32(&crdy[sl][1]);
                tag = t0 == t1 ? t0 : 0u;
                cbar();
#pragma unroll
                for (int j = 0; j < kFmBatch; j++) {
                    v.w[j] = cw[sl][j][lane];
                    v.u[j] = cu[sl][j][lane & (kFmNC - 1)];
                }
                b4 = cbase[sl][lane & 3];
            };
            for (int b = 0; b < nb; b++) {
                const uint32_t g = g0 + (uint32_t)b;
                const int i0 = b * kFmBatch;
                if (lane == 0) {      // publish the state at this batch's start
                    const int sl = (int)(g % kFmRing);
                    sst[sl][0] = theta;
                    sst[sl][1] = d;
                    sst[sl][2] = __float_as_uint(pe);
                    cbar();
                    lds_st_u32(&sst[sl][3], g + 1u);
                }
                if (b == 0) fetch(g, cc, cb4, ctag);
                else cc = nx, cb4 = nb4, ctag = ntag;
#ifdef LDSP_TUNING
                n_late += __builtin_amdgcn_readfirstlane(ctag) != g + 1u;
#endif
                bool miss = false;
                if (__builtin_amdgcn_readfirstlane(ctag) != g + 1u) {   // not ready when prefetched
                    const uint64_t tw = wall_clock64();
                    do {
                        // no helper within kFmWaitTicks: the batch is stepped directly (exact either way)
                        if (wall_clock64() - tw > kFmWaitTicks) {
                            miss = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        fetch(g, cc, cb4, ctag);
#ifdef LDSP_TUNING
                        n_spin++;
#endif
                    } while (__builtin_amdgcn_readfirstlane(ctag) != g + 1u);
                }
                const uint32_t th0 = theta, d0 = d;
                const float pe0 = pe;
                int u4 = 0;
#pragma unroll
                for (int j = 0; j < kFmBatch; j++) {
                    // every candidate's step at once (the lanes): its pe and C(alpha pe) /
                    // C(beta pe) -- the same operations as fm_step -- while the scalar
                    // unit finds the true index; then the step is three readlanes
                    const float pk = (float)(0.999 * (double)pe + cc.w[j]);
                    uint32_t ck = lm_constrain_fr(pk * mco);
                    // formed here, as soon as pe is known: the compiler otherwise pairs it
                    // with the next step's (packed f32 ops), which puts that step's pe on
                    // this step's path to its index
                    asm volatile("" : "+v"(ck));
                    const uint32_t idx = ((theta + (1u << 21)) >> 22) & 0x3ffu;
                    const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)cb4, j);
                    const uint32_t off = (idx - bj) & 0x3ffu;
                    miss |= off >= (uint32_t)kFmNC;
                    const int ln = __builtin_amdgcn_readfirstlane((int)(off & (kFmNC - 1)));
                    pe = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pk), ln));
                    const uint32_t ca = (uint32_t)__builtin_amdgcn_readlane((int)ck, ln);
                    const uint32_t cbt = (uint32_t)__builtin_amdgcn_readlane((int)ck, ln + 32);
                    // u into lane j of u4, stored once per batch
                    const int ub = __builtin_amdgcn_readlane(__float_as_int(cc.u[j]), ln);
                    u4 = lane == j ? ub : u4;
                    d += ca;
                    theta += cbt;
                    theta += d;
                    // the next batch's candidates, read while the last steps of this one run
                    // (late enough for the helpers, early enough to hide the LDS latency)
                    if (j == 1 && b + 1 < nb) fetch(g + 1u, nx, nb4, ntag);
                }
                if (!miss) {
                    up[lane < kFmBatch ? i0 + lane : kFmChunk + lane] = __int_as_float(u4);
                } else {         // an index left its window: redo the batch directly
#ifdef LDSP_TUNING
                    n_miss++;
#endif
                    theta = th0;
                    d = d0;
                    pe = pe0;
                    for (int j = 0; j < kFmBatch; j++) {
                        const float u = fm_step(sp[i0 + j], tab, theta, d, pe, alpha, beta);
                        up[(i0 + j) * (lane == 0) + uoff] = u;
                    }
                }
            }
            for (int i = nb * kFmBatch; i < cnt; i++) {
                const float u = fm_step(sp[i], tab, theta, d, pe, alpha, beta);
                up[i * (lane == 0) + uoff] = u;
            }
        } else if ((wave == 1 || wave == 2) && c < nch) {
            // helper wave - 1: entries lane + 64 (wave - 1) of every batch of this chunk
            const int hw = wave - 1;
            const int e = lane + 64 * hw;
            for (int b = 0; b < nb; b++) {
                const uint32_t g = g0 + (uint32_t)b;
                const uint32_t gs = g >= (uint32_t)kFmHor ? g - (uint32_t)kFmHor : 0u;   // state source batch
                const int sl = (int)(gs % kFmRing);
                if (__builtin_amdgcn_readfirstlane(lds_ld_u32(&sst[sl][3])) != gs + 1u) {
                    const uint64_t tw = wall_clock64();
                    bool late = false;
                    do {
#ifdef LDSP_TUNING
                        n_hwait++;
#endif
                        if (wall_clock64() - tw > kFmWaitTicks) {   // the chain steps this batch directly
                            late = true;
                            break;
                        }
                    } while (__builtin_amdgcn_readfirstlane(lds_ld_u32(&sst[sl][3])) != gs + 1u);
                    if (late) continue;
                }
                cbar();
                const uint32_t th = sst[sl][0], dd = sst[sl][1];
                const float pp = __uint_as_float(sst[sl][2]);
                const uint32_t h0 = (g - gs) * (uint32_t)kFmBatch;
                const int o = (int)(g % kFmRing);
                const uint32_t bse = fm_base(th, dd, pp, alpha, beta, h0 + (uint32_t)(e / kFmNC));
                float z, u;
                fm_eval(sp, b * kFmBatch, cnt, tab, bse, e, z, u);
                const int j = e / kFmNC, k = e % kFmNC;
                const double w = 0.001 * (double)z;
                cw[o][j][k] = w;
                cw[o][j][k + 32] = w;
                cu[o][j][k] = u;
                if (k == 0) cbase[o][j] = bse;
                cbar();
                if (lane == 0) lds_st_u32(&crdy[o][hw], g + 1u);
            }
        } else if (wave == 3) {
            const int nxt = 1 - cur;        // holds chunk c - 1 (results) and receives chunk c + 1
            const long pb = (c - 1) * kFmChunk, nbs = (c + 1) * kFmChunk;
            for (int i = lane; i < kFmChunk; i += 64) {
                if (c >= 1 && pb + i < n) {
                    const float x = sb[nxt][i], u = ub[nxt][i];
                    lo[pb + i] = x + u;
                    ro[pb + i] = x - u;
                }
                if (c + 1 < nch) sb[nxt][i] = nbs + i < n ? s[nbs + i] : 0.0f;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        st->theta = theta;
        st->dtheta = d;
        st->pe = pe;
    }
#ifdef LDSP_TUNING
    if (lane == 0 && wave < 3)
        printf("k_fm_pll wave %d: n %ld misses %u late %u spins %u helper_waits %u\n", wave, n, n_miss, n_late, n_spin,
               n_hwait);
#endif
}

__global__ void __launch_bounds__(256) k_interleave2(const float* __restrict__ a, const float* __restrict__ b, long n,
                                                     float2* __restrict__ y)
{
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) y[i] = make_float2(a[i], b[i]);
}

// AmpModem usb / lsb (liquid ampmodem_demod_ssb[_pll_carrier] -> firhilbf_c2r_execute,
// see oracle/liquid_restate.c): v1 = x[n - m] mixed down by the PLL's table index
// (cmul_down order), then per output
//   yi = re z[n - 2M],  yq = sum_j hq[j] im z[n - 4M + 1 + 2j]  (sequential, oldest first)
//   y  = 0.5f * (usb ? yi - yq : yi + yq) / mod_index
// over z = the 4M - 1 samples of history ++ this call's input.
__global__ void __launch_bounds__(256) k_ssb_v1(const uint32_t* __restrict__ idx, const float2* __restrict__ x,
                                                const float2* __restrict__ dhist, int m, const float* __restrict__ tab,
                                                long n, float2* __restrict__ v1)
{
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const float2 u = i >= m ? x[i - m] : dhist[i];
        const uint32_t k = idx[i] & 0x3ffu;
        const float sn = tab[k], cs = tab[(k + 256) & 0x3ffu];
        v1[i] = make_float2(u.x * cs - u.y * (-sn), u.x * (-sn) + u.y * cs);
    }
}

constexpr int kHilTile = 1024;        // outputs per workgroup
constexpr int kHilMaxM = 64;          // semi-length bound of the LDS tile

__global__ void __launch_bounds__(256) k_ssb_c2r(const float2* __restrict__ x, const float2* __restrict__ hist, long n,
                                                 const float* __restrict__ hq, int M, int usb, float mod_index,
                                                 float* __restrict__ y)
{
    __shared__ float2 z[kHilTile + 4 * kHilMaxM];
    __shared__ float h[2 * kHilMaxM];
    const int H = 4 * M - 1;              // history samples
    const long b0 = (long)blockIdx.x * kHilTile;
    const int cnt = (int)min((long)kHilTile, n - b0);
    for (int t = threadIdx.x; t < 2 * M; t += 256) h[t] = hq[t];
    for (int t = threadIdx.x; t < cnt + H; t += 256) {
        const long g = b0 - H + t;        // z index
        z[t] = g >= 0 ? x[g] : hist[g + H];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < cnt; t += 256) {
        // output b0 + t: z tile offset of sample n - k is t + H - k
        const float yi = z[t + H - 2 * M].x;
        float yq = 0.0f;
        for (int j = 0; j < 2 * M; j++) yq += h[j] * z[t + 2 * j].y;
        const float s = usb ? yi - yq : yi + yq;
        y[b0 + t] = 0.5f * s / mod_index;
    }
}

unsigned grid_for(size_t n) { return (unsigned)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 16384)); }

} // namespace

void bytes_to_iq(const void* x, void* y, size_t n, hipStream_t s)
{
    if (n == 0) return;
    LDSP_PROF(s, "k_bytes_to_iq");
    hipLaunchKernelGGL(k_bytes_to_iq, dim3(grid_for(n)), dim3(256), 0, s, (const short2*)x, (float2*)y, (long)n);
    LDSP_HIP(hipGetLastError());
}

void delay(bool cplx, const void* x, const void* hist, void* hist_out, size_t n, int D, void* y, hipStream_t s)
{
    const unsigned g = grid_for(std::max<size_t>(n, (size_t)D));
    LDSP_PROF(s, "k_delay");
    if (cplx)
        hipLaunchKernelGGL(k_delay<float2>, dim3(g), dim3(256), 0, s, (const float2*)x, (const float2*)hist,
                           (float2*)hist_out, (long)n, D, (float2*)y);
    else
        hipLaunchKernelGGL(k_delay<float>, dim3(g), dim3(256), 0, s, (const float*)x, (const float*)hist,
                           (float*)hist_out, (long)n, D, (float*)y);
    LDSP_HIP(hipGetLastError());
}

void ssb_v1(const void* idx, const void* x, const void* dhist, int m, const float* table, size_t n, void* v1,
            hipStream_t s)
{
    if (n == 0) return;
    LDSP_PROF(s, "k_ssb_v1");
    hipLaunchKernelGGL(k_ssb_v1, dim3(grid_for(n)), dim3(256), 0, s, (const uint32_t*)idx, (const float2*)x,
                       (const float2*)dhist, m, table, (long)n, (float2*)v1);
    LDSP_HIP(hipGetLastError());
}

void ssb_c2r(const void* x, const void* hist, size_t n, const float* hq, int M, int usb, float mod_index, float* y,
             hipStream_t s)
{
    if (n == 0) return;
    LDSP_REQUIRE(M >= 2 && M <= kHilMaxM, "ssb_c2r: Hilbert semi-length out of range");
    LDSP_PROF(s, "k_ssb_c2r");
    hipLaunchKernelGGL(k_ssb_c2r, dim3((unsigned)((n + kHilTile - 1) / kHilTile)), dim3(256), 0, s, (const float2*)x,
                       (const float2*)hist, (long)n, hq, M, usb, mod_index, y);
    LDSP_HIP(hipGetLastError());
}

void freqdem(const void* x, const void* prev, void* prev_out, size_t n, float ref, float* y, hipStream_t s)
{
    LDSP_PROF(s, "k_freqdem");
    hipLaunchKernelGGL(k_freqdem, dim3(grid_for(n)), dim3(256), 0, s, (const float2*)x, (const float2*)prev,
                       (float2*)prev_out, (long)n, ref, y);
    LDSP_HIP(hipGetLastError());
}

void fm_pll(const float* s, size_t n, FmState* st, const float* table, float* l, float* r, hipStream_t strm)
{
    if (n == 0) return;
    LDSP_PROF(strm, "k_fm_pll");
    hipLaunchKernelGGL(k_fm_pll, dim3(1), dim3(256), 0, strm, s, (long)n, st, table, l, r);
    LDSP_HIP(hipGetLastError());
}

void interleave2(const float* a, const float* b, size_t n, float* y, hipStream_t strm)
{
    if (n == 0) return;
    LDSP_PROF(strm, "k_interleave2");
    hipLaunchKernelGGL(k_interleave2, dim3(grid_for(n)), dim3(256), 0, strm, a, b, (long)n, (float2*)y);
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
