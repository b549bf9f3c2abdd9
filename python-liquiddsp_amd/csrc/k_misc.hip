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
constexpr int kFmCand = 16;      // candidate table indices per sample (64 lanes / kFmBatch)

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
// the input sample and the table index.  So wave 0 runs the chain in batches of
// kFmBatch samples and, beside batch b (in the same basic block, so the two
// instruction streams interleave), evaluates atan2 and u for batch b + 1 at
// kFmCand candidate indices per sample in its 64 lanes: indices around the
// trajectory extrapolated from the state at batch b's start with the phase error
// held (theta_h = theta + h (C(beta pe) + d) + C(alpha pe) h (h + 1) / 2).  The
// chain step then only looks its index up (readlane) -- the same bits the direct
// evaluation gives.  A batch in which some index falls outside its candidate
// window (a few per thousand batches on FM composite signals,
// scripts/analysis: fm_h2) is redone with the direct step from the saved state.
// Waves 1-3 store chunk c - 1's l / r and stream chunk c + 1 of s into the LDS
// double buffer while wave 0 walks chunk c.
struct FmCand {
    float z, u;          // this lane's atan2 and mixer output
    uint32_t base;       // first candidate index of this lane's sample
};

__device__ __forceinline__ FmCand fm_cands(const float* sp, int i0, int cnt, const float* tab, uint32_t theta,
                                           uint32_t d, float pe, float alpha, float beta, int h0, int lane)
{
    const int j = lane / kFmCand;
    const uint32_t h = (uint32_t)(h0 + j);
    const uint32_t ca = lm_constrain(pe * alpha), cb = lm_constrain(pe * beta);
    const uint32_t pred = theta + h * (cb + d) + ca * (h * (h + 1) / 2);
    FmCand c;
    c.base = (((pred + (1u << 21)) >> 22) - kFmCand / 2) & 0x3ffu;
    const uint32_t idx = (c.base + (uint32_t)(lane % kFmCand)) & 0x3ffu;
    const float x = sp[min(i0 + j, cnt - 1)];   // past the chunk's last batch: a value never used
    const float sn = tab[idx];
    const float cs = tab[(idx + 256) & 0x3ffu];
    const float r1 = x * cs - 0.0f * (-sn);
    const float i1 = x * (-sn) + 0.0f * cs;
    c.z = lm_atan2f_vsel(i1, r1);
    c.u = r1 * cs - i1 * (-sn);
    return c;
}

__global__ void __launch_bounds__(256) k_fm_pll(const float* __restrict__ s, long n, FmState* st,
                                                const float* __restrict__ table, float* __restrict__ lo,
                                                float* __restrict__ ro)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ float tab[1024];
    __shared__ float sb[2][kFmChunk + kFmBatch];
    __shared__ float ub[2][kFmChunk + 64];     // + 64: lanes 1..63 of wave 0 store their (identical) u here
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += 256) tab[i] = table[i];
    const long nch = (n + kFmChunk - 1) / kFmChunk;
    for (int i = tid; i < kFmChunk; i += 256) sb[0][i] = i < n ? s[i] : 0.0f;
    uint32_t theta = st->theta, d = st->dtheta;
    float pe = st->pe;
    const float alpha = st->alpha, beta = st->beta;
    __syncthreads();
    for (long c = 0; c <= nch; c++) {
        const int cur = (int)(c & 1);
        if (tid < 64 && c < nch) {
            const int lane = tid;
            const long base = c * kFmChunk;
            const int cnt = (int)min((long)kFmChunk, n - base);
            const float* sp = sb[cur];
            float* up = ub[cur];
            const int nb = cnt / kFmBatch;
            // lane 0 stores the chain's u; the other lanes store the same value past the chunk
            const int uoff = lane == 0 ? 0 : kFmChunk + lane;
            FmCand cc{};
            if (nb > 0) cc = fm_cands(sp, 0, cnt, tab, theta, d, pe, alpha, beta, 0, lane);
            for (int b = 0; b < nb; b++) {
                const int i0 = b * kFmBatch;
                // no branch around it: the candidates share a basic block with the chain steps
                const FmCand nx = fm_cands(sp, i0 + kFmBatch, cnt, tab, theta, d, pe, alpha, beta, kFmBatch, lane);
                const uint32_t th0 = theta, d0 = d;
                const float pe0 = pe;
                bool miss = false;
#pragma unroll
                for (int j = 0; j < kFmBatch; j++) {
                    const uint32_t idx = ((theta + (1u << 21)) >> 22) & 0x3ffu;
                    const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)cc.base, j * kFmCand);
                    const uint32_t off = (idx - bj) & 0x3ffu;
                    miss |= off >= (uint32_t)kFmCand;
                    const int ln = __builtin_amdgcn_readfirstlane(j * kFmCand + (int)(off & (kFmCand - 1)));
                    const float z = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cc.z), ln));
                    const float u = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cc.u), ln));
                    pe = (float)(0.999 * (double)pe + 0.001 * (double)z);
                    up[(i0 + j) * (lane == 0) + uoff] = u;
                    d += lm_constrain(pe * alpha);
                    theta += lm_constrain(pe * beta);
                    theta += d;
                }
                if (miss) {      // an index left its window: redo the batch directly
                    theta = th0;
                    d = d0;
                    pe = pe0;
                    for (int j = 0; j < kFmBatch; j++) {
                        const float u = fm_step(sp[i0 + j], tab, theta, d, pe, alpha, beta);
                        up[(i0 + j) * (lane == 0) + uoff] = u;
                    }
                }
                cc = nx;
            }
            for (int i = nb * kFmBatch; i < cnt; i++) {
                const float u = fm_step(sp[i], tab, theta, d, pe, alpha, beta);
                up[i * (lane == 0) + uoff] = u;
            }
        } else if (tid >= 64) {
            const int nxt = 1 - cur;        // holds chunk c - 1 (results) and receives chunk c + 1
            const long pb = (c - 1) * kFmChunk, nb = (c + 1) * kFmChunk;
            for (int i = tid - 64; i < kFmChunk; i += 192) {
                if (c >= 1 && pb + i < n) {
                    const float x = sb[nxt][i], u = ub[nxt][i];
                    lo[pb + i] = x + u;
                    ro[pb + i] = x - u;
                }
                if (c + 1 < nch) sb[nxt][i] = nb + i < n ? s[nb + i] : 0.0f;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        st->theta = theta;
        st->dtheta = d;
        st->pe = pe;
    }
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
