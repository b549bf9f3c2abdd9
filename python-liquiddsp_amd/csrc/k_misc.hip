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

// Per sample (demod.hpp:61-79; nco_crcf_mix_down with the 1024-entry table):
//   (r1, i1) = (s + 0j) e^{-j theta};  pe = (float)(0.999 pe + 0.001 atan2(i1, r1))
//   (r2, i2) = (r1, i1) e^{-j theta};  dtheta += C(alpha pe); theta += C(beta pe) + dtheta
//   l = s + r2, r = s - r2
// The chain theta -> index -> atan2 -> pe -> C() -> theta is walked by one
// lane (~130 dependent instructions per sample).  Evaluating atan2 for the
// next sample at the 64 indices around the predicted one in the other lanes
// (the prediction theta + dtheta is within 3 cells here) was measured slower:
// the compiler cannot interleave the two instruction streams of one wave.
// Waves 1-3 store chunk c - 1's l / r and stream chunk c + 1 of s into the
// LDS double buffer while lane 0 walks chunk c.
__global__ void __launch_bounds__(256) k_fm_pll(const float* __restrict__ s, long n, FmState* st,
                                                const float* __restrict__ table, float* __restrict__ lo,
                                                float* __restrict__ ro)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ float tab[1024];
    __shared__ float sb[2][kFmChunk];
    __shared__ float ub[2][kFmChunk];
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
        if (tid == 0 && c < nch) {
            const long base = c * kFmChunk;
            const int cnt = (int)min((long)kFmChunk, n - base);
            const float* sp = sb[cur];
            float* up = ub[cur];
            for (int i = 0; i < cnt; i++) {
                const float x = sp[i];
                const uint32_t idx = ((theta + (1u << 21)) >> 22) & 0x3ffu;
                const float sn = tab[idx];
                const float cs = tab[(idx + 256) & 0x3ffu];
                const float r1 = x * cs - 0.0f * (-sn);
                const float i1 = x * (-sn) + 0.0f * cs;
                pe = (float)(0.999 * (double)pe + 0.001 * (double)lm_atan2f(i1, r1));
                up[i] = r1 * cs - i1 * (-sn);
                d += lm_constrain(pe * alpha);
                theta += lm_constrain(pe * beta);
                theta += d;
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
