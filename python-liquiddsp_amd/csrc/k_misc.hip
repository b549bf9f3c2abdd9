// k_misc.hip -- small streaming kernels for the rest of the receive-path API:
//   bytes_to_iq  (reference src/utility.hpp:61-69): int16 (I, Q) -> complex64 / 32767
//   Delay        (src/utility.hpp:5-57, wdelay read-then-push): y[n] = x[n - nd - 1]
//   FreqDem      (src/demod.hpp:189-219 -> freqdem_demodulate_block):
//                y[n] = cargf(conjf(x[n-1]) x[n]) * ref, ref = 1 / (2 pi kf)
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

} // namespace k
} // namespace ldsp
