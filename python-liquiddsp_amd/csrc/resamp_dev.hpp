// resamp_dev.hpp -- the resampler's per-output arithmetic (liquid resamp_*_execute
// -> firpfb dot product, reference src/resampler.hpp:160-172), shared by the
// resampler kernels (k_fir.hip) and the IIR -> resampler fusion
// (k_iir_modal.hip), so both produce the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ldsp {
namespace k {

// smallest input index j with P0 + k*step - j*2^24 <= 0xffffff: output k's window ends at input j
__device__ __forceinline__ long resamp_j(uint64_t P0, uint64_t k, uint32_t step)
{
    const long long num = (long long)(P0 + k * (uint64_t)step) - 0xffffffLL;
    return num <= 0 ? 0 : (long)((num + 0xffffffLL) >> 24);
}

// the first output k whose window ends at or after input J (inverse of resamp_j)
__device__ __forceinline__ uint64_t resamp_kmin(uint64_t P0, long J, uint32_t step)
{
    const long long t = (long long)J * (1LL << 24) - 1 - (long long)P0;
    return t < 0 ? 0 : (uint64_t)t / step + 1;
}

// complex taps (cccf): C99 complex product, sequential accumulation
__device__ __forceinline__ void rs_mac(float2& r, float2 h, float2 v)
{
    r.x = r.x + (h.x * v.x - h.y * v.y);
    r.y = r.y + (h.x * v.y + h.y * v.x);
}

// real taps on complex samples (crcf): componentwise sequential accumulation
__device__ __forceinline__ void rs_mac_cr(float2& r, float h, float2 v)
{
    r.x = r.x + h * v.x;
    r.y = r.y + h * v.y;
}

} // namespace k
} // namespace ldsp
