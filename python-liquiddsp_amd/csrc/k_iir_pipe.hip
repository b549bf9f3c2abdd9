// k_iir_pipe.hip -- exact (float32, bit-identical) SOS cascade for gfx950: the
// sequential recursion of k_iir_seq (reference src/iirfilter.hpp:292-298 ->
// iirfilt_crcf_execute_block -> iirfiltsos_execute_df2) with the sections of both
// components evaluated side by side in one wave.  Compiled without SLP
// vectorisation (Makefile): paired v_pk_mul_f32 / v_pk_add_f32 cost more
// operand moves than they save here.
#include "kernels.hpp"
#include "ldsp_common.hpp"

namespace ldsp {
namespace k {

namespace {

// Section-pipelined exact SOS cascade (the float32 recursion of k_iir_seq, the same
// operations in the same order): one lane per (component, section) -- lane 16 c + s
// -- so each VALU instruction advances every section of both components at once.
// Skewed by two steps per section: at step t lane s runs sample t - 2 s, and its
// input is lane s - 1's output of step t - 2 (a DPP row shift; the first lane of a
// row takes the input sample instead), so the cross-lane chain spans two steps and
// a step is ~11 instructions, issue-bound, instead of ~36 per component.  Wave 0
// steps; waves 1-3 stage input tiles into LDS (re / im planes) and store output
// tiles.  Fill and drain steps (a lane before its first or after its last sample)
// keep the lane's state unchanged.
constexpr int kPipeT = 2048;          // steps per tile (multiple of 8)
constexpr int kPipeThreads = 256;

struct PipeLane {
    float a1, a2, b0, b1, b2;
    float p1, p2, p3;                 // the section's v0 history (latest first)
    float y1, y2;                     // its outputs of the last two steps
};

template <bool CHECK>
__device__ __forceinline__ void pipe_step(PipeLane& L, float xin, int rel)
{
    // rel = t - 2 s: this lane's sample index (CHECK: the lane is active iff 0 <= rel < n, tested by the caller)
    const float in = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(xin), __float_as_int(L.y2), 0x111,
                                                                0xf, 0xf, false));
    const float v0 = (in - L.a1 * L.p1) - L.a2 * L.p2;
    const float y = (L.b0 * v0 + L.b1 * L.p1) + L.b2 * L.p2;
    if (CHECK && rel) {               // inactive lane: state unchanged (its output is never used)
        L.y2 = L.y1;
        L.y1 = y;
        return;
    }
    L.p3 = L.p2;
    L.p2 = L.p1;
    L.p1 = v0;
    L.y2 = L.y1;
    L.y1 = y;
}

__global__ void __launch_bounds__(kPipeThreads) k_iir_pipe(IirDesc d, const float* __restrict__ x, long n, int ncomp,
                                                           float* __restrict__ state, float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
    constexpr int R = 3 * kPipeT;                 // output ring (steps), see below
    __shared__ __attribute__((aligned(16))) float xin[2][2][kPipeT + 16];      // [tile parity][component][step - t0] (+ read-ahead padding)
    __shared__ __attribute__((aligned(16))) float yr[2][R];   // [component][step mod R]: the last lane's output
    __shared__ __attribute__((aligned(16))) float junk[64 * 8];   // the other lanes' output writes
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int L = d.nsos;
    const long D = 2 * (L - 1);                   // skew of the last section: sample t - D leaves it at step t
    const long nsteps = n + D;
    const long ntiles = (nsteps + kPipeT - 1) / kPipeT;
    const int fs = 3 * L;
    // staging waves: input tile k into xin[k & 1]; output sample r sits at ring
    // slot (r + D) mod R, so output tile j is complete after the barrier that
    // ends step tile j + 1, and is stored during tile j + 2
    auto stage_in = [&](long k) {
        const long base = k * kPipeT;
        for (int i = tid - 64; i < kPipeT; i += kPipeThreads - 64) {
            const long g = base + i;
            if (ncomp == 2) {
                const float2 v = g < n ? reinterpret_cast<const float2*>(x)[g] : make_float2(0.0f, 0.0f);
                xin[k & 1][0][i] = v.x;
                xin[k & 1][1][i] = v.y;
            } else {
                xin[k & 1][0][i] = g < n ? x[g] : 0.0f;
            }
        }
    };
    auto stage_out = [&](long j) {
        const long base = j * kPipeT;
        for (int i = tid - 64; i < kPipeT; i += kPipeThreads - 64) {
            const long g = base + i;
            if (g >= n) break;
            const long q = (g + D) % R;
            if (ncomp == 2)
                reinterpret_cast<float2*>(y)[g] = make_float2(yr[0][q], yr[1][q]);
            else
                y[g] = yr[0][q];
        }
    };
    const int c = lane >> 4, s = lane & 15;
    const bool mine = c < ncomp && s < L;         // a real (component, section) lane
    PipeLane P;
    {
        const int sc = s < L ? s : 0;
        P.a1 = s < L ? d.a[3 * sc + 1] : 0.0f;
        P.a2 = s < L ? d.a[3 * sc + 2] : 0.0f;
        P.b0 = s < L ? d.b[3 * sc] : 0.0f;
        P.b1 = s < L ? d.b[3 * sc + 1] : 0.0f;
        P.b2 = s < L ? d.b[3 * sc + 2] : 0.0f;
        const float* st = state + (c < ncomp ? c : 0) * fs + 3 * sc;
        P.p1 = mine ? st[0] : 0.0f;
        P.p2 = mine ? st[1] : 0.0f;
        P.p3 = mine ? st[2] : 0.0f;
        P.y1 = 0.0f;
        P.y2 = 0.0f;
    }
    if (wave != 0) stage_in(0);
    __syncthreads();
    const int cin = c < ncomp ? c : 0;
    const bool outl = mine && s == L - 1;
    const long D8 = (D + 7) / 8 * 8;
    for (long k = 0; k < ntiles; k++) {
        if (wave != 0) {
            if (k + 1 < ntiles) stage_in(k + 1);
            if (k >= 2) stage_out(k - 2);
        } else {
            const long t0 = k * kPipeT, t1 = min(nsteps, t0 + kPipeT);
            const float* xi = xin[k & 1][cin];
            float* ring = yr[outl ? c : 0];
            const long ro = t0 % R;                  // ring slot of step t0 (R is a multiple of kPipeT)
            // [fa, fb): 8-step groups in which every lane is active (D <= t and t < n)
            const long fa = max(t0, min(t1, D8));
            const long fb = fa + max(0l, (min(t1, n) - fa) / 8 * 8);
            auto check = [&](long t) {               // a fill / drain step: inactive lanes keep their state
                const long rel = t - 2 * s;
                pipe_step<true>(P, xi[t - t0], (rel < 0 || rel >= n) ? 1 : 0);
                if (outl) ring[ro + (t - t0)] = P.y1;
            };
            for (long t = t0; t < fa; t++) check(t);
            if (fa < fb) {
                const float4* ip = reinterpret_cast<const float4*>(xi + (fa - t0));
                float4* op = reinterpret_cast<float4*>(outl ? ring + ro + (fa - t0) : junk + lane * 8);
                const int ost = outl ? 2 : 0;
                float4 na = ip[0], nb = ip[1];
                for (long t = fa; t < fb; t += 8) {
                    const float4 ca = na, cb = nb;
                    na = ip[2];                      // the next group's inputs (padding covers the last)
                    nb = ip[3];
                    ip += 2;
                    float4 oa, ob;
                    pipe_step<false>(P, ca.x, 0);
                    oa.x = P.y1;
                    pipe_step<false>(P, ca.y, 0);
                    oa.y = P.y1;
                    pipe_step<false>(P, ca.z, 0);
                    oa.z = P.y1;
                    pipe_step<false>(P, ca.w, 0);
                    oa.w = P.y1;
                    pipe_step<false>(P, cb.x, 0);
                    ob.x = P.y1;
                    pipe_step<false>(P, cb.y, 0);
                    ob.y = P.y1;
                    pipe_step<false>(P, cb.z, 0);
                    ob.z = P.y1;
                    pipe_step<false>(P, cb.w, 0);
                    ob.w = P.y1;
                    op[0] = oa;
                    op[1] = ob;
                    op += ost;
                }
            }
            for (long t = fb; t < t1; t++) check(t);
        }
        __syncthreads();
    }
    if (wave != 0) {
        for (long j = max(0l, ntiles - 2); j < ntiles; j++) stage_out(j);
    } else if (mine) {
        float* st = state + c * fs + 3 * s;
        st[0] = P.p1;
        st[1] = P.p2;
        st[2] = P.p3;
    }
}

} // namespace

void iir_pipe(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, void* y, hipStream_t s)
{
    if (n == 0) return;
    LDSP_REQUIRE(d.sos && d.nsos >= 1 && d.nsos <= kIirPipeMaxSos, "iir_pipe: 1..8 second-order sections");
    LDSP_PROF(s, "k_iir_pipe");
    hipLaunchKernelGGL(k_iir_pipe, dim3(1), dim3(kPipeThreads), 0, s, d, (const float*)x, (long)n, cplx ? 2 : 1, state,
                       (float*)y);
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
