// k_pll.hip -- exact AmpModem phase-locked loop on gfx950
// (ampmodem_demod_dsb_pll_carrier / ampmodem_demod_dsb_pll_costas behind
// reference src/demod.hpp:294 ampmodem_demodulate_block).
//
// Per sample n the loop does (nco_crcf mixer, 1024-entry table):
//   i_n = ((theta_n + 2^21) >> 22) & 1023
//   v0 = x0_n conj(e^{j2pi i_n/1024}),  v1 = x1_n conj(e^{j2pi i_n/1024})
//   phi = carg(v0) (carrier) | tanh(re v0) im v0 (Costas)
//   d_{n+1} = d_n + C(alpha phi);  theta_{n+1} = theta_n + C(beta phi) + d_{n+1}
//   out_n = re(v1) / mod_index
// The state (theta, d) is uint32 and enters the update only through the table
// index i_n.  So for two trajectories whose indices agree, the offset
// (dtheta, dd) between them evolves linearly: dd stays, dtheta grows by dd per
// sample.  Exact trajectories never coalesce (the quantised phase detector
// keeps a residual), so chunk-parallel speculation cannot be verified by state
// equality as for the AGC; instead:
//   k_pll_cand : every chunk of C samples runs W samples early from an
//                extrapolated state and records, per sample, its phase and the
//                kick / output differences of the neighbouring indices i-1, i+1;
//   k_pll_walk : one workgroup walks the chunks in order with the exact offset
//                of the true trajectory from the candidate; a 64-lane ballot
//                finds the next sample whose true index differs, only that
//                sample is recomputed (a table lookup of the recorded neighbour
//                for |di| = 1, the full loop step otherwise), the offset is
//                updated, and the output is patched.  Waves 1-3 stream the next
//                chunk's records into an LDS double buffer meanwhile.
// The result is bit-identical to the sequential loop (k_pll_seq, also used for
// short calls); ~2 % of samples need a repair on locked AM signals.
#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kChunk = 1024;      // candidate chunk = walker block
constexpr int kWarm = 2048;       // candidate warm-up

__device__ __forceinline__ uint32_t tidx(uint32_t th) { return ((th + (1u << 21)) >> 22) & 0x3ffu; }

struct PllIn {
    const float2* x0;     // lowpass(x)
    const float2* x;      // raw input (x1 = x delayed by m)
    const float2* hist;   // m samples before x[0]
    int m;
    const float* table;
    float mod_index;
    int costas;
};

__device__ __forceinline__ float2 x1_at(const PllIn& in, long n)
{
    const long g = n - in.m;
    return g >= 0 ? in.x[g] : in.hist[g + in.m];
}

// one evaluation of the phase detector at table index i
struct Kick {
    uint32_t k1, k2;
    float out;
};
__device__ __forceinline__ Kick pll_eval(const float* tab, uint32_t i, float2 u0, float2 u1, float alpha, float beta,
                                         float mod_index, int costas)
{
    const float sn = tab[i];
    const float cs = tab[(i + 256) & 0x3ffu];
    const float v0r = u0.x * cs - u0.y * (-sn);
    const float v0i = u0.x * (-sn) + u0.y * cs;
    const float v1r = u1.x * cs - u1.y * (-sn);
    const float phi = costas ? lm_tanhf(v0r) * v0i : lm_atan2f(v0i, v0r);
    Kick k;
    k.k1 = lm_constrain(phi * alpha);
    k.k2 = lm_constrain(phi * beta);
    k.out = v1r / mod_index;
    return k;
}

// ------------------------------------------------------------------ sequential
constexpr int kSeqChunk = 2048;

__global__ void __launch_bounds__(256) k_pll_seq(PllIn in, long n, AmpState* st, float* __restrict__ y)
{
    __shared__ float tab[1024];
    __shared__ float2 b0[kSeqChunk], b1[kSeqChunk];
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += 256) tab[i] = in.table[i];
    uint32_t theta = st->theta, d = st->dtheta;
    const float alpha = st->alpha, beta = st->beta;
    for (long base = 0; base < n; base += kSeqChunk) {
        const int cnt = (int)min((long)kSeqChunk, n - base);
        __syncthreads();
        for (int i = tid; i < cnt; i += 256) {
            b0[i] = in.x0[base + i];
            b1[i] = x1_at(in, base + i);
        }
        __syncthreads();
        if (tid == 0) {
            for (int i = 0; i < cnt; i++) {
                const Kick k = pll_eval(tab, tidx(theta), b0[i], b1[i], alpha, beta, in.mod_index, in.costas);
                d += k.k1;
                theta += k.k2 + d;
                y[base + i] = k.out;
            }
        }
    }
    if (tid == 0) {
        st->theta = theta;
        st->dtheta = d;
    }
}

// ------------------------------------------------------------------ candidates
// records (SoA, stride npad): th, dk1m, dk2m, dk1p, dk2p (uint32), om, op (float)
struct CandBuf {
    uint32_t* th;
    uint32_t* dk;         // [4][npad]: dk1(i-1), dk2(i-1), dk1(i+1), dk2(i+1)   (difference to index i)
    float* om;            // [2][npad]: output at i-1, i+1
    uint32_t* cs;         // [nch][2] candidate state at chunk start
    uint32_t* ce;         // [nch][2] candidate state at chunk end
    long npad;
};

__global__ void __launch_bounds__(64) k_pll_cand(PllIn in, long n, const AmpState* st, long nch, CandBuf cb,
                                                 float* __restrict__ y)
{
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) tab[i] = in.table[i];
    __syncthreads();
    const long k = (long)blockIdx.x * 64 + threadIdx.x;
    if (k >= nch) return;
    const long s0 = k * kChunk, s1 = min(n, s0 + kChunk);
    const float alpha = st->alpha, beta = st->beta;
    uint32_t theta = st->theta, d = st->dtheta;
    long w0 = s0 - kWarm;
    if (w0 <= 0) {
        w0 = 0;                                       // exact: from the true state
    } else {
        theta = st->theta + (uint32_t)((uint64_t)w0 * d);   // constant-frequency extrapolation
    }
    for (long i = w0; i < s0; i++) {
        const Kick kk = pll_eval(tab, tidx(theta), in.x0[i], x1_at(in, i), alpha, beta, in.mod_index, in.costas);
        d += kk.k1;
        theta += kk.k2 + d;
    }
    cb.cs[2 * k] = theta;
    cb.cs[2 * k + 1] = d;
    for (long i = s0; i < s1; i++) {
        const float2 u0 = in.x0[i], u1 = x1_at(in, i);
        const uint32_t ic = tidx(theta);
        const Kick kc = pll_eval(tab, ic, u0, u1, alpha, beta, in.mod_index, in.costas);
        const Kick km = pll_eval(tab, (ic - 1) & 0x3ffu, u0, u1, alpha, beta, in.mod_index, in.costas);
        const Kick kp = pll_eval(tab, (ic + 1) & 0x3ffu, u0, u1, alpha, beta, in.mod_index, in.costas);
        cb.th[i] = theta;
        cb.dk[i] = km.k1 - kc.k1;
        cb.dk[cb.npad + i] = km.k2 - kc.k2;
        cb.dk[2 * cb.npad + i] = kp.k1 - kc.k1;
        cb.dk[3 * cb.npad + i] = kp.k2 - kc.k2;
        cb.om[i] = km.out;
        cb.om[cb.npad + i] = kp.out;
        y[i] = kc.out;
        d += kc.k1;
        theta += kc.k2 + d;
    }
    cb.ce[2 * k] = theta;
    cb.ce[2 * k + 1] = d;
}

// ------------------------------------------------------------------ walker
struct WalkBuf {
    uint32_t th[kChunk];
    uint32_t dk[4][kChunk];
    float om[2][kChunk];
    uint32_t cs[2], ce[2];
};

__device__ __forceinline__ void walk_load(WalkBuf& b, const CandBuf& cb, long chunk, long n, int t, int nt)
{
    const long s0 = chunk * kChunk;
    const int cnt = (int)min((long)kChunk, n - s0);
    for (int i = t; i < cnt; i += nt) {
        b.th[i] = cb.th[s0 + i];
        b.dk[0][i] = cb.dk[s0 + i];
        b.dk[1][i] = cb.dk[cb.npad + s0 + i];
        b.dk[2][i] = cb.dk[2 * cb.npad + s0 + i];
        b.dk[3][i] = cb.dk[3 * cb.npad + s0 + i];
        b.om[0][i] = cb.om[s0 + i];
        b.om[1][i] = cb.om[cb.npad + s0 + i];
    }
    if (t == 0) {
        b.cs[0] = cb.cs[2 * chunk];
        b.cs[1] = cb.cs[2 * chunk + 1];
        b.ce[0] = cb.ce[2 * chunk];
        b.ce[1] = cb.ce[2 * chunk + 1];
    }
}

__global__ void __launch_bounds__(256) k_pll_walk(PllIn in, long n, AmpState* st, long nch, CandBuf cb,
                                                  float* __restrict__ y)
{
    __shared__ float tab[1024];
    __shared__ WalkBuf buf[2];
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    for (int i = tid; i < 1024; i += 256) tab[i] = in.table[i];
    walk_load(buf[0], cb, 0, n, tid, 256);
    __syncthreads();
    const float alpha = st->alpha, beta = st->beta;
    uint32_t th_t = st->theta, d_t = st->dtheta;      // true state at the current chunk start
    for (long c = 0; c < nch; c++) {
        const int cur = (int)(c & 1);
        if (wave != 0) {
            if (c + 1 < nch) walk_load(buf[cur ^ 1], cb, c + 1, n, tid - 64, 192);
        } else {
            const WalkBuf& b = buf[cur];
            const long s0 = c * kChunk;
            const int cnt = (int)min((long)kChunk, n - s0);
            uint32_t dth = th_t - b.cs[0];            // offset of the true trajectory (exact, mod 2^32)
            uint32_t dd = d_t - b.cs[1];
            int p = 0;                                // dth is the offset at local sample p
            for (int wb = 0; wb < cnt; wb += 64) {
                const int nl = wb + lane;
                const bool valid = nl < cnt;
                const uint32_t thc = valid ? b.th[nl] : 0u;
                const uint32_t ic = tidx(thc);
                while (true) {
                    const uint32_t pred = thc + dth + (uint32_t)(nl - p) * dd;
                    const bool mis = valid && nl >= p && tidx(pred) != ic;
                    const unsigned long long mask = __ballot(mis);
                    if (mask == 0) break;
                    const int j = __ffsll((long long)mask) - 1;
                    const int ns = wb + j;                                   // local sample to repair
                    const uint32_t thn = __builtin_amdgcn_readlane(thc, j);
                    const uint32_t dthn = dth + (uint32_t)(ns - p) * dd;     // offset at ns
                    const uint32_t it = tidx(thn + dthn), icn = tidx(thn);
                    const uint32_t di = (it - icn) & 0x3ffu;
                    uint32_t dk1, dk2;
                    float out;
                    if (di == 0x3ffu) {
                        dk1 = b.dk[0][ns];
                        dk2 = b.dk[1][ns];
                        out = b.om[0][ns];
                    } else if (di == 1u) {
                        dk1 = b.dk[2][ns];
                        dk2 = b.dk[3][ns];
                        out = b.om[1][ns];
                    } else {                                                 // rare: full step
                        const float2 u0 = in.x0[s0 + ns], u1 = x1_at(in, s0 + ns);
                        const Kick kt = pll_eval(tab, it, u0, u1, alpha, beta, in.mod_index, in.costas);
                        const Kick kc = pll_eval(tab, icn, u0, u1, alpha, beta, in.mod_index, in.costas);
                        dk1 = kt.k1 - kc.k1;
                        dk2 = kt.k2 - kc.k2;
                        out = kt.out;
                    }
                    if (lane == 0) y[s0 + ns] = out;
                    dth = dthn + dd + dk1 + dk2;
                    dd = dd + dk1;
                    p = ns + 1;
                }
            }
            // true state at the chunk end = candidate end + offset propagated to cnt
            th_t = b.ce[0] + dth + (uint32_t)(cnt - p) * dd;
            d_t = b.ce[1] + dd;
        }
        __syncthreads();
    }
    if (tid == 0) {
        st->theta = th_t;
        st->dtheta = d_t;
    }
}

__global__ void k_delay_hist(const float2* __restrict__ x, const float2* __restrict__ hist, float2* __restrict__ hist_out,
                             long n, int m)
{
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
        const long g = n - m + j;
        hist_out[j] = g >= 0 ? x[g] : hist[g + m];
    }
}

} // namespace

size_t pll_scratch_bytes(size_t n)
{
    const size_t nch = (n + kChunk - 1) / kChunk;
    const size_t npad = nch * kChunk;
    return npad * 4 * 7 + nch * 16 + 256;
}

void ampmodem_pll(const void* x0, const void* x, const void* hist, void* hist_out, int m, size_t n, AmpState* st,
                  const float* table, float mod_index, int costas, float* y, void* scratch, hipStream_t s)
{
    if (n == 0) return;
    PllIn in;
    in.x0 = (const float2*)x0;
    in.x = (const float2*)x;
    in.hist = (const float2*)hist;
    in.m = m;
    in.table = table;
    in.mod_index = mod_index;
    in.costas = costas;
    if (n < (size_t)4 * kWarm || scratch == nullptr) {
        hipLaunchKernelGGL(k_pll_seq, dim3(1), dim3(256), 0, s, in, (long)n, st, y);
        LDSP_HIP(hipGetLastError());
    } else {
        const long nch = (long)((n + kChunk - 1) / kChunk);
        CandBuf cb;
        cb.npad = nch * kChunk;
        char* p = (char*)scratch;
        cb.th = (uint32_t*)p;
        cb.dk = (uint32_t*)(p + (size_t)cb.npad * 4);
        cb.om = (float*)(p + (size_t)cb.npad * 4 * 5);
        cb.cs = (uint32_t*)(p + (size_t)cb.npad * 4 * 7);
        cb.ce = cb.cs + 2 * nch;
        hipLaunchKernelGGL(k_pll_cand, dim3((unsigned)((nch + 63) / 64)), dim3(64), 0, s, in, (long)n,
                           (const AmpState*)st, nch, cb, y);
        LDSP_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_pll_walk, dim3(1), dim3(256), 0, s, in, (long)n, st, nch, cb, y);
        LDSP_HIP(hipGetLastError());
    }
    // delay-line history for the next call (m samples); k_pll_* read the old one
    hipLaunchKernelGGL(k_delay_hist, dim3(1), dim3(64), 0, s, (const float2*)x, (const float2*)hist, (float2*)hist_out,
                       (long)n, m);
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
