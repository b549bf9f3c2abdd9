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
//   k_pll_cand : every chunk of 256 samples runs W samples early from an
//                extrapolated state and records, per sample, its phase and the
//                kick / output differences of the neighbouring indices i-1, i+1;
//   k_pll_walk : one workgroup walks 1024-sample blocks in order with the exact offset
//                of the true trajectory from the candidate; a 64-lane ballot
//                finds the next sample whose true index differs, only that
//                sample is recomputed (a table lookup of the recorded neighbour
//                for |di| = 1, the full loop step otherwise), the offset is
//                updated, and the output is patched.  Waves 1-7 stream the next
//                block's records into an LDS double buffer meanwhile.
// The result is bit-identical to the sequential loop (k_pll_seq, also used for
// short calls); ~2 % of samples need a repair on locked AM signals.
#include <cstdlib>

#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kBlk = 1024;        // walker block
constexpr int kCand = 256;        // candidate chunk
constexpr int kSub = kBlk / kCand;
constexpr int kWarm = 1024;       // candidate warm-up (locks the loop; 2048 gives no fewer repairs)

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

__global__ void __launch_bounds__(256) k_pll_seq(PllIn in, long n, AmpState* st, int gcur, float* __restrict__ y)
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
        st->gth[1 - gcur] = theta;     // exact: the next call's candidates start on the true state
        st->gd[1 - gcur] = d;
    }
}

// ------------------------------------------------------------------ candidates
// Candidate chunks are kCand samples; the walker consumes blocks of kBlk =
// kSub candidate chunks.  Records (AoS, 8 words = 32 B per sample, npad = nblk*kBlk):
//   th (candidate phase), u = (th + 2^21) mod 2^22 (position inside the table
//   cell), dk1(i-1), dk2(i-1), dk1(i+1), dk2(i+1) (kick differences to index
//   i), output at i-1, i+1 (float bits).
struct CandBuf {
    uint4* rec;           // [npad][2]
    uint32_t* cs;         // [nsub][2] candidate state at chunk start
    uint32_t* ce;         // [nsub][2] candidate state at chunk end
    unsigned long long* stats;   // walker counters: repairs, -, walk ticks, barrier-wait ticks
    long npad;
    int norep;            // timing experiment (LDSP_DEBUG_PLL=2, counting kernel only): skip every repair
};

__device__ __forceinline__ const float2* x1_ptr(const PllIn& in, long i)
{
    const long g = i - in.m;
    return g >= 0 ? in.x + g : in.hist + (g + in.m);
}

// Run the loop over [a, b) with the inputs software-pipelined kB samples ahead
// (the loads are off the theta dependence chain).  REC: record the candidate.
constexpr int kB = 8;
template <bool REC>
__device__ __forceinline__ void cand_run(const PllIn& in, const float* tab, long a, long b, float alpha, float beta,
                                         uint32_t& theta, uint32_t& d, const CandBuf& cb, float* __restrict__ y)
{
    if (a >= b) return;
    float2 n0[kB], n1[kB];
#pragma unroll
    for (int j = 0; j < kB; j++) {
        const long i = min(a + j, b - 1);
        n0[j] = in.x0[i];
        n1[j] = *x1_ptr(in, i);
    }
    for (long i = a; i < b; i += kB) {
        float2 c0[kB], c1[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) {
            c0[j] = n0[j];
            c1[j] = n1[j];
        }
        if (i + kB < b) {
#pragma unroll
            for (int j = 0; j < kB; j++) {
                const long ii = min(i + kB + j, b - 1);
                n0[j] = in.x0[ii];
                n1[j] = *x1_ptr(in, ii);
            }
        }
#pragma unroll
        for (int j = 0; j < kB; j++) {
            if (i + j < b) {
                const uint32_t ic = tidx(theta);
                const Kick kc = pll_eval(tab, ic, c0[j], c1[j], alpha, beta, in.mod_index, in.costas);
                if (REC) {
                    const long s = i + j;
                    const uint32_t jl = (uint32_t)(s & 63);
                    const Kick km = pll_eval(tab, (ic - 1) & 0x3ffu, c0[j], c1[j], alpha, beta, in.mod_index, in.costas);
                    const Kick kp = pll_eval(tab, (ic + 1) & 0x3ffu, c0[j], c1[j], alpha, beta, in.mod_index, in.costas);
                    const uint32_t d1m = km.k1 - kc.k1, d1p = kp.k1 - kc.k1;
                    cb.rec[2 * s] = make_uint4(theta + (1u << 21), __float_as_uint(kc.out), d1m, km.k2 - kc.k2 - jl * d1m);
                    cb.rec[2 * s + 1] = make_uint4(d1p, kp.k2 - kc.k2 - jl * d1p, __float_as_uint(km.out),
                                                   __float_as_uint(kp.out));
                }
                d += kc.k1;
                theta += kc.k2 + d;
            }
        }
    }
}

// Candidate chunk k starts `warm` samples early from the guess state (the
// previous call's last candidate end state, or the true state after a reset or a
// sequential call), extrapolated at constant frequency.  The guess is never the
// true state of a walk still in progress, so this kernel can overlap the
// previous call's walker; the walker carries the exact offset either way.
__global__ void __launch_bounds__(64) k_pll_cand(PllIn in, long n, AmpState* st, int gcur, long nchc, CandBuf cb,
                                                 float* __restrict__ y, int warm)
{
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) tab[i] = in.table[i];
    __syncthreads();
    const long k = (long)blockIdx.x * 64 + threadIdx.x;
    if (k >= nchc) return;
    const long s0 = k * kCand, s1 = min(n, s0 + kCand);
    const float alpha = st->alpha, beta = st->beta;
    const uint32_t g_th = st->gth[gcur];
    uint32_t d = st->gd[gcur];
    uint32_t theta = g_th;
    long w0 = s0 - warm;
    if (w0 <= 0) {
        w0 = 0;
    } else {
        theta = g_th + (uint32_t)((uint64_t)w0 * d);   // constant-frequency extrapolation
    }
    cand_run<false>(in, tab, w0, s0, alpha, beta, theta, d, cb, y);
    cb.cs[2 * k] = theta;
    cb.cs[2 * k + 1] = d;
    cand_run<true>(in, tab, s0, s1, alpha, beta, theta, d, cb, y);
    cb.ce[2 * k] = theta;
    cb.ce[2 * k + 1] = d;
    if (k == nchc - 1) {                 // guess for the next call (other slot: every thread read [gcur])
        st->gth[1 - gcur] = theta;
        st->gd[1 - gcur] = d;
    }
}

// ------------------------------------------------------------------ walker
struct WalkBuf {
    uint4 rec[kBlk * 2];
    uint32_t cs[kSub * 2], ce[kSub * 2];
};

constexpr int kWalkThreads = 512;
constexpr int kLoaders = kWalkThreads - 64;       // waves 1..7
constexpr int kVec = kBlk * 2;                    // uint4 per block
constexpr int kLoadSlots = (kVec + kLoaders - 1) / kLoaders;

struct LoadRegs {
    uint4 v[kLoadSlots];
    uint32_t w;
};

// Unconditional (clamped) loads: predicated loads into the same registers made
// the compiler serialise them with a vmcnt wait each, i.e. one HBM round trip
// per slot in every block.
__device__ __forceinline__ void walk_fetch(LoadRegs& r, const CandBuf& cb, long blk, int lt)
{
    const uint4* src = cb.rec + blk * kVec;
#pragma unroll
    for (int k = 0; k < kLoadSlots; k++) r.v[k] = src[min(lt + k * kLoaders, kVec - 1)];
    const int wi = min(lt, 4 * kSub - 1);
    const uint32_t* wsrc = wi < 2 * kSub ? cb.cs + blk * 2 * kSub + wi : cb.ce + blk * 2 * kSub + wi - 2 * kSub;
    r.w = *wsrc;
}

__device__ __forceinline__ void walk_store(WalkBuf& b, const LoadRegs& r, int lt)
{
#pragma unroll
    for (int k = 0; k < kLoadSlots; k++) {
        const int q = lt + k * kLoaders;
        if (q < kVec) b.rec[q] = r.v[k];
    }
    if (lt < 2 * kSub) b.cs[lt] = r.w;
    else if (lt < 4 * kSub) b.ce[lt - 2 * kSub] = r.w;
}

// LDS-DMA record streaming (global_load_lds_dwordx4: each lane's 16 B land at
// M0 + 16 lane, no VGPR staging, no compiler-inserted waits).  Loader wave w
// (0..6) moves the 1 KiB pieces w, w + 7, ... of a block's 32 KiB of records;
// wave 0 also moves the 2 x 8 chunk-state words.  Every loader wave issues
// the same number of DMAs per block (kDmaPer, padding with a repeat of its
// last piece), so one immediate s_waitcnt vmcnt covers the two blocks still
// in flight.
constexpr int kPieces = kBlk * 2 * 16 / 1024;              // 32
constexpr int kLoadWaves = kWalkThreads / 64 - 1;          // 7
constexpr int kDmaPer = (kPieces + kLoadWaves - 1) / kLoadWaves + 2;   // 5 pieces + 2 state DMAs
static_assert(kDmaPer == 7, "walker DMA wait count below assumes 7 DMAs per loader wave per block");

// M0 is compiler-reserved: save / set / restore it inside one statement
// (cdna_hip_programming.md LDS-DMA recipe); asm loads are invisible to hipcc's
// waitcnt bookkeeping, the walker counts them itself (s_waitcnt vmcnt(N)).
__device__ __forceinline__ void dma16(uint32_t lds_byte, const void* g)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds_byte)
                 : "memory");
}
__device__ __forceinline__ void dma4(uint32_t lds_byte, const void* g)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds_byte)
                 : "memory");
}

__device__ __forceinline__ void walk_dma(WalkBuf& b, const CandBuf& cb, long blk, int lw, int lane)
{
    const char* src = (const char*)(cb.rec + blk * kVec);
    const uint32_t base = (uint32_t)(uintptr_t)&b.rec[0];
#pragma unroll
    for (int t = 0; t < kDmaPer - 2; t++) {
        const int piece = min(lw + t * kLoadWaves, kPieces - 1);        // a repeat is harmless
        dma16(base + piece * 1024, src + piece * 1024 + lane * 16);
    }
    // chunk states: 8 cs words, 8 ce words (lanes 0..7; the instruction still counts once in vmcnt)
    const int wl = lane & 7;
    if (lane < 8) {
        dma4((uint32_t)(uintptr_t)&b.cs[0], cb.cs + blk * 2 * kSub + wl);
        dma4((uint32_t)(uintptr_t)&b.ce[0], cb.ce + blk * 2 * kSub + wl);
    }
}

// Inputs of the rare full step (true index more than one cell from the candidate's).
struct FullCtx {
    const float2* x0;
    const float2* x;
    const float2* hist;
    const float* table;
    int m, costas;
    float alpha, beta, mod_index;
    int norep;
};

// Kick differences and output of the true index (icand + t) at global sample sg;
// w = candidate theta + 2^21 (record word 0).
__device__ __noinline__ uint4 pll_full(FullCtx fc, uint32_t w, uint32_t t, long sg)
{
    const uint32_t ic = w >> 22;
    const uint32_t it = (ic + t) & 0x3ffu;
    const long g = sg - fc.m;
    const float2 u0 = fc.x0[sg], u1 = g >= 0 ? fc.x[g] : fc.hist[g + fc.m];
    const Kick kt = pll_eval(fc.table, it, u0, u1, fc.alpha, fc.beta, fc.mod_index, fc.costas);
    const Kick kc = pll_eval(fc.table, ic, u0, u1, fc.alpha, fc.beta, fc.mod_index, fc.costas);
    return make_uint4(kt.k1 - kc.k1, kt.k2 - kc.k2, __float_as_uint(kt.out), 0u);
}

__device__ __forceinline__ uint32_t rl(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }

// v + lane * dk1.  F24: every kick difference fits 24 signed bits (host check:
// |k1| <= alpha 2^31, so |dk1| < 2^23 when alpha <= 2^-9), one v_mad_i32_i24.
template <bool F24>
__device__ __forceinline__ uint32_t mad_lane(uint32_t lane, uint32_t dk1, uint32_t v)
{
    if (F24) {
        uint32_t r;
        asm volatile("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(lane), "s"(dk1), "v"(v));
        return r;
    }
    return v + lane * dk1;
}

// pout = lane is set in `bit` ? so : pout  (one v_cndmask_b32 with an SGPR lane mask)
__device__ __forceinline__ uint32_t sel_lane(uint32_t pout, uint32_t so, unsigned long long bit)
{
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(pout), "v"(so), "s"(bit));
    return r;
}

// Walker state per lane-block of 64 samples.  Record words (k_pll_cand):
//   R0 = (w = th + 2^21, candidate output, dk1(i-1), dk2'(i-1))
//   R1 = (dk1(i+1), dk2'(i+1), output(i-1), output(i+1))
// with dk2' = dk2 - (s mod 64) dk1, so that a repair at lane j adds
// dk2' + lane dk1 to the offset of every lane (only lanes > j matter).
// v = u + offset per lane, u = w mod 2^22 the candidate's position in its
// table cell: the true index equals the candidate's iff v < 2^22; it is one
// cell up iff 2^22 <= v < 2^23, one down iff v >= 2^32 - 2^22, else |di| > 1.

// Any-distance repair loop over the lanes in M, in order (block tails, the
// rare |di| > 1 samples): the direction is decided on the scalar unit and
// |di| > 1 re-evaluates the loop step (pll_full).  By value in and out: a
// reference would put the caller's registers on the stack.
struct WalkRegs {
    uint32_t v, pout, DD, nrep;
};
template <bool F24>
__device__ __noinline__ WalkRegs walk_generic(uint4 R0, uint4 R1, WalkRegs r, unsigned long long M, long sg0, int lane,
                                              FullCtx fc)
{
    uint32_t DD = __builtin_amdgcn_readfirstlane(r.DD);
    unsigned long long mask = __builtin_amdgcn_ballot_w64(r.v > 0x3fffffu) & M;
    while (mask != 0) {
        const int j = __builtin_ctzll(mask);
        const uint32_t vj = rl(r.v, j);
        uint32_t dk1, dk2p, ob;
        if (vj - 0x400000u < 0x400000u) {
            dk1 = rl(R1.x, j);
            dk2p = rl(R1.y, j);
            ob = rl(R1.w, j);
        } else if (vj >= 0xffc00000u) {
            dk1 = rl(R0.z, j);
            dk2p = rl(R0.w, j);
            ob = rl(R1.z, j);
        } else {
            const uint4 f = pll_full(fc, rl(R0.x, j), vj >> 22, sg0 + j);
            dk1 = __builtin_amdgcn_readfirstlane(f.x);
            dk2p = __builtin_amdgcn_readfirstlane(f.y) - (uint32_t)j * dk1;
            ob = __builtin_amdgcn_readfirstlane(f.z);
        }
        r.pout = lane == j ? ob : r.pout;
        r.v = mad_lane<F24>((uint32_t)lane, dk1, r.v) + dk2p;
        DD += dk1;
        r.nrep++;
        M &= (~0ull << j) << 1;
        mask = __builtin_amdgcn_ballot_w64(r.v > 0x3fffffu) & M;
    }
    r.DD = DD;
    return r;
}

// Full lane-block fast path, assuming every repaired lane is one cell away:
// per repair one ff1, three direction selects, two readlanes, two lane selects
// (the output, and v at the repair for the check below), a 24-bit
// multiply-add and an add for the offsets, one ballot.  Afterwards one ballot
// over the repaired lanes checks that assumption; if any was |di| > 1 (rare:
// loop unlocked) the whole block is redone by walk_generic from its start.
template <bool F24, bool STATS>
__device__ __forceinline__ void walk_block(const uint4& R0, const uint4& R1, uint32_t& v, uint32_t& DD, float* yb,
                                           long sg0, int lane, const FullCtx& fc, unsigned& nrep)
{
    const uint32_t v_in = v, dd_in = DD;
    uint32_t pout = R0.y, vrep = 0;
    unsigned long long PM = 0;
    unsigned long long mask = __builtin_amdgcn_ballot_w64(v > 0x3fffffu);
    if (STATS && fc.norep) mask = 0;
    unsigned cnt = 0;
    while (mask != 0) {
        const int j = __builtin_ctzll(mask);
        const bool upl = v < 0x800000u;                               // one cell up (else down)
        const uint32_t s1 = upl ? R1.x : R0.z;
        const uint32_t s2 = upl ? R1.y : R0.w;
        const uint32_t so = upl ? R1.w : R1.z;
        const uint32_t dk1 = rl(s1, j), dk2p = rl(s2, j);
        const unsigned long long bit = 1ull << j;
        pout = sel_lane(pout, so, bit);
        vrep = sel_lane(vrep, v, bit);
        PM |= bit;
        v = mad_lane<F24>((uint32_t)lane, dk1, v) + dk2p;
        DD += dk1;
        if (STATS) cnt++;
        mask = __builtin_amdgcn_ballot_w64(v > 0x3fffffu) & ((~0ull << j) << 1);
    }
    if (__builtin_expect((__builtin_amdgcn_ballot_w64(vrep + 0x400000u > 0xbfffffu) & PM) != 0, 0)) {
        WalkRegs r{v_in, R0.y, dd_in, nrep};
        r = walk_generic<F24>(R0, R1, r, ~0ull, sg0, lane, fc);
        v = r.v;
        pout = r.pout;
        DD = __builtin_amdgcn_readfirstlane(r.DD);
        if (STATS) nrep = __builtin_amdgcn_readfirstlane(r.nrep);
    } else if (STATS) {
        nrep += cnt;
    }
    yb[lane] = __uint_as_float(pout);
}

__device__ __forceinline__ void load_sub(uint4 (&D)[4][2], const WalkBuf& b, int sub, int lane)
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = sub * kCand + q * 64 + lane;
        D[q][0] = b.rec[2 * i];
        D[q][1] = b.rec[2 * i + 1];
    }
}

// The four lane-blocks of one candidate chunk.
template <bool F24, bool STATS>
__device__ __forceinline__ void walk_sub(const uint4 (&D)[4][2], int sub, uint32_t& off, uint32_t& DD, float* yb, long s0,
                                         int lane, const FullCtx& fc, unsigned& nrep)
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int base = sub * kCand + q * 64;
        const uint32_t u = D[q][0].x & 0x3fffffu;
        uint32_t v = u + off;
        if (STATS && fc.norep >= 2) {
            if (fc.norep == 2) yb[base + lane] = __uint_as_float(D[q][0].y);
            off = v - u + 64u * DD;
            continue;
        }
        walk_block<F24, STATS>(D[q][0], D[q][1], v, DD, yb + base, s0 + base, lane, fc, nrep);
        off = v - u + 64u * DD;
    }
}

// Wave 0 walks block c; waves 1-7 DMA the records of block c + 3 into the LDS
// ring meanwhile.  Per lane the walker carries off = the exact offset of the
// true trajectory from the current candidate chunk at its sample (affine in
// the lane: K + lane DD), DD = the frequency offset (wave-uniform).
template <bool F24, bool STATS>
__global__ void __launch_bounds__(kWalkThreads) k_pll_walk(PllIn in, long n, AmpState* st, long nblk, CandBuf cb,
                                                           float* __restrict__ y)
{
    __shared__ WalkBuf buf[4];           // ring: block c in buf[c & 3], DMA'd three blocks ahead
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: keeps the walk on SALU
    const int lane = tid & 63;
    const int lw = wave - 1;             // loader wave index 0..6
    if (wave != 0) {
        for (long b0 = 0; b0 < 3 && b0 < nblk; b0++) walk_dma(buf[b0], cb, b0, lw, lane);
        // block 0 landed: at most the DMAs of blocks 1 and 2 still in flight
        if (nblk > 2) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        else if (nblk > 1) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    FullCtx fc;
    fc.x0 = in.x0;
    fc.x = in.x;
    fc.hist = in.hist;
    fc.table = in.table;
    fc.m = in.m;
    fc.costas = in.costas;
    fc.alpha = st->alpha;
    fc.beta = st->beta;
    fc.mod_index = in.mod_index;
    fc.norep = STATS ? cb.norep : 0;
    uint32_t th_t = st->theta, d_t = st->dtheta;      // true state at the current block start
    unsigned long long cyc_walk = 0, cyc_wait = 0;
    unsigned nrep = 0;
    for (long c = 0; c < nblk; c++) {
        const unsigned long long t0 = STATS ? wall_clock64() : 0;
        if (wave != 0) {
            // slot (c + 3) & 3 held block c - 1, released by the previous barrier
            if (c + 3 < nblk) walk_dma(buf[(c + 3) & 3], cb, c + 3, lw, lane);
            // block c + 1 must have landed before the barrier below publishes it
            if (c + 3 < nblk) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
            else if (c + 2 < nblk) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            const WalkBuf& b = buf[c & 3];
            const long s0 = c * kBlk;
            const int cnt = (int)min((long)kBlk, n - s0);
            float* yb = y + s0;
            // candidate chunk start / end states of the block (cs[0..7], ce[0..7]) in one LDS read
            const uint32_t csce = lane < 2 * kSub ? b.cs[lane] : (lane < 4 * kSub ? b.ce[lane - 2 * kSub] : 0u);
            uint32_t DD = d_t - rl(csce, 1);
            uint32_t off = th_t - rl(csce, 0) + (uint32_t)lane * DD;
            uint4 D0[4][2], D1[4][2];
            load_sub(D0, b, 0, lane);
            int last = 0;
            if (cnt == kBlk) {
#pragma unroll
                for (int sub = 0; sub < kSub; sub++) {
                    if (sub > 0) {                                  // next candidate chunk: rebase the offset
                        const uint32_t dth = rl(csce, 2 * kSub + 2 * sub - 2) - rl(csce, 2 * sub);
                        const uint32_t dd = rl(csce, 2 * kSub + 2 * sub - 1) - rl(csce, 2 * sub + 1);
                        off += dth + (uint32_t)lane * dd;
                        DD += dd;
                    }
                    if (sub & 1) {
                        if (sub + 1 < kSub) load_sub(D0, b, sub + 1, lane);
                        walk_sub<F24, STATS>(D1, sub, off, DD, yb, s0, lane, fc, nrep);
                    } else {
                        if (sub + 1 < kSub) load_sub(D1, b, sub + 1, lane);
                        walk_sub<F24, STATS>(D0, sub, off, DD, yb, s0, lane, fc, nrep);
                    }
                }
                last = kSub - 1;
            } else {
                for (int sub = 0; sub * kCand < cnt; sub++) {
                    if (sub > 0) {
                        const uint32_t dth = rl(csce, 2 * kSub + 2 * sub - 2) - rl(csce, 2 * sub);
                        const uint32_t dd = rl(csce, 2 * kSub + 2 * sub - 1) - rl(csce, 2 * sub + 1);
                        off += dth + (uint32_t)lane * dd;
                        DD += dd;
                    }
                    load_sub(D0, b, sub, lane);
                    for (int q = 0; q < 4; q++) {
                        const int base = sub * kCand + q * 64;
                        const int nvalid = min(64, cnt - base);
                        if (nvalid <= 0) break;
                        const uint32_t u = D0[q][0].x & 0x3fffffu;
                        uint32_t v = u + off;
                        const unsigned long long M = nvalid == 64 ? ~0ull : ((1ull << nvalid) - 1ull);
                        WalkRegs r{v, D0[q][0].y, DD, nrep};
                        r = walk_generic<F24>(D0[q][0], D0[q][1], r, M, s0 + base, lane, fc);
                        v = r.v;
                        DD = __builtin_amdgcn_readfirstlane(r.DD);
                        nrep = __builtin_amdgcn_readfirstlane(r.nrep);
                        if (lane < nvalid) yb[base + lane] = __uint_as_float(r.pout);
                        off = v - u + (uint32_t)nvalid * DD;
                    }
                    last = sub;
                }
            }
            // true state at the block end = candidate end + offset there (lane 0 of off)
            th_t = b.ce[2 * last] + __builtin_amdgcn_readfirstlane(off);
            d_t = b.ce[2 * last + 1] + DD;
        }
        // LDS-only barrier: __syncthreads() would also drain the loaders' global fetch of
        // block c + 2 (vmcnt(0)), putting an HBM round trip into every block
        const unsigned long long t1 = STATS ? wall_clock64() : 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (STATS) {
            const unsigned long long t2 = wall_clock64();
            cyc_walk += t1 - t0;
            cyc_wait += t2 - t1;
        }
    }
    if (tid == 0) {
        st->theta = th_t;
        st->dtheta = d_t;
        if (STATS) {
            cb.stats[0] = nrep;
            cb.stats[1] = 0;
            cb.stats[2] = cyc_walk;
            cb.stats[3] = cyc_wait;
        }
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
    const size_t nblk = (n + kBlk - 1) / kBlk;
    const size_t npad = nblk * kBlk;
    return npad * 32 + nblk * kSub * 16 + 256;
}

size_t pll_stats_offset(size_t n)
{
    const size_t nblk = (n + kBlk - 1) / kBlk;
    return nblk * kBlk * 32 + nblk * kSub * 16;
}

bool pll_parallel(size_t n) { return n >= (size_t)4 * kWarm; }

static PllIn pll_in(const PllCall& c)
{
    PllIn in;
    in.x0 = (const float2*)c.x0;
    in.x = (const float2*)c.x;
    in.hist = (const float2*)c.hist;
    in.m = c.m;
    in.table = c.table;
    in.mod_index = c.mod_index;
    in.costas = c.costas;
    return in;
}

static CandBuf cand_buf(const PllCall& c)
{
    const long nblk = (long)((c.n + kBlk - 1) / kBlk);
    CandBuf cb;
    cb.npad = nblk * kBlk;
    char* p = (char*)c.scratch;
    cb.rec = (uint4*)p;
    cb.cs = (uint32_t*)(p + (size_t)cb.npad * 32);
    cb.ce = cb.cs + 2 * nblk * kSub;
    cb.stats = (unsigned long long*)(p + pll_stats_offset(c.n));
    static const int dbg = std::getenv("LDSP_DEBUG_PLL") ? std::atoi(std::getenv("LDSP_DEBUG_PLL")) : 0;
    cb.norep = dbg >= 2 ? dbg - 1 : 0;     // 2: skip repairs; 3: skip the lane-block walk; 4: 3 without stores
    return cb;
}

void pll_front(const PllCall& c, hipStream_t s)
{
    if (c.n == 0) return;
    // delay-line history for the next call (m samples); this call's kernels read the old one
    {
        LDSP_PROF(s, "k_delay_hist");
        hipLaunchKernelGGL(k_delay_hist, dim3(1), dim3(64), 0, s, (const float2*)c.x, (const float2*)c.hist,
                           (float2*)c.hist_out, (long)c.n, c.m);
    }
    LDSP_HIP(hipGetLastError());
    if (!pll_parallel(c.n)) return;
    const long nchc = (long)((c.n + kCand - 1) / kCand);
    {
        LDSP_PROF(s, "k_pll_cand");
        static const int warm = std::getenv("LDSP_PLL_WARM") ? std::atoi(std::getenv("LDSP_PLL_WARM")) : kWarm;
        hipLaunchKernelGGL(k_pll_cand, dim3((unsigned)((nchc + 63) / 64)), dim3(64), 0, s, pll_in(c), (long)c.n, c.st,
                           c.gcur, nchc, cand_buf(c), c.y, warm);
    }
    LDSP_HIP(hipGetLastError());
}

void pll_back(const PllCall& c, hipStream_t s)
{
    if (c.n == 0) return;
    if (!pll_parallel(c.n)) {
        {
            LDSP_PROF(s, "k_pll_seq");
            hipLaunchKernelGGL(k_pll_seq, dim3(1), dim3(256), 0, s, pll_in(c), (long)c.n, c.st, c.gcur, c.y);
        }
        LDSP_HIP(hipGetLastError());
        return;
    }
    const long nblk = (long)((c.n + kBlk - 1) / kBlk);
    {
        LDSP_PROF(s, "k_pll_walk");
        static const bool stats = std::getenv("LDSP_DEBUG_PLL") != nullptr;
        const dim3 g(1), blk(kWalkThreads);
        const PllIn in = pll_in(c);
        const CandBuf cb = cand_buf(c);
        if (c.alpha_host <= 1.0f / 512.0f) {
            if (stats) hipLaunchKernelGGL((k_pll_walk<true, true>), g, blk, 0, s, in, (long)c.n, c.st, nblk, cb, c.y);
            else hipLaunchKernelGGL((k_pll_walk<true, false>), g, blk, 0, s, in, (long)c.n, c.st, nblk, cb, c.y);
        } else {
            if (stats) hipLaunchKernelGGL((k_pll_walk<false, true>), g, blk, 0, s, in, (long)c.n, c.st, nblk, cb, c.y);
            else hipLaunchKernelGGL((k_pll_walk<false, false>), g, blk, 0, s, in, (long)c.n, c.st, nblk, cb, c.y);
        }
    }
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
