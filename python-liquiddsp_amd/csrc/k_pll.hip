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
//                extrapolated state and records, per sample, its phase word
//                and output (the neighbouring index a repair needs is evaluated
//                later, by k_pll_entries, and only at the entries); in carrier
//                mode it also builds the walker's offset model (the chunk scan,
//                cand_scan_fold), which Costas calls run as k_pll_scan;
//   k_pll_walk : one workgroup walks 1024-sample blocks in order with the exact offset
//                of the true trajectory from the candidate; a 64-lane ballot
//                finds the next sample whose true index differs, only that
//                sample is recomputed (a table lookup of the recorded neighbour
//                for |di| = 1, the full loop step otherwise), the offset is
//                updated, and the output is patched.  Waves 1-7 stream the next
//                block's records into an LDS double buffer meanwhile.
// The result is bit-identical to the sequential loop (k_pll_seq, also used for
// short calls); ~2 % of samples need a repair on locked AM signals.
#include <atomic>
#include <cstdlib>
#include <random>

#include "batch.hpp"
#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

constexpr int kCand = 256;        // candidate chunk
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
    int out_idx;          // SSB carrier: the sample's table index (as float bits) is its output
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
                                         float mod_index, int costas, int out_idx)
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
    k.out = out_idx ? __uint_as_float(i) : v1r / mod_index;
    return k;
}

// After a launch's state stores (one thread): release them, then advance the
// hand-off epoch (AmpState::wepoch) that an early-launched walker waits on.
// Monotonic (atomic max): a predecessor that publishes after its successor timed
// out waiting for it cannot move the epoch backwards.
__device__ __forceinline__ void amp_publish(AmpState* st, uint32_t next)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_max(&st->wepoch, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ sequential
constexpr int kSeqChunk = 2048;

template <bool COSTAS>
__device__ __forceinline__ void k_pll_seq_body(PllIn in, long n, AmpState* st, int gcur, float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
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
                const Kick k = pll_eval(tab, tidx(theta), b0[i], b1[i], alpha, beta, in.mod_index, COSTAS ? 1 : 0, in.out_idx);
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
        amp_publish(st, st->wepoch + 1u);
    }
}
struct PllSeqArgs {
    PllIn in;
    long n;
    AmpState* st;
    int gcur;
    float* y;
};

template <bool COSTAS>
__global__ void __launch_bounds__(256) k_pll_seq(PllSeqArgs a) { k_pll_seq_body<COSTAS>(a.in, a.n, a.st, a.gcur, a.y); }
template <bool COSTAS>
__global__ void __launch_bounds__(256) k_pll_seq_many(::ldsp::Many<PllSeqArgs> m)
{
    const PllSeqArgs& a = m.a[blockIdx.y];
    k_pll_seq_body<COSTAS>(a.in, a.n, a.st, a.gcur, a.y);
}


// Carrier-mode sequential loop with candidate kicks (the technique of
// k_fm_pll, k_misc.hip): a step's kicks and output are a function of the
// sample and the table index only, so wave 0 evaluates them for the next batch
// of kSqBatch samples at kSqCand indices each (around the trajectory
// extrapolated with the last kicks held) beside the current batch's steps, and
// a step is an index lookup plus two adds.  A step whose index leaves its
// window is evaluated with pll_eval.  Same bits as k_pll_seq.
constexpr int kSqBatch = 4;
constexpr int kSqCand = 16;

struct SqCand {
    uint32_t k1, k2, base;
    float out;
};

__device__ __forceinline__ SqCand sq_cands(const float2* b0, const float2* b1, int i0, int cnt, const float* tab,
                                           uint32_t theta, uint32_t d, uint32_t k1h, uint32_t k2h, float alpha,
                                           float beta, float mod_index, int out_idx, int h0, int lane)
{
    const int j = lane / kSqCand;
    const uint32_t h = (uint32_t)(h0 + j);
    const uint32_t pred = theta + h * (k2h + d) + k1h * (h * (h + 1) / 2);
    SqCand c;
    c.base = (tidx(pred) - kSqCand / 2) & 0x3ffu;
    const uint32_t i = (c.base + (uint32_t)(lane % kSqCand)) & 0x3ffu;
    const int q = min(i0 + j, cnt - 1);      // past the chunk's last batch: a value never used
    const float2 u0 = b0[q], u1 = b1[q];
    const float sn = tab[i];
    const float cs = tab[(i + 256) & 0x3ffu];
    const float v0r = u0.x * cs - u0.y * (-sn);
    const float v0i = u0.x * (-sn) + u0.y * cs;
    const float v1r = u1.x * cs - u1.y * (-sn);
    const float phi = lm_atan2f_vsel(v0i, v0r);
    c.k1 = lm_constrain(phi * alpha);
    c.k2 = lm_constrain(phi * beta);
    c.out = out_idx ? __uint_as_float(i) : v1r / mod_index;
    return c;
}

__device__ __forceinline__ void k_pll_seqc_body(PllIn in, long n, AmpState* st, int gcur, float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ float tab[1024];
    __shared__ float2 b0[kSeqChunk], b1[kSeqChunk];
    __shared__ float ob[kSeqChunk + 64];      // + 64: lanes 1..63 of wave 0 store their (identical) outputs here
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += 256) tab[i] = in.table[i];
    uint32_t theta = st->theta, d = st->dtheta;
    uint32_t k1h = 0, k2h = 0;                // the last step's kicks (the prediction holds them)
    const float alpha = st->alpha, beta = st->beta;
    for (long base = 0; base < n; base += kSeqChunk) {
        const int cnt = (int)min((long)kSeqChunk, n - base);
        __syncthreads();
        for (int i = tid; i < cnt; i += 256) {
            b0[i] = in.x0[base + i];
            b1[i] = x1_at(in, base + i);
        }
        __syncthreads();
        if (tid < 64) {
            const int lane = tid;
            const int ooff = lane == 0 ? 0 : kSeqChunk + lane;
            const int nb = cnt / kSqBatch;
            SqCand cc{};
            uint32_t nredo = 0;
            if (nb > 0)
                cc = sq_cands(b0, b1, 0, cnt, tab, theta, d, k1h, k2h, alpha, beta, in.mod_index, in.out_idx, 0, lane);
            for (int b = 0; b < nb; b++) {
                const int i0 = b * kSqBatch;
                const SqCand nx = sq_cands(b0, b1, i0 + kSqBatch, cnt, tab, theta, d, k1h, k2h, alpha, beta,
                                           in.mod_index, in.out_idx, kSqBatch, lane);
                // A sample whose index left its window is evaluated directly and the
                // batch goes on from the state it gives (scripts/analysis/pll_predict.py:
                // a third of the batches miss at horizons 4..7 on the bench signal, mostly
                // in their last samples, so re-running whole batches cost ~4x the misses).
                bool miss = false;
#pragma unroll
                for (int j = 0; j < kSqBatch; j++) {
                    const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)cc.base, j * kSqCand);
                    const uint32_t off = (tidx(theta) - bj) & 0x3ffu;
                    float o;
                    if (off < (uint32_t)kSqCand) {
                        const int ln = __builtin_amdgcn_readfirstlane(j * kSqCand + (int)off);
                        k1h = (uint32_t)__builtin_amdgcn_readlane((int)cc.k1, ln);
                        k2h = (uint32_t)__builtin_amdgcn_readlane((int)cc.k2, ln);
                        o = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cc.out), ln));
                    } else {
                        miss = true;
                        const Kick k = pll_eval(tab, tidx(theta), b0[i0 + j], b1[i0 + j], alpha, beta, in.mod_index, 0,
                                                    in.out_idx);
                        k1h = k.k1;
                        k2h = k.k2;
                        o = k.out;
                    }
                    d += k1h;
                    theta += k2h + d;
                    ob[(i0 + j) * (lane == 0) + ooff] = o;
                }
                nredo += miss ? 1u : 0u;
                cc = nx;
            }
            for (int i = nb * kSqBatch; i < cnt; i++) {
                const Kick k = pll_eval(tab, tidx(theta), b0[i], b1[i], alpha, beta, in.mod_index, 0, in.out_idx);
                d += k.k1;
                theta += k.k2 + d;
                k1h = k.k1;
                k2h = k.k2;
                ob[i * (lane == 0) + ooff] = k.out;
            }
            if (tid == 0) {
                st->sq_batches += (uint32_t)nb;
                st->sq_redone += nredo;
            }
        }
        __syncthreads();
        for (int i = tid; i < cnt; i += 256) y[base + i] = ob[i];
    }
    if (tid == 0) {
        st->theta = theta;
        st->dtheta = d;
        st->gth[1 - gcur] = theta;     // exact: the next call's candidates start on the true state
        st->gd[1 - gcur] = d;
        amp_publish(st, st->wepoch + 1u);
    }
}

struct PllSeqcArgs {
    PllIn in;
    long n;
    AmpState* st;
    int gcur;
    float* y;
};
__device__ __forceinline__ void k_pll_seqc_run(const PllSeqcArgs& a) { k_pll_seqc_body(a.in, a.n, a.st, a.gcur, a.y); }
LDSP_KERNEL_PAIR(k_pll_seqc, PllSeqcArgs, k_pll_seqc_run, 256)


// ------------------------------------------------------------------ candidates
// Candidate chunks of kCand samples.  Per sample the candidate kernel writes
// its output to y and its phase word w = theta + 2^21 (4 B; the table index is
// w >> 22), and per chunk its start / end state and its entry count (see the
// walker).  The kicks at the candidate's index and at the neighbouring index
// i -+ 1 -- what a repair substitutes -- are evaluated by k_pll_entries for the
// entries only (~1/4 of the samples, in parallel): the candidate's serial loop
// does one phase-detector evaluation per sample, and stores 8 B per sample (it
// stored a 16-B record (w, k1, k2, out) until round 6: 67 MB per 1.6 M samples
// for this kernel and 66 MB for k_pll_entries, which read it back).
constexpr int kBlkE = 512;        // walker block: entries
struct CandBuf {
    uint32_t* rw;         // [npad] candidate phase word w = theta + 2^21 per sample
    uint32_t* eout;       // [nblkE][kBlkE] candidate output at each entry (the undo of a failed walker block)
    uint32_t* cs;         // [nchc][2] candidate state at chunk start
    uint32_t* ce;         // [nchc][2] candidate state at chunk end
    uint32_t* cnt;        // [nchc] entries per chunk
    uint32_t* eoff;       // [nchc] index of the chunk's first entry
    uint32_t* pth;        // [nchc] P_theta(k)   (walker offset model, below)
    uint32_t* pd;         // [nchc] P_d(k)
    uint32_t* ne;         // total entries
    uint32_t* hk;         // [nchc] Costas: chunk k's candidate locked half a turn from chunk 0's (re-run)
    uint32_t* bbase;      // [nblkE] S_blk: sample base of walker block c
    uint4* ent;           // [nblkE][2][kBlkE] entry records
    unsigned long long* stats;   // walker counters (LDSP_DEBUG_PLL)
    unsigned long long* lb;      // [nchc / 64][2][3] the folded scan's look-back granules {value, epoch}
    uint32_t ep;          // this call's look-back epoch (never 0)
    long nchc;
    int costas;           // Costas phase detector (two stable points half a turn apart)
    uint32_t B;           // risky margin (table-cell units of 2^-22)
    int dbg;              // 0; 1 counters; 2 counters + every lane-block through the generic path; 3 no repairs (timing)
};

__device__ __forceinline__ bool risky(uint32_t w, uint32_t B) { return ((w + B) & 0x3fffffu) < 2u * B; }

__device__ __forceinline__ const float2* x1_ptr(const PllIn& in, long i)
{
    const long g = i - in.m;
    return g >= 0 ? in.x + g : in.hist + (g + in.m);
}

// Run the loop over [a, b) with the inputs software-pipelined kB samples ahead
// (the loads are off the theta dependence chain), whole batches without a
// per-sample bound check (in a one-wave chain each exec-mask branch costs
// several issue slots per sample), then the tail.  REC: record the candidate,
// write its output, count the chunk's entries.
constexpr int kB = 8;
template <bool REC>
__device__ __forceinline__ void cand_step(const PllIn& in, const float* tab, long s, long a, long b, float2 c0,
                                          float2 c1, float alpha, float beta, uint32_t& theta, uint32_t& d,
                                          const CandBuf& cb, uint32_t& rec, float& yo, uint32_t& nent)
{
    const uint32_t ic = tidx(theta);
    const Kick kc = pll_eval(tab, ic, c0, c1, alpha, beta, in.mod_index, in.costas, in.out_idx);
    if (REC) {
        const uint32_t w = theta + (1u << 21);
        rec = w;
        yo = kc.out;
        nent += (risky(w, cb.B) || s == a || s == b - 1) ? 1u : 0u;
    }
    d += kc.k1;
    theta += kc.k2 + d;
}

template <bool REC>
__device__ __forceinline__ void cand_run(const PllIn& in, const float* tab, long a, long b, float alpha, float beta,
                                         uint32_t& theta, uint32_t& d, const CandBuf& cb, float* __restrict__ y,
                                         uint32_t& nent)
{
    if (a >= b) return;
    const long full = a + (b - a) / kB * kB;
    float2 n0[kB], n1[kB];
#pragma unroll
    for (int j = 0; j < kB; j++) {
        const long i = min(a + j, b - 1);
        n0[j] = in.x0[i];
        n1[j] = *x1_ptr(in, i);
    }
    long i = a;
    for (; i < full; i += kB) {
        float2 c0[kB], c1[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) {
            c0[j] = n0[j];
            c1[j] = n1[j];
        }
#pragma unroll
        for (int j = 0; j < kB; j++) {
            const long ii = min(i + kB + j, b - 1);
            n0[j] = in.x0[ii];
            n1[j] = *x1_ptr(in, ii);
        }
        // REC: the group's phase words and outputs are kept in registers and
        // stored back to back after it, so each lane's 32 B of each reach L2 as
        // whole pieces (stored one sample at a time, ~1 us apart, the partly
        // written lines were evicted by the streaming kernels beside this one
        // and reached HBM several times over).
        uint32_t r0[kB];
        float yo[kB];
#pragma unroll
        for (int j = 0; j < kB; j++)
            cand_step<REC>(in, tab, i + j, a, b, c0[j], c1[j], alpha, beta, theta, d, cb, r0[j], yo[j], nent);
        if (REC) {
#pragma unroll
            for (int j = 0; j < kB; j++) cb.rw[i + j] = r0[j];
#pragma unroll
            for (int j = 0; j < kB; j++) y[i + j] = yo[j];
        }
    }
    for (; i < b; i++) {
        uint32_t r0;
        float yo;
        cand_step<REC>(in, tab, i, a, b, in.x0[i], *x1_ptr(in, i), alpha, beta, theta, d, cb, r0, yo, nent);
        if (REC) {
            cb.rw[i] = r0;
            y[i] = yo;
        }
    }
}

// Approximate loop step for the carrier candidates' warm-up (never for a
// record or an output).  Its only product is chunk k's start state, a guess the
// walker corrects through the exact offset whatever it is (a candidate from an
// exact warm-up is itself only a guess: its offset from the true trajectory
// settles at ~2^17 and never reaches 0), so the warm-up
// needs the loop's dynamics, not its bits: the same table cell (the loop's
// quantisation, which sets where it settles), hardware sin / cos of that cell's
// angle for the table entries, a minimax atan2 (|error| < 1e-5 rad: a kick
// error of ~2^8 phase units against the 2^19 margin), and float -> int
// conversions for constrain (|phi beta| / 2pi < 1/2, so the wrap of a negative
// kick is the int32 -> uint32 conversion).  ~25 dependent instructions a step
// instead of ~110 for the exact one (atan2 alone ~70).
__device__ __forceinline__ float atan2_approx(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mn * __builtin_amdgcn_rcpf(mx > 0.0f ? mx : 1.0f);
    const float s = a * a;
    float r = fmaf(fmaf(fmaf(-0.0464964749f, s, 0.15931422f), s, -0.327622764f), s * a, a);
    r = ay > ax ? 1.57079637f - r : r;
    r = x < 0.0f ? 3.14159274f - r : r;
    return y < 0.0f ? -r : r;
}

__device__ __forceinline__ void cand_warm_approx(const PllIn& in, long a, long b, float alpha, float beta,
                                                 uint32_t& theta, uint32_t& d)
{
    if (a >= b) return;
    constexpr float kRadToPhase = 683565275.57643158f;      // 2^32 / (2 pi)
    const float as = alpha * kRadToPhase, bs = beta * kRadToPhase;
    const long full = a + (b - a) / kB * kB;
    float2 nx[kB];
#pragma unroll
    for (int j = 0; j < kB; j++) nx[j] = in.x0[min(a + j, b - 1)];
    long i = a;
    for (; i < full; i += kB) {
        float2 cx[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) cx[j] = nx[j];
#pragma unroll
        for (int j = 0; j < kB; j++) nx[j] = in.x0[min(i + kB + j, b - 1)];
#pragma unroll
        for (int j = 0; j < kB; j++) {
            const float ang = (float)tidx(theta) * 6.1359231515e-03f;      // 2 pi / 1024
            const float sn = __sinf(ang), cs = __cosf(ang);
            // v0 = x0 conj(e^{j ang})
            const float v0r = fmaf(cx[j].x, cs, cx[j].y * sn), v0i = fmaf(cx[j].y, cs, -(cx[j].x * sn));
            const float phi = atan2_approx(v0i, v0r);
            d += (uint32_t)(int)(phi * as);
            theta += (uint32_t)(int)(phi * bs) + d;
        }
    }
    for (; i < b; i++) {
        const float2 c = in.x0[i];
        const float ang = (float)tidx(theta) * 6.1359231515e-03f;
        const float sn = __sinf(ang), cs = __cosf(ang);
        const float v0r = fmaf(c.x, cs, c.y * sn), v0i = fmaf(c.y, cs, -(c.x * sn));
        const float phi = atan2_approx(v0i, v0r);
        d += (uint32_t)(int)(phi * as);
        theta += (uint32_t)(int)(phi * bs) + d;
    }
}

// Candidate chunk k starts `warm` samples early from the guess state (the
// previous call's last candidate end state, or the true state after a reset or a
// sequential call), extrapolated at constant frequency.  The guess is never the
// true state of a walk still in progress, so this kernel can overlap the
// previous call's walker; the walker carries the exact offset either way.
// from_true: start from the true state instead of the guess (Costas, whose
// front waits for the previous walk: chunk 0 is then the true trajectory's branch).
// The carrier chunk scan (k_pll_scan with flip 0, below) folded into this
// kernel: one launch fewer per call.  The scan's term for chunk k,
//     dd_k = ce_d[k-1] - cs_d[k],  c_k = (ce_th[k-1] - k K ce_d[k-1]) - (cs_th[k] - k K cs_d[k])
// (K = kCand), splits into a part of chunk k - 1's end state and a part of
// chunk k's start state, so chunk j contributes E_j = (cnt_j, ce_d[j],
// ce_th[j] - (j + 1) K ce_d[j]) to every LATER chunk's prefix and I_j = (0,
// -cs_d[j], (j K) cs_d[j] - cs_th[j]) (j > 0) to its own and later ones:
//     eoff[k] = sum_{j<k} E.cnt,  P_d(k) = sum_{j<k} E.d + sum_{j<=k} I.d,  P_th likewise.
// A workgroup's 64 chunks (its lanes) thus reduce to one aggregate without its
// neighbours' states; workgroups chain the aggregates with a decoupled
// look-back over {value, epoch} granules (the k_iir_modal protocol: a granule
// counts only when its tag is this call's epoch), the lanes reading 64
// predecessors at a time.  All additions are mod 2^32, as in k_pll_scan, so
// the order of the sums does not change a bit.  A predecessor is dispatched
// before its successor, so the wait ends; it is bounded anyway (wait_ticks,
// then the state is flagged like a walker's timed-out wait).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)v, d);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v += (uint32_t)__shfl_xor((int)v, d);
    return v;
}

__device__ __forceinline__ void cand_scan_fold(AmpState* st, const CandBuf& cb, long k, bool valid, uint32_t nent,
                                               uint32_t cs_th, uint32_t cs_d, uint32_t ce_th, uint32_t ce_d)
{
    const int lane = (int)threadIdx.x;
    const long b = blockIdx.x;
    uint32_t e0 = 0, e1 = 0, e2 = 0, i1 = 0, i2 = 0;
    if (valid) {
        e0 = nent;
        e1 = ce_d;
        e2 = ce_th - (uint32_t)((k + 1) * kCand) * ce_d;
        if (k > 0) {
            i1 = 0u - cs_d;
            i2 = (uint32_t)(k * kCand) * cs_d - cs_th;
        }
    }
    const uint32_t s0 = wave_incl_scan(e0, lane), s1 = wave_incl_scan(e1, lane), s2 = wave_incl_scan(e2, lane);
    const uint32_t t1 = wave_incl_scan(i1, lane), t2 = wave_incl_scan(i2, lane);
    const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)s0, 63);
    const uint32_t g1 = (uint32_t)__builtin_amdgcn_readlane((int)(s1 + t1), 63);
    const uint32_t g2 = (uint32_t)__builtin_amdgcn_readlane((int)(s2 + t2), 63);
    const unsigned long long tag = (unsigned long long)cb.ep << 32;
    unsigned long long* const rec = cb.lb + (size_t)b * 6;      // [0..2] aggregate, [3..5] inclusive prefix
    if (lane == 0) {
        __hip_atomic_store(rec + 0, tag | g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rec + 1, tag | g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rec + 2, tag | g2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint32_t p0 = 0, p1 = 0, p2 = 0;      // the prefix of every earlier workgroup
    if (b > 0) {
        long j0 = b - 1;
        const unsigned long long tw = wall_clock64(), wmax = st->wait_ticks;
        for (;;) {
            // lane i: workgroup j0 - i; both of its records in one round trip, and
            // only a lane that has neither polls again
            const long j = j0 - lane;
            uint32_t v0 = 0, v1 = 0, v2 = 0;
            int s = j >= 0 ? 0 : 3;                      // before chunk 0: an inclusive zero
            bool first = true;
            for (;;) {
                if (s == 0) {
                    // the first read takes both records; a re-poll only the aggregate
                    // (a predecessor publishes it first), with a pause long enough
                    // that waiting lanes do not load the memory system the
                    // concurrent kernels stream through
                    const unsigned long long* r = cb.lb + (size_t)j * 6;
                    unsigned long long q[6];
#pragma unroll
                    for (int e = 0; e < 3; e++) q[e] = __hip_atomic_load(r + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (first) {
#pragma unroll
                        for (int e = 3; e < 6; e++) q[e] = __hip_atomic_load(r + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (first && (q[3] >> 32) == cb.ep && (q[4] >> 32) == cb.ep && (q[5] >> 32) == cb.ep) {
                        s = 2;
                        v0 = (uint32_t)q[3], v1 = (uint32_t)q[4], v2 = (uint32_t)q[5];
                    } else if ((q[0] >> 32) == cb.ep && (q[1] >> 32) == cb.ep && (q[2] >> 32) == cb.ep) {
                        s = 1;
                        v0 = (uint32_t)q[0], v1 = (uint32_t)q[1], v2 = (uint32_t)q[2];
                    }
                }
                first = false;
                const unsigned long long inc = __builtin_amdgcn_ballot_w64(s >= 2);
                const int f = inc ? __builtin_ctzll(inc) : 64;
                const unsigned long long need = f == 64 ? ~0ull : ((1ull << f) - 1ull);
                if (!(__builtin_amdgcn_ballot_w64(s == 0) & need)) break;
                if (wall_clock64() - tw > wmax) break;
                __builtin_amdgcn_s_sleep(32);
            }
            const unsigned long long inc = __builtin_amdgcn_ballot_w64(s >= 2);
            const int f = inc ? __builtin_ctzll(inc) : 64;
            if (__builtin_amdgcn_ballot_w64(s == 0) & (f == 64 ? ~0ull : ((1ull << f) - 1ull))) {   // timed out
                if (lane == 0) {
                    st->werr = 1u;
                    if (st->herr) __hip_atomic_store(st->herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                break;
            }
            const bool take = lane <= f;                 // aggregates before the first inclusive prefix, and it
            p0 += wave_sum_u32(take ? v0 : 0u);
            p1 += wave_sum_u32(take ? v1 : 0u);
            p2 += wave_sum_u32(take ? v2 : 0u);
            if (f < 64) break;
            j0 -= 64;
        }
    }
    if (lane == 0) {
        __hip_atomic_store(rec + 3, tag | (p0 + g0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rec + 4, tag | (p1 + g1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(rec + 5, tag | (p2 + g2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!valid) return;
    const uint32_t ea = p0 + s0 - e0;
    cb.eoff[k] = ea;
    cb.pd[k] = p1 + (s1 - e1) + t1;
    cb.pth[k] = p2 + (s2 - e2) + t2;
    const uint32_t blk = (ea + kBlkE - 1) / kBlkE;     // first walker block starting at or after ea
    if ((uint64_t)blk * kBlkE < (uint64_t)ea + nent) cb.bbase[blk] = (uint32_t)(k * kCand);
    if (k == cb.nchc - 1) *cb.ne = ea + nent;
}

__device__ __forceinline__ void cand_chunk(PllIn in, long n, AmpState* st, int gcur, CandBuf cb, float* __restrict__ y,
                                           int warm, int from_true, int approx, const float* tab, long k,
                                           uint32_t& nent, uint32_t& cs_th, uint32_t& cs_d, uint32_t& ce_th,
                                           uint32_t& ce_d);

__device__ __forceinline__ void k_pll_cand_body(PllIn in, long n, AmpState* st, int gcur, CandBuf cb,
                                                 float* __restrict__ y, int warm, int from_true, int approx, int fold)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) tab[i] = in.table[i];
    __syncthreads();
    const long k = (long)blockIdx.x * 64 + threadIdx.x;
    const bool valid = k < cb.nchc;
    uint32_t nent = 0, cs_th = 0, cs_d = 0, ce_th = 0, ce_d = 0;
    if (valid) cand_chunk(in, n, st, gcur, cb, y, warm, from_true, approx, tab, k, nent, cs_th, cs_d, ce_th, ce_d);
    if (fold) cand_scan_fold(st, cb, k, valid, nent, cs_th, cs_d, ce_th, ce_d);   // the whole wave, converged
}

// Chunk k's candidate (k_pll_cand_body): start / end state and entry count.
__device__ __forceinline__ void cand_chunk(PllIn in, long n, AmpState* st, int gcur, CandBuf cb, float* __restrict__ y,
                                           int warm, int from_true, int approx, const float* tab, long k,
                                           uint32_t& nent, uint32_t& cs_th, uint32_t& cs_d, uint32_t& ce_th,
                                           uint32_t& ce_d)
{
    const long s0 = k * kCand, s1 = min(n, s0 + kCand);
    const float alpha = st->alpha, beta = st->beta;
    const uint32_t g_th = from_true ? st->theta : st->gth[gcur];
    uint32_t d = from_true ? st->dtheta : st->gd[gcur];
    uint32_t theta = g_th;
    long w0 = s0 - warm;
    if (w0 <= 0) {
        w0 = 0;
    } else {
        theta = g_th + (uint32_t)((uint64_t)w0 * d);   // constant-frequency extrapolation
    }
    if (approx) cand_warm_approx(in, w0, s0, alpha, beta, theta, d);
    else cand_run<false>(in, tab, w0, s0, alpha, beta, theta, d, cb, y, nent);
    cb.cs[2 * k] = theta;
    cb.cs[2 * k + 1] = d;
    cs_th = theta, cs_d = d;
    cand_run<true>(in, tab, s0, s1, alpha, beta, theta, d, cb, y, nent);
    cb.ce[2 * k] = theta;
    cb.ce[2 * k + 1] = d;
    cb.cnt[k] = nent;
    ce_th = theta, ce_d = d;
    if (k == cb.nchc - 1) {              // guess for the next call (other slot: every thread read [gcur])
        st->gth[1 - gcur] = theta;
        st->gd[1 - gcur] = d;
    }
}

struct PllCandArgs {
    PllIn in;
    long n;
    AmpState* st;
    int gcur;
    CandBuf cb;
    float* y;
    int warm;
    int from_true;
    int approx;
    int fold;             // carrier: the chunk scan (k_pll_scan, flip 0) folded in
};
__device__ __forceinline__ void k_pll_cand_run(const PllCandArgs& a) { k_pll_cand_body(a.in, a.n, a.st, a.gcur, a.cb, a.y, a.warm, a.from_true, a.approx, a.fold); }
LDSP_KERNEL_PAIR(k_pll_cand, PllCandArgs, k_pll_cand_run, 64)


// Costas: re-run the chunks the first scan marked (hk) from their start state
// turned by half a turn, so every candidate sits in chunk 0's branch.
__device__ __forceinline__ void k_pll_reflip_body(PllIn in, long n, AmpState* st, CandBuf cb, float* __restrict__ y)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) tab[i] = in.table[i];
    __syncthreads();
    const long k = (long)blockIdx.x * 64 + threadIdx.x;
    if (k >= cb.nchc || cb.hk[k] == 0u) return;
    const long s0 = k * kCand, s1 = min(n, s0 + kCand);
    uint32_t theta = cb.cs[2 * k] + (1u << 31), d = cb.cs[2 * k + 1];
    cb.cs[2 * k] = theta;
    uint32_t nent = 0;
    cand_run<true>(in, tab, s0, s1, st->alpha, st->beta, theta, d, cb, y, nent);
    cb.ce[2 * k] = theta;
    cb.ce[2 * k + 1] = d;
    cb.cnt[k] = nent;
}

struct PllReflipArgs {
    PllIn in;
    long n;
    AmpState* st;
    CandBuf cb;
    float* y;
};
__device__ __forceinline__ void k_pll_reflip_run(const PllReflipArgs& a) { k_pll_reflip_body(a.in, a.n, a.st, a.cb, a.y); }
LDSP_KERNEL_PAIR(k_pll_reflip, PllReflipArgs, k_pll_reflip_run, 64)


// ------------------------------------------------------------------ walker offset model
// The true trajectory T and chunk k's candidate C_k (samples [b_k, b_k + 256))
// differ by f(s) = T_theta(s) - C_k,theta(s) (uint32).  While their table
// indices agree, f grows by the constant frequency offset per sample; at a
// chunk boundary it jumps by ce[k-1] - cs[k]; a sample whose true index
// differs (a repair, kick differences dk1, dk2) adds dk2 + (s - r) dk1 to
// every later f(s).  So, globally,
//     f(s) = K + s D + A(s),   A(s) = P_theta(k) + s P_d(k)   (k = chunk of s)
// with P_d(k) = sum_{k' <= k} (ce[k'-1].d - cs[k'].d),
//      P_theta(k) = sum_{k' <= k} (ce[k'-1].theta - cs[k'].theta - b_k' (ce[k'-1].d - cs[k'].d)),
// and (K, D) changed only by repairs: K += dk2 - r dk1, D += dk1.  The true
// index equals the candidate's iff u(s) + f(s) < 2^22 (u = w mod 2^22, the
// candidate's position in its table cell).
//
// Sparse walk: a sample whose u lies at least B from both cell edges ("safe")
// cannot differ while |f(s)| <= B.  The walker visits only the other samples
// ("entries": the risky ones plus the first and last sample of every chunk).
// Between two consecutive entries p < e of one chunk f is affine with the
// values f_post(p) (after p's repair, if any) and f_pre(e) at its ends, so
// |f| <= B holds on the whole gap iff it holds at both ends -- which the walker
// checks wherever a gap is non-empty; if a check fails the lane-block is
// redone sample by sample (walk_fallback).  The result is the sequential
// loop's, bit for bit.

// Exclusive scan over chunks (one workgroup): entry offsets, P_theta, P_d,
// the total entry count and the sample base of every walker block.
// Costas (phase error tanh(re v0) im v0) locks to either of two points half a
// turn apart, and independently warmed-up candidates pick one at random.  With
// flip = 1 the scan only marks, in hk[k], the chunks an odd number of
// near-half-turn boundary jumps away from chunk 0 (k_pll_reflip re-runs them
// from their start state + pi, a genuine trajectory in chunk 0's branch), and a
// second scan with flip = 0 builds the model.  (The sine table is not exactly
// odd, so a half-turn-shifted candidate cannot stand in for a re-run.)
__device__ __forceinline__ uint32_t half_flip(uint32_t dth, int flip)
{
    return flip ? ((dth + (1u << 30)) >> 31) : 0u;
}

// 256 threads (4 waves): a 1024-thread workgroup needs 16 free wave slots on one
// CU, which a full-GPU filter launch on another stream keeps taking -- with 8
// batched channels the scan waited up to 3 ms for a CU (scripts/batched_timeline.py).
constexpr int kScanT = 256;
__device__ __forceinline__ void k_pll_scan_body(CandBuf cb, int flip)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ uint32_t sa[kScanT], sb[kScanT], sc[kScanT], sh[kScanT];
    const int t = threadIdx.x;
    const long per = (cb.nchc + kScanT - 1) / kScanT;
    const long k0 = min(cb.nchc, (long)t * per), k1 = min(cb.nchc, k0 + per);
    uint32_t a = 0, b = 0, c = 0, h = 0;
    // (unrolled: the loads of later chunks issue before the sums of earlier ones)
#pragma unroll 8
    for (long k = k0; k < k1; k++) {
        a += cb.cnt[k];
        if (k > 0) {
            const uint32_t dd = cb.ce[2 * k - 1] - cb.cs[2 * k + 1];
            const uint32_t dth = cb.ce[2 * k - 2] - cb.cs[2 * k];
            const uint32_t fl = half_flip(dth, flip);
            b += dd;
            c += dth - (fl << 31) - (uint32_t)(k * kCand) * dd;
            h ^= fl;
        }
    }
    sa[t] = a;
    sb[t] = b;
    sc[t] = c;
    sh[t] = h;
    __syncthreads();
    for (int off = 1; off < kScanT; off <<= 1) {        // inclusive Hillis-Steele
        const uint32_t pa = t >= off ? sa[t - off] : 0u, pb = t >= off ? sb[t - off] : 0u,
                       pc = t >= off ? sc[t - off] : 0u, ph = t >= off ? sh[t - off] : 0u;
        __syncthreads();
        sa[t] += pa;
        sb[t] += pb;
        sc[t] += pc;
        sh[t] ^= ph;
        __syncthreads();
    }
    uint32_t ea = sa[t] - a, eb = sb[t] - b, ec = sc[t] - c, eh = sh[t] ^ h;     // exclusive
#pragma unroll 8
    for (long k = k0; k < k1; k++) {
        if (k > 0) {
            const uint32_t dd = cb.ce[2 * k - 1] - cb.cs[2 * k + 1];
            const uint32_t dth = cb.ce[2 * k - 2] - cb.cs[2 * k];
            const uint32_t fl = half_flip(dth, flip);
            eb += dd;
            ec += dth - (fl << 31) - (uint32_t)(k * kCand) * dd;
            eh ^= fl;
        }
        cb.pd[k] = eb;
        cb.pth[k] = ec;
        cb.hk[k] = eh;
        cb.eoff[k] = ea;
        const uint32_t m = cb.cnt[k];
        const uint32_t blk = (ea + kBlkE - 1) / kBlkE;       // first walker block starting at or after ea
        if ((uint64_t)blk * kBlkE < (uint64_t)ea + m) cb.bbase[blk] = (uint32_t)(k * kCand);
        ea += m;
    }
    if (t == kScanT - 1) *cb.ne = sa[kScanT - 1];
}

struct PllScanArgs {
    CandBuf cb;
    int flip;
};
__device__ __forceinline__ void k_pll_scan_run(const PllScanArgs& a) { k_pll_scan_body(a.cb, a.flip); }
LDSP_KERNEL_PAIR(k_pll_scan, PllScanArgs, k_pll_scan_run, kScanT)


// Entry records, one wave per chunk (4 samples per lane).  Per entry (SoA per
// walker block: E0[kBlkE], E1[kBlkE]), with srel = s - S_blk (< 2^17):
//   E0 = (c, W, srel, L' - dk2)
//        x = c + Kb + srel D = f(s) - lo; event iff x > W, [lo, lo + W] being
//        the no-repair interval of f cut to [-B, B] when a neighbouring gap is
//        non-empty (the gap to the previous / next entry)
//   E1 = (dk1, dk2 - srel dk1, out, span) for the one crossing direction possible
//        while |f| < 2^21 (up if u >= 2^21, else down); the repair was right iff
//        x_post - L' <= span (see below), i.e. x_pre - (L' - dk2) <= span with the
//        offset before the repair (x_post = x_pre + dk2), which the walker keeps.
// The tail of the last walker block is padded with W = ~0 (never an event).
__device__ __forceinline__ void k_pll_entries_body(PllIn in, const AmpState* st, CandBuf cb, long n)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ float tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) tab[i] = in.table[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const long k = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= cb.nchc) return;
    const float alpha = st->alpha, beta = st->beta;
    const long b0 = k * kCand;
    const int nv = (int)min((long)kCand, n - b0);
    uint32_t R0[4];
    unsigned long long M[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int i = r * 64 + lane;
        const long sg = b0 + min(i, nv - 1);
        R0[r] = cb.rw[sg];
        M[r] = __builtin_amdgcn_ballot_w64(i < nv && (risky(R0[r], cb.B) || i == 0 || i == nv - 1));
    }
    const uint32_t pth = cb.pth[k], pd = cb.pd[k];
    uint32_t e = cb.eoff[k];
    const int B = (int)cb.B;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int i = r * 64 + lane;
        const bool me = (M[r] >> lane) & 1ull;
        const bool prev = lane > 0 ? ((M[r] >> (lane - 1)) & 1ull) : (r > 0 ? (M[r > 0 ? r - 1 : 0] >> 63) : 1ull);
        const bool next = lane < 63 ? ((M[r] >> (lane + 1)) & 1ull) : (r < 3 ? (M[r < 3 ? r + 1 : 3] & 1ull) : 1ull);
        const uint32_t rank = e + (uint32_t)__builtin_popcountll(M[r] & ((1ull << lane) - 1ull));
        e += (uint32_t)__builtin_popcountll(M[r]);
        if (!me) continue;
        const bool lne = i > 0 && !prev, rne = i < nv - 1 && !next;
        const long s = b0 + i;
        const uint32_t blk = rank / kBlkE, idx = rank % kBlkE;
        const uint32_t srel = (uint32_t)(s - (long)cb.bbase[blk]);
        const uint32_t w = R0[r], u = w & 0x3fffffu;
        const uint32_t A = pth + (uint32_t)s * pd;
        int lo = -(int)u, hi = (1 << 22) - 1 - (int)u;
        if (lne || rne) {
            lo = max(lo, -B);
            hi = min(hi, B);
        }
        const bool up = u >= (1u << 21);
        // the loop at the neighbouring table index (one cell up or down) minus the
        // candidate's own step (re-evaluated here from the same inputs: the same bits
        // as k_pll_cand's), whose output is kept for the undo of a failed walker block
        const uint32_t ic = w >> 22;
        const float2 ex0 = in.x0[s], ex1 = *x1_ptr(in, s);
        const Kick kc = pll_eval(tab, ic, ex0, ex1, alpha, beta, in.mod_index, in.costas, in.out_idx);
        const Kick kn = pll_eval(tab, (up ? ic + 1 : ic - 1) & 0x3ffu, ex0, ex1, alpha, beta, in.mod_index,
                                 in.costas, in.out_idx);
        const uint32_t dk1 = kn.k1 - kc.k1, dk2 = kn.k2 - kc.k2;
        const uint32_t out = __float_as_uint(kn.out);
        cb.eout[(size_t)blk * kBlkE + idx] = __float_as_uint(kc.out);
        // A repair here is right iff f_pre (the offset before it) lies in the
        // intersection of: the presumed one-cell crossing, [-B, B] if the left gap
        // is non-empty, and [-B - dk2, B - dk2] (f_post within B) if the right one
        // is.  All three are small signed intervals, so their intersection is one,
        // checked on the walker's snapshot x_post = f_pre - lo + dk2.
        long fl = up ? (1l << 22) - (long)u : -(1l << 22) - (long)u;
        long fh = fl + (1l << 22) - 1;
        if (lne) {
            fl = max(fl, (long)-B);
            fh = min(fh, (long)B);
        }
        if (rne) {
            const long d2 = (long)(int)dk2;
            fl = max(fl, -(long)B - d2);
            fh = min(fh, (long)B - d2);
        }
        const uint32_t Lp = fl <= fh ? (uint32_t)(fl - lo) + dk2 : 0x80000000u;   // empty: always redo
        const uint32_t span = fl <= fh ? (uint32_t)(fh - fl) : 0u;
        uint4* E = cb.ent + (size_t)blk * 2 * kBlkE;
        // stored as L' - dk2: the walker tests its pre-repair snapshot, x_pre = x_post - dk2
        E[idx] = make_uint4(A - (uint32_t)lo, (uint32_t)(hi - lo), srel, Lp - dk2);
        E[kBlkE + idx] = make_uint4(dk1, dk2 - srel * dk1, out, span);
    }
    if (k == cb.nchc - 1) {              // pad the last walker block: events never fire there
        const uint32_t ne = e, end = (ne + kBlkE - 1) / kBlkE * kBlkE;
        for (uint32_t t = ne + lane; t < end; t += 64)
            cb.ent[(size_t)(t / kBlkE) * 2 * kBlkE + t % kBlkE] = make_uint4(0u, ~0u, 0u, 0u);
    }
}

struct PllEntriesArgs {
    PllIn in;
    const AmpState* st;
    CandBuf cb;
    long n;
};
__device__ __forceinline__ void k_pll_entries_run(const PllEntriesArgs& a) { k_pll_entries_body(a.in, a.st, a.cb, a.n); }
LDSP_KERNEL_PAIR(k_pll_entries, PllEntriesArgs, k_pll_entries_run, 256)


// ------------------------------------------------------------------ walker
struct WalkBufE {
    uint4 e[2][kBlkE];
    uint32_t hdr[4];
};

constexpr int kWalkThreads = 512;
constexpr int kLoadWaves = kWalkThreads / 64 - 1;             // 7
constexpr int kPieces = 2 * kBlkE * 16 / 1024;                // 16 x 1 KiB per block
constexpr int kDmaPer = (kPieces + kLoadWaves - 1) / kLoadWaves + 1;   // 3 pieces + the block header
static_assert(kDmaPer == 4, "walker DMA wait counts below assume 4 DMAs per loader wave per block");
constexpr int kRing = 8;             // LDS ring of walker blocks (8 x 16 KiB), DMA'd kRing - 1 ahead

// Loader wave: wait until at most k blocks' DMAs (kDmaPer each) are still in flight.
__device__ __forceinline__ void vm_wait_blocks(long k)
{
    switch (k <= 0 ? 0 : (k >= kRing - 2 ? kRing - 2 : (int)k)) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    }
}
static_assert(kRing == 8, "vm_wait_blocks covers up to 6 blocks in flight");

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

// Loader wave lw (0..6) moves the 1 KiB pieces lw, lw + 7, ... of a block's
// 16 KiB of entries (a repeat of its last piece pads every wave to the same
// DMA count) and the block header word.
__device__ __forceinline__ void walk_dma(WalkBufE& b, const CandBuf& cb, long blk, int lw, int lane)
{
    const char* src = (const char*)(cb.ent + blk * 2 * kBlkE);
    const uint32_t base = (uint32_t)(uintptr_t)&b.e[0][0];
#pragma unroll
    for (int t = 0; t < kDmaPer - 1; t++) {
        const int piece = min(lw + t * kLoadWaves, kPieces - 1);
        dma16(base + piece * 1024, src + piece * 1024 + lane * 16);
    }
    if (lane == 0) dma4((uint32_t)(uintptr_t)&b.hdr[0], cb.bbase + blk);
}

// Inputs of a full loop step (true index any number of cells from the candidate's).
struct FullCtx {
    const float2* x0;
    const float2* x;
    const float2* hist;
    const float* table;
    int m, costas, out_idx;
    float alpha, beta, mod_index;
};

__device__ __forceinline__ uint32_t rl(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// v + a * dk1.  F24: a < 2^23 and every kick difference fits 24 signed bits
// (host check: |k1| <= alpha 2^31, so |dk1| < 2^23 when alpha <= 2^-9), one v_mad_i32_i24.
template <bool F24>
__device__ __forceinline__ uint32_t mad_lane(uint32_t a, uint32_t dk1, uint32_t v)
{
    if (F24) {
        uint32_t r;
        asm volatile("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(dk1), "v"(v));
        return r;
    }
    return v + a * dk1;
}

// pout = lane is set in `bit` ? so : pout  (one v_cndmask_b32 with an SGPR lane mask)
__device__ __forceinline__ uint32_t sel_lane(uint32_t pout, uint32_t so, unsigned long long bit)
{
    uint32_t r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(pout), "v"(so), "s"(bit));
    return r;
}

// Walker state (wave-uniform): f(s) = Kb + (s - S) D + A(s), S = the current walker block's sample base.
struct WState {
    uint32_t Kb, D, nrep, nfb, nlb, nsame;
};

// Generic walk of every sample in [sa, sb] (the samples of one lane-block's
// entries and the gaps between them): 64 consecutive samples per step, the
// candidate records, offset model and loop inputs of kFbPre steps loaded up front
// into registers (one memory round trip for a whole lane-block's range instead of
// one per step and per full repair), each repair applied at the true index.  A
// repair at one of the lane-block's entries that crosses the one cell its entry
// record allows (E1) takes that record's kick differences and output (the same
// pll_eval k_pll_entries ran); any other one (a gap sample, or two or more cells)
// evaluates the loop step in full against the candidate's recorded kicks.  Used
// where the sparse walk cannot prove a gap clean, and for every lane-block in
// the LDSP_DEBUG_PLL=2 check (which evaluates every repair in full).
constexpr int kFbPre = 4;      // 64-sample steps loaded up front (a lane-block's range is ~4)

struct FbKick {
    uint32_t dk1, dk2p, out;
};
// walk_fallback's rare full loop step (kept out of line: inlined, its code and
// registers made every repair of the loop around it ~150 instructions long)
__device__ __noinline__ FbKick fb_full_step(const float* tab, uint32_t wj, uint32_t cell, float2 u0v, float2 u1v,
                                            int j, uint32_t rrel, FullCtx fc)
{
    const float2 u0 = make_float2(__uint_as_float(rl(__float_as_uint(u0v.x), j)),
                                  __uint_as_float(rl(__float_as_uint(u0v.y), j)));
    const float2 u1 = make_float2(__uint_as_float(rl(__float_as_uint(u1v.x), j)),
                                  __uint_as_float(rl(__float_as_uint(u1v.y), j)));
    const Kick kt = pll_eval(tab, ((wj >> 22) + cell) & 0x3ffu, u0, u1, fc.alpha, fc.beta, fc.mod_index, fc.costas,
                             fc.out_idx);
    // the candidate's own step at its index (k_pll_cand's bits)
    const Kick kc = pll_eval(tab, (wj >> 22) & 0x3ffu, u0, u1, fc.alpha, fc.beta, fc.mod_index, fc.costas,
                             fc.out_idx);
    FbKick r;
    r.dk1 = rfl(kt.k1 - kc.k1);
    r.dk2p = rfl(kt.k2 - kc.k2) - rrel * r.dk1;
    r.out = rfl(__float_as_uint(kt.out));
    return r;
}

__device__ __noinline__ WState walk_fallback(WState g, long sa, long sb, uint32_t S, CandBuf cb, FullCtx fc,
                                             const float* tab, float* y, int lane, uint32_t esrel, uint32_t edk1,
                                             uint32_t edk2p, uint32_t eout, int nv)
{
    const unsigned long long emask = nv >= 64 ? ~0ull : nv <= 0 ? 0ull : ((1ull << nv) - 1ull);
    const bool use_e1 = cb.dbg != 2;
    for (long b0 = sa; b0 <= sb; b0 += 64l * kFbPre) {
        // every input of kFbPre steps in registers before the first: the record
        // (candidate phase word, kicks), the offset model and the full step's two
        // samples -- a repair that needs the full loop step reads them lane by lane.
        // (Fully unrolled with guards, not a break: a loop-indexed array would live
        // in scratch memory.)
        uint32_t R[kFbPre];
        uint32_t A[kFbPre];
        float2 U0[kFbPre], U1[kFbPre];
#pragma unroll
        for (int q = 0; q < kFbPre; q++) {
            const long s = min(b0 + 64l * q + lane, sb);
            R[q] = cb.rw[s];
            const long k = s / kCand;
            A[q] = cb.pth[k] + (uint32_t)s * cb.pd[k];
            U0[q] = fc.x0[s];
            const long gi = s - fc.m;
            U1[q] = gi >= 0 ? fc.x[gi] : fc.hist[gi + fc.m];
        }
#pragma unroll
        for (int q = 0; q < kFbPre; q++) {
            const long base = b0 + 64l * q;
            if (base <= sb) {
                const unsigned long long M = __builtin_amdgcn_ballot_w64(base + lane <= sb);
                const uint32_t srel = (uint32_t)(base + lane - (long)S);
                uint32_t v = (R[q] & 0x3fffffu) + g.Kb + srel * g.D + A[q];
                unsigned long long mask = __builtin_amdgcn_ballot_w64(v > 0x3fffffu) & M;
                // the step's repaired outputs: lane j of yv, stored once after the step
                uint32_t yv = 0;
                unsigned long long rep = 0;
                while (mask != 0) {
                    const int j = __builtin_ctzll(mask);
                    const uint32_t vj = rl(v, j), wj = rl(R[q], j);
                    const uint32_t rrel = (uint32_t)j + (uint32_t)(base - (long)S);
                    const uint32_t cell = vj >> 22;            // true index - candidate's (mod 1024)
                    const unsigned long long em = __builtin_amdgcn_ballot_w64(esrel == rrel) & emask;
                    uint32_t dk1, dk2p, out;
                    if (use_e1 && em != 0 && cell == ((wj & 0x3fffffu) >= (1u << 21) ? 1u : 1023u)) {
                        const int L = __builtin_ctzll(em);
                        dk1 = rl(edk1, L);
                        dk2p = rl(edk2p, L);                  // dk2 - srel dk1
                        out = rl(eout, L);
                    } else {
                        // the loop step at the true index (any number of cells from the
                        // candidate's), evaluated in full; the candidate's kicks from its record
                        const FbKick fk = fb_full_step(tab, wj, cell, U0[q], U1[q], j, rrel, fc);
                        dk1 = fk.dk1;
                        dk2p = fk.dk2p;
                        out = fk.out;
                    }
                    yv = lane == j ? out : yv;
                    rep |= 1ull << j;
                    g.Kb += dk2p;
                    g.D += dk1;
                    g.nrep++;
                    v += dk2p + srel * dk1;
                    mask = __builtin_amdgcn_ballot_w64(v > 0x3fffffu) & M & ((~0ull << j) << 1);
                }
                if ((rep >> lane) & 1ull) y[base + lane] = __uint_as_float(yv);
            }
        }
    }
    return g;
}

// One lane-block of 64 entries (lanes >= nv are padding or the next lane-block's:
// their W = ~0 or they are checked again there -- only s_last uses nv).
// Every repair is assumed to be the one crossing the entry allows (E1): per
// repair one ff1, two readlanes, a 24-bit multiply-add, an add, one lane
// select (x after the repair) and one ballot.  Afterwards, over the repaired
// lanes: the crossing was that one cell, f_pre is within B where the left
// gap is non-empty and f_post within B where the right gap is; else the
// lane-block is redone by walk_fallback from its saved state.  The repaired
// outputs are stored only then.
// Where the previous lane-block ended (its srel register, valid lanes and
// block base): the first sample a fallback of this lane-block must redo.  Only
// read on that rare path, so no lane-block waits for a readlane.
struct PrevLB {
    uint32_t srel;
    int nv;
    uint32_t S;
    bool first;
};

template <bool F24, bool STATS>
__device__ __forceinline__ void walk_lb(const uint4& E0, const uint4& E1, int nv, WState& g, uint32_t S, PrevLB& prev,
                                        const CandBuf& cb, const FullCtx& fc, const float* tab, float* y, int lane)
{
    const uint32_t srel = E0.z, sx = srel;
    uint32_t x = E0.x + g.Kb + srel * g.D;
    unsigned long long mask = __builtin_amdgcn_ballot_w64(x > E0.y);
    if (STATS && cb.dbg == 2) mask = 1;
    if (STATS && cb.dbg == 3) mask = 0;      // timing only: no repairs (wrong output)
    const unsigned long long mask0 = mask;
    if (mask != 0) {
        const WState g0 = g;
        uint32_t Kb = rfl(g.Kb), D = rfl(g.D);       // scalar accumulators
        uint32_t xpost = 0;
        unsigned long long PM = 0;
        if (F24) {
            // The repair chain, hand-scheduled (15 instructions; s_and sets SCC for
            // the back branch, no s_cmp): per repair j = ff1(mask); dk1, dk2' =
            // lane j's (readlane); snapshot lane j's x (pre-repair); x += dk2' +
            // srel dk1 in every lane; mask = events after j.  Exec is the full wave here.
            uint32_t j, dk1, dk2;
            unsigned long long bit, above;
            asm volatile(
                "1:\n\t"
                "s_ff1_i32_b64 %[j], %[mask]\n\t"
                "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t"
                "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t"
                "s_lshl_b64 %[bit], 1, %[j]\n\t"
                "s_lshl_b64 %[above], -2, %[j]\n\t"
                "s_or_b64 %[pm], %[pm], %[bit]\n\t"
                "v_cndmask_b32_e64 %[xp], %[xp], %[x], %[bit]\n\t"
                "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t"
                "v_add_u32 %[x], %[dk2], %[x]\n\t"
                "s_add_u32 %[kb], %[kb], %[dk2]\n\t"
                "s_add_u32 %[d], %[d], %[dk1]\n\t"
                "v_cmp_gt_u32_e64 %[mask], %[x], %[w]\n\t"
                "s_and_b64 %[mask], %[mask], %[above]\n\t"
                "s_cbranch_scc1 1b"
                : [x] "+v"(x), [xp] "+v"(xpost), [mask] "+s"(mask), [pm] "+s"(PM), [kb] "+s"(Kb), [d] "+s"(D),
                  [j] "=&s"(j), [dk1] "=&s"(dk1), [dk2] "=&s"(dk2), [bit] "=&s"(bit), [above] "=&s"(above)
                : [e1x] "v"(E1.x), [e1y] "v"(E1.y), [sx] "v"(sx), [w] "v"(E0.y)
                : "scc");
        } else {
            do {
                const int j = __builtin_ctzll(mask);
                const uint32_t dk1 = rl(E1.x, j), dk2p = rl(E1.y, j);
                const unsigned long long bit = 1ull << j;
                PM |= bit;
                xpost = sel_lane(xpost, x, bit);          // pre-repair offset (E0.w = L' - dk2)
                x = mad_lane<F24>(sx, dk1, x) + dk2p;
                D += dk1;
                Kb += dk2p;
                mask = __builtin_amdgcn_ballot_w64(x > E0.y) & ((~0ull << j) << 1);
            } while (mask != 0);
        }
        // every repaired lane: x_pre - (L' - dk2) <= span (E0.w, E1.w: k_pll_entries)
        unsigned long long bad = __builtin_amdgcn_ballot_w64(xpost - E0.w > E1.w) & PM;
        if (STATS && cb.dbg == 2) bad = 1;
        if (__builtin_expect(bad != 0, 0)) {
            WState r = g0;
            r.nfb++;
            const long s_first = prev.first ? 0l : (long)prev.S + rl(prev.srel, prev.nv - 1) + 1;
            r = walk_fallback(r, s_first, (long)S + rl(srel, nv - 1), S, cb, fc, tab, y, lane, E0.z, E1.x, E1.y,
                              E1.z, nv);
            g.Kb = rfl(r.Kb);
            g.D = rfl(r.D);
            g.nrep = rfl(r.nrep);
            g.nfb = rfl(r.nfb);
        } else {
            // store the repaired lanes' outputs with exec = PM
            float* yb = y + S;
            asm volatile("s_mov_b64 exec, %[pm]\n\t"
                         "global_store_dword %[off], %[v], %[base]\n\t"
                         "s_mov_b64 exec, -1"
                         :
                         : [pm] "s"(PM), [off] "v"(srel << 2), [v] "v"(E1.z), [base] "s"(yb)
                         : "memory", "exec");
            g.Kb = Kb;
            g.D = D;
            g.nrep += (unsigned)__builtin_popcountll(PM);    // live counters (ldsp_ampmodem_walk_stats)
            if (STATS) {
                g.nlb++;
                g.nsame += PM == mask0 ? 1u : 0u;
            }
        }
    }
    prev.srel = srel;
    prev.nv = nv;
    prev.S = S;
    prev.first = false;
}

// The F24 lane-block, hand-scheduled end to end.  x holds this lane-block's
// offsets with every earlier repair applied; the next lane-block's (xn) are
// formed from Kb, D before this block's repairs and carried through them in
// the repair loop (two VALU ops per repair placed in the v_cmp -> s_and
// shadow), so no lane-block starts with a multiply on its critical path.  The
// interval test of the repaired lanes follows the loop in the same block.
template <bool STATS>
__device__ __forceinline__ void walk_lb24(const uint4& E0, const uint4& E1, int nv, WState& g, uint32_t S, PrevLB& prev,
                                          const CandBuf& cb, const FullCtx& fc, const float* tab, float* y, int lane,
                                          uint32_t& x, unsigned long long& mask, uint32_t e0nx, uint32_t sxn, uint32_t wn,
                                          float* yb)
{
    const uint32_t srel = E0.z;
    const uint32_t W = (STATS && cb.dbg == 3) ? ~0u : E0.y;       // dbg 3: timing only, no repairs
    if (STATS && cb.dbg == 3) wn = ~0u;
    uint32_t Kb = rfl(g.Kb), D = rfl(g.D);
    const uint32_t Kb0 = Kb, D0 = D;
    uint32_t xn, xp, t, off, j, dk1, dk2, nr;
    unsigned long long PM, bad, bit, above;
    const unsigned long long m0 = mask;          // (STATS only)
    // per repair: ff1, two readlanes, x += dk2' + srel dk1 (24-bit mad), the
    // lane's post-repair x kept, the next events; Kb, D and the next
    // lane-block's offsets follow in the shadow of the v_cmp.  Afterwards the
    // interval test and the repaired outputs' store with exec = PM (empty when
    // the test fails: walk_fallback then redoes the lane-block).  mask: this
    // lane-block's events on entry, the next lane-block's on exit (formed
    // beside the interval test, so the two VALU -> SALU hand-offs overlap).
    asm volatile(
        "v_mul_lo_u32 %[t], %[d], %[sxn]\n\t"
        "v_add3_u32 %[xn], %[e0nx], %[kb], %[t]\n\t"
        "v_lshlrev_b32 %[off], 2, %[sx]\n\t"
        "s_mov_b64 %[pm], 0\n\t"
        "s_cmp_eq_u64 %[mask], 0\n\t"
        "s_cbranch_scc1 2f\n"
        "1:\n\t"
        "s_ff1_i32_b64 %[j], %[mask]\n\t"
        "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t"
        "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t"
        "s_lshl_b64 %[bit], 1, %[j]\n\t"
        "s_lshl_b64 %[above], -2, %[j]\n\t"
        "s_or_b64 %[pm], %[pm], %[bit]\n\t"
        "v_cndmask_b32_e64 %[xp], %[xp], %[x], %[bit]\n\t"
        "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t"
        "v_add_u32 %[x], %[dk2], %[x]\n\t"
        "s_add_u32 %[kb], %[kb], %[dk2]\n\t"
        "s_add_u32 %[d], %[d], %[dk1]\n\t"
        "v_cmp_gt_u32_e64 %[mask], %[x], %[w]\n\t"
        "v_mad_i32_i24 %[xn], %[sxn], %[dk1], %[xn]\n\t"
        "v_add_u32 %[xn], %[dk2], %[xn]\n\t"
        "s_and_b64 %[mask], %[mask], %[above]\n\t"
        "s_cbranch_scc0 2f\n\t"
        "s_ff1_i32_b64 %[j], %[mask]\n\t"
        "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t"
        "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t"
        "s_lshl_b64 %[bit], 1, %[j]\n\t"
        "s_lshl_b64 %[above], -2, %[j]\n\t"
        "s_or_b64 %[pm], %[pm], %[bit]\n\t"
        "v_cndmask_b32_e64 %[xp], %[xp], %[x], %[bit]\n\t"
        "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t"
        "v_add_u32 %[x], %[dk2], %[x]\n\t"
        "s_add_u32 %[kb], %[kb], %[dk2]\n\t"
        "s_add_u32 %[d], %[d], %[dk1]\n\t"
        "v_cmp_gt_u32_e64 %[mask], %[x], %[w]\n\t"
        "v_mad_i32_i24 %[xn], %[sxn], %[dk1], %[xn]\n\t"
        "v_add_u32 %[xn], %[dk2], %[xn]\n\t"
        "s_and_b64 %[mask], %[mask], %[above]\n\t"
        "s_cbranch_scc0 2f\n\t"
        "s_ff1_i32_b64 %[j], %[mask]\n\t"
        "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t"
        "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t"
        "s_lshl_b64 %[bit], 1, %[j]\n\t"
        "s_lshl_b64 %[above], -2, %[j]\n\t"
        "s_or_b64 %[pm], %[pm], %[bit]\n\t"
        "v_cndmask_b32_e64 %[xp], %[xp], %[x], %[bit]\n\t"
        "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t"
        "v_add_u32 %[x], %[dk2], %[x]\n\t"
        "s_add_u32 %[kb], %[kb], %[dk2]\n\t"
        "s_add_u32 %[d], %[d], %[dk1]\n\t"
        "v_cmp_gt_u32_e64 %[mask], %[x], %[w]\n\t"
        "v_mad_i32_i24 %[xn], %[sxn], %[dk1], %[xn]\n\t"
        "v_add_u32 %[xn], %[dk2], %[xn]\n\t"
        "s_and_b64 %[mask], %[mask], %[above]\n\t"
        "s_cbranch_scc0 2f\n\t"
        "s_ff1_i32_b64 %[j], %[mask]\n\t"
        "v_readlane_b32 %[dk1], %[e1x], %[j]\n\t"
        "v_readlane_b32 %[dk2], %[e1y], %[j]\n\t"
        "s_lshl_b64 %[bit], 1, %[j]\n\t"
        "s_lshl_b64 %[above], -2, %[j]\n\t"
        "s_or_b64 %[pm], %[pm], %[bit]\n\t"
        "v_cndmask_b32_e64 %[xp], %[xp], %[x], %[bit]\n\t"
        "v_mad_i32_i24 %[x], %[sx], %[dk1], %[x]\n\t"
        "v_add_u32 %[x], %[dk2], %[x]\n\t"
        "s_add_u32 %[kb], %[kb], %[dk2]\n\t"
        "s_add_u32 %[d], %[d], %[dk1]\n\t"
        "v_cmp_gt_u32_e64 %[mask], %[x], %[w]\n\t"
        "v_mad_i32_i24 %[xn], %[sxn], %[dk1], %[xn]\n\t"
        "v_add_u32 %[xn], %[dk2], %[xn]\n\t"
        "s_and_b64 %[mask], %[mask], %[above]\n\t"
        "s_cbranch_scc1 1b\n"
        "2:\n\t"
        "v_cmp_gt_u32_e64 %[mask], %[xn], %[wn]\n\t"
        "v_sub_u32 %[t], %[xp], %[lp]\n\t"
        "v_cmp_gt_u32_e64 %[bad], %[t], %[span]\n\t"
        "s_bcnt1_i32_b64 %[nr], %[pm]\n\t"
        "s_and_b64 %[bad], %[bad], %[pm]\n\t"
        "s_cmp_eq_u64 %[bad], 0\n\t"
        "s_cselect_b64 exec, %[pm], 0\n\t"
        "global_store_dword %[off], %[out], %[yb]\n\t"
        "s_mov_b64 exec, -1"
        : [x] "+v"(x), [xn] "=&v"(xn), [xp] "=&v"(xp), [t] "=&v"(t), [off] "=&v"(off), [mask] "+s"(mask),
          [pm] "=&s"(PM), [bad] "=&s"(bad), [kb] "+s"(Kb), [d] "+s"(D), [j] "=&s"(j),
          [dk1] "=&s"(dk1), [dk2] "=&s"(dk2), [bit] "=&s"(bit), [above] "=&s"(above), [nr] "=&s"(nr)
        : [e1x] "v"(E1.x), [e1y] "v"(E1.y), [sx] "v"(srel), [sxn] "v"(sxn), [e0nx] "v"(e0nx), [w] "v"(W), [wn] "v"(wn),
          [lp] "v"(E0.w), [span] "v"(E1.w), [out] "v"(E1.z), [yb] "s"(yb)
        : "scc", "exec", "memory");
    g.Kb = Kb;
    g.D = D;
    g.nrep += nr;                                // live counters (ldsp_ampmodem_walk_stats)
    if (STATS && m0 != 0) {
        g.nlb++;
        g.nsame += PM == m0 ? 1u : 0u;
    }
    if (STATS && cb.dbg == 2 && nv > 0) bad = 1;
    if (__builtin_expect(bad != 0, 0)) {         // (never in a padding lane-block: nv <= 0 there)
        WState r = g;
        r.Kb = Kb0;
        r.D = D0;
        r.nrep -= nr;
        r.nfb++;
        const long s_first = prev.first ? 0l : (long)prev.S + rl(prev.srel, prev.nv - 1) + 1;
        r = walk_fallback(r, s_first, (long)S + rl(srel, nv - 1), S, cb, fc, tab, y, lane, E0.z, E1.x, E1.y, E1.z,
                          nv);
        g.Kb = rfl(r.Kb);
        g.D = rfl(r.D);
        g.nrep = rfl(r.nrep);
        g.nfb = rfl(r.nfb);
        xn = e0nx + g.Kb + sxn * g.D;
        mask = __builtin_amdgcn_ballot_w64(xn > wn);
    }
    x = xn;
    prev.srel = srel;
    prev.nv = nv;
    prev.S = S;
    prev.first = false;
}

// ---- The walker's block loop as one asm statement (product path).  Per walker
// block c (entries already in v100-v163, LB0's offsets / events carried in from
// the previous block): the 8 lane-blocks (WL_LB), each followed by the LDS
// reads of the NEXT block's entries of that lane-block into its own registers
// (free once it is done), so no block starts by waiting for the LDS; block
// c + 1's header (its sample base) is read at the start of block c and its first
// lane-block's offsets are formed in lane-block 7 (sxn = srel + S_{c+1} - S_c),
// so the events of the next block's first lane-block are known when it starts.
// Then the interval-test check (exit to the C++ fallback on failure, state of the
// block's start in kb0 / d0 / nrep0), the rebase Kb += (S_{c+1} - S_c) D, the
// barrier with the loader waves and the slot bookkeeping, all on SALU.  The
// loaders guarantee blocks c + 1 and c + 2 landed at the barrier ending block c.
// Repaired outputs are stored at y + 4 (S + srel) through a 32-bit offset
// (n < 2^30 PCM samples per call, checked on the host).
#define WL_PF(A, B, OFS_A, OFS_B)                                                                           \
    "ds_read_b128 v[" #A "], %[ln] offset:" #OFS_A "\n\t"                                                  \
    "ds_read_b128 v[" #B "], %[ln] offset:" #OFS_B "\n\t"
// Per repair (exec-masked): j = ff1(VCC); exec = the lanes above j; dk1, dk2' = lane
// j's (readlane, which ignores exec); x += dk2' + srel dk1 in those lanes only; VCC =
// their events (a VOPC writes 0 for inactive lanes, so VCC is already "events after
// j": no s_and on the chain, and the loop branches on VCCZ).  Lane j itself keeps its
// pre-repair offset, so after the loop the repaired lanes are exactly those whose x
// is still > W (PM), and the interval test reads x_pre - (L' - dk2) <= span (E0.w).
// No snapshot, no PM bookkeeping, no next-lane-block update inside the loop: the next
// lane-block's offsets are formed once from the final Kb, D (v_mul_lo + v_add3) and
// its events compared into VCC before this lane-block's store / test, which hide the
// compare's latency before the next lane-block's VCCZ branch.
#define WX_REP(E1X, E1Y, SX, W, X)                                                                         \
    "s_ff1_i32_b64 %[j], vcc\n\t"                                                                          \
    "s_lshl_b64 exec, -2, %[j]\n\t"                                                                        \
    "v_readlane_b32 %[dk1], " E1X ", %[j]\n\t"                                                             \
    "v_readlane_b32 %[dk2], " E1Y ", %[j]\n\t"                                                             \
    "v_mad_i32_i24 " X ", " SX ", %[dk1], " X "\n\t"                                                       \
    "v_add_u32 " X ", %[dk2], " X "\n\t"                                                                   \
    "s_add_u32 %[kb], %[kb], %[dk2]\n\t"                                                                   \
    "s_add_u32 %[d], %[d], %[dk1]\n\t"                                                                     \
    "v_cmp_gt_u32_e32 vcc, " X ", " W "\n\t"
// The lane-block transition: the next lane-block's offsets (v_mul_lo, quarter
// rate, then v_add3) are the critical path into its VCCZ branch, so the
// independent work -- this lane-block's repaired mask, store offset and interval
// test -- is issued between the multiply and the add and the store between the
// add and the compare, instead of after them (in-order issue: an instruction
// waiting on a result holds every later one).
#define WL_LB(E0X, E0Y, E0Z, E0W, E1X, E1Y, E1Z, E1W, N0X, N0Y, SXN, X, XN, TAIL)                           \
    "s_cbranch_vccz 2f\n"                                                                                  \
    "1:\n\t"                                                                                               \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccnz 1b\n"                                                    \
    "3:\n\t"                                                                                               \
    "s_mov_b64 exec, -1\n"                                                                                 \
    "2:\n\t"                                                                                               \
    "v_mul_lo_u32 %[t2], %[d], " SXN "\n\t"                                                                \
    "v_cmp_gt_u32_e64 %[pm], " X ", " E0Y "\n\t"                                                           \
    "v_lshl_add_u32 %[off], " E0Z ", 2, %[s4]\n\t"                                                         \
    "v_sub_u32 %[t], " X ", " E0W "\n\t"                                                                   \
    "v_sub_u32_e64 %[t], %[t], " E1W " clamp\n\t"                                                          \
    "v_add3_u32 " XN ", " N0X ", %[kb], %[t2]\n\t"                                                         \
    "s_mov_b64 exec, %[pm]\n\t"                                                                            \
    "global_store_dword %[off], " E1Z ", %[yb]\n\t"                                                        \
    "v_or_b32 %[acc], %[acc], %[t]\n\t"                                                                    \
    "s_mov_b64 exec, -1\n\t"                                                                               \
    "v_cmp_gt_u32_e32 vcc, " XN ", " N0Y "\n\t"                                                            \
    "s_bcnt1_i32_b64 %[nr], %[pm]\n\t"                                                                     \
    "s_add_u32 %[nrep], %[nrep], %[nr]\n\t" TAIL
#ifdef LDSP_TUNING
// Round 4's lane-block order (timing A/B against WL_LB: k_pll_walk VAR 128)
#define WL_LB_ORIG(E0X, E0Y, E0Z, E0W, E1X, E1Y, E1Z, E1W, N0X, N0Y, SXN, X, XN, TAIL)                           \
    "s_cbranch_vccz 2f\n"                                                                                  \
    "1:\n\t"                                                                                               \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccnz 1b\n"                                                    \
    "3:\n\t"                                                                                               \
    "s_mov_b64 exec, -1\n"                                                                                 \
    "2:\n\t"                                                                                               \
    "v_mul_lo_u32 %[t], %[d], " SXN "\n\t"                                                                 \
    "v_add3_u32 " XN ", " N0X ", %[kb], %[t]\n\t"                                                          \
    "v_cmp_gt_u32_e64 %[pm], " X ", " E0Y "\n\t"                                                           \
    "v_lshl_add_u32 %[off], " E0Z ", 2, %[s4]\n\t"                                                         \
    "v_sub_u32 %[t], " X ", " E0W "\n\t"                                                                   \
    "v_sub_u32_e64 %[t], %[t], " E1W " clamp\n\t"                                                          \
    "v_cmp_gt_u32_e32 vcc, " XN ", " N0Y "\n\t"                                                            \
    "s_mov_b64 exec, %[pm]\n\t"                                                                            \
    "global_store_dword %[off], " E1Z ", %[yb]\n\t"                                                        \
    "v_or_b32 %[acc], %[acc], %[t]\n\t"                                                                    \
    "s_mov_b64 exec, -1\n\t"                                                                               \
    "s_bcnt1_i32_b64 %[nr], %[pm]\n\t"                                                                     \
    "s_add_u32 %[nrep], %[nrep], %[nr]\n\t" TAIL
// Timing variants of the product loop (tuning build, k_pll_walk VAR 32 / 64; wrong
// outputs): NOREP skips every repair loop (the lane-block transitions, stores and
// tests alone), NOST drops the store / interval test / repair count (loop + transitions).
#define WL_LB_NOREP(E0X, E0Y, E0Z, E0W, E1X, E1Y, E1Z, E1W, N0X, N0Y, SXN, X, XN, TAIL)                     \
    "s_branch 2f\n"                                                                                        \
    "2:\n\t"                                                                                               \
    "v_mul_lo_u32 %[t], %[d], " SXN "\n\t"                                                                 \
    "v_add3_u32 " XN ", " N0X ", %[kb], %[t]\n\t"                                                          \
    "v_cmp_gt_u32_e64 %[pm], " X ", " E0Y "\n\t"                                                           \
    "v_lshl_add_u32 %[off], " E0Z ", 2, %[s4]\n\t"                                                         \
    "v_sub_u32 %[t], " X ", " E0W "\n\t"                                                                   \
    "v_sub_u32_e64 %[t], %[t], " E1W " clamp\n\t"                                                          \
    "v_cmp_gt_u32_e32 vcc, " XN ", " N0Y "\n\t"                                                            \
    "s_mov_b64 exec, %[pm]\n\t"                                                                            \
    "global_store_dword %[off], " E1Z ", %[yb]\n\t"                                                        \
    "s_mov_b64 exec, -1\n\t"                                                                               \
    "s_bcnt1_i32_b64 %[nr], %[pm]\n\t"                                                                     \
    "s_add_u32 %[nrep], %[nrep], %[nr]\n\t" TAIL
#define WL_LB_NOST(E0X, E0Y, E0Z, E0W, E1X, E1Y, E1Z, E1W, N0X, N0Y, SXN, X, XN, TAIL)                      \
    "s_cbranch_vccz 2f\n"                                                                                  \
    "1:\n\t"                                                                                               \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccnz 1b\n"                                                    \
    "3:\n\t"                                                                                               \
    "s_mov_b64 exec, -1\n"                                                                                 \
    "2:\n\t"                                                                                               \
    "v_mul_lo_u32 %[t], %[d], " SXN "\n\t"                                                                 \
    "v_add3_u32 " XN ", " N0X ", %[kb], %[t]\n\t"                                                          \
    "v_cmp_gt_u32_e32 vcc, " XN ", " N0Y "\n\t" TAIL
// HELPER: the walker's side of a design where other waves store the repaired
// outputs and count the repairs: the repaired lanes' test via a select (no exec
// switch), the offsets written to LDS for the helpers (timing only: one junk slot)
#define WL_LB_HELPER(E0X, E0Y, E0Z, E0W, E1X, E1Y, E1Z, E1W, N0X, N0Y, SXN, X, XN, TAIL)                    \
    "s_cbranch_vccz 2f\n"                                                                                  \
    "1:\n\t"                                                                                               \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccz 3f\n\t"                                                  \
    WX_REP(E1X, E1Y, E0Z, E0Y, X) "s_cbranch_vccnz 1b\n"                                                    \
    "3:\n\t"                                                                                               \
    "s_mov_b64 exec, -1\n"                                                                                 \
    "2:\n\t"                                                                                               \
    "v_mul_lo_u32 %[t], %[d], " SXN "\n\t"                                                                 \
    "v_add3_u32 " XN ", " N0X ", %[kb], %[t]\n\t"                                                          \
    "v_cmp_gt_u32_e64 %[pm], " X ", " E0Y "\n\t"                                                           \
    "v_sub_u32 %[t], " X ", " E0W "\n\t"                                                                   \
    "v_sub_u32_e64 %[t], %[t], " E1W " clamp\n\t"                                                          \
    "v_cmp_gt_u32_e32 vcc, " XN ", " N0Y "\n\t"                                                            \
    "v_cndmask_b32_e64 %[t], 0, %[t], %[pm]\n\t"                                                           \
    "v_or_b32 %[acc], %[acc], %[t]\n\t"                                                                    \
    "ds_write_b32 %[xs], " X "\n\t" TAIL
#endif
#define WL_LBQ(LBM, a, b, c, d, e, f, g, h, n0, n1, n2, X, XN, TAIL)                                         \
    LBM("v" #a, "v" #b, "v" #c, "v" #d, "v" #e, "v" #f, "v" #g, "v" #h, "v" #n0, "v" #n1, "v" #n2, X, XN, TAIL)

#define WALK_ASM(LBM)                                                                                    \
    asm volatile(                                                                                                     \
        /* prologue: block c's entries, block c + 1's header, LB0's offsets / events */                               \
        "v_mov_b32 %[lh], %[sn]\n\t"                                                                                  \
        "v_add_u32 %[ln], %[sn], %[l16]\n\t"                                                                          \
        "ds_read_b128 v[100:103], %[la]\n\t"                                                                          \
        "ds_read_b128 v[104:107], %[la] offset:8192\n\t"                                                              \
        "ds_read_b128 v[108:111], %[la] offset:1024\n\t"                                                              \
        "ds_read_b128 v[112:115], %[la] offset:9216\n\t"                                                              \
        "ds_read_b128 v[116:119], %[la] offset:2048\n\t"                                                              \
        "ds_read_b128 v[120:123], %[la] offset:10240\n\t"                                                             \
        "ds_read_b128 v[124:127], %[la] offset:3072\n\t"                                                              \
        "ds_read_b128 v[128:131], %[la] offset:11264\n\t"                                                             \
        "ds_read_b128 v[132:135], %[la] offset:4096\n\t"                                                              \
        "ds_read_b128 v[136:139], %[la] offset:12288\n\t"                                                             \
        "ds_read_b128 v[140:143], %[la] offset:5120\n\t"                                                              \
        "ds_read_b128 v[144:147], %[la] offset:13312\n\t"                                                             \
        "ds_read_b128 v[148:151], %[la] offset:6144\n\t"                                                              \
        "ds_read_b128 v[152:155], %[la] offset:14336\n\t"                                                             \
        "ds_read_b128 v[156:159], %[la] offset:7168\n\t"                                                              \
        "ds_read_b128 v[160:163], %[la] offset:15360\n\t"                                                             \
        "ds_read_b32 v164, %[lh] offset:16384\n\t"                                                                    \
        "s_lshl_b32 %[s4], %[S], 2\n\t"                                                                               \
        "s_mov_b32 %[kb0], %[kb]\n\t"                                                                                 \
        "s_mov_b32 %[d0], %[d]\n\t"                                                                                   \
        "s_mov_b32 %[nrep0], %[nrep]\n\t"                                                                             \
        "v_mov_b32 %[acc], 0\n\t"                                                                                     \
        "s_waitcnt lgkmcnt(0)\n\t"                                                                                    \
        "v_mul_lo_u32 %[t], %[d], v102\n\t"                                                                           \
        "v_add3_u32 %[xa], v100, %[kb], %[t]\n\t"                                                                     \
        "v_cmp_gt_u32_e32 vcc, %[xa], v101\n"                                                                         \
        "9:\n\t"                                                                                                      \
        WL_LBQ(LBM, 100, 101, 102, 103, 104, 105, 106, 107, 108, 109, 110, "%[xa]", "%[xb]",                               \
               WL_PF(100:103, 104:107, 0, 8192))                                                                      \
        WL_LBQ(LBM, 108, 109, 110, 111, 112, 113, 114, 115, 116, 117, 118, "%[xb]", "%[xa]",                               \
               WL_PF(108:111, 112:115, 1024, 9216))                                                                   \
        WL_LBQ(LBM, 116, 117, 118, 119, 120, 121, 122, 123, 124, 125, 126, "%[xa]", "%[xb]",                               \
               WL_PF(116:119, 120:123, 2048, 10240))                                                                  \
        WL_LBQ(LBM, 124, 125, 126, 127, 128, 129, 130, 131, 132, 133, 134, "%[xb]", "%[xa]",                               \
               WL_PF(124:127, 128:131, 3072, 11264))                                                                  \
        WL_LBQ(LBM, 132, 133, 134, 135, 136, 137, 138, 139, 140, 141, 142, "%[xa]", "%[xb]",                               \
               WL_PF(132:135, 136:139, 4096, 12288))                                                                  \
        WL_LBQ(LBM, 140, 141, 142, 143, 144, 145, 146, 147, 148, 149, 150, "%[xb]", "%[xa]",                               \
               WL_PF(140:143, 144:147, 5120, 13312))                                                                  \
        WL_LBQ(LBM, 148, 149, 150, 151, 152, 153, 154, 155, 156, 157, 158, "%[xa]", "%[xb]",                               \
               WL_PF(148:151, 152:155, 6144, 14336))                                                                  \
        /* lane-block 7: its N0 is the next block's lane-block 0 (read after LB 0; the */                             \
        /* header of block c + 1 was the first read of this block) */                                                 \
        "s_waitcnt lgkmcnt(13)\n\t"                                                                                   \
        "v_readfirstlane_b32 %[snx], v164\n\t"                                                                        \
        "s_sub_u32 %[dS], %[snx], %[S]\n\t"                                                                           \
        "v_add_u32 %[sx7], %[dS], v102\n\t"                                                                           \
        LBM("v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v100", "v101", "%[sx7]", "%[xb]",      \
              "%[xa]", "")                                                                                            \
        /* block end */                                                                                               \
        "v_cmp_ne_u32_e64 %[bad], 0, %[acc]\n\t"                                                                      \
        "s_mul_i32 %[tS], %[dS], %[d]\n\t"                                                                            \
        "s_cmp_lg_u64 %[bad], 0\n\t"                                                                                  \
        "s_cbranch_scc1 8f\n\t"                                                                                       \
        "v_mov_b32 %[s7], v158\n\t"                                                                                   \
        WL_PF(156:159, 160:163, 7168, 15360)                                                                          \
        "s_add_u32 %[kb], %[kb], %[tS]\n\t"                                                                           \
        "s_mov_b32 %[Sp], %[S]\n\t"                                                                                   \
        "s_mov_b32 %[S], %[snx]\n\t"                                                                                  \
        "s_lshl_b32 %[s4], %[S], 2\n\t"                                                                               \
        "s_mov_b32 %[kb0], %[kb]\n\t"                                                                                 \
        "s_mov_b32 %[d0], %[d]\n\t"                                                                                   \
        "s_mov_b32 %[nrep0], %[nrep]\n\t"                                                                             \
        "v_mov_b32 %[acc], 0\n\t"                                                                                     \
        "s_add_u32 %[c], %[c], 1\n\t"                                                                                 \
        "s_add_u32 %[sn], %[sn], %[slot]\n\t"                                                                         \
        "s_cmp_eq_u32 %[sn], %[rend]\n\t"                                                                             \
        "s_cselect_b32 %[sn], %[ring], %[sn]\n\t"                                                                     \
        "s_waitcnt lgkmcnt(0)\n\t"                                                                                    \
        "s_barrier\n\t"                                                                                               \
        "v_mov_b32 %[lh], %[sn]\n\t"                                                                                  \
        "v_add_u32 %[ln], %[sn], %[l16]\n\t"                                                                          \
        "ds_read_b32 v164, %[lh] offset:16384\n\t"                                                                    \
        "s_cmp_lt_u32 %[c], %[nblk]\n\t"                                                                              \
        "s_cbranch_scc1 9b\n"                                                                                         \
        "8:\n\t"                                                                                                      \
        "s_waitcnt lgkmcnt(0)"                                                                                        \
        : [xa] "=&v"(xa), [xb] "=&v"(xb), [t] "=&v"(t), [t2] "=&v"(t2), [off] "=&v"(off), [acc] "=&v"(acc),          \
          [sx7] "=&v"(sx7), [ln] "=&v"(ln), [lh] "=&v"(lh), [s7] "+v"(s7),                                            \
          [pm] "=&s"(pm), [bad] "=&s"(bad),                                                                           \
          [kb] "+s"(kb), [d] "+s"(d), [nrep] "+s"(nrep), [c] "+s"(c), [S] "+s"(S), [Sp] "+s"(Sprev),                  \
          [kb0] "=&s"(kb0), [d0] "=&s"(d0), [nrep0] "=&s"(nrep0), [sn] "+s"(sn),                                      \
          [j] "=&s"(j), [dk1] "=&s"(dk1), [dk2] "=&s"(dk2), [nr] "=&s"(nr), [snx] "=&s"(snx), [dS] "=&s"(dS),         \
          [tS] "=&s"(tS), [s4] "=&s"(s4)                                                                              \
        : [la] "v"(la), [l16] "v"(lane16), [nblk] "s"(nblk), [ring] "s"(ring), [rend] "s"(rend), [slot] "s"(kSlot), \
          [xs] "v"(xs),   \
          [yb] "s"(y)                                                                                                 \
        : "scc", "vcc", "exec", "memory", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109",\
          "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",     \
          "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135",     \
          "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148",     \
          "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161",     \
          "v162", "v163", "v164");

struct WalkLoop {
    uint32_t c, kb, d, nrep;          // block index; offset model; live repair count
    uint32_t kb0, d0, nrep0;          // at the start of block c (the fallback's entry state)
    uint32_t S, Sprev;                // sample base of block c and of the last block completed here
    uint32_t s7;                      // srel register of that block's lane-block 7 (fallback bookkeeping)
};

// Runs blocks c .. nblk - 1 until one fails its interval test (returns with c = that
// block, not yet barriered) or all are done (c = nblk).  PV: 0 the product, 1 / 2 the
// tuning build's timing variants (WL_LB_NOREP / WL_LB_NOST).
template <int PV>
__device__ __forceinline__ void walk_asm_loop(WalkLoop& w, uint32_t nblk, uint32_t ring, float* y, uint32_t lane16,
                                              uint32_t xs = 0)
{
    constexpr uint32_t kSlot = (uint32_t)sizeof(WalkBufE);
    static_assert(sizeof(WalkBufE) == 16400, "slot stride below");
    const uint32_t rend = ring + kRing * kSlot;
    const uint32_t la = ring + (w.c % kRing) * kSlot + lane16;        // block c's entries (prologue)
    uint32_t sn = ring + ((w.c + 1) % kRing) * kSlot;                  // slot of block c + 1
    uint32_t xa, xb, t, t2, off, acc, sx7, ln, lh, s7 = w.s7;
    uint32_t j, dk1, dk2, nr, snx, dS, tS, s4;
    unsigned long long pm, bad;
    uint32_t kb = w.kb, d = w.d, nrep = w.nrep, c = w.c, S = w.S, Sprev = w.Sprev, kb0, d0, nrep0;
    if constexpr (PV == 0) {
        WALK_ASM(WL_LB);
    }
#ifdef LDSP_TUNING
    else if constexpr (PV == 1) {
        WALK_ASM(WL_LB_NOREP);
    } else if constexpr (PV == 2) {
        WALK_ASM(WL_LB_NOST);
    } else if constexpr (PV == 4) {
        WALK_ASM(WL_LB_ORIG);
    } else {
        WALK_ASM(WL_LB_HELPER);
    }
#endif
    w.c = c;
    w.kb = kb;
    w.d = d;
    w.nrep = nrep;
    w.kb0 = kb0;
    w.d0 = d0;
    w.nrep0 = nrep0;
    w.S = S;
    w.Sprev = Sprev;
    w.s7 = s7;
}

// Wave 0 walks the entries of block c; waves 1-7 DMA the entries of block c + kRing - 1
// into the LDS ring meanwhile.
template <bool F24, bool STATS, int VAR = 0>
__device__ __forceinline__ void k_pll_walk_body(PllIn in, long n, AmpState* st, CandBuf cb,
                                                           float* __restrict__ y, uint32_t wexp)
{
    LDSP_LATENCY_CRITICAL();
    __shared__ WalkBufE buf[kRing];      // ring: block c in buf[c % kRing], DMA'd kRing - 1 blocks ahead
    __shared__ float wtab[1024];         // NCO table for the fallback's full loop steps
#ifdef LDSP_TUNING
    __shared__ uint32_t xscratch[64];    // timing variant 96 (WL_LB_HELPER) writes its offsets here
#endif
    // Own the CU: 8 waves x 256 VGPRs fill every SIMD's register file, so no wave of
    // the kernels running beside the walk (the next call's AGC, candidates, ...)
    // is placed on the walker's SIMD and takes issue slots from its serial chain.
    asm volatile("" ::: "v255");
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: keeps the walk on SALU
    const int lane = tid & 63;
    const int lw = wave - 1;             // loader wave index 0..6
    const uint32_t NE = rfl(*(volatile uint32_t*)cb.ne);
    const long nblk = ((long)NE + kBlkE - 1) / kBlkE;
    if (wave != 0) {
        for (long b0 = 0; b0 < kRing - 1 && b0 < nblk; b0++) walk_dma(buf[b0], cb, b0, lw, lane);
        // blocks 0 and 1 landed: at most the DMAs of blocks 2 .. kRing - 2 still in flight
        vm_wait_blocks(min(5l, nblk - 2));
    }
    for (int i = tid; i < 1024; i += kWalkThreads) wtab[i] = in.table[i];
    __syncthreads();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // Hand-off: the launch may be resident before the previous call's walk (or
    // sequential loop) has stored the true state -- it then holds its CU and has
    // its first blocks in LDS when the state arrives, instead of waiting for a
    // whole CU to drain after it.  Wave 0 waits for the state's epoch, bounded
    // (AmpState::wait_ticks, 1 s): on a timeout the state is flagged (werr, and the
    // host-mapped herr that the next call's entry checks) and the host raises.
    unsigned long long t_act = 0;
    if (wave == 0) {
        const unsigned long long tw = wall_clock64();
        const unsigned long long wmax = st->wait_ticks;
        while (__hip_atomic_load(&st->wepoch, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < wexp) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - tw > wmax) {
                if (lane == 0) {
                    st->werr = 1u;
                    if (st->herr) __hip_atomic_store(st->herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                break;
            }
        }
        t_act = wall_clock64();
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
    fc.out_idx = in.out_idx;
    fc.alpha = st->alpha;
    fc.beta = st->beta;
    fc.mod_index = in.mod_index;
    WState g;
    // (coherent loads: the state was stored by another launch during this one)
    g.Kb = __hip_atomic_load(&st->theta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - cb.cs[0];   // f(0) = K
    g.D = __hip_atomic_load(&st->dtheta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - cb.cs[1];   // (block 0: S = 0)
    g.nrep = 0;
    g.nfb = 0;
    g.nlb = 0;
    g.nsame = 0;
    uint32_t S = 0;
    PrevLB prev{0u, 1, 0u, true};
    unsigned long long cyc_walk = 0, cyc_wait = 0;
#ifdef LDSP_TUNING
    unsigned long long cyc_undo = 0, cyc_fb = 0;      // product loop's block redos: undo pass, fallback lane-blocks
#endif
    static_assert(VAR == 0 || VAR == 32 || VAR == 64 || VAR == 96 || VAR == 128, "walker variant");
    if constexpr (F24 && !STATS) {
        // the product path: the block loop in one asm statement (walk_asm_loop)
        if (wave != 0) {
            for (long c = 0; c < nblk; c++) {
                // slot (c + kRing - 1) % kRing held block c - 1, released by the previous barrier
                if (c + kRing - 1 < nblk) walk_dma(buf[(c + kRing - 1) % kRing], cb, c + kRing - 1, lw, lane);
                // blocks c + 1 and c + 2 must have landed before the barrier ending block c
                vm_wait_blocks(min(5l, nblk - c - 3));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
        } else {
            WalkLoop w{0u, rfl(g.Kb), rfl(g.D), 0u, 0u, 0u, 0u, 0u, 0u, 0u};
            const uint32_t ring = (uint32_t)(uintptr_t)&buf[0];
            while (w.c < (uint32_t)nblk) {
                const uint32_t c0 = w.c;
                const uint32_t Sn = rfl(buf[c0 % kRing].hdr[0]);
                w.kb += (Sn - w.S) * w.d;
                w.S = Sn;
#ifdef LDSP_TUNING
                walk_asm_loop<VAR / 32>(w, (uint32_t)nblk, ring, y, (uint32_t)lane * 16u,
                                        (uint32_t)(uintptr_t)&xscratch[lane]);
#else
                walk_asm_loop<VAR / 32>(w, (uint32_t)nblk, ring, y, (uint32_t)lane * 16u);
#endif
                if (w.c > c0) prev = PrevLB{w.s7, 64, w.Sprev, false};
                if (w.c >= (uint32_t)nblk) break;
#ifdef LDSP_TUNING
                const unsigned long long tf0 = wall_clock64();      // fallback cost (stats[2], stats[3])
#endif
                // block c failed its interval test: undo its speculative stores (the
                // candidates' outputs at every entry), then redo it lane-block by
                // lane-block from its entry state (each rewrite lands after the previous one)
                const long c = w.c;
                const WalkBufE& b = buf[c % kRing];
                const int cnt = (int)min((long)kBlkE, (long)NE - c * kBlkE);
                S = w.S;
                float* yb = y + S;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                {
                    // every load first (one round trip), then the stores
                    uint32_t sr[kBlkE / 64], cw[kBlkE / 64];
#pragma unroll
                    for (int q = 0; q < kBlkE / 64; q++) {
                        sr[q] = b.e[0][q * 64 + lane].z;
                        cw[q] = cb.eout[(size_t)c * kBlkE + q * 64 + lane];
                    }
#pragma unroll
                    for (int q = 0; q < kBlkE / 64; q++)
                        if (q * 64 + lane < cnt) y[S + sr[q]] = __uint_as_float(cw[q]);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef LDSP_TUNING
                const unsigned long long tu1 = wall_clock64();
                cyc_undo += tu1 - tf0;
#endif
                g.Kb = w.kb0;
                g.D = w.d0;
                g.nrep = w.nrep0;
                for (int q = 0; q < kBlkE / 64; q++) {
                    const uint4 C0 = b.e[0][q * 64 + lane], C1 = b.e[1][q * 64 + lane];
                    const uint4 N0 = b.e[0][min(q + 1, kBlkE / 64 - 1) * 64 + lane];
                    uint32_t x = C0.x + g.Kb + C0.z * g.D;
                    unsigned long long mk = __builtin_amdgcn_ballot_w64(x > C0.y);
#ifdef LDSP_TUNING
                    const unsigned long long tq0 = wall_clock64();
                    const uint32_t nfb0 = g.nfb;
#endif
                    walk_lb24<false>(C0, C1, min(64, cnt - q * 64), g, S, prev, cb, fc, wtab, y, lane, x, mk, N0.x,
                                     N0.z, N0.y, yb);
#ifdef LDSP_TUNING
                    if (g.nfb != nfb0) cyc_fb += wall_clock64() - tq0;
#endif
                }
                w.kb = rfl(g.Kb);
                w.d = rfl(g.D);
                w.nrep = rfl(g.nrep);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                w.c++;
#ifdef LDSP_TUNING
                cyc_walk += wall_clock64() - tf0;
                cyc_wait++;
#endif
            }
            g.Kb = w.kb;
            g.D = w.d;
            g.nrep = w.nrep;
            S = w.S;
        }
    }
    for (long c = 0; c < ((F24 && !STATS) ? 0 : nblk); c++) {
        const unsigned long long t0 = STATS ? wall_clock64() : 0;
        if (wave != 0) {
            // slot (c + kRing - 1) % kRing held block c - 1, released by the previous barrier
            if (c + kRing - 1 < nblk) walk_dma(buf[(c + kRing - 1) % kRing], cb, c + kRing - 1, lw, lane);
            // block c + 1 must have landed before the barrier below publishes it
            vm_wait_blocks(nblk - c - 2);
        } else {
            const WalkBufE& b = buf[c % kRing];
            const uint32_t Sn = rfl(b.hdr[0]);
            g.Kb += (Sn - S) * g.D;
            S = Sn;
            const int cnt = (int)min((long)kBlkE, (long)NE - c * kBlkE);
            // software-pipelined LDS reads: the next lane-block's entries are always
            // fetched (clamped), so every wait is the same lgkmcnt
            uint4 A0 = b.e[0][lane], A1 = b.e[1][lane];
            if constexpr (F24) {
                // entries two lane-blocks ahead: lane-block q + 1's E0 feeds q's asm.
                // Straight-line over all 8 lane-blocks: the last block's tail is
                // padded with W = ~0 (k_pll_entries), where nothing is ever repaired.
                uint4 N0 = b.e[0][64 + lane], N1 = b.e[1][64 + lane];
                uint32_t x = A0.x + g.Kb + A0.z * g.D;
                unsigned long long mk = __builtin_amdgcn_ballot_w64(x > ((STATS && cb.dbg == 3) ? ~0u : A0.y));
                float* yb = y + S;
#pragma unroll
                for (int q = 0; q < kBlkE / 64; q++) {
                    const int qn = min(q + 2, kBlkE / 64 - 1) * 64 + lane;
                    const uint4 M0 = b.e[0][qn], M1 = b.e[1][qn];
                    walk_lb24<STATS>(A0, A1, min(64, cnt - q * 64), g, S, prev, cb, fc, wtab, y, lane, x, mk, N0.x, N0.z,
                                     N0.y, yb);
                    A0 = N0;
                    A1 = N1;
                    N0 = M0;
                    N1 = M1;
                }
            } else {
#pragma unroll
                for (int q = 0; q < kBlkE / 64; q++) {
                    const int qn = min(q + 1, kBlkE / 64 - 1) * 64 + lane;
                    const uint4 N0 = b.e[0][qn], N1 = b.e[1][qn];
                    if (q * 64 >= cnt) break;
                    walk_lb<F24, STATS>(A0, A1, min(64, cnt - q * 64), g, S, prev, cb, fc, wtab, y, lane);
                    A0 = N0;
                    A1 = N1;
                }
            }
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
        // true state after the last sample: the last chunk's candidate end state + f(n)
        const long L = cb.nchc - 1;
        const uint32_t pd = cb.pd[L];
        st->theta = cb.ce[2 * L] + g.Kb + (uint32_t)(n - (long)S) * g.D + cb.pth[L] + (uint32_t)n * pd;
        st->dtheta = cb.ce[2 * L + 1] + g.D + pd;
        st->wact += wall_clock64() - t_act;
        st->wact_n += 1;
        amp_publish(st, wexp + 1u);
        cb.stats[0] = g.nrep;
        cb.stats[1] = g.nfb;
        cb.stats[4] = NE;
#ifdef LDSP_TUNING
        if (F24 && !STATS) {             // product loop: 10 ns ticks in fallback block redos; their count
            cb.stats[2] = cyc_walk;      // | undo ticks << 16 | fallback lane-block ticks << 40
            cb.stats[3] = cyc_wait | (min(cyc_undo, 0xffffffull) << 16) | (min(cyc_fb, 0xffffffull) << 40);
        }
#endif
        if (STATS) {
            cb.stats[2] = cyc_walk;
            cb.stats[3] = cyc_wait;
            cb.stats[5] = g.nlb;
            cb.stats[6] = g.nsame;
        }
    }
}
struct PllWalkArgs {
    PllIn in;
    long n;
    AmpState* st;
    CandBuf cb;
    float* y;
    uint32_t wexp;
};

template <bool F24, bool STATS, int VAR = 0>
__global__ void __launch_bounds__(kWalkThreads) k_pll_walk(PllWalkArgs a) { k_pll_walk_body<F24, STATS, VAR>(a.in, a.n, a.st, a.cb, a.y, a.wexp); }
template <bool F24, bool STATS, int VAR = 0>
__global__ void __launch_bounds__(kWalkThreads) k_pll_walk_many(::ldsp::Many<PllWalkArgs> m)
{
    const PllWalkArgs& a = m.a[blockIdx.y];
    k_pll_walk_body<F24, STATS, VAR>(a.in, a.n, a.st, a.cb, a.y, a.wexp);
}


__device__ __forceinline__ void k_delay_hist_body(const float2* __restrict__ x, const float2* __restrict__ hist, float2* __restrict__ hist_out,
                             long n, int m)
{
    LDSP_LATENCY_CRITICAL();
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) {
        const long g = n - m + j;
        hist_out[j] = g >= 0 ? x[g] : hist[g + m];
    }
}
struct DelayHistArgs {
    const float2* x;
    const float2* hist;
    float2* hist_out;
    long n;
    int m;
};
__device__ __forceinline__ void k_delay_hist_run(const DelayHistArgs& a) { k_delay_hist_body(a.x, a.hist, a.hist_out, a.n, a.m); }
LDSP_KERNEL_PAIR(k_delay_hist, DelayHistArgs, k_delay_hist_run, 64)


} // namespace

// Scratch layout (16-byte aligned pieces): phase words | cs | ce | cnt | eoff | pth | pd |
// hk | ne | bbase | entries | entry outputs | look-back granules | stats (256 B).
struct PllLayout {
    size_t rw, cs, ce, cnt, eoff, pth, pd, hk, ne, bbase, ent, eout, lb, stats, total;
    long nchc, nblkE;
};
static size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }
static PllLayout pll_layout(size_t n)
{
    PllLayout L;
    L.nchc = (long)((n + kCand - 1) / kCand);
    L.nblkE = (long)((n + kBlkE - 1) / kBlkE);     // entries <= samples
    const size_t nc = (size_t)L.nchc;
    size_t o = 0;
    L.rw = o;    o = al16(o + nc * kCand * 4);
    L.cs = o;    o = al16(o + nc * 8);
    L.ce = o;    o = al16(o + nc * 8);
    L.cnt = o;   o = al16(o + nc * 4);
    L.eoff = o;  o = al16(o + nc * 4);
    L.pth = o;   o = al16(o + nc * 4);
    L.pd = o;    o = al16(o + nc * 4);
    L.hk = o;    o = al16(o + nc * 4);
    L.ne = o;    o = al16(o + 4);
    L.bbase = o; o = al16(o + (size_t)L.nblkE * 4);
    L.ent = o;   o = al16(o + (size_t)L.nblkE * 2 * kBlkE * 16);
    L.eout = o;  o = al16(o + (size_t)L.nblkE * kBlkE * 4);
    L.lb = o;    o = al16(o + (size_t)((nc + 63) / 64) * 6 * 8);
    L.stats = o; o += 256;
    L.total = o;
    return L;
}

size_t pll_scratch_bytes(size_t n) { return pll_layout(n).total; }

size_t pll_stats_offset(size_t n) { return pll_layout(n).stats; }

void delay_hist(const void* x, const void* hist, void* hist_out, size_t n, int m, hipStream_t s)
{
    if (m <= 0) return;
    // one-wave workgroups, one sample per lane: a copy on the chain's critical path
    // that any free wave slot can take (a 256-thread workgroup waited up to 1.5 ms
    // behind a full-GPU filter launch with 8 batched channels)
    launch("k_delay_hist", k_delay_hist, k_delay_hist_many, dim3((unsigned)((m + 63) / 64)), dim3(64), 0, s,
           DelayHistArgs{(const float2*)x, (const float2*)hist, (float2*)hist_out, (long)n, m});
    LDSP_HIP(hipGetLastError());
}

// Costas mode: candidates + walk beat the one-lane loop (~0.57 us per sample)
// from kParMin (1 280) samples: their latency is the warm-up plus one recorded chunk
// (~0.94 ms), then the walk.
static const size_t kParMin = (size_t)LDSP_KNOB("LDSP_PLL_PARMIN", 1280L);
// Carrier mode: the candidate-kick sequential loop (k_pll_seqc, ~0.25 us per
// sample) against candidates + walk.  With exact candidate warm-ups the
// candidates alone took 643 us for a README block (65 536 IQ -> 1 573 PCM
// samples) and the threshold was 2 048; with the approximate warm-up
// (cand_warm_approx) the parallel path wins from ~1 k samples: README blocks on
// one stream 0.69 -> 0.54 ms (95 -> 120 MS/s), numpy blocks 0.89 -> 0.74 ms
// (profiles/r05h_readme_blocks_*.json).
static const size_t kParMinCarrier = (size_t)LDSP_KNOB("LDSP_PLL_PARMIN_CARRIER", 1024L);
bool pll_parallel(size_t n, int costas) { return n >= (costas ? kParMin : kParMinCarrier); }

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
    in.out_idx = c.out_idx;
    return in;
}

static std::atomic<int> g_margin_override{0};    // ldsp_debug_pll_margin

static CandBuf cand_buf(const PllCall& c)
{
    const PllLayout L = pll_layout(c.n);
    char* p = (char*)c.scratch;
    CandBuf cb;
    cb.rw = (uint32_t*)(p + L.rw);
    cb.eout = (uint32_t*)(p + L.eout);
    cb.cs = (uint32_t*)(p + L.cs);
    cb.ce = (uint32_t*)(p + L.ce);
    cb.cnt = (uint32_t*)(p + L.cnt);
    cb.eoff = (uint32_t*)(p + L.eoff);
    cb.pth = (uint32_t*)(p + L.pth);
    cb.pd = (uint32_t*)(p + L.pd);
    cb.hk = (uint32_t*)(p + L.hk);
    cb.costas = c.costas;
    cb.ne = (uint32_t*)(p + L.ne);
    cb.bbase = (uint32_t*)(p + L.bbase);
    cb.ent = (uint4*)(p + L.ent);
    cb.stats = (unsigned long long*)(p + L.stats);
    cb.lb = (unsigned long long*)(p + L.lb);
    cb.ep = 0u;
    cb.nchc = L.nchc;
    // risky margin B: with the carrier PLL |f| stays below 2^19 on ~99.6 % of the
    // samples of the AM chain (walker counters), and 2B / 2^22 = 1/4 of the samples
    // are entries.  The Costas detector's gain vanishes at the message's zero
    // crossings, |f| often exceeds 2^20 there, and gap proofs would fail: B = 2^21
    // makes every sample an entry (no gaps; 11 ms instead of 190 ms per 1.6 M
    // samples of locked DSB-SC, scripts/pll_stress.py).
    static const int lb_env = LDSP_KNOB("LDSP_PLL_LOGB", 0);
    const int lb = g_margin_override.load() ? g_margin_override.load() : lb_env;
    cb.B = 1u << std::max(8, std::min(21, lb ? lb : (c.costas ? 21 : 19)));
    static const int dbg = LDSP_KNOB("LDSP_DEBUG_PLL", 0);
    cb.dbg = dbg;
    return cb;
}

int pll_margin_override(int log2_b)
{
    return g_margin_override.exchange(log2_b);
}

void pll_front(const PllCall& c, hipStream_t s)
{
    if (c.n == 0) return;
    // delay-line history for the next call (m samples); this call's kernels read the old one
    launch("k_delay_hist", k_delay_hist, k_delay_hist_many, dim3((unsigned)((c.m + 63) / 64)), dim3(64), 0, s,
           DelayHistArgs{(const float2*)c.x, (const float2*)c.hist, (float2*)c.hist_out, (long)c.n, c.m});
    if (!pll_parallel(c.n, c.costas)) return;
    CandBuf cb = cand_buf(c);
    // carrier: the chunk scan runs inside k_pll_cand (cand_scan_fold); Costas
    // keeps the two scans around its re-flip
    static const bool fold_knob = LDSP_KNOB("LDSP_PLL_FOLD", 1) != 0;
    // (not inside a many-call: there the scan is one merged launch for every
    // object, and candidate workgroups that share CUs with the concurrent filter
    // launches finish unevenly, so the look-back waits: 8 batched channels 2-5 %
    // slower, scripts/fold_batched_ab.sh)
    const bool fold = fold_knob && !c.costas && !batch_active();
    if (fold) {
        // a look-back epoch no granule in this process has carried (a random start:
        // nor one left in reused device memory, but with 2^-32 odds)
        static std::atomic<uint32_t> ep{(uint32_t)std::random_device{}() | 1u};
        uint32_t e;
        do e = ep.fetch_add(1u); while (e == 0u);
        cb.ep = e;
    }
    {
        static const int warm = LDSP_KNOB("LDSP_PLL_WARM", kWarm);
        // carrier loop: approximate warm-up (cand_warm_approx); Costas keeps the exact one
        // (its two stable points make the warm-up's branch matter, k_pll_reflip)
        static const int approx = LDSP_KNOB("LDSP_PLL_WARM_APPROX", 1);
        launch("k_pll_cand", k_pll_cand, k_pll_cand_many, dim3((unsigned)((cb.nchc + 63) / 64)), dim3(64), 0, s,
               PllCandArgs{pll_in(c), (long)c.n, c.st, c.gcur, cb, c.y, warm, c.costas,
                           (approx && !c.costas) ? 1 : 0, fold ? 1 : 0});
    }
    if (c.costas) {
        launch("k_pll_scan", k_pll_scan, k_pll_scan_many, dim3(1), dim3(kScanT), 0, s, PllScanArgs{cb, 1});
        launch("k_pll_reflip", k_pll_reflip, k_pll_reflip_many, dim3((unsigned)((cb.nchc + 63) / 64)), dim3(64), 0, s,
               PllReflipArgs{pll_in(c), (long)c.n, c.st, cb, c.y});
    }
    if (!fold) launch("k_pll_scan", k_pll_scan, k_pll_scan_many, dim3(1), dim3(kScanT), 0, s, PllScanArgs{cb, 0});
    launch("k_pll_entries", k_pll_entries, k_pll_entries_many, dim3((unsigned)((cb.nchc + 3) / 4)), dim3(256), 0, s,
           PllEntriesArgs{pll_in(c), (const AmpState*)c.st, cb, (long)c.n});
}

void pll_back(const PllCall& c, hipStream_t s)
{
    if (c.n == 0) return;
    if (!pll_parallel(c.n, c.costas)) {
        if (c.costas)
            launch("k_pll_seq", k_pll_seq<true>, k_pll_seq_many<true>, dim3(1), dim3(256), 0, s,
                   PllSeqArgs{pll_in(c), (long)c.n, c.st, c.gcur, c.y});
        else
            launch("k_pll_seqc", k_pll_seqc, k_pll_seqc_many, dim3(1), dim3(256), 0, s,
                   PllSeqcArgs{pll_in(c), (long)c.n, c.st, c.gcur, c.y});
        return;
    }
    {
        static const bool stats = LDSP_KNOB("LDSP_DEBUG_PLL", 0) != 0;
        // the walker stores repaired outputs through 32-bit byte offsets from y
        LDSP_REQUIRE(c.n < (size_t(1) << 30), "ampmodem: at most 2^30 samples per call");
        const dim3 g(1), blk(kWalkThreads);
        const PllWalkArgs a{pll_in(c), (long)c.n, c.st, cand_buf(c), c.y, c.wexp};
#define WALK_LAUNCH(F, S, V) launch("k_pll_walk", k_pll_walk<F, S, V>, k_pll_walk_many<F, S, V>, g, blk, 0, s, a)
        if (c.alpha_host <= 1.0f / 512.0f) {
#ifdef LDSP_TUNING
            // timing variants (k_pll_walk VAR): read per call
            const int var = LDSP_KNOB("LDSP_WALK_VARIANT", 0);
            if (!stats && var > 0) {
                switch (var) {
                case 32: WALK_LAUNCH(true, false, 32); break;
                case 64: WALK_LAUNCH(true, false, 64); break;
                case 96: WALK_LAUNCH(true, false, 96); break;
                case 128: WALK_LAUNCH(true, false, 128); break;
                default: break;
                }
                return;
            }
#endif
            if (stats) WALK_LAUNCH(true, true, 0);
            else WALK_LAUNCH(true, false, 0);
        } else {
            if (stats) WALK_LAUNCH(false, true, 0);
            else WALK_LAUNCH(false, false, 0);
        }
#undef WALK_LAUNCH
    }
}

} // namespace k
} // namespace ldsp
