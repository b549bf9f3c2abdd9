// k_agc.hip -- AGC (agc_crcf) and AmpModem PLL kernels for gfx950, plus the
// math test hook.
//
// AGC (reference src/agc.hpp:109-128 AGC::execute -> agc_crcf_execute per
// sample, squelch status polled per sample, output zeroed in SIGNALLO/ENABLED):
// the gain loop is a nonlinear recurrence, so it is evaluated exactly as the
// sequential algorithm, but in parallel chunks: every chunk starts W samples
// early from a guessed state (gain from the local input power), and because the
// loop forgets its initial state the float32 trajectory coalesces bit-for-bit
// with the true one inside the warm-up.  Chunks whose guessed start state
// differs from the predecessor's end state are repaired run by run
// (k_agc_runfix), and a single-wave verifier re-checks every chunk and re-runs
// any leftover, so the output is always identical to the sequential evaluation.
// (The AmpModem PLL lives in k_pll.hip.)
#include "batch.hpp"
#include "kernels.hpp"
#include "ldsp_common.hpp"
#include "ldsp_math.hpp"

namespace ldsp {
namespace k {

namespace {

enum { SQ_UNKNOWN = 0, SQ_ENABLED, SQ_RISE, SQ_SIGNALHI, SQ_FALL, SQ_SIGNALLO, SQ_TIMEOUT, SQ_DISABLED };

struct AgcReg {
    float g, y2p;
    int mode;
    unsigned int timer;
};

__device__ __forceinline__ float ldnt(const float* p) { return __builtin_nontemporal_load(p); }

// Input extended by the previous call's last H samples: x[i] for i >= 0,
// hist[H + i] for -H <= i < 0 (history kept for the speculative warm-ups).
struct XExt {
    const float2* x;
    const float2* hist;
    long H;
    __device__ __forceinline__ float2 operator[](long i) const { return i >= 0 ? x[i] : hist[H + i]; }
};
__device__ __forceinline__ unsigned ldntu(const unsigned* p) { return __builtin_nontemporal_load(p); }

// AGC(_squelch_update_mode)
__device__ __forceinline__ void agc_squelch(AgcReg& r, const AgcState& p)
{
    if (r.mode == SQ_DISABLED) return;      // threshold test unused in this mode
    const float rssi = (float)(-20.0 * log10((double)r.g));
    const bool ex = rssi > p.threshold;
    switch (r.mode) {
    case SQ_ENABLED: r.mode = ex ? SQ_RISE : SQ_ENABLED; break;
    case SQ_RISE: r.mode = ex ? SQ_SIGNALHI : SQ_FALL; break;
    case SQ_SIGNALHI: r.mode = ex ? SQ_SIGNALHI : SQ_FALL; break;
    case SQ_FALL:
        r.mode = ex ? SQ_SIGNALHI : SQ_SIGNALLO;
        r.timer = p.timeout;
        break;
    case SQ_SIGNALLO:
        r.timer--;
        if (r.timer == 0) r.mode = SQ_TIMEOUT;
        else if (ex) r.mode = SQ_SIGNALHI;
        break;
    case SQ_TIMEOUT: r.mode = SQ_ENABLED; break;
    default: break;
    }
}

// AGC(_execute) + the python-liquiddsp wrapper's zeroing (agc.hpp:114-126).
// SQ = false: squelch disabled for the whole call (the state's mode is
// SQ_DISABLED and stays so: no mode update, no zeroing), decided once per call
// instead of per sample.  The gain update for y2p <= 1e-6 is a multiply by 1
// (a select, not a branch around the transcendentals).
template <bool SQ>
__device__ __forceinline__ float2 agc_step(AgcReg& r, const AgcState& p, float2 x)
{
    const float a = x.x * r.g, b = x.y * r.g;
    const float y2 = a * a - b * (-b);
    r.y2p = (float)((1.0 - (double)p.alpha) * (double)r.y2p + (double)(p.alpha * y2));
    float2 y;
    if (p.locked) {
        y = make_float2(a, b);
    } else {
        const float f = lm_expf_loop(-0.5f * p.alpha * lm_logf_loop(r.y2p));
        r.g *= (r.y2p > 1e-6f) ? f : 1.0f;
        r.g = (r.g > 1e6f) ? 1e6f : r.g;
        if (SQ) agc_squelch(r, p);
        y = make_float2(a * p.scale, b * p.scale);
    }
    if (SQ && (r.mode == SQ_SIGNALLO || r.mode == SQ_ENABLED)) {
        y.x *= 0.0f;
        y.y *= 0.0f;
    }
    return y;
}

// Approximate step (hardware v_log_f32 / v_exp_f32, float32 smoothing): used
// only to bring a chunk's guessed state within a few ulps of the true
// trajectory before the exact warm-up (never for outputs).  kt = -alpha ln(2) / 2
// (the caller's, loop-invariant).
template <bool SQ>
__device__ __forceinline__ void agc_step_approx(AgcReg& r, const AgcState& p, float2 x, float kt)
{
    const float a = x.x * r.g, b = x.y * r.g;
    const float y2 = a * a - b * (-b);
    // the smoothing exactly as agc_step: its float32 rounding would bias y2p (error ~1 ulp / alpha)
    r.y2p = (float)((1.0 - (double)p.alpha) * (double)r.y2p + (double)(p.alpha * y2));
    if (!p.locked) {
        // g *= expf(-0.5 alpha ln y2p) with the exact loop's rounding structure (factor
        // rounded to float, then one float multiply): ln from v_log_f32 (its error is
        // scaled by alpha/2, far below an ulp of the factor), exp by a short series
        // in fused multiply-adds (its error ~1e-11, also far below that ulp).  The
        // factor then rounds like lm_expf's almost always, so this trajectory tracks
        // the exact one within a few ulps instead of drifting by its own rounding
        // noise.
        const float t = kt * __builtin_amdgcn_logf(r.y2p);
        const float u = t * __builtin_fmaf(t, __builtin_fmaf(t, __builtin_fmaf(t, 0.041666668f, 0.16666667f), 0.5f), 1.0f);
        r.g *= (r.y2p > 1e-6f) ? 1.0f + u : 1.0f;
        r.g = (r.g > 1e6f) ? 1e6f : r.g;
        if (SQ) agc_squelch(r, p);
    }
}

// Both loops run whole batches of kA / kB samples without a per-sample bound
// check (the lanes of a chunk kernel all run the same length, but the compiler
// cannot know that: a per-sample check became an exec-mask branch around every
// step), loads software-pipelined one batch ahead (addresses clamped, so the
// prefetch needs no check either), then the tail.  In a one-wave dependent
// chain every instruction costs ~4 cycles of issue.
template <bool SQ, class X>
__device__ __forceinline__ void agc_run_approx_t(AgcReg& r, const AgcState& p, const X& x, long a, long b)
{
#ifndef LDSP_AGC_KA
#define LDSP_AGC_KA 16
#endif
    constexpr int kA = LDSP_AGC_KA;
    if (a >= b) return;
    const float kt = -0.5f * p.alpha * 0.69314718056f;
    const long full = a + (b - a) / kA * kA;
    float2 nx[kA];
#pragma unroll
    for (int j = 0; j < kA; j++) nx[j] = x[min(a + j, b - 1)];
    long i = a;
    for (; i < full; i += kA) {
        float2 cx[kA];
#pragma unroll
        for (int j = 0; j < kA; j++) cx[j] = nx[j];
#pragma unroll
        for (int j = 0; j < kA; j++) nx[j] = x[min(i + kA + j, b - 1)];
#pragma unroll
        for (int j = 0; j < kA; j++) agc_step_approx<SQ>(r, p, cx[j], kt);
    }
    for (; i < b; i++) agc_step_approx<SQ>(r, p, x[i], kt);
}
template <class X>
__device__ __forceinline__ void agc_run_approx(AgcReg& r, const AgcState& p, const X& x, long a, long b)
{
    if (p.mode == SQ_DISABLED) agc_run_approx_t<false>(r, p, x, a, b);
    else agc_run_approx_t<true>(r, p, x, a, b);
}

// Run the AGC over x[a, b) (exact).  OUT: write y/status.
#ifndef LDSP_AGC_KB
#define LDSP_AGC_KB 8
#endif
constexpr int kB = LDSP_AGC_KB;
template <bool OUT, bool SQ, class X>
__device__ __forceinline__ void agc_run_t(AgcReg& r, const AgcState& p, const X& x, long a, long b,
                                          float2* __restrict__ y, uint8_t* __restrict__ status)
{
    if (a >= b) return;
    const long full = a + (b - a) / kB * kB;
    float2 nx[kB];
#pragma unroll
    for (int j = 0; j < kB; j++) nx[j] = x[min(a + j, b - 1)];
    long i = a;
    for (; i < full; i += kB) {
        float2 cx[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) cx[j] = nx[j];
#pragma unroll
        for (int j = 0; j < kB; j++) nx[j] = x[min(i + kB + j, b - 1)];
#pragma unroll
        for (int j = 0; j < kB; j++) {
            const float2 v = agc_step<SQ>(r, p, cx[j]);
            if (OUT) {
                y[i + j] = v;
                if (status) status[i + j] = (uint8_t)r.mode;
            }
        }
    }
    for (; i < b; i++) {
        const float2 v = agc_step<SQ>(r, p, x[i]);
        if (OUT) {
            y[i] = v;
            if (status) status[i] = (uint8_t)r.mode;
        }
    }
}
template <bool OUT, class X>
__device__ __forceinline__ void agc_run(AgcReg& r, const AgcState& p, const X& x, long a, long b,
                                        float2* __restrict__ y, uint8_t* __restrict__ status)
{
    if (p.mode == SQ_DISABLED) agc_run_t<OUT, false>(r, p, x, a, b, y, status);
    else agc_run_t<OUT, true>(r, p, x, a, b, y, status);
}

// A chunk's exact run with its state checkpointed every kAgcCp samples
// (STORE: the chunk kernel records its speculative trajectory) or compared
// with those checkpoints (!STORE: a re-run from the true state stops at the
// first checkpoint its state equals bit for bit -- from there the stored
// outputs and end state are the true ones, so a re-run costs the trajectories'
// coalescence time, ~110 samples on the bench chain, instead of the chunk;
// every checkpoint it passes without a match is rewritten, so the checkpoints
// always describe the trajectory the stored outputs hold).
// cpk: the chunk's kAgcCp-spaced states, [j][4 words] for offsets kAgcCp (j + 1)
// < chunk length.  Returns true when a re-run coalesced (r then holds the state
// at that checkpoint; the caller takes the stored end state).
constexpr int kAgcCp = 64;
static_assert(kAgcCp % kB == 0, "checkpoints fall on batch ends");
__device__ __forceinline__ bool cp_equal(const AgcReg& r, const unsigned* c)
{
    return c[0] == __float_as_uint(r.g) && c[1] == __float_as_uint(r.y2p) && c[2] == (unsigned)r.mode &&
           c[3] == r.timer;
}
template <bool STORE, bool SQ>
__device__ __forceinline__ bool agc_run_cp_t(AgcReg& r, const AgcState& p, const float2* __restrict__ x, long a, long b,
                                             float2* __restrict__ y, uint8_t* __restrict__ status, unsigned* cpk)
{
    if (a >= b) return false;
    const long full = a + (b - a) / kB * kB;
    float2 nx[kB];
#pragma unroll
    for (int j = 0; j < kB; j++) nx[j] = x[min(a + j, b - 1)];
    long i = a;
    for (; i < full; i += kB) {
        float2 cx[kB];
#pragma unroll
        for (int j = 0; j < kB; j++) cx[j] = nx[j];
#pragma unroll
        for (int j = 0; j < kB; j++) nx[j] = x[min(i + kB + j, b - 1)];
#pragma unroll
        for (int j = 0; j < kB; j++) {
            const float2 v = agc_step<SQ>(r, p, cx[j]);
            y[i + j] = v;
            if (status) status[i + j] = (uint8_t)r.mode;
        }
        const long o = i + kB - a;                     // samples done
        if (o % kAgcCp == 0 && i + kB < b) {
            unsigned* c = cpk + (o / kAgcCp - 1) * 4;
            if (!STORE && cp_equal(r, c)) return true;
            // the outputs up to here are this run's now: so is the checkpoint (a later
            // re-run of this chunk must compare against the trajectory the outputs hold)
            c[0] = __float_as_uint(r.g);
            c[1] = __float_as_uint(r.y2p);
            c[2] = (unsigned)r.mode;
            c[3] = r.timer;
        }
    }
    for (; i < b; i++) {
        const float2 v = agc_step<SQ>(r, p, x[i]);
        y[i] = v;
        if (status) status[i] = (uint8_t)r.mode;
    }
    return false;
}
template <bool STORE>
__device__ __forceinline__ bool agc_run_cp(AgcReg& r, const AgcState& p, const float2* __restrict__ x, long a, long b,
                                           float2* __restrict__ y, uint8_t* __restrict__ status, unsigned* cpk)
{
    if (p.mode == SQ_DISABLED) return agc_run_cp_t<STORE, false>(r, p, x, a, b, y, status, cpk);
    return agc_run_cp_t<STORE, true>(r, p, x, a, b, y, status, cpk);
}

// One lane runs the loop; the wave stages the input through LDS 2048 samples
// at a time so the loop never waits on a global load.
__device__ __forceinline__ void k_agc_seq_body(const float2* __restrict__ x, long n, AgcState* st,
                                                float2* __restrict__ y, uint8_t* __restrict__ status)
{
    LDSP_LATENCY_CRITICAL();
    constexpr int kS = 2048;
    __shared__ float2 xs[kS];
    const AgcState p = *st;
    AgcReg r{p.g, p.y2p, p.mode, p.timer};
    for (long base = 0; base < n; base += kS) {
        const int cnt = (int)min((long)kS, n - base);
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += 64) xs[i] = x[base + i];
        __syncthreads();
        if (threadIdx.x == 0) agc_run<true>(r, p, (const float2*)xs, 0, cnt, y + base, status ? status + base : nullptr);
    }
    if (threadIdx.x == 0) {
        st->g = r.g;
        st->y2p = r.y2p;
        st->mode = r.mode;
        st->timer = r.timer;
    }
}
struct AgcSeqArgs {
    const float2* x;
    long n;
    AgcState* st;
    float2* y;
    uint8_t* status;
};
__device__ __forceinline__ void k_agc_seq_run(const AgcSeqArgs& a) { k_agc_seq_body(a.x, a.n, a.st, a.y, a.status); }
LDSP_KERNEL_PAIR(k_agc_seq, AgcSeqArgs, k_agc_seq_run, 64)


// scratch: [nchunks][2 (start, end)][4 words: g, y2p, mode, timer]
// Chunk k's exact run starts W samples early (w0 = s0 - W) from a guessed
// state.  The guess comes from an approximate pass (agc_step_approx) over the
// Wa samples before w0, itself started from y2p = 1 and the gain that
// normalises the mean power of the kPow samples before it; that brings the
// guess within a few ulps of the true trajectory, so the exact float32 loop
// coalesces bit for bit within ~100 samples typically (a few thousand at
// worst; chunks that have not are re-run by k_agc_runfix / k_agc_verify).
constexpr int kPow = kAgcPow;
// H > 0 (speculative call): the H samples before x[0] come from hist and every
// chunk, chunk 0 included, starts from a guess (H >= W + Wa + kPow), so the
// kernel never reads the true state and may overlap the previous call's
// back half; chunk 0 is then checked against the true state like any other.
__device__ __forceinline__ void k_agc_chunks_body(const float2* __restrict__ x, const float2* __restrict__ hist, long H,
                                                   long n, const AgcState* st, int C, int W, int Wa, long nch,
                                                   unsigned* __restrict__ sc, float2* __restrict__ y,
                                                   uint8_t* __restrict__ status, int tsa, unsigned* cp)
{
    LDSP_LATENCY_CRITICAL();
    const long chunk = (long)blockIdx.x * 64 + threadIdx.x;
    if (chunk >= nch) return;
    const AgcState p = *st;
    const XExt xe{x, hist, H};
    const long lo = -H;                  // earliest sample available
    const long s0 = chunk * C, s1 = min(n, s0 + C);
    long w0 = s0 - W;
    AgcReg r;
    bool guessed = false;                // the chunk starts from a guess (checked by the flag pass)
    if (tsa & 3) {
        // small call (H = 0): the true state at x[0] is known, and the approximate
        // loop started from it stays bit-identical to the exact one for thousands of
        // samples in almost every case, so each chunk approximates from the call
        // start to its own start (0.16 vs 0.43 us per step); a chunk whose start
        // came out different is flagged against its predecessor and re-run.
        r = AgcReg{p.g, p.y2p, p.mode, p.timer};
        agc_run_approx(r, p, xe, 0, s0);
        w0 = s0;
    } else if (w0 <= lo) {
        w0 = lo;
        r = AgcReg{p.g, p.y2p, p.mode, p.timer};
    } else {
        guessed = true;
        long a0 = w0 - Wa;
        if (a0 <= lo) {
            a0 = lo;
            r = AgcReg{p.g, p.y2p, p.mode, p.timer};
        } else {
            r.y2p = 1.0f;
            r.mode = (p.mode == SQ_DISABLED) ? SQ_DISABLED : SQ_ENABLED;
            r.timer = 0;
            if (p.locked) {
                r.g = p.g;                          // gain frozen while locked
            } else {
                const long a = max(lo, a0 - kPow);
                const long m = a0 - a;
                double pw = 0.0;
                if (m > 0) {
                    double acc[4] = {0.0, 0.0, 0.0, 0.0};
                    for (long i = a; i < a0; i += 16) {
                        float2 v[16];
#pragma unroll
                        for (int j = 0; j < 16; j++) v[j] = xe[min(i + j, a0 - 1)];
#pragma unroll
                        for (int j = 0; j < 16; j++)
                            if (i + j < a0) acc[j & 3] += (double)v[j].x * v[j].x + (double)v[j].y * v[j].y;
                    }
                    pw = (acc[0] + acc[1] + acc[2] + acc[3]) / (double)m;
                }
                const double g = pw > 1e-12 ? 1.0 / sqrt(pw) : 1e6;
                r.g = (float)(g > 1e6 ? 1e6 : g);
            }
        }
        agc_run_approx(r, p, xe, a0, w0);
    }
    agc_run<false>(r, p, xe, w0, s0, y, status);
    if (tsa & 2) {
        if ((tsa & 4) && chunk > 0) r.g = __uint_as_float(__float_as_uint(r.g) + 1u);   // test hook: every start off by 1 ulp
        // one-wave small call: check and repair in this kernel (no flags /
        // runfix / verify launches).  Chunk j is right iff its start state
        // equals chunk j-1's true end state bit for bit; a chunk that is not is
        // re-run from that end state by lane 0, in order, and its successor
        // compared again.  Chunk 0 started from the true state.
        const AgcReg s = r;
        agc_run<true>(r, p, x, s0, s1, y, status);
        const int lane = threadIdx.x;
        auto differs = [&](const AgcReg& e_prev) {
            return __float_as_uint(s.g) != __float_as_uint(e_prev.g) ||
                   __float_as_uint(s.y2p) != __float_as_uint(e_prev.y2p) || s.mode != e_prev.mode ||
                   s.timer != e_prev.timer;
        };
        // (the shuffles run on every lane: a lane reading an inactive one gets garbage)
        auto up = [&](const AgcReg& e) {
            return AgcReg{__shfl_up(e.g, 1), __shfl_up(e.y2p, 1), __shfl_up(e.mode, 1), __shfl_up(e.timer, 1)};
        };
        AgcReg pe = up(r);
        uint64_t bad = __ballot(lane >= 1 && differs(pe));
        int reruns = 0;
        while (bad) {
            reruns++;
            const int j = __builtin_ctzll(bad);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");    // chunk j's first outputs are stored
            AgcReg e{__shfl(r.g, j - 1), __shfl(r.y2p, j - 1), __shfl(r.mode, j - 1), __shfl(r.timer, j - 1)};
            if (lane == 0) agc_run<true>(e, p, x, (long)j * C, min(n, (long)j * C + C), y, status);
            const AgcReg f{__shfl(e.g, 0), __shfl(e.y2p, 0), __shfl(e.mode, 0), __shfl(e.timer, 0)};
            if (lane == j) r = f;
            pe = up(r);
            bad = __ballot(lane > j && differs(pe));
        }
        if (lane == (int)(nch - 1)) {
            AgcState* so = const_cast<AgcState*>(st);
            so->g = r.g;
            so->y2p = r.y2p;
            so->mode = r.mode;
            so->timer = r.timer;
            if (reruns) so->pad[0] += reruns;     // ldsp_debug_agc_tsa_reruns
        }
        return;
    }
    if ((tsa & 8) && guessed && (chunk & 1)) r.g = __uint_as_float(__float_as_uint(r.g) + 1u);   // test hook
    unsigned* gs = sc + chunk * 8;
    gs[0] = __float_as_uint(r.g);
    gs[1] = __float_as_uint(r.y2p);
    gs[2] = (unsigned)r.mode;
    gs[3] = r.timer;
    if (cp) agc_run_cp<true>(r, p, x, s0, s1, y, status, cp + chunk * (C / kAgcCp) * 4);
    else agc_run<true>(r, p, x, s0, s1, y, status);
    gs[4] = __float_as_uint(r.g);
    gs[5] = __float_as_uint(r.y2p);
    gs[6] = (unsigned)r.mode;
    gs[7] = r.timer;
}
struct AgcChunksArgs {
    const float2* x;
    const float2* hist;
    long H;
    long n;
    const AgcState* st;
    int C;
    int W;
    int Wa;
    long nch;
    unsigned* sc;
    float2* y;
    uint8_t* status;
    int tsa;
    unsigned* cp;
};
__device__ __forceinline__ void k_agc_chunks_run(const AgcChunksArgs& a) { k_agc_chunks_body(a.x, a.hist, a.H, a.n, a.st, a.C, a.W, a.Wa, a.nch, a.sc, a.y, a.status, a.tsa, a.cp); }
LDSP_KERNEL_PAIR(k_agc_chunks, AgcChunksArgs, k_agc_chunks_run, 64)


// One-wave small call (tsa 2) with the call's input staged in LDS first: the
// approximate loop of every lane runs up to its chunk's start over the same
// prefix of x, and from global memory each batch of loads costs an L2 / HBM
// round trip on the dependent chain (~0.13 us a step); from LDS the loop is
// compute-bound.  Otherwise the tsa 2 path of k_agc_chunks.
constexpr long kAgcSmallMax = 8192;      // samples staged (64 KB of LDS)
__device__ __forceinline__ void k_agc_small_body(const float2* __restrict__ x, long n, AgcState* st, int C, long nch,
                                                  float2* __restrict__ y, uint8_t* __restrict__ status, int perturb)
{
    LDSP_LATENCY_CRITICAL();
    extern __shared__ float2 xs[];
    const int lane = threadIdx.x;
    for (long i = lane; i < n; i += 64) xs[i] = x[i];
    __syncthreads();
    const long chunk = lane;
    if (chunk >= nch) return;
    const AgcState p = *st;
    const float2* xl = xs;
    const long s0 = chunk * C, s1 = min(n, s0 + C);
    AgcReg r{p.g, p.y2p, p.mode, p.timer};
    agc_run_approx(r, p, xl, 0, s0);
    if (perturb && chunk > 0) r.g = __uint_as_float(__float_as_uint(r.g) + 1u);   // test hook
    const AgcReg s = r;
    agc_run<true>(r, p, xl, s0, s1, y, status);
    auto differs = [&](const AgcReg& e_prev) {
        return __float_as_uint(s.g) != __float_as_uint(e_prev.g) || __float_as_uint(s.y2p) != __float_as_uint(e_prev.y2p) ||
               s.mode != e_prev.mode || s.timer != e_prev.timer;
    };
    auto up = [&](const AgcReg& e) {
        return AgcReg{__shfl_up(e.g, 1), __shfl_up(e.y2p, 1), __shfl_up(e.mode, 1), __shfl_up(e.timer, 1)};
    };
    AgcReg pe = up(r);
    uint64_t bad = __ballot(lane >= 1 && differs(pe));
    int reruns = 0;
    while (bad) {
        reruns++;
        const int j = __builtin_ctzll(bad);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        AgcReg e{__shfl(r.g, j - 1), __shfl(r.y2p, j - 1), __shfl(r.mode, j - 1), __shfl(r.timer, j - 1)};
        if (lane == 0) agc_run<true>(e, p, xl, (long)j * C, min(n, (long)j * C + C), y, status);
        const AgcReg f{__shfl(e.g, 0), __shfl(e.y2p, 0), __shfl(e.mode, 0), __shfl(e.timer, 0)};
        if (lane == j) r = f;
        pe = up(r);
        bad = __ballot(lane > j && differs(pe));
    }
    if (lane == (int)(nch - 1)) {
        st->g = r.g;
        st->y2p = r.y2p;
        st->mode = r.mode;
        st->timer = r.timer;
        if (reruns) st->pad[0] += reruns;     // ldsp_debug_agc_tsa_reruns
    }
}
struct AgcSmallArgs {
    const float2* x;
    long n;
    AgcState* st;
    int C;
    long nch;
    float2* y;
    uint8_t* status;
    int perturb;
};
__device__ __forceinline__ void k_agc_small_run(const AgcSmallArgs& a) { k_agc_small_body(a.x, a.n, a.st, a.C, a.nch, a.y, a.status, a.perturb); }
LDSP_KERNEL_PAIR(k_agc_small, AgcSmallArgs, k_agc_small_run, 64)


// Parallel repair round over runs of failed chunks.  flags (k_agc_flags)
// mark the chunks whose guessed start state differs from the predecessor's
// end state; one thread per run start (flagged chunk with an unflagged
// predecessor, whose end state is the true one) re-runs the whole run in
// order from that end state, then keeps going through unflagged chunks until
// its state equals a chunk's stored start state bit for bit (from there the
// stored chunks are the true trajectory).  It stops early at the next run's
// start, whose own thread began from a stale state: the next flags pass
// catches that.  One round replaces the ~R/2 parity rounds a run of R failed
// chunks needed.
// End state (g, y2p, mode, timer) of chunk k - 1; for chunk 0 of a
// speculative call, the true state the previous call left in st.
__device__ __forceinline__ unsigned pred_word(const unsigned* sc, const AgcState* st, long k, int i)
{
    if (k > 0) return ldntu(sc + (k - 1) * 8 + 4 + i);
    const unsigned* w = (const unsigned*)st;
    return ldntu(w + (i == 0 ? 0 : i == 1 ? 1 : i == 2 ? 5 : 6));
}

__device__ __forceinline__ bool agc_flag(const unsigned long long* flags, long c)
{
    return (flags[c >> 6] >> (c & 63)) & 1ull;
}

__device__ __forceinline__ void k_agc_runfix_body(const float2* __restrict__ x, long n, const AgcState* st, int C,
                                                   long nch, unsigned* __restrict__ sc,
                                                   const unsigned long long* __restrict__ flags,
                                                   float2* __restrict__ y, uint8_t* __restrict__ status, unsigned* dbg,
                                                   unsigned* cp)
{
    LDSP_LATENCY_CRITICAL();
    const long k = (long)blockIdx.x * 64 + threadIdx.x;
    if (k >= nch || !agc_flag(flags, k) || (k > 0 && agc_flag(flags, k - 1))) return;
    const AgcState p = *st;
    AgcReg r{__uint_as_float(pred_word(sc, st, k, 0)), __uint_as_float(pred_word(sc, st, k, 1)),
             (int)pred_word(sc, st, k, 2), pred_word(sc, st, k, 3)};
    bool inrun = true;
    for (long m = k; m < nch; m++) {
        unsigned* gs = sc + m * 8;
        if (m > k) {
            const bool b = agc_flag(flags, m);
            if (!(inrun && b)) {
                if (b) break;                               // the next run's start
                inrun = false;
                if (ldntu(gs) == __float_as_uint(r.g) && ldntu(gs + 1) == __float_as_uint(r.y2p) &&
                    ldntu(gs + 2) == (unsigned)r.mode && ldntu(gs + 3) == r.timer)
                    break;                                  // coalesced with the stored trajectory
            }
        }
        if (dbg) atomicAdd(dbg, 1u);
        atomicAdd((unsigned*)&st->pad[2], 1u);              // ldsp_debug_agc_reruns (runfix)
        gs[0] = __float_as_uint(r.g);
        gs[1] = __float_as_uint(r.y2p);
        gs[2] = (unsigned)r.mode;
        gs[3] = r.timer;
        const long s0 = m * C;
        if (cp && agc_run_cp<false>(r, p, x, s0, min(n, s0 + C), y, status, cp + m * (C / kAgcCp) * 4)) {
            // coalesced with the stored trajectory: its outputs and end state stand
            r = AgcReg{__uint_as_float(ldntu(gs + 4)), __uint_as_float(ldntu(gs + 5)), (int)ldntu(gs + 6), ldntu(gs + 7)};
            continue;
        }
        if (!cp) agc_run<true>(r, p, x, s0, min(n, s0 + C), y, status);
        gs[4] = __float_as_uint(r.g);
        gs[5] = __float_as_uint(r.y2p);
        gs[6] = (unsigned)r.mode;
        gs[7] = r.timer;
    }
}
// The same repair with one wave per run: chunk m of the run is processed in
// windows of 64 segments of `seg` samples; lane j brings the window's true
// start state to its segment by the approximate loop (from the chunk staged in
// LDS: the small-call technique, which from a true state tracks the exact
// trajectory bit for bit almost always) and runs its segment exactly; a lane
// whose start differs from its left neighbour's exact end is re-run by lane 0
// from that end, in order.  After each window the true states at the chunk's
// checkpoints in it are compared with the stored ones: at the first match the
// stored trajectory from there on is the true one (outputs, later checkpoints,
// end state), so the chunk is done -- a chunk costs ~min(coalescence, C)
// approximate + seg exact steps per window instead of its coalescence time in
// exact steps.  Records, checkpoints, stop rules and outputs are those of
// k_agc_runfix.
struct AgcLdsX {                 // absolute sample index -> the chunk staged in LDS
    const float2* xs;
    long base;
    __device__ __forceinline__ float2 operator[](long i) const { return xs[i - base]; }
};
__device__ __forceinline__ bool agc_reg_eq(const AgcReg& a, const AgcReg& b)
{
    return __float_as_uint(a.g) == __float_as_uint(b.g) && __float_as_uint(a.y2p) == __float_as_uint(b.y2p) &&
           a.mode == b.mode && a.timer == b.timer;
}
__device__ __forceinline__ AgcReg agc_reg_shfl(const AgcReg& e, int src)
{
    return AgcReg{__shfl(e.g, src), __shfl(e.y2p, src), __shfl(e.mode, src), __shfl(e.timer, src)};
}
// One chunk m of a repair, from its true start state T, by one wave (the chunk
// staged in LDS, windows of 64 segments of `seg` samples, the approximate loop to
// each segment, exact segments, in-order re-runs of segments whose start missed,
// exit at the first checkpoint that meets the stored trajectory).  Leaves T = the
// chunk's true end state and records it in gs[4..7] unless the stored one stands.
__device__ __forceinline__ void agc_chunk_wide(const float2* __restrict__ x, long n, const AgcState& p, int C,
                                               int seg, long m, unsigned* gs, unsigned* cpm, float2* xs,
                                               float2* __restrict__ y, uint8_t* __restrict__ status, AgcReg& T)
{
    const int lane = threadIdx.x;
    const long s0 = m * C, s1 = min(n, s0 + C);
    const int cnt = (int)(s1 - s0);
    __syncthreads();                                    // the previous chunk's reads of xs are done
    for (int i = lane; i < cnt; i += 64) xs[i] = x[s0 + i];
    __syncthreads();
    const AgcLdsX xl{xs, s0};
    bool joined = false;                                // met the stored trajectory at a checkpoint
    for (long w0 = s0; w0 < s1; w0 += 64L * seg) {
        const long a = min(s1, w0 + (long)lane * seg), b = min(s1, a + seg);
        AgcReg r = T;
        agc_run_approx(r, p, xl, w0, a);
        AgcReg S = r;                                   // this segment's start (a guess for lane > 0)
        agc_run<true>(r, p, xl, a, b, y, status);
        // lanes whose start is not their left neighbour's exact end: re-run in order
        // (the shuffles on every lane: a lane reading an inactive one gets garbage)
        AgcReg pe = agc_reg_shfl(r, lane > 0 ? lane - 1 : 0);
        uint64_t bad = __ballot(lane >= 1 && a < b && !agc_reg_eq(S, pe));
        while (bad) {
            const int j = __builtin_ctzll(bad);
            const AgcReg e = agc_reg_shfl(r, j - 1);
            AgcReg f = e;
            if (lane == 0) agc_run<true>(f, p, xl, w0 + (long)j * seg, min(s1, w0 + (long)j * seg + seg), y, status);
            f = agc_reg_shfl(f, 0);
            if (lane == j) {
                S = e;
                r = f;
            }
            pe = agc_reg_shfl(r, lane > 0 ? lane - 1 : 0);
            bad = __ballot(lane > j && a < b && !agc_reg_eq(S, pe));
        }
        // the true states at the checkpoints in this window (chunk offsets 64 (q + 1) < cnt)
        const long o = a - s0;
        bool match = false;
        if (cpm && a < s1 && o > 0 && o % kAgcCp == 0) {
            unsigned* c = cpm + (o / kAgcCp - 1) * 4;
            match = cp_equal(S, c);
            if (!match) {
                c[0] = __float_as_uint(S.g);
                c[1] = __float_as_uint(S.y2p);
                c[2] = (unsigned)S.mode;
                c[3] = S.timer;
            }
        }
        if (__ballot(match)) {
            joined = true;
            break;
        }
        T = agc_reg_shfl(r, (int)min(63L, (s1 - 1 - w0) / seg));   // the window's true end state
    }
    if (joined) {
        // the stored end state stands (every lane reads it: T stays wave-uniform)
        T = AgcReg{__uint_as_float(ldntu(gs + 4)), __uint_as_float(ldntu(gs + 5)), (int)ldntu(gs + 6), ldntu(gs + 7)};
    } else if (lane == 0) {
        gs[4] = __float_as_uint(T.g);
        gs[5] = __float_as_uint(T.y2p);
        gs[6] = (unsigned)T.mode;
        gs[7] = T.timer;
    }
}
__device__ __forceinline__ void k_agc_runfix_wide_body(const float2* __restrict__ x, long n, const AgcState* st,
                                                        int C, int seg, long nch, unsigned* __restrict__ sc,
                                                        const unsigned long long* __restrict__ flags,
                                                        float2* __restrict__ y, uint8_t* __restrict__ status,
                                                        unsigned* dbg, unsigned* cp)
{
    LDSP_LATENCY_CRITICAL();
    extern __shared__ float2 xs[];
    const long k = blockIdx.x;
    const int lane = threadIdx.x;
    if (k >= nch || !agc_flag(flags, k) || (k > 0 && agc_flag(flags, k - 1))) return;
    const AgcState p = *st;
    AgcReg T{__uint_as_float(pred_word(sc, st, k, 0)), __uint_as_float(pred_word(sc, st, k, 1)),
             (int)pred_word(sc, st, k, 2), pred_word(sc, st, k, 3)};
    bool inrun = true;
#ifdef LDSP_AGC_TRACE
    const long t_start = wall_clock64();
    int n_chunks = 0;
#endif
    for (long m = k; m < nch; m++) {
        unsigned* gs = sc + m * 8;
        if (m > k) {
            const bool b = agc_flag(flags, m);
            if (!(inrun && b)) {
                if (b) break;                               // the next run's start
                inrun = false;
                if (ldntu(gs) == __float_as_uint(T.g) && ldntu(gs + 1) == __float_as_uint(T.y2p) &&
                    ldntu(gs + 2) == (unsigned)T.mode && ldntu(gs + 3) == T.timer)
                    break;                                  // coalesced with the stored trajectory
            }
        }
        unsigned* cpm = cp ? cp + m * (C / kAgcCp) * 4 : nullptr;
        if (lane == 0) {
            if (dbg) atomicAdd(dbg, 1u);
            atomicAdd((unsigned*)&st->pad[2], 1u);          // ldsp_debug_agc_reruns (runfix)
            gs[0] = __float_as_uint(T.g);
            gs[1] = __float_as_uint(T.y2p);
            gs[2] = (unsigned)T.mode;
            gs[3] = T.timer;
        }
        agc_chunk_wide(x, n, p, C, seg, m, gs, cpm, xs, y, status, T);
#ifdef LDSP_AGC_TRACE
        n_chunks++;
#endif
    }
#ifdef LDSP_AGC_TRACE
    if (lane == 0)
        printf("runfix k=%ld chunks=%d us=%.1f\n", k, n_chunks, (wall_clock64() - t_start) * 0.01);
#endif
}

struct AgcRunfixArgs {
    const float2* x;
    long n;
    const AgcState* st;
    int C;
    long nch;
    unsigned* sc;
    const unsigned long long* flags;
    float2* y;
    uint8_t* status;
    unsigned* dbg;
    unsigned* cp;
    int seg;          // k_agc_runfix_wide: samples per lane per window
};
__device__ __forceinline__ void k_agc_runfix_run(const AgcRunfixArgs& a) { k_agc_runfix_body(a.x, a.n, a.st, a.C, a.nch, a.sc, a.flags, a.y, a.status, a.dbg, a.cp); }
LDSP_KERNEL_PAIR(k_agc_runfix, AgcRunfixArgs, k_agc_runfix_run, 64)
__device__ __forceinline__ void k_agc_runfix_wide_run(const AgcRunfixArgs& a) { k_agc_runfix_wide_body(a.x, a.n, a.st, a.C, a.seg, a.nch, a.sc, a.flags, a.y, a.status, a.dbg, a.cp); }
LDSP_KERNEL_PAIR(k_agc_runfix_wide, AgcRunfixArgs, k_agc_runfix_wide_run, 64)


// Parallel pre-check: bit c of flags[c / 64] = chunk c's start state differs
// from chunk c-1's end state (after the repair rounds).
// spec: 1 = every chunk started from a guess (chunk 0 is compared with the true
// state); 2 = the same, but chunk 0 is presumed right (repair rounds that run
// before the previous call has produced the true state; k_agc_verify then
// checks chunk 0 directly).
__device__ __forceinline__ void k_agc_flags_body(int C, int W, long nch, const unsigned* __restrict__ sc,
                                                  const AgcState* st, int spec, unsigned long long* __restrict__ flags)
{
    LDSP_LATENCY_CRITICAL();
    const long kk = (long)blockIdx.x * 64 + threadIdx.x;
    bool bad = false;
    if (kk < nch && (spec == 2 ? kk >= 1 : spec ? true : (kk >= 1 && kk * C - W > 0))) {
#pragma unroll
        for (int i = 0; i < 4; i++) bad |= sc[kk * 8 + i] != pred_word(sc, st, kk, i);
    }
    const unsigned long long m = __ballot(bad);
    if (threadIdx.x == 0) flags[blockIdx.x] = m;
}
struct AgcFlagsArgs {
    int C;
    int W;
    long nch;
    const unsigned* sc;
    const AgcState* st;
    int spec;
    unsigned long long* flags;
};
__device__ __forceinline__ void k_agc_flags_run(const AgcFlagsArgs& a) { k_agc_flags_body(a.C, a.W, a.nch, a.sc, a.st, a.spec, a.flags); }
LDSP_KERNEL_PAIR(k_agc_flags, AgcFlagsArgs, k_agc_flags_run, 64)


// WIDE: each re-run by the whole wave (agc_chunk_wide, the chunk staged in
// dynamic LDS) instead of lane 0 alone -- the re-runs are serial, chunk after
// chunk, so their latency is the verifier's.
template <bool WIDE>
__device__ __forceinline__ void k_agc_verify_body(const float2* __restrict__ x, long n, AgcState* st, int C, int W,
                                                   int spec, long nch, unsigned* __restrict__ sc,
                                                   const unsigned long long* __restrict__ flags, float2* __restrict__ y,
                                                   uint8_t* __restrict__ status, unsigned* dbg, unsigned* cp, int seg)
{
    LDSP_LATENCY_CRITICAL();
    const int lane = threadIdx.x;
    const AgcState p = *st;
    const long nw = (nch + 63) / 64;
    long k = spec ? 0 : 1;
    // chunk k's predecessor was re-run, or (spec 2) chunk 0 was presumed right by
    // the repair rounds: compare states, not the flag
    bool direct = spec == 2;
    while (k < nch) {
        long kb;
        if (direct) {
            bool bad = false;
            if ((spec || k * C - W > 0) && lane < 4) bad = ldntu(sc + k * 8 + lane) != pred_word(sc, st, k, lane);
            if (__ballot(bad) == 0) {
                direct = false;
                k++;
                continue;
            }
            kb = k;
        } else {
            // flags of 64 x 64 chunks per step (k_agc_flags)
            const long wk = k >> 6;
            unsigned long long w = (wk + lane < nw) ? flags[wk + lane] : 0ull;
            if (lane == 0) w &= ~0ull << (k & 63);
            const unsigned long long bm = __ballot(w != 0ull);
            if (bm == 0) {
                k = (wk + 64) << 6;
                continue;
            }
            const int L = __builtin_ctzll(bm);
            const unsigned long long wd =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(w >> 32), L) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w, L);
            kb = ((wk + L) << 6) + __builtin_ctzll(wd);
            if (kb >= nch) break;
        }
        if constexpr (WIDE) {
            extern __shared__ float2 xs[];
            AgcReg T{__uint_as_float(pred_word(sc, st, kb, 0)), __uint_as_float(pred_word(sc, st, kb, 1)),
                     (int)pred_word(sc, st, kb, 2), pred_word(sc, st, kb, 3)};
            agc_chunk_wide(x, n, p, C, seg, kb, sc + kb * 8, cp ? cp + kb * (C / kAgcCp) * 4 : nullptr, xs, y, status, T);
            if (lane == 0) {
                if (dbg) dbg[0]++;
                st->pad[1]++;                               // ldsp_debug_agc_reruns (verifier)
            }
        } else if (lane == 0) {
            AgcReg r{__uint_as_float(pred_word(sc, st, kb, 0)), __uint_as_float(pred_word(sc, st, kb, 1)),
                     (int)pred_word(sc, st, kb, 2), pred_word(sc, st, kb, 3)};
            unsigned* en = sc + kb * 8;
            if (cp && agc_run_cp<false>(r, p, x, kb * C, min(n, kb * C + C), y, status, cp + kb * (C / kAgcCp) * 4))
                r = AgcReg{__uint_as_float(ldntu(en + 4)), __uint_as_float(ldntu(en + 5)), (int)ldntu(en + 6),
                           ldntu(en + 7)};      // coalesced: the stored end state stands
            else if (!cp)
                agc_run<true>(r, p, x, kb * C, min(n, kb * C + C), y, status);
            if (dbg) dbg[0]++;
            st->pad[1]++;                                   // ldsp_debug_agc_reruns (verifier)
            en[4] = __float_as_uint(r.g);
            en[5] = __float_as_uint(r.y2p);
            en[6] = (unsigned)r.mode;
            en[7] = r.timer;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        k = kb + 1;
        direct = true;
    }
    if (lane == 0) {
        const unsigned* e = sc + (nch - 1) * 8 + 4;
        st->g = __uint_as_float(ldntu(e));
        st->y2p = __uint_as_float(ldntu(e + 1));
        st->mode = (int)ldntu(e + 2);
        st->timer = ldntu(e + 3);
    }
}
struct AgcVerifyArgs {
    const float2* x;
    long n;
    AgcState* st;
    int C;
    int W;
    int spec;
    long nch;
    unsigned* sc;
    const unsigned long long* flags;
    float2* y;
    uint8_t* status;
    unsigned* dbg;
    unsigned* cp;
    int seg;          // k_agc_verify_wide: samples per lane per window
};
__device__ __forceinline__ void k_agc_verify_run(const AgcVerifyArgs& a) { k_agc_verify_body<false>(a.x, a.n, a.st, a.C, a.W, a.spec, a.nch, a.sc, a.flags, a.y, a.status, a.dbg, a.cp, a.seg); }
LDSP_KERNEL_PAIR(k_agc_verify, AgcVerifyArgs, k_agc_verify_run, 64)
__device__ __forceinline__ void k_agc_verify_wide_run(const AgcVerifyArgs& a) { k_agc_verify_body<true>(a.x, a.n, a.st, a.C, a.W, a.spec, a.nch, a.sc, a.flags, a.y, a.status, a.dbg, a.cp, a.seg); }
LDSP_KERNEL_PAIR(k_agc_verify_wide, AgcVerifyArgs, k_agc_verify_wide_run, 64)


__global__ void k_math_eval(int fn, const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ y,
                            long n)
{
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float r = 0.0f;
    switch (fn) {
    case 0: r = lm_expf(a[i]); break;
    case 1: r = lm_logf(a[i]); break;
    case 2: r = lm_atan2f(a[i], b[i]); break;
    case 3: r = lm_tanhf(a[i]); break;
    case 4: r = __uint_as_float(lm_constrain(a[i])); break;
    case 5: r = lm_expf_loop(a[i]); break;
    case 6: r = lm_logf_loop(a[i]); break;
    case 7: r = lm_atan2f_vsel(a[i], b[i]); break;
    case 8: r = __uint_as_float(lm_constrain_fr(a[i])); break;
    default: break;
    }
    y[i] = r;
}

} // namespace

void agc_seq(const void* x, size_t n, AgcState* st, void* y, uint8_t* status, hipStream_t s)
{
    if (n == 0) return;
    launch("k_agc_seq", k_agc_seq, k_agc_seq_many, dim3(1), dim3(64), 0, s,
           AgcSeqArgs{(const float2*)x, (long)n, st, (float2*)y, status});
}

size_t agc_flags_offset_words(long nchunks) { return (size_t)nchunks * 8 + 8; }     // after records + debug words
// then the flag words, then the checkpoints: [nchunks][C / kAgcCp][4 words] (chunk-parallel calls)
static size_t agc_cp_offset_words(long nchunks) { return agc_flags_offset_words(nchunks) + 2 * ((nchunks + 63) / 64 + 64); }
size_t agc_scratch_bytes(long nchunks, int C)
{
    return (agc_cp_offset_words(nchunks) + (size_t)nchunks * (size_t)(C / kAgcCp) * 4) * 4;
}
// checkpoints for chunks of C >= 2 kAgcCp samples outside the small-call paths
static unsigned* agc_cp(const SpecPlan& p)
{
    return (!(p.tsa & 3) && p.C >= 2 * kAgcCp && p.C % kAgcCp == 0) ? (unsigned*)p.scratch + agc_cp_offset_words(p.nchunks)
                                                                      : nullptr;
}

// the one-wave-per-run repair (k_agc_runfix_wide) for the large chunk-parallel calls
static bool agc_runfix_wide(const SpecPlan& p)
{
    static const bool on = LDSP_KNOB("LDSP_AGC_WIDE", 1) != 0;     // tuning build: A/B against k_agc_runfix
    return on && !(p.tsa & 3) && p.C % 64 == 0 && p.C >= 64 && p.C <= 4096;
}

// samples per lane per window of k_agc_runfix_wide: a window costs ~64 seg
// approximate + seg exact steps, and the repair stops at the first window
// whose checkpoints meet the stored trajectory
static int agc_runfix_seg(const SpecPlan& p)
{
    static const int seg = (int)LDSP_KNOB("LDSP_AGC_WSEG", 4);
    return std::max(1, std::min(seg, p.C / 64));
}

void agc_spec_front(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status, hipStream_t s)
{
    if (n == 0) return;
    if ((p.tsa & 2) && p.nchunks <= 64 && (long)n <= kAgcSmallMax) {
        launch("k_agc_chunks", k_agc_small, k_agc_small_many, dim3(1), dim3(64), n * sizeof(float2), s,
               AgcSmallArgs{(const float2*)x, (long)n, st, p.C, p.nchunks, (float2*)y, status, (p.tsa & 4) ? 1 : 0});
        return;
    }
    launch("k_agc_chunks", k_agc_chunks, k_agc_chunks_many, dim3((unsigned)((p.nchunks + 63) / 64)), dim3(64), 0, s,
           AgcChunksArgs{(const float2*)x, (const float2*)p.hist, (long)p.H, (long)n, (const AgcState*)st, p.C, p.W,
                         p.Wa, p.nchunks, (unsigned*)p.scratch, (float2*)y, status, p.tsa, agc_cp(p)});
}

static void agc_rounds(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status, int spec,
                       hipStream_t s)
{
    unsigned long long* flags = (unsigned long long*)((unsigned*)p.scratch + agc_flags_offset_words(p.nchunks));
    const unsigned nb = (unsigned)((p.nchunks + 63) / 64);
    for (int round = 0; round <= p.rounds; round++) {
        launch("k_agc_flags", k_agc_flags, k_agc_flags_many, dim3(nb), dim3(64), 0, s,
               AgcFlagsArgs{p.C, p.W, p.nchunks, (const unsigned*)p.scratch, (const AgcState*)st, spec, flags});
        if (round == p.rounds) break;
        const AgcRunfixArgs ra{(const float2*)x, (long)n, (const AgcState*)st, p.C, p.nchunks, (unsigned*)p.scratch,
                               (const unsigned long long*)flags, (float2*)y, status, p.dbg ? p.dbg + round : nullptr,
                               agc_cp(p), agc_runfix_seg(p)};
        if (agc_runfix_wide(p))
            launch("k_agc_runfix", k_agc_runfix_wide, k_agc_runfix_wide_many, dim3((unsigned)p.nchunks), dim3(64),
                   (size_t)p.C * sizeof(float2), s, ra);
        else
            launch("k_agc_runfix", k_agc_runfix, k_agc_runfix_many, dim3(nb), dim3(64), 0, s, ra);
    }
}

static void agc_verify(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status, int spec,
                       hipStream_t s)
{
    unsigned long long* flags = (unsigned long long*)((unsigned*)p.scratch + agc_flags_offset_words(p.nchunks));
    const AgcVerifyArgs va{(const float2*)x, (long)n, st, p.C, p.W, spec, p.nchunks, (unsigned*)p.scratch,
                           (const unsigned long long*)flags, (float2*)y, status, p.dbg ? p.dbg + p.rounds : nullptr,
                           agc_cp(p), agc_runfix_seg(p)};
    if (agc_runfix_wide(p))
        launch("k_agc_verify", k_agc_verify_wide, k_agc_verify_wide_many, dim3(1), dim3(64),
               (size_t)p.C * sizeof(float2), s, va);
    else
        launch("k_agc_verify", k_agc_verify, k_agc_verify_many, dim3(1), dim3(64), 0, s, va);
}

void agc_spec_back(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status, hipStream_t s)
{
    if (n == 0) return;
    const int spec = p.H > 0 ? 1 : 0;
    agc_rounds(x, n, st, p, y, status, spec, s);
    agc_verify(x, n, st, p, y, status, spec, s);
}

void agc_spec_repair(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status,
                     hipStream_t s)
{
    if (n == 0) return;
    agc_rounds(x, n, st, p, y, status, 2, s);
}

void agc_spec_verify(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status,
                     hipStream_t s)
{
    if (n == 0) return;
    agc_verify(x, n, st, p, y, status, 2, s);
}

void math_eval(int fn, const float* a, const float* b, float* y, size_t n, hipStream_t s)
{
    if (n == 0) return;
    {
        LDSP_PROF(s, "k_math_eval");
        hipLaunchKernelGGL(k_math_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fn, a, b, y, (long)n);
    }
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
