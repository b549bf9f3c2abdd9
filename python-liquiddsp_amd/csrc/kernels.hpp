// kernels.hpp -- host launchers for the gfx950 kernels of libldsp.
// All pointers are device pointers; every launcher only enqueues on `s`.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace ldsp {
namespace k {

// ------------------------------------------------------------------ FIR
// y[i] = scale * sum_{k<L} h[k] xv[i-k], xv[j<0] = hist[j + L - 1]; writes the
// new history (last L-1 samples of xv) to hist_out.  taps_pad has
// ceil(L/16)*16 floats (zero padded).  fast: register-blocked FMA kernel;
// exact: liquid dotprod order (oldest sample first, separate mul and add).
constexpr int kFirMaxTaps = 8192;
void fir_fast(bool cplx, const void* x, const void* hist, void* hist_out, size_t n,
              const float* taps_pad, int L, float scale, void* y, hipStream_t s);
void fir_exact(bool cplx, const void* x, const void* hist, void* hist_out, size_t n,
               const float* taps_rev, int L, float scale, void* y, hipStream_t s);
// history update only (n == 0 calls skip the kernels)

// Overlap-save FFT convolution (complex samples, real taps), k_firfft.hip.
// P = history samples per window (L - 1 <= P <= 512, multiple of 64); the
// window has fir_fft_points(P) = 512 (P <= 128) or 1024 points.
// H[N] = scale * FFT(h) / N for that N; tw = Stockham twiddles
// exp(-2 pi i r k / (Ns R)) laid out [pass][r-1][k]:
//   N = 512 : (Ns, R) = (8, 8), (64, 8)      -> kFft512Tw entries
//   N = 1024: (Ns, R) = (16, 16), (256, 4)   -> kFft1024Tw entries
constexpr int kFft512Tw = 7 * 8 + 7 * 64;
constexpr int kFft1024Tw = 15 * 16 + 3 * 256;
int fir_fft_points(int P);
// Optional NCO mix fused into the window loads (table NCO, nco_crcf_mix_block_*):
// sample i enters as x[i] e^{-+j theta}, theta = theta0 + i dtheta; hist then
// holds mixed samples, like the filter's own history after a separate mix.
struct NcoFuse {
    uint32_t theta0, dtheta;
    bool down;
    const float* table;   // device sine table (1024)
};
void fir_fft(const void* x, const void* hist, void* hist_out, size_t n, int L, int P, const void* H, const void* tw,
             void* y, hipStream_t s, const NcoFuse* nco = nullptr);

// ------------------------------------------------------------------ resampler
struct ResampPlan {
    uint64_t P0;          // phase at call start (resamp "phase", < 2^24 + step)
    uint32_t step;        // round(2^24 / rate)
    int bits_index;       // 24 - log2(npfb)
    int sub_len;          // taps per branch (2m)
    int npfb;
    size_t K;             // outputs of this call
    int KB;               // outputs per workgroup
    int span_max;         // LDS samples per workgroup
    int tile = 0;         // 1: k_resamp_tile (span streamed into LDS with 16-byte loads), KB from resamp_tile_outputs
};
// Outputs per workgroup of the tile kernel (0: its LDS would not fit; use the others).
int resamp_tile_outputs(uint32_t step, int sub_len, int npfb, bool cplx, bool real_taps);
// sub: [npfb][sub_len] branch taps reversed (cccf: complex64 with imag 0; rrrf, crcf: float)
void resamp(bool cplx, bool real_taps, const void* x, const void* hist, void* hist_out, size_t n, const float* sub,
            const ResampPlan& p, void* y, hipStream_t s);

// ------------------------------------------------------------------ NCO
void nco_mix(const void* x, void* y, size_t n, uint32_t theta0, uint32_t dtheta, const float* table,
             bool down, int type, hipStream_t s);

// ------------------------------------------------------------------ IIR
// Structure of one IIR filter for the kernels.  SOS: nsos sections b[3],a[3]
// (a0 == 1); TF: nb, na coefficients (a0 == 1), nv = max(nb, na).
constexpr int kIirMaxState = 16;
struct IirDesc {
    int sos;              // 1 SOS cascade, 0 TF
    int nsos;
    int nb, na, nv;
    int D;                // state dimension (SOS: 2 nsos, TF: nv - 1)
    const float* b;       // device coefficients
    const float* a;
};
// Sequential float32 evaluation (bit-exact with the liquid recursion).
// state: float[2][3*nsos] (SOS) or float[2][nv] (TF); cplx -> 2 components.
void iir_seq(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, void* y, hipStream_t s);
// Sections per cascade of the exact kernel below.
constexpr int kIirSectMaxSos = 8;
// The same recursion with one wave per section and one workgroup per (object,
// component) (k_iir_sect.hip); mergeable in many-calls.  iir_seq uses it for SOS
// cascades of <= kIirSectMaxSos sections.
void iir_sect(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, void* y, hipStream_t s);
int iir_sect_trace(void* dev_buf);     // diagnostics: ldsp_debug_iir_sect_trace
// Float64 chunked linear scan.  state64: double[2][D] (the DF-II delay line in
// the layout used by the scan); Apow: double[D*D] matrices: [0] = A^C,
// [1 + l] = A^{C G 2^l} prepared by the host (see IirScanPlan).
struct IirScanPlan {
    int C;                // samples per chunk
    long nchunks;
    int G;                // chunks per scan thread (1024 scan threads)
    int levels;           // 10 = log2(1024)
    const double* AC;     // A^C           [D*D]
    const double* AG;     // A^{C*G*2^l}    [levels][D*D]
    double* local;        // [nchunks][ncomp][D] scratch: chunk end state from zero
    double* carry;        // [nchunks][ncomp][D] scratch: chunk start state
};
void iir_scan(bool cplx, const IirDesc& d, const void* x, size_t n, double* state64, const IirScanPlan& p,
              void* y, hipStream_t s);
// Blocked float64 scan for state dimension D <= kIirBlkMaxD (k_iir_blk):
// chunks of 256 samples, 256 chunks per block.  hb/ha: host copies of the
// float32 coefficients (SOS [nsos][3] or TF [nb] / [na]), passed by value.
constexpr int kIirBlkMaxD = 8;
constexpr int kIirBlkChunk = 256;
constexpr int kIirBlkChunks = 256;
struct IirBlkPlan {
    long nchunks, nblk;
    int G;                // blocks per carry thread
    const double* AL;     // A^{256 * 2^l}, l = 0..7             [8][D*D]
    const double* AB;     // A^{65536}                            [D*D]
    const double* AG;     // A^{65536 * G * 2^l}, l = 0..9         [10][D*D]
    double* local;        // [nchunks][ncomp][D]
    double* blocal;       // [nblk][ncomp][D]
    double* bstart;       // [nblk][ncomp][D]
};
// iq16: x holds int16 (I, Q) pairs, converted on load as bytes_to_iq does
void iir_blk(bool cplx, const IirDesc& d, const float* hb, const float* ha, const void* x, size_t n, double* state64,
             const IirBlkPlan& p, void* y, hipStream_t s, bool iq16 = false);
// Single-pass float64 scan in modal coordinates (k_iir_modal.hip): the filter
// as M <= 8 parallel sections (one per pole pair or real pole) in direct form,
// w_n = u_n - a1 w_{n-1} - a2 w_{n-2}, y = d u + sum_k c1 w_{n-1} + c2 w_{n-2}
// (modal.hpp).  One wave = 64 chunks of kIirModalChunk samples; each unit's
// start state is the look-back sum over the J <= kIirModalJmax units before it
// (valid when max|lambda|^(2048 J) < 2^-70).  State layout (st_in / st_out,
// distinct buffers): double [ncomp][M][w_n, w_{n-1}].
constexpr int kIirModalMax = 8;
constexpr int kIirModalChunk = 32;
constexpr int kIirModalJmax = 64;
struct IirModalCoef {     // kernel argument
    int M;
    double a1[kIirModalMax], a2[kIirModalMax];   // section denominators
    double c1[kIirModalMax], c2[kIirModalMax];   // section outputs
    double d;                                    // direct term
};
struct IirModalPlan {
    int J;                // look-back depth (units)
    const double* PS;     // [6][M][4]   A_k^(32 * 2^l), l = 0..5 (2 x 2, row-major)
    const double* PL;     // [64][M][4]  A_k^(32 t), t = lane
    const double* PB;     // [J][M][4]   A_k^(2048 i)
    uint64_t* agg;        // [nunits][ncomp][M * 4] {32-bit half, epoch} granules (zeroed when allocated)
    uint32_t epoch;       // per call, never 0
    int recompute = 0;    // test hook: every wave recomputes its predecessors instead of reading them
    int one_xcd = 0;      // small call: every unit on the XCD of block 0 (a grid of 8 x units, the
                          // blocks of the other XCDs return at once), so no unit recomputes a predecessor
    int variant = 0;      // tuning builds only (timing experiments, wrong outputs): bit 0 no look-back,
                          // bit 1 no pass 2, bit 2 no pass 1 / scan; bit 3 stagger the first
                          // round of workgroups by (variant >> 4) sleeps (outputs unchanged)
};
// IIR -> resampler fusion (liquiddsp.filter_resample, k_iir_modal<RS>): each unit's
// filter outputs stay in LDS and feed the resampler outputs whose sub_len-sample
// window lies inside the unit (the resampler's own arithmetic, resamp_dev.hpp);
// the unit's first and last H = sub_len - 1 outputs go to `side`, from which
// k_iir_resamp_edges computes the outputs whose window straddles a unit boundary
// (and the resampler's new history).  The filter outputs never reach HBM.
struct IirResampFuse {
    const float* sub;     // [npfb][sub_len] branch taps, reversed (ResampObj::sub; complex interleaved if ctaps)
    uint64_t P0;          // the resampler's phase at the call's start
    uint32_t step;
    int bits_index, sub_len;
    int ctaps;            // complex taps (resamp_cccf, the ComplexResampler): rs_mac over both components
    long K;               // outputs of the call
    float* side;          // [units][2][H][ncomp]: head (first H) and tail (last H, right-aligned) outputs
    float* y;             // resampler outputs ([K][ncomp] floats)
};
size_t iir_resamp_side_bytes(size_t n, int sub_len, bool cplx);
void iir_modal_resamp(bool cplx, const IirModalCoef& cf, const void* x, size_t n, const double* st_in,
                      double* st_out, const IirModalPlan& p, const IirResampFuse& f, const void* hist,
                      void* hist_out, hipStream_t s);
long iir_modal_units(size_t n);   // workgroups (2048-sample look-back units) of a call
void iir_modal(bool cplx, const IirModalCoef& cf, const void* x, size_t n, const double* st_in, double* st_out,
               const IirModalPlan& p, void* y, hipStream_t s, bool iq16 = false);
// Speculative exact evaluation for fast-decaying filters: chunks start from a
// zero state W samples early; a verifier re-runs any chunk whose guessed
// start state differs bit-wise from its predecessor's end state.
struct SpecPlan {
    int C;                // samples per chunk
    int W;                // warm-up samples (exact)
    int Wa = 0;           // AGC: approximate warm-up before the exact one
    int rounds = 0;       // AGC: parallel repair rounds before the sequential verifier
    unsigned* dbg = nullptr;   // AGC debug: per-round re-run counters (LDSP_DEBUG_AGC)
    long nchunks;
    void* scratch;        // device scratch (states: start-guess and end per chunk)
    const void* hist = nullptr;   // AGC: the H input samples before x[0] (H > 0: every chunk speculative)
    int H = 0;
    int tsa = 0;          // AGC small call: every chunk approximates from the true state up to its start
                          // (2: one wave, which also checks and repairs the chunks in order;
                          // | 4: test hook, every chunk's start state 1 ulp off;
                          // | 8: test hook, chunk-parallel call: odd chunks start 1 ulp off)
};
// scratch for iir_spec: chunk states + verifier flag words
size_t spec_flags_offset(long nchunks, int ncomp, int fs);
size_t spec_scratch_bytes(long nchunks, int ncomp, int fs);
void iir_spec(bool cplx, const IirDesc& d, const void* x, size_t n, float* state, const SpecPlan& p, void* y,
              hipStream_t s);

// ------------------------------------------------------------------ AGC
struct AgcState {         // device-resident agc_crcf state
    float g, y2p, alpha, scale;
    int locked, mode;
    unsigned int timer, timeout;
    float threshold;
    int pad[3];           // test counters: [0] small-call in-kernel re-runs, [1] verifier re-runs, [2] runfix re-runs
};
constexpr int kAgcPow = 256;     // samples whose mean power sets a chunk's guessed gain
void agc_seq(const void* x, size_t n, AgcState* st, void* y, uint8_t* status, hipStream_t s);
size_t agc_scratch_bytes(long nchunks, int C);
// Chunk-parallel exact AGC in two halves.  Front: the chunks (reads only the
// parameters when p.H > 0, so it may run while the previous call's back half
// still advances the state).  Back: flag / repair rounds and the verifier
// against the true state, which it then advances.
void agc_spec_front(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status,
                    hipStream_t s);
void agc_spec_back(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status,
                   hipStream_t s);
// A speculative call's back half in two parts: the repair rounds over chunks
// 1.. (chunk 0 presumed right: they read only the chunk records, so they may
// run while the previous call is still producing the true state), then -- after
// it -- the verifier, which checks chunk 0 against the true state, re-runs
// whatever the rounds left and advances the state: the only AGC work on the
// chain from one call to the next.
void agc_spec_repair(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status,
                     hipStream_t s);
void agc_spec_verify(const void* x, size_t n, AgcState* st, const SpecPlan& p, void* y, uint8_t* status,
                     hipStream_t s);
// hist_out = the last m samples of (hist, x[0, n)) (complex), for the next call.
void delay_hist(const void* x, const void* hist, void* hist_out, size_t n, int m, hipStream_t s);

// ------------------------------------------------------------------ AmpModem
struct AmpState {         // device-resident PLL state
    uint32_t theta, dtheta;   // true loop state (written by the walker / sequential loop)
    float alpha, beta;
    uint32_t gth[2], gd[2];   // ping-pong guess of the state at the next call's start (candidate end state)
    uint32_t sq_batches;      // k_pll_seqc diagnostics, cumulative: candidate batches stepped,
    uint32_t sq_redone;       //   and batches with a step evaluated by pll_eval (an index left its window)
    // hand-off: every launch that writes theta / dtheta advances wepoch after them
    // (release); a walker launched early waits until wepoch equals its call's index
    uint32_t wepoch;
    uint32_t werr;            // 1: a walker's hand-off wait timed out (the host raises)
    unsigned long long wact;  // walker ticks (10 ns) from hand-off to end, cumulative
    unsigned long long wact_n;
    unsigned long long wait_ticks;   // bound of the hand-off wait (10 ns ticks; 1 s unless a test shortens it)
    uint32_t* herr;           // host-mapped flag the walker also sets on a timeout: checked at every call's
                              // entry, so a timed-out walk is never returned silently (capi.cpp amp_check_err)
};
// One AmpModem / BroadcastAM PLL call.  x0 = lowpass(x) (precomputed), x1 =
// delay_m(x) via hist (m samples before x[0]); writes Re(v1)/mod (carrier) or
// the final output (Costas) to y.  scratch (pll_scratch_bytes(n)) holds the
// candidate records of the chunk-parallel exact path (k_pll.hip).
struct PllCall {
    const void* x0;
    const void* x;
    const void* hist;     // m samples before x[0]
    void* hist_out;       // m samples before the next call's x[0]
    int m;
    size_t n;
    AmpState* st;
    int gcur;             // candidates start from st->gth/gd[gcur], leave the next guess in [1 - gcur]
    const float* table;
    float mod_index;
    int costas;
    int out_idx;          // 1: write each sample's table index (uint32 bits) instead of its output (SSB: the
                          //    Hilbert stage recomputes v1 from it)
    float alpha_host;
    float* y;
    void* scratch;
    uint32_t wexp;        // launches that wrote the PLL state before this call's (AmpState::wepoch)
};
size_t pll_scratch_bytes(size_t n);
size_t pll_stats_offset(size_t n);     // 4 x u64 walker counters inside the scratch (debug)
// True when the call runs as candidates + walker (else one sequential loop in pll_back).
bool pll_parallel(size_t n, int costas);
// Front half: the delay-line history for the next call and (parallel calls)
// the candidate chunks.  Reads only the guess state, never the true state, so
// it may run while the previous call's pll_back is still walking.
void pll_front(const PllCall& c, hipStream_t s);
int pll_margin_override(int log2_b);       // diagnostics: 0 = default; returns the previous value
// Back half: the exact walk over the candidates (or the sequential loop);
// reads and advances the true state, so it must follow the previous call's back half.
void pll_back(const PllCall& c, hipStream_t s);

// ------------------------------------------------------------------ debug
void math_eval(int fn, const float* a, const float* b, float* y, size_t n, hipStream_t s);

// k_misc.hip: bytes_to_iq, delay line, frequency discriminator
void bytes_to_iq(const void* x, void* y, size_t n, hipStream_t s);
void delay(bool cplx, const void* x, const void* hist, void* hist_out, size_t n, int D, void* y, hipStream_t s);
void freqdem(const void* x, const void* prev, void* prev_out, size_t n, float ref, float* y, hipStream_t s);
// AmpModem usb / lsb: v1 = delay_m(x) mixed down by the per-sample table index idx
// (the PLL stage's out_idx output); Hilbert c2r over x (4M - 1 samples of history
// before x[0]) -> 0.5 * sideband / mod_index.
void ssb_v1(const void* idx, const void* x, const void* dhist, int m, const float* table, size_t n, void* v1,
            hipStream_t s);
void ssb_c2r(const void* x, const void* hist, size_t n, const float* hq, int M, int usb, float mod_index, float* y,
             hipStream_t s);
struct FmState {          // FMStereo mixer loop state (device-resident)
    uint32_t theta, dtheta;
    float pe, alpha, beta;
};
void fm_pll(const float* s, size_t n, FmState* st, const float* table, float* l, float* r, hipStream_t strm);
void interleave2(const float* a, const float* b, size_t n, float* y, hipStream_t strm);

} // namespace k
} // namespace ldsp
