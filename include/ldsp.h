/*
 * ldsp.h -- C ABI of libldsp, the MI355X (gfx950) streaming-DSP library that
 * replaces the liquid-dsp calls behind python-liquiddsp's hot path.
 *
 * Every entry point below names the reference interface it replaces
 * (colbyAtCRI/python-liquiddsp, paths relative to the repository root) and the
 * liquid-dsp routine that interface calls.  The pybind11 module `liquiddsp`
 * (python-liquiddsp_amd/pybind/liquiddsp_module.cpp) binds these with the same
 * class names, keyword arguments and properties as src/wrapper.cpp; a ctypes or
 * other FFI binding can call them directly.
 *
 * Conventions
 *  - All functions return LDSP_OK (0) or a negative LDSP_E* code; the message
 *    of the last failure on the calling thread is ldsp_last_error().
 *  - Handles are independent; calls on one handle must not overlap in time and
 *    must be issued on one stream (or be externally ordered).
 *  - Sample buffers: complex samples are interleaved float32 (re, im) =
 *    numpy.complex64; real samples float32.  `mem` says whether x / y are host
 *    pointers (LDSP_MEM_HOST: the call stages through the device and returns
 *    after the result is in y) or device pointers (LDSP_MEM_DEVICE: the call
 *    only enqueues work on `stream` (a hipStream_t, NULL = default stream) and
 *    returns immediately).
 *  - Streaming state (filter history, resampler / NCO phase, IIR state, AGC
 *    gain, PLL) lives in device memory owned by the handle and carries across
 *    calls exactly like the liquid objects' internal state.
 *  - Objects can be created and configured without a GPU (design, properties,
 *    freqresponse are host-side); device memory is allocated on first execute.
 */
#ifndef LDSP_H
#define LDSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDSP_OK      0
#define LDSP_EINVAL (-1)   /* invalid configuration / argument (Python ValueError) */
#define LDSP_ENOMEM (-2)   /* allocation failure */
#define LDSP_EHIP   (-3)   /* HIP runtime failure or no GPU (Python RuntimeError) */
#define LDSP_ERANGE (-4)   /* output capacity too small */
#define LDSP_EUNSUP (-5)   /* configuration not implemented */

#define LDSP_MEM_HOST   0
#define LDSP_MEM_DEVICE 1

/* execution modes (exact = bit-identical to the sequential CPU restatement) */
#define LDSP_MODE_FAST  0
#define LDSP_MODE_EXACT 1
#define LDSP_MODE_DIRECT 2   /* FIR only: fast direct form (bitwise invariant to how a stream is cut into calls) */

const char *ldsp_last_error(void);
int ldsp_version(void);
int ldsp_device_count(int *n);
int ldsp_stream_synchronize(void *stream);

/* Page-locked host buffers for LDSP_MEM_HOST calls (no reference counterpart:
 * the reference returns pageable numpy arrays from every __call__,
 * src/firfilter.hpp:25-35, src/iirfilter.hpp:292-298, src/resampler.hpp:144-152).
 * An LDSP_MEM_HOST call whose x or y lies in page-locked memory (from here, or
 * hipHostMalloc / hipHostRegister) copies it by DMA directly instead of through
 * the library's staging buffer, so a chain of host calls that hands one call's
 * output to the next skips two host copies per hand-over.  Blocks are pooled:
 * ldsp_host_free keeps up to 256 MB of them for reuse.  ldsp_host_alloc fails
 * with LDSP_ENOMEM once 1 GB is handed out (callers then use pageable memory). */
int ldsp_host_alloc(size_t bytes, void **p);
int ldsp_host_free(void *p);

/* Test hook: the per-thread staging pools of LDSP_MEM_HOST calls.  A thread
 * takes one pool per device on its first host call and returns it to a
 * process-wide free list when it exits, so *total (pools ever created) stays at
 * the number of threads making host calls concurrently; *idle = pools on the
 * free list. */
int ldsp_debug_host_pools(size_t *total, size_t *idle);

/* Test hook: evaluate the loop transcendentals (ldsp_math.hpp) on the device.
 * fn: 0 exp, 1 log, 2 atan2(a, b), 3 tanh, 4 constrain (y as uint32 bits);
 * 5 exp, 6 log through the loops' fast paths (lm_*_loop); 7 atan2(a, b) in its
 * select-only form (lm_atan2f_vsel: the candidate evaluations of k_pll_seqc and
 * k_fm_pll); 8 constrain through v_fract (lm_constrain_fr: k_fm_pll's chain).
 * a, b, y are device pointers of n floats. */
int ldsp_debug_math_eval(int fn, const float *a, const float *b, float *y, size_t n, void *stream);

/* Test hook (host only, no device): check the loops' fast paths (ldsp_math.hpp
 * lm_logf_fast, lm_expf_fast) against the general functions on every stride-th
 * float bit pattern in [begin, end) that lies in the fast range (fn 0 log,
 * 1 exp).  *checked: patterns in the fast range; *mismatches: how many differ in
 * any bit. */
int ldsp_debug_math_fastcheck(int fn, uint32_t begin, uint32_t end, uint32_t stride, uint64_t *checked,
                              uint64_t *mismatches);

/* Per-kernel device timing (no reference counterpart; measurement support for
 * bench.py).  While enabled every kernel launch is bracketed by a HIP event
 * pair on its stream; the report lists "name calls total_ms" lines. */
int ldsp_profile_enable(int on);
int ldsp_profile_reset(void);
/* time only the launches of the kernel named `kernel` (NULL or "": every kernel) */
int ldsp_profile_only(const char *kernel);
int ldsp_profile_report(char *buf, size_t cap, size_t *len);

/* ------------------------------------------------------------------------
 * FIR filter: firfilt_rrrf (cplx=0) / firfilt_crcf (cplx=1), real taps.
 * Replaces RealFIRFilter (src/firfilter.hpp:13-35, firfilt_rrrf_create /
 * firfilt_rrrf_execute_block), RealDCBlocker (firfilter.hpp:42-44,
 * firfilt_rrrf_create_dc_blocker), RealKaiserBessel (firfilter.hpp:56-61,
 * firfilt_rrrf_create_kaiser + set_scale) and the crcf filter used inside
 * demod.hpp:105,135-136 (new class ComplexFIRFilter).
 * ---------------------------------------------------------------------- */
typedef struct ldsp_firfilt_s *ldsp_firfilt_t;
int ldsp_firfilt_create(const float *h, unsigned int n, int cplx, ldsp_firfilt_t *q);
int ldsp_firfilt_create_kaiser(unsigned int n, float fc, float as, float mu, int cplx, ldsp_firfilt_t *q);
int ldsp_firfilt_create_dc_blocker(unsigned int m, float as, int cplx, ldsp_firfilt_t *q);
int ldsp_firfilt_destroy(ldsp_firfilt_t q);
int ldsp_firfilt_reset(ldsp_firfilt_t q);
int ldsp_firfilt_set_scale(ldsp_firfilt_t q, float scale);
int ldsp_firfilt_get_scale(ldsp_firfilt_t q, float *scale);
int ldsp_firfilt_get_length(ldsp_firfilt_t q, unsigned int *n);
int ldsp_firfilt_get_taps(ldsp_firfilt_t q, float *h);
/* mode: LDSP_MODE_FAST (default; complex data with 48 <= L <= 1025 taps uses
 * overlap-save FFT convolution, HBM-bound), LDSP_MODE_DIRECT (register-blocked
 * direct form), LDSP_MODE_EXACT (liquid dot-product order, bit-identical). */
int ldsp_firfilt_set_mode(ldsp_firfilt_t q, int mode);
int ldsp_firfilt_get_mode(ldsp_firfilt_t q, int *mode);
/* firfilt_*_freqresponse (firfilter.hpp:23-27) */
int ldsp_firfilt_freqresponse(ldsp_firfilt_t q, float f, float *re, float *im);
/* firfilt_*_execute_block (firfilter.hpp:29-35): y[i] = scale * sum_k h[k] x[i-k] */
int ldsp_firfilt_execute(ldsp_firfilt_t q, const void *x, size_t n, void *y, int mem, void *stream);

/* ------------------------------------------------------------------------
 * Arbitrary-rate polyphase resampler: resamp_rrrf (cplx=0) / resamp_cccf
 * (cplx=1).  Replaces RealResampler / ComplexResampler
 * (src/resampler.hpp:72-173: resamp_*_create(rate, m, fc, As, npfb),
 * resamp_*_execute per sample, set_rate, reset, print).
 * ---------------------------------------------------------------------- */
typedef struct ldsp_resamp_s *ldsp_resamp_t;
/* cplx: 0 resamp_rrrf, 1 resamp_cccf (ComplexResampler), 2 resamp_crcf (complex
 * samples, real taps: CResampler) */
int ldsp_resamp_create(float rate, unsigned int m, float fc, float as, unsigned int npfb, int cplx,
                       ldsp_resamp_t *q);
/* resamp_*_create_default(rate): RResampler / CResampler (src/resampler.hpp:10-13,
 * 46-49; wrapper.cpp:15-23).  m = 7, fc = 0.25, As = 60, npfb = 256 (liquid-dsp
 * resamp.proto.c defaults, recalled: parity unpinned). */
int ldsp_resamp_create_default(float rate, int kind, ldsp_resamp_t *q);
int ldsp_resamp_destroy(ldsp_resamp_t q);
int ldsp_resamp_reset(ldsp_resamp_t q);
int ldsp_resamp_set_rate(ldsp_resamp_t q, float rate);
int ldsp_resamp_get_rate(ldsp_resamp_t q, float *rate);
/* npfb (after power-of-two rounding), step, current phase, taps per branch */
int ldsp_resamp_get_info(ldsp_resamp_t q, unsigned int *npfb, uint32_t *step, uint32_t *phase,
                         unsigned int *sub_len);
int ldsp_resamp_get_taps(ldsp_resamp_t q, float *h, unsigned int cap, unsigned int *n);
/* number of outputs the next execute of n inputs will produce (host-side, exact) */
int ldsp_resamp_num_outputs(ldsp_resamp_t q, size_t n, size_t *nout);
int ldsp_resamp_execute(ldsp_resamp_t q, const void *x, size_t n, void *y, size_t cap, size_t *nout,
                        int mem, void *stream);

/* ------------------------------------------------------------------------
 * NCO: nco_crcf (type 0 = LIQUID_NCO table, 1 = LIQUID_VCO).  Replaces NCO
 * (src/nco.hpp:4-81): frequency / phase accessors, PLL helpers and
 * nco_crcf_mix_block_up / _down (nco.hpp:66-80).
 * ---------------------------------------------------------------------- */
typedef struct ldsp_nco_s *ldsp_nco_t;
int ldsp_nco_create(int type, ldsp_nco_t *q);
int ldsp_nco_destroy(ldsp_nco_t q);
int ldsp_nco_reset(ldsp_nco_t q);
int ldsp_nco_set_frequency(ldsp_nco_t q, float f);
int ldsp_nco_get_frequency(ldsp_nco_t q, float *f);
int ldsp_nco_adjust_frequency(ldsp_nco_t q, float df);
int ldsp_nco_set_phase(ldsp_nco_t q, float phi);
int ldsp_nco_get_phase(ldsp_nco_t q, float *phi);
int ldsp_nco_adjust_phase(ldsp_nco_t q, float dphi);
int ldsp_nco_pll_set_bandwidth(ldsp_nco_t q, float bw);
int ldsp_nco_pll_step(ldsp_nco_t q, float dphi);
int ldsp_nco_get_state(ldsp_nco_t q, uint32_t *theta, uint32_t *dtheta);
int ldsp_nco_set_state(ldsp_nco_t q, uint32_t theta, uint32_t dtheta);
int ldsp_nco_mix(ldsp_nco_t q, const void *x, size_t n, void *y, int down, int mem, void *stream);

/* NCO mix fused into a complex FIR: y = fir(nco.mix_down(x)) (down = 1) or
 * fir(nco.mix_up(x)), the chain of BASELINE config 3 (reference src/nco.hpp:74-80
 * NCO::mix_down, then src/firfilter.hpp:29-35 execute_block).  Advances the NCO
 * phase by n * dtheta and the filter's history exactly as ldsp_nco_mix followed
 * by ldsp_firfilt_execute would, with the same output bits; on the filter's
 * overlap-save path (fast mode, table NCO) the mixed samples are formed as the
 * filter loads x and never reach memory (16 B per sample instead of 32).  The
 * filter must be complex (firfilt_crcf); both objects on the buffer's device. */
int ldsp_nco_mix_firfilt(ldsp_nco_t nco, ldsp_firfilt_t fir, const void *x, size_t n, void *y, int down, int mem,
                         void *stream);

/* ------------------------------------------------------------------------
 * IIR filter: iirfilt_rrrf (cplx=0) / iirfilt_crcf (cplx=1).  Replaces
 * ComplexIIRFilter / RealIIRFilter (src/iirfilter.hpp:243-356,
 * iirfilt_*_create_prototype(..., LIQUID_IIRDES_SOS, ...)), the
 * C/R{Lowpass,Highpass,Bandpass,Bandstop}IIR family (iirfilter.hpp:61-241),
 * CIIRFilter / RIIRFilter raw transfer functions (iirfilter.hpp:30-34,140-144,
 * iirfilt_*_create) and DeemphasisFilter (iirfilter.hpp:358-392).
 * ftype: 0 butter 1 cheby1 2 cheby2 3 ellip 4 bessel;
 * btype: 0 lowpass 1 highpass 2 bandpass 3 bandstop.
 * Mode FAST evaluates the cascade as a chunked linear scan in float64 (more
 * accurate than liquid's float32 recursion): in one pass over memory in the
 * filter's modal coordinates when they are well-conditioned, else as a blocked
 * scan of the SOS state; EXACT runs the float32 direct-form II recursion
 * (bit-identical to the restatement): sequentially, or -- for filters that
 * forget their state within 16 384 samples (de-emphasis, DC blockers) -- as
 * speculative chunks started early from zero whose start states a verifier
 * checks bit for bit against their predecessors' (the same bits).  Fast mode
 * takes that path for those filters too.
 * ---------------------------------------------------------------------- */
typedef struct ldsp_iirfilt_s *ldsp_iirfilt_t;
int ldsp_iirfilt_create_prototype(int ftype, int btype, unsigned int order, float fc, float f0,
                                  float ap, float as, int cplx, ldsp_iirfilt_t *q);
int ldsp_iirfilt_create_sos(const float *B, const float *A, unsigned int nsos, int cplx,
                            ldsp_iirfilt_t *q);
int ldsp_iirfilt_create_tf(const float *b, unsigned int nb, const float *a, unsigned int na, int cplx,
                           ldsp_iirfilt_t *q);
/* Test / diagnostic hooks for the fast-mode evaluation.  The fast mode runs the
 * single-pass modal scan (k_iir_modal) when the filter's modal form passed its
 * host check at creation (ok = 1: modes M, look-back depth J in 2048-sample
 * units, check error err), else the blocked SOS-coordinate scan.  path: 0
 * automatic, 1 force the blocked scan, 2 require the modal scan (LDSP_EINVAL
 * when the filter has none), 3 the modal scan with every look-back recomputed
 * from the input (the path a wave takes when a predecessor is late).  A forced
 * path also replaces the speculative exact path of fast-decaying filters;
 * exact mode is unaffected. */
int ldsp_debug_iir_path(ldsp_iirfilt_t q, int path);
/* Diagnostics, no reference counterpart: while dev_buf (device memory, at least
 * objects x 2 x 9 x 4 uint64) is set, every exact SOS launch (k_iir_sect)
 * writes per (object, component, section wave) the shader clocks spent waiting
 * for its input / ring space, forming its input tile, in its recursion, and in
 * all.  NULL turns it off.  Not thread-safe; for timing studies. */
int ldsp_debug_iir_sect_trace(void *dev_buf);
int ldsp_debug_iir_modal_info(ldsp_iirfilt_t q, int *ok, int *modes, int *lookback, double *err);
int ldsp_iirfilt_destroy(ldsp_iirfilt_t q);
int ldsp_iirfilt_reset(ldsp_iirfilt_t q);
int ldsp_iirfilt_set_mode(ldsp_iirfilt_t q, int mode);
int ldsp_iirfilt_get_nsos(ldsp_iirfilt_t q, unsigned int *nsos);
int ldsp_iirfilt_get_sos(ldsp_iirfilt_t q, float *B, float *A);
int ldsp_iirfilt_freqresponse(ldsp_iirfilt_t q, float f, float *re, float *im);
int ldsp_iirfilt_execute(ldsp_iirfilt_t q, const void *x, size_t n, void *y, int mem, void *stream);
/* bytes_to_iq fused into the filter (replaces the pair
 * `filter(bytes_to_iq(raw))`, src/utility.hpp:61-69 + iirfilter.hpp:292-298):
 * x holds n native int16 (I, Q) pairs (4 n bytes), each converted to
 * (float)v / 32767.0f exactly as bytes_to_iq does; y receives n complex64
 * outputs, the same bits as ldsp_bytes_to_iq followed by ldsp_iirfilt_execute.
 * Complex filters only (LDSP_EINVAL otherwise).  The blocked float64 scan (the
 * default fast mode) converts on load, so the input is read at 4 B per sample;
 * the exact and speculative paths convert with one extra pass first. */
int ldsp_iirfilt_execute_iq16(ldsp_iirfilt_t q, const void *x, size_t n, void *y, int mem, void *stream);
/* resamp(iirfilt(x)) in one call: the chain's first two stages (reference
 * README.md:53-54, src/iirfilter.hpp:292-298 then src/resampler.hpp:160-172;
 * an opt-in fusion, not a reference entry point).  y receives the resampler's
 * outputs (*nout = ldsp_resamp_num_outputs(rs, n), at most cap), the same bits
 * and the same state updates of both objects as ldsp_iirfilt_execute into a
 * scratch buffer followed by ldsp_resamp_execute on it.  When the filter takes
 * the modal scan (fast mode) the filter outputs never reach HBM; otherwise the
 * two calls run.  Both objects complex (complex64) or both real. */
int ldsp_iirfilt_resamp_execute(ldsp_iirfilt_t q, ldsp_resamp_t rs, const void *x, size_t n, void *y, size_t cap,
                                size_t *nout, int mem, void *stream);

/* ------------------------------------------------------------------------
 * AGC: agc_crcf.  Replaces AGC (src/agc.hpp:4-149).  execute implements
 * AGC::execute (agc.hpp:109-128): agc_crcf_execute per sample, squelch status
 * polled per sample, output zeroed in SIGNALLO / ENABLED.  When `status` is
 * non-NULL it receives the per-sample squelch status (host array of n bytes;
 * the call then synchronises) so the caller can replay onRise callbacks.
 * ---------------------------------------------------------------------- */
typedef struct ldsp_agc_s *ldsp_agc_t;
int ldsp_agc_create(ldsp_agc_t *q);
/* Test hook: small AGC calls (the one-wave chunk path, 320 <= n < the
 * chunk-parallel threshold) start every chunk but the first 1 ulp away from its
 * approximated state, so the in-kernel check re-runs each of them from its
 * predecessor's end state; the output stays bit-identical to agc_crcf. */
int ldsp_debug_agc_tsa_perturb(ldsp_agc_t q, int on);
/* chunks re-run by that in-kernel check since the object was created */
int ldsp_debug_agc_tsa_reruns(ldsp_agc_t q, unsigned int *count);
/* Test hooks for chunk-parallel calls (above the small-call range): with
 * perturb on, every odd chunk starts from its guessed state with the gain 1 ulp
 * off, so the flag pass marks it and the repair rounds / the verifier re-run it
 * from its predecessor's true end state (output still bit-identical to
 * agc_crcf).  rounds: parallel repair rounds before the one-wave verifier (-1 =
 * the default, 1; 0 = the verifier alone re-runs every flagged chunk).
 * reruns: chunks re-run since the object was created, by the repair rounds
 * (*runfix) and by the verifier (*verify). */
int ldsp_debug_agc_perturb(ldsp_agc_t q, int on);
int ldsp_debug_agc_rounds(ldsp_agc_t q, int rounds);
int ldsp_debug_agc_reruns(ldsp_agc_t q, unsigned int *runfix, unsigned int *verify);
int ldsp_agc_destroy(ldsp_agc_t q);
int ldsp_agc_reset(ldsp_agc_t q);
int ldsp_agc_set_bandwidth(ldsp_agc_t q, float bw);
int ldsp_agc_get_bandwidth(ldsp_agc_t q, float *bw);
int ldsp_agc_lock(ldsp_agc_t q, int on);
int ldsp_agc_squelch_enable(ldsp_agc_t q, int on);
int ldsp_agc_squelch_set_threshold(ldsp_agc_t q, float t);
int ldsp_agc_squelch_get_threshold(ldsp_agc_t q, float *t);
int ldsp_agc_squelch_set_timeout(ldsp_agc_t q, unsigned int t);
int ldsp_agc_squelch_get_status(ldsp_agc_t q, int *status);
int ldsp_agc_get_gain(ldsp_agc_t q, float *g);
int ldsp_agc_set_gain(ldsp_agc_t q, float g);
int ldsp_agc_get_scale(ldsp_agc_t q, float *s);
int ldsp_agc_set_scale(ldsp_agc_t q, float s);
int ldsp_agc_get_signal_level(ldsp_agc_t q, float *x);
int ldsp_agc_set_signal_level(ldsp_agc_t q, float x);
int ldsp_agc_get_rssi(ldsp_agc_t q, float *r);
int ldsp_agc_set_rssi(ldsp_agc_t q, float r);
int ldsp_agc_set_mode(ldsp_agc_t q, int mode);
int ldsp_agc_execute(ldsp_agc_t q, const void *x, size_t n, void *y, uint8_t *status, int mem,
                     void *stream);

/* ------------------------------------------------------------------------
 * AM demodulator: ampmodem (type 0 dsb, 1 usb, 2 lsb).  Replaces AmpModem
 * (src/demod.hpp:221-307: ampmodem_create(mod, type, suppressed_carrier),
 * ampmodem_demodulate_block, ampmodem_reset).  dsb: carrier PLL (carrier) or
 * Costas loop (suppressed); usb / lsb: the carrier PLL then a Hilbert c2r
 * (carrier), or the Hilbert c2r alone (suppressed).
 * ---------------------------------------------------------------------- */
typedef struct ldsp_ampmodem_s *ldsp_ampmodem_t;
int ldsp_ampmodem_create(float mod_index, int type, int suppressed_carrier, ldsp_ampmodem_t *q);
int ldsp_ampmodem_destroy(ldsp_ampmodem_t q);
int ldsp_ampmodem_reset(ldsp_ampmodem_t q);
int ldsp_ampmodem_get_pll_state(ldsp_ampmodem_t q, uint32_t *theta, uint32_t *dtheta);
/* The designs inside (liquid ampmodem_create): carrier lowpass (2m+1 = 51 taps,
 * firfilt_crcf_create_kaiser(51, 0.01, 40, 0)), DC blocker (51 taps,
 * firfilt_rrrf_create_dc_blocker(25, 20)) and the usb / lsb Hilbert transform's
 * 2m = 50 quadrature taps (firhilbf_create(25, 60), see firhilb.proto.c).  Any
 * pointer may be NULL.  Host only. */
int ldsp_ampmodem_get_taps(ldsp_ampmodem_t q, float *lowpass, float *dcblock, float *hilbert);
int ldsp_ampmodem_demodulate(ldsp_ampmodem_t q, const void *x, size_t n, void *y, int mem,
                             void *stream);
/* Diagnostics, no reference counterpart: the exact PLL walk of the last call
 * that ran chunk-parallel (k_pll.hip) -- entries visited, repairs (samples
 * whose true table index differed from the candidate's) and lane-blocks redone
 * sample by sample.  All zero after a sequential (short) call.  Synchronises. */
int ldsp_ampmodem_walk_stats(ldsp_ampmodem_t q, uint64_t *entries, uint64_t *repairs,
                             uint64_t *fallbacks);
/* Diagnostics, no reference counterpart: the carrier-mode short-call loop
 * (k_pll_seqc, calls below 2 048 samples), cumulative since the object's first
 * call: candidate batches stepped and batches redone directly because a table
 * index left its candidate window.  Synchronises. */
int ldsp_ampmodem_seq_stats(ldsp_ampmodem_t q, uint64_t *batches, uint64_t *redone);
/* Diagnostics, no reference counterpart: walker clock counters of the last
 * chunk-parallel call (shader clocks spent walking / waiting at the per-block
 * barrier), written only by the timing variants of a tuning build (zero
 * otherwise).  Synchronises. */
int ldsp_ampmodem_walk_clocks(ldsp_ampmodem_t q, uint64_t *walk, uint64_t *wait);
/* Diagnostics, no reference counterpart: the chunk-parallel walker's active time,
 * cumulative since the object was created -- 10 ns ticks from the moment a walk
 * has the previous call's state (a walker may be dispatched before that and wait
 * on the device) to its end, and the number of walks.  Raises LDSP_EHIP if a
 * walker's wait timed out.  Synchronises. */
int ldsp_ampmodem_walk_active(ldsp_ampmodem_t q, uint64_t *ticks, uint64_t *count);
/* Diagnostics, no reference counterpart: the walker's entry margin B = 2^log2_b
 * for the calls that follow (8..21; 0 restores the default).  A narrower
 * margin leaves fewer entries and fails more gap proofs, so more lane-blocks
 * are redone sample by sample -- the tests use it to exercise that path.
 * Returns the previous setting. */
int ldsp_debug_pll_margin(int log2_b);
/* Test hook, no reference counterpart: the bound of an early-dispatched
 * walker's wait for the previous call's PLL state (10 ns ticks; 0 restores the
 * default 1 s), and a skew added to the epoch the object's next walker waits for
 * (a skew of 1 makes it wait for a launch that never comes, so it times out).
 * A timed-out walk raises LDSP_EHIP at the object's next call or state read
 * until ldsp_ampmodem_reset.  Synchronises. */
int ldsp_debug_ampmodem_handoff(ldsp_ampmodem_t q, uint64_t wait_ticks, int epoch_skew);
/* Diagnostics, no reference counterpart: the walker's early hand-off for the
 * calls that follow (1 on, the default; 0 off: every walker waits for the
 * previous walk in stream order, so a kernel trace's k_pll_walk duration is the
 * walk itself; -1 restores the default).  Returns the previous setting. */
int ldsp_debug_walk_early(int on);

/* ------------------------------------------------------------------------
 * Broadcast AM demodulator.  Replaces BroadcastAM (src/demod.hpp:93-153,
 * wrapper.cpp:259-262): carrier PLL (Kaiser lowpass 2m+1, wdelaycf(m), NCO
 * PLL bw 0.001) followed by a cheby2 SOS highpass DC blocker (order 3,
 * fc 20/48000, Ap 0.5, As 20).  The PLL stage is bit-exact; the DC blocker
 * runs in LDSP_MODE_FAST (fp64 scan) by default, LDSP_MODE_EXACT on request.
 * `pre` (optional, device-or-host like y) receives re(v1) before the blocker.
 * ---------------------------------------------------------------------- */
typedef struct ldsp_bcastam_s *ldsp_bcastam_t;
int ldsp_bcastam_create(unsigned int m, ldsp_bcastam_t *q);
int ldsp_bcastam_destroy(ldsp_bcastam_t q);
int ldsp_bcastam_reset(ldsp_bcastam_t q);
int ldsp_bcastam_set_mode(ldsp_bcastam_t q, int mode);
int ldsp_bcastam_get_mode(ldsp_bcastam_t q, int *mode);
int ldsp_bcastam_demodulate(ldsp_bcastam_t q, const void *x, size_t n, void *y, void *pre, int mem,
                            void *stream);

/* ------------------------------------------------------------------------
 * Frequency demodulator.  Replaces FreqDem (src/demod.hpp:189-219,
 * wrapper.cpp:183-187 -> freqdem_create(kf), freqdem_demodulate_block):
 * y[n] = cargf(conjf(x[n-1]) x[n]) / (2 pi kf), bit-exact.
 * ---------------------------------------------------------------------- */
typedef struct ldsp_freqdem_s *ldsp_freqdem_t;
int ldsp_freqdem_create(float kf, ldsp_freqdem_t *q);
int ldsp_freqdem_destroy(ldsp_freqdem_t q);
int ldsp_freqdem_reset(ldsp_freqdem_t q);
int ldsp_freqdem_get_kf(ldsp_freqdem_t q, float *kf);
int ldsp_freqdem_demodulate(ldsp_freqdem_t q, const void *x, size_t n, void *y, int mem, void *stream);

/* ------------------------------------------------------------------------
 * FM stereo receiver.  Replaces FMStereo (src/demod.hpp:4-85, wrapper.cpp:264-267):
 * freqdem(4) -> composite mixer loop (NCO, PLL bandwidth 0.1, one-pole phase
 * error) -> 75 us de-emphasis per channel -> resamp_rrrf_create_default
 * (pcm_rate / iq_rate) per channel; output interleaved (L, R) float32.
 * Bit-exact; the mixer loop is inherently sequential (one lane).  reset()
 * resets only the resamplers, like the reference.  pcm_rate > iq_rate is
 * LDSP_EUNSUP.  num_outputs counts floats (2 per output pair).
 * ---------------------------------------------------------------------- */
typedef struct ldsp_fmstereo_s *ldsp_fmstereo_t;
int ldsp_fmstereo_create(float iq_rate, float pcm_rate, ldsp_fmstereo_t *q);
int ldsp_fmstereo_destroy(ldsp_fmstereo_t q);
int ldsp_fmstereo_reset(ldsp_fmstereo_t q);
int ldsp_fmstereo_num_outputs(ldsp_fmstereo_t q, size_t n, size_t *nout);
int ldsp_fmstereo_get_state(ldsp_fmstereo_t q, uint32_t *theta, uint32_t *dtheta, float *pe);
int ldsp_fmstereo_execute(ldsp_fmstereo_t q, const void *x, size_t n, void *y, size_t cap, size_t *nout,
                          int mem, void *stream);

/* ------------------------------------------------------------------------
 * Sample delay line.  Replaces Delay (src/utility.hpp:5-57, wrapper.cpp:25-28):
 * separate real (wdelayf) and complex (wdelaycf) lines of nd, read-then-push,
 * i.e. y[n] = x[n - nd - 1].  set_delay re-creates (zeroes) both lines.
 * ---------------------------------------------------------------------- */
typedef struct ldsp_delay_s *ldsp_delay_t;
int ldsp_delay_create(unsigned int nd, ldsp_delay_t *q);
int ldsp_delay_destroy(ldsp_delay_t q);
int ldsp_delay_set_delay(ldsp_delay_t q, unsigned int nd);
int ldsp_delay_get_delay(ldsp_delay_t q, unsigned int *nd);
int ldsp_delay_execute(ldsp_delay_t q, const void *x, size_t n, int cplx, void *y, int mem, void *stream);

/* ------------------------------------------------------------------------
 * Raw IQ conversion.  Replaces bytes_to_iq (src/utility.hpp:61-69,
 * wrapper.cpp:13): interleaved native int16 (I, Q) -> complex64 / 32767.
 * nbytes / 4 samples are converted (a trailing partial sample is ignored).
 * ---------------------------------------------------------------------- */
int ldsp_bytes_to_iq(const void *in, size_t nbytes, void *y, int mem, void *stream);

/* ------------------------------------------------------------------------
 * Many-calls: one call each on C independent objects of one class (no
 * reference counterpart -- the reference's SDR callback runs one channel's
 * chain per call, README.md:53-58; SURVEY 7 H5 / 8(e): channels batched on one
 * GPU).  Equivalent to calling the single-object execute on q[0], .., q[C-1]
 * in turn on `stream`, bit for bit, but every kernel runs as ONE launch for
 * all objects that take the same path (blockIdx.y = object), so a step of C
 * channels issues as many launches as one channel's.  Device pointers only;
 * all objects get n input samples; the objects must be distinct.
 * iirfilt_resamp: nout[c] receives object c's output count (cap per object).
 * ---------------------------------------------------------------------- */
int ldsp_agc_execute_many(ldsp_agc_t *q, const void *const *x, size_t n, void *const *y, int C, void *stream);
int ldsp_ampmodem_demodulate_many(ldsp_ampmodem_t *q, const void *const *x, size_t n, void *const *y, int C,
                                  void *stream);
int ldsp_iirfilt_execute_many(ldsp_iirfilt_t *q, const void *const *x, size_t n, void *const *y, int C,
                              void *stream);
int ldsp_iirfilt_resamp_execute_many(ldsp_iirfilt_t *q, ldsp_resamp_t *rs, const void *const *x, size_t n,
                                     void *const *y, size_t cap, size_t *nout, int C, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LDSP_H */
