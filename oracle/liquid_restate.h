/*
 * liquid_restate.h -- C API of the CPU restatement (oracle) of the liquid-dsp
 * algorithms that python-liquiddsp's streaming hot path calls.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product library.
 * See liquid_restate.c for the per-function citations and the "parity
 * unpinned" statement.
 */
#ifndef LIQUID_RESTATE_H
#define LIQUID_RESTATE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- firdes ---------------------------------------------------------- */
float ora_kaiser_beta_As(float as);
float ora_kaiser(unsigned int i, unsigned int wlen, float beta);
float ora_besseli0f(float z);
float ora_lngammaf(float z);
float ora_sincf(float x);
int   ora_firdes_kaiser(unsigned int n, float fc, float as, float mu, float *h);
int   ora_firdes_notch(unsigned int m, float f0, float as, float *h);

/* ---- math (deterministic transcendentals, ora_math.h) ----------------- */
void ora_math_eval(int fn, const float *a, const float *b, float *y, size_t n);

/* ---- firfilt (rrrf: cplx=0, crcf: cplx=1) ----------------------------- */
typedef struct ora_firfilt_s *ora_firfilt;
ora_firfilt ora_firfilt_create(const float *h, unsigned int n, int cplx);
ora_firfilt ora_firfilt_create_kaiser(unsigned int n, float fc, float as, float mu, int cplx);
ora_firfilt ora_firfilt_create_dc_blocker(unsigned int m, float as, int cplx);
void  ora_firfilt_destroy(ora_firfilt q);
void  ora_firfilt_reset(ora_firfilt q);
void  ora_firfilt_set_scale(ora_firfilt q, float s);
float ora_firfilt_get_scale(ora_firfilt q);
unsigned int ora_firfilt_get_length(ora_firfilt q);
void  ora_firfilt_get_taps(ora_firfilt q, float *h);
void  ora_firfilt_freqresponse(ora_firfilt q, float f, float *re, float *im);
void  ora_firfilt_execute_block(ora_firfilt q, const float *x, size_t n, float *y);

/* ---- resamp (rrrf: kind 0, cccf: kind 2) ------------------------------ */
typedef struct ora_resamp_s *ora_resamp;
ora_resamp ora_resamp_create_default(float rate, int kind);   /* kind: 0 rrrf, 1 crcf, 2 cccf */
ora_resamp ora_resamp_create(float rate, unsigned int m, float fc, float as,
                             unsigned int npfb, int kind);
void     ora_resamp_destroy(ora_resamp q);
void     ora_resamp_reset(ora_resamp q);
int      ora_resamp_set_rate(ora_resamp q, float rate);
float    ora_resamp_get_rate(ora_resamp q);
uint32_t ora_resamp_get_step(ora_resamp q);
uint32_t ora_resamp_get_phase(ora_resamp q);
unsigned int ora_resamp_get_npfb(ora_resamp q);
unsigned int ora_resamp_get_taps(ora_resamp q, float *h);  /* prototype h (n-1 taps used) */
size_t   ora_resamp_execute_block(ora_resamp q, const float *x, size_t n, float *y);

/* ---- nco -------------------------------------------------------------- */
typedef struct ora_nco_s *ora_nco;
ora_nco  ora_nco_create(int type);   /* 0 = LIQUID_NCO (table), 1 = LIQUID_VCO */
void     ora_nco_destroy(ora_nco q);
void     ora_nco_reset(ora_nco q);
uint32_t ora_nco_constrain(float theta);
void     ora_nco_set_frequency(ora_nco q, float dtheta);
void     ora_nco_adjust_frequency(ora_nco q, float df);
float    ora_nco_get_frequency(ora_nco q);
void     ora_nco_set_phase(ora_nco q, float phi);
void     ora_nco_adjust_phase(ora_nco q, float dphi);
float    ora_nco_get_phase(ora_nco q);
void     ora_nco_pll_set_bandwidth(ora_nco q, float bw);
void     ora_nco_pll_step(ora_nco q, float dphi);
void     ora_nco_get_state(ora_nco q, uint32_t *theta, uint32_t *dtheta);
void     ora_nco_set_state(ora_nco q, uint32_t theta, uint32_t dtheta);
void     ora_nco_get_table(ora_nco q, float *tab1024);
void     ora_nco_mix_block_up(ora_nco q, const float *x, float *y, size_t n);
void     ora_nco_mix_block_down(ora_nco q, const float *x, float *y, size_t n);

/* ---- iirdes / iirfilt ------------------------------------------------- */
int ora_iirdes(int ftype, int btype, int format, unsigned int n, float fc,
               float f0, float ap, float as, float *B, float *A);
void ora_iirdes_dzpk(int ftype, int btype, unsigned int n, float fc, float f0,
                     float ap, float as, float *zd, float *pd, float *kd);
typedef struct ora_iirfilt_s *ora_iirfilt;
ora_iirfilt ora_iirfilt_create_sos(const float *B, const float *A, unsigned int nsos, int cplx);
ora_iirfilt ora_iirfilt_create_tf(const float *b, unsigned int nb, const float *a,
                                  unsigned int na, int cplx);
ora_iirfilt ora_iirfilt_create_prototype(int ftype, int btype, int format,
                                         unsigned int order, float fc, float f0,
                                         float ap, float as, int cplx);
void ora_iirfilt_destroy(ora_iirfilt q);
void ora_iirfilt_reset(ora_iirfilt q);
unsigned int ora_iirfilt_get_nsos(ora_iirfilt q);
void ora_iirfilt_get_sos(ora_iirfilt q, float *B, float *A);
void ora_iirfilt_freqresponse(ora_iirfilt q, float f, float *re, float *im);
void ora_iirfilt_execute_block(ora_iirfilt q, const float *x, size_t n, float *y);
/* float64 evaluation of the same difference equations (accuracy "truth") */
void ora_iirfilt_execute_block_f64(ora_iirfilt q, const float *x, size_t n, float *y);

/* ---- agc -------------------------------------------------------------- */
typedef struct ora_agc_s *ora_agc;
ora_agc ora_agc_create(void);
void  ora_agc_destroy(ora_agc q);
void  ora_agc_reset(ora_agc q);
void  ora_agc_set_bandwidth(ora_agc q, float bw);
float ora_agc_get_bandwidth(ora_agc q);
void  ora_agc_lock(ora_agc q, int on);
void  ora_agc_squelch_enable(ora_agc q, int on);
void  ora_agc_squelch_set_threshold(ora_agc q, float t);
float ora_agc_squelch_get_threshold(ora_agc q);
void  ora_agc_squelch_set_timeout(ora_agc q, unsigned int t);
int   ora_agc_squelch_get_status(ora_agc q);
float ora_agc_get_gain(ora_agc q);
void  ora_agc_set_gain(ora_agc q, float g);
float ora_agc_get_scale(ora_agc q);
void  ora_agc_set_scale(ora_agc q, float s);
float ora_agc_get_signal_level(ora_agc q);
void  ora_agc_set_signal_level(ora_agc q, float x);
float ora_agc_get_rssi(ora_agc q);
void  ora_agc_set_rssi(ora_agc q, float r);
void  ora_agc_get_state(ora_agc q, float *g, float *y2p, int *mode, unsigned int *timer);
void  ora_agc_set_state(ora_agc q, float g, float y2p, int mode, unsigned int timer);
/* python-liquiddsp AGC::execute semantics (src/agc.hpp:109-128): per sample
 * status in `status` (may be NULL), zeroing in SIGNALLO/ENABLED. */
void  ora_agc_execute_wrapper(ora_agc q, const float *x, size_t n, float *y, uint8_t *status);

/* ---- ampmodem --------------------------------------------------------- */
typedef struct ora_ampmodem_s *ora_ampmodem;
ora_ampmodem ora_ampmodem_create(float mod_index, int type, int suppressed_carrier);
void ora_ampmodem_destroy(ora_ampmodem q);
void ora_ampmodem_reset(ora_ampmodem q);
void ora_ampmodem_demodulate_block(ora_ampmodem q, const float *x, size_t n, float *y);
void ora_ampmodem_get_pll_state(ora_ampmodem q, uint32_t *theta, uint32_t *dtheta);
/* firfilt taps used inside (lowpass 2m+1 taps, dcblock 2m+1 taps) */
void ora_ampmodem_get_taps(ora_ampmodem q, float *lowpass, float *dcblock);
/* the Hilbert transform's 2m quadrature taps (usb / lsb) */
void ora_ampmodem_get_hilbert_taps(ora_ampmodem q, float *hq);

/* ---- firhilbf (complex -> real) ---------------------------------------- */
typedef struct ora_firhilb_s *ora_firhilb;
ora_firhilb ora_firhilb_create(unsigned int m, float as);
void ora_firhilb_destroy(ora_firhilb q);
void ora_firhilb_reset(ora_firhilb q);
void ora_firhilb_get_taps(ora_firhilb q, float *hq);
/* y0: lower sideband retained, y1: upper sideband retained */
void ora_firhilb_c2r_block(ora_firhilb q, const float *x, size_t n, float *y0, float *y1);

/* ---- AMRadio chain (README.md:41-58) ---------------------------------- */
typedef struct ora_amradio_s *ora_amradio;
ora_amradio ora_amradio_create(float bandwidth, float iq_rate, float pcm_rate, int iir_f64);
void   ora_amradio_destroy(ora_amradio q);
size_t ora_amradio_max_out(ora_amradio q, size_t n);
size_t ora_amradio_execute(ora_amradio q, const float *x, size_t n, float *y);

/* ---- freqdem, BroadcastAM ------------------------------------------- */
typedef struct ora_freqdem_s *ora_freqdem;
ora_freqdem ora_freqdem_create(float kf);
void ora_freqdem_destroy(ora_freqdem q);
void ora_freqdem_reset(ora_freqdem q);
void ora_freqdem_demodulate_block(ora_freqdem q, const float *x, size_t n, float *y);
typedef struct ora_bcastam_s *ora_bcastam;
ora_bcastam ora_bcastam_create(unsigned int m, int iir_f64);
void ora_bcastam_destroy(ora_bcastam q);
void ora_bcastam_reset(ora_bcastam q);
void ora_bcastam_demodulate_block(ora_bcastam q, const float *x, size_t n, float *pre, float *y, int iir_f64);

/* ---- FMStereo (src/demod.hpp:4-85) ------------------------------------ */
typedef struct ora_fmstereo_s *ora_fmstereo;
ora_fmstereo ora_fmstereo_create(float iq_rate, float pcm_rate);
void ora_fmstereo_destroy(ora_fmstereo q);
void ora_fmstereo_reset(ora_fmstereo q);
/* y: interleaved (L, R) pairs, capacity 2 n; returns the number of floats written.
 * dbg (optional, 4 n floats): per sample s, re(sc) after the second mix, the
 * phase error, theta bits (internal checks) */
size_t ora_fmstereo_execute(ora_fmstereo q, const float *x, size_t n, float *y, float *dbg);
void ora_fmstereo_get_state(ora_fmstereo q, uint32_t *theta, uint32_t *dtheta, float *pe);
void ora_fmstereo_set_state(ora_fmstereo q, uint32_t theta, uint32_t dtheta, float pe);

#ifdef __cplusplus
}
#endif
#endif
