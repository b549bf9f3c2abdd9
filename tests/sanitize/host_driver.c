/* Host-only exercise of libldsp's C ABI under ASan / UBSan (sanitizers
 * on host code; the GPU pool runs none).  Linked against the library built with
 * `make -C python-liquiddsp_amd asan` (capi / design / modal host code
 * instrumented, kernel objects as built) and run without a GPU by
 * tests/test_sanitizers.py: every designer (iirdes all prototypes x bands x
 * orders, firdes, resampler, AmpModem / FMStereo / BroadcastAM setup), every
 * property, the error paths (NULL handles, invalid designs, capacities) and the
 * execute calls that must fail cleanly with LDSP_EHIP when no device exists.
 * Exit status 0 = every check held; the sanitizers abort on the first report. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ldsp.h"

static int fails = 0;
#define CHECK(c)                                                                    \
    do {                                                                            \
        if (!(c)) {                                                                 \
            fprintf(stderr, "check failed at %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, \
                    ldsp_last_error());                                             \
            fails++;                                                                \
        }                                                                           \
    } while (0)

static void iir_designs(void)
{
    const float fcs[] = {0.0075f, 0.1f, 0.3f};
    for (int ft = 0; ft < 5; ft++)
        for (int bt = 0; bt < 4; bt++)
            for (unsigned order = 1; order <= 10; order++)
                for (int k = 0; k < 3; k++)
                    for (int cplx = 0; cplx < 2; cplx++) {
                        ldsp_iirfilt_t q = NULL;
                        int rc = ldsp_iirfilt_create_prototype(ft, bt, order, fcs[k], 0.25f, 0.7f, 60.0f, cplx, &q);
                        if (rc != LDSP_OK) {
                            CHECK(q == NULL && strlen(ldsp_last_error()) > 0);
                            continue;
                        }
                        unsigned nsos = 0;
                        CHECK(ldsp_iirfilt_get_nsos(q, &nsos) == LDSP_OK && nsos >= 1 && nsos <= 16);
                        float B[3 * 16], A[3 * 16];
                        CHECK(ldsp_iirfilt_get_sos(q, B, A) == LDSP_OK);
                        for (int i = 0; i < 8; i++) {
                            float re = 0, im = 0;
                            CHECK(ldsp_iirfilt_freqresponse(q, -0.5f + i / 8.0f, &re, &im) == LDSP_OK);
                        }
                        int ok = 0, modes = 0, lb = 0;
                        double err = 0;
                        CHECK(ldsp_debug_iir_modal_info(q, &ok, &modes, &lb, &err) == LDSP_OK);
                        CHECK(ldsp_iirfilt_set_mode(q, LDSP_MODE_EXACT) == LDSP_OK);
                        CHECK(ldsp_iirfilt_reset(q) == LDSP_OK);
                        CHECK(ldsp_iirfilt_destroy(q) == LDSP_OK);
                    }
    /* transfer-function and SOS constructors, de-emphasis */
    const float x = expf(-1.0f / (75e-6f * 48000.0f));
    const float b[1] = {1.0f - x}, a[2] = {1.0f, -x};
    ldsp_iirfilt_t q = NULL;
    CHECK(ldsp_iirfilt_create_tf(b, 1, a, 2, 0, &q) == LDSP_OK);
    float re, im;
    CHECK(ldsp_iirfilt_freqresponse(q, 0.1f, &re, &im) == LDSP_OK);
    CHECK(ldsp_iirfilt_destroy(q) == LDSP_OK);
    const float b5[5] = {0.1f, 0.2f, 0.3f, 0.2f, 0.1f}, a5[5] = {1.0f, -0.5f, 0.25f, -0.125f, 0.0625f};
    CHECK(ldsp_iirfilt_create_tf(b5, 5, a5, 5, 1, &q) == LDSP_OK);
    CHECK(ldsp_iirfilt_destroy(q) == LDSP_OK);
    const float Bs[6] = {1, 2, 1, 1, 0, -1}, As[6] = {1, -0.5f, 0.2f, 1, 0.1f, 0.3f};
    CHECK(ldsp_iirfilt_create_sos(Bs, As, 2, 1, &q) == LDSP_OK);
    CHECK(ldsp_iirfilt_destroy(q) == LDSP_OK);
    /* invalid: a0 = 0, no coefficients, bad cutoff */
    const float az[2] = {0.0f, 1.0f};
    q = NULL;
    CHECK(ldsp_iirfilt_create_tf(b, 1, az, 2, 0, &q) != LDSP_OK && q == NULL);
    CHECK(ldsp_iirfilt_create_tf(b, 0, a, 2, 0, &q) != LDSP_OK);
    CHECK(ldsp_iirfilt_create_prototype(2, 0, 8, 0.7f, 0.3f, 0.7f, 60.0f, 1, &q) != LDSP_OK);
    CHECK(ldsp_iirfilt_create_prototype(2, 0, 0, 0.1f, 0.3f, 0.7f, 60.0f, 1, &q) != LDSP_OK);
}

static void fir_designs(void)
{
    for (unsigned n = 1; n <= 1100; n += 37)
        for (int cplx = 0; cplx < 2; cplx++) {
            ldsp_firfilt_t q = NULL;
            if (ldsp_firfilt_create_kaiser(n, 0.1f, 60.0f, 0.0f, cplx, &q) != LDSP_OK) continue;
            unsigned len = 0;
            CHECK(ldsp_firfilt_get_length(q, &len) == LDSP_OK && len == n);
            float* h = (float*)malloc(sizeof(float) * n);
            CHECK(ldsp_firfilt_get_taps(q, h) == LDSP_OK);
            free(h);
            float re, im;
            CHECK(ldsp_firfilt_freqresponse(q, 0.05f, &re, &im) == LDSP_OK);
            CHECK(ldsp_firfilt_set_scale(q, 0.5f) == LDSP_OK);
            for (int m = 0; m < 3; m++) CHECK(ldsp_firfilt_set_mode(q, m) == LDSP_OK);
            CHECK(ldsp_firfilt_set_mode(q, 9) != LDSP_OK);
            CHECK(ldsp_firfilt_destroy(q) == LDSP_OK);
        }
    ldsp_firfilt_t q = NULL;
    CHECK(ldsp_firfilt_create_dc_blocker(25, 20.0f, 0, &q) == LDSP_OK);
    CHECK(ldsp_firfilt_destroy(q) == LDSP_OK);
    const float h3[3] = {0.25f, 0.5f, 0.25f};
    CHECK(ldsp_firfilt_create(h3, 3, 1, &q) == LDSP_OK);
    float y[8], xx[16] = {0};
    CHECK(ldsp_firfilt_execute(q, xx, 8, y, LDSP_MEM_HOST, NULL) == LDSP_EHIP);   /* no device */
    CHECK(ldsp_firfilt_destroy(q) == LDSP_OK);
    CHECK(ldsp_firfilt_create(h3, 0, 1, &q) != LDSP_OK);
    CHECK(ldsp_firfilt_create_kaiser(0, 0.1f, 60.0f, 0.0f, 1, &q) != LDSP_OK);
    CHECK(ldsp_firfilt_create_kaiser(51, 0.6f, 60.0f, 0.0f, 1, &q) != LDSP_OK);
}

static void resamplers(void)
{
    const float rates[] = {0.004f, 0.024f, 0.3f, 0.5f, 1.0f, 1.7f, 7.3f};
    for (int r = 0; r < 7; r++)
        for (int kind = 0; kind < 3; kind++) {
            ldsp_resamp_t q = NULL;
            if (ldsp_resamp_create(rates[r], 20, 0.024f, 60.0f, 13, kind, &q) != LDSP_OK) continue;
            size_t nout = 0;
            for (size_t n = 0; n < 200000; n = n * 3 + 1) CHECK(ldsp_resamp_num_outputs(q, n, &nout) == LDSP_OK);
            unsigned npfb, sub;
            uint32_t step, phase;
            CHECK(ldsp_resamp_get_info(q, &npfb, &step, &phase, &sub) == LDSP_OK);
            unsigned nt = 0;
            CHECK(ldsp_resamp_get_taps(q, NULL, 0, &nt) == LDSP_OK);
            float* h = (float*)malloc(sizeof(float) * (nt ? nt : 1));
            CHECK(ldsp_resamp_get_taps(q, h, nt, &nt) == LDSP_OK);
            free(h);
            CHECK(ldsp_resamp_set_rate(q, rates[(r + 1) % 7]) == LDSP_OK);
            float got = 0;
            CHECK(ldsp_resamp_get_rate(q, &got) == LDSP_OK);
            float xx[64] = {0}, y[8];
            /* too small an output: LDSP_ERANGE before any device work */
            CHECK(ldsp_resamp_execute(q, xx, 32, y, 0, &nout, LDSP_MEM_HOST, NULL) != LDSP_OK);
            CHECK(ldsp_resamp_reset(q) == LDSP_OK);
            CHECK(ldsp_resamp_destroy(q) == LDSP_OK);
        }
    for (int kind = 0; kind < 2; kind++) {
        ldsp_resamp_t q = NULL;
        CHECK(ldsp_resamp_create_default(0.024f, kind, &q) == LDSP_OK);
        CHECK(ldsp_resamp_destroy(q) == LDSP_OK);
    }
    ldsp_resamp_t q = NULL;
    CHECK(ldsp_resamp_create(-1.0f, 20, 0.024f, 60.0f, 13, 1, &q) != LDSP_OK);
    CHECK(ldsp_resamp_create(0.5f, 0, 0.024f, 60.0f, 13, 1, &q) != LDSP_OK);
    CHECK(ldsp_resamp_create(0.5f, 20, 0.6f, 60.0f, 13, 1, &q) != LDSP_OK);
}

static void loops(void)
{
    for (int t = 0; t < 2; t++) {
        ldsp_nco_t q = NULL;
        CHECK(ldsp_nco_create(t, &q) == LDSP_OK);
        float f = 0;
        CHECK(ldsp_nco_set_frequency(q, 0.3f) == LDSP_OK && ldsp_nco_get_frequency(q, &f) == LDSP_OK);
        CHECK(ldsp_nco_adjust_frequency(q, -0.1f) == LDSP_OK && ldsp_nco_set_phase(q, -2.0f) == LDSP_OK);
        CHECK(ldsp_nco_adjust_phase(q, 7.0f) == LDSP_OK && ldsp_nco_get_phase(q, &f) == LDSP_OK);
        CHECK(ldsp_nco_pll_set_bandwidth(q, 0.001f) == LDSP_OK);
        for (int i = 0; i < 100; i++) CHECK(ldsp_nco_pll_step(q, 0.01f * (i - 50)) == LDSP_OK);
        uint32_t th, dth;
        CHECK(ldsp_nco_get_state(q, &th, &dth) == LDSP_OK && ldsp_nco_set_state(q, th, dth) == LDSP_OK);
        CHECK(ldsp_nco_reset(q) == LDSP_OK && ldsp_nco_destroy(q) == LDSP_OK);
    }
    ldsp_agc_t g = NULL;
    CHECK(ldsp_agc_create(&g) == LDSP_OK);
    float v;
    CHECK(ldsp_agc_set_bandwidth(g, 0.02f) == LDSP_OK && ldsp_agc_get_bandwidth(g, &v) == LDSP_OK);
    CHECK(ldsp_agc_lock(g, 1) == LDSP_OK && ldsp_agc_lock(g, 0) == LDSP_OK);
    CHECK(ldsp_agc_squelch_enable(g, 1) == LDSP_OK && ldsp_agc_squelch_set_threshold(g, -30.0f) == LDSP_OK);
    CHECK(ldsp_agc_squelch_get_threshold(g, &v) == LDSP_OK && ldsp_agc_squelch_set_timeout(g, 7) == LDSP_OK);
    int st = 0;
    CHECK(ldsp_agc_squelch_get_status(g, &st) == LDSP_OK);
    CHECK(ldsp_agc_set_gain(g, 3.0f) == LDSP_OK && ldsp_agc_get_gain(g, &v) == LDSP_OK);
    CHECK(ldsp_agc_set_scale(g, 0.01f) == LDSP_OK && ldsp_agc_get_scale(g, &v) == LDSP_OK);
    CHECK(ldsp_agc_set_signal_level(g, 2.0f) == LDSP_OK && ldsp_agc_get_signal_level(g, &v) == LDSP_OK);
    CHECK(ldsp_agc_set_rssi(g, -20.0f) == LDSP_OK && ldsp_agc_get_rssi(g, &v) == LDSP_OK);
    CHECK(ldsp_debug_agc_perturb(g, 1) == LDSP_OK && ldsp_debug_agc_rounds(g, 0) == LDSP_OK);
    CHECK(ldsp_debug_agc_rounds(g, 99) != LDSP_OK);
    float xx[64] = {0}, y[64];
    CHECK(ldsp_agc_execute(g, xx, 32, y, NULL, LDSP_MEM_HOST, NULL) == LDSP_EHIP);
    CHECK(ldsp_agc_reset(g) == LDSP_OK && ldsp_agc_destroy(g) == LDSP_OK);

    for (int type = 0; type < 3; type++)
        for (int sup = 0; sup < 2; sup++) {
            ldsp_ampmodem_t q = NULL;
            CHECK(ldsp_ampmodem_create(0.5f, type, sup, &q) == LDSP_OK);
            float lp[51], dc[51], hq[200];
            CHECK(ldsp_ampmodem_get_taps(q, lp, dc, hq) == LDSP_OK);
            uint32_t t1, t2;
            CHECK(ldsp_ampmodem_get_pll_state(q, &t1, &t2) == LDSP_OK);
            CHECK(ldsp_ampmodem_demodulate(q, xx, 16, y, LDSP_MEM_HOST, NULL) == LDSP_EHIP);
            CHECK(ldsp_ampmodem_reset(q) == LDSP_OK && ldsp_ampmodem_destroy(q) == LDSP_OK);
        }
    ldsp_ampmodem_t am = NULL;
    CHECK(ldsp_ampmodem_create(0.5f, 7, 0, &am) != LDSP_OK);

    ldsp_bcastam_t b = NULL;
    CHECK(ldsp_bcastam_create(25, &b) == LDSP_OK);
    int mode = 0;
    CHECK(ldsp_bcastam_set_mode(b, 1) == LDSP_OK && ldsp_bcastam_get_mode(b, &mode) == LDSP_OK);
    CHECK(ldsp_bcastam_destroy(b) == LDSP_OK);
    ldsp_freqdem_t fd = NULL;
    CHECK(ldsp_freqdem_create(4.0f, &fd) == LDSP_OK && ldsp_freqdem_get_kf(fd, &v) == LDSP_OK);
    CHECK(ldsp_freqdem_destroy(fd) == LDSP_OK);
    ldsp_fmstereo_t fm = NULL;
    CHECK(ldsp_fmstereo_create(600000.0f, 48000.0f, &fm) == LDSP_OK);
    size_t nout = 0;
    CHECK(ldsp_fmstereo_num_outputs(fm, 65536, &nout) == LDSP_OK && nout > 0);
    CHECK(ldsp_fmstereo_destroy(fm) == LDSP_OK);
    ldsp_delay_t d = NULL;
    unsigned nd = 0;
    CHECK(ldsp_delay_create(25, &d) == LDSP_OK && ldsp_delay_set_delay(d, 40) == LDSP_OK);
    CHECK(ldsp_delay_get_delay(d, &nd) == LDSP_OK && nd == 40 && ldsp_delay_destroy(d) == LDSP_OK);
}

static void misc(void)
{
    CHECK(ldsp_version() > 0);
    int n = -1;
    CHECK(ldsp_device_count(&n) == LDSP_OK && n == 0);
    CHECK(ldsp_device_count(NULL) != LDSP_OK);
    CHECK(ldsp_firfilt_destroy(NULL) == LDSP_OK);             /* destroy(NULL) is a no-op */
    CHECK(ldsp_firfilt_reset(NULL) != LDSP_OK);
    CHECK(ldsp_agc_set_gain(NULL, 1.0f) != LDSP_OK);
    uint64_t checked = 0, mism = 0;
    CHECK(ldsp_debug_math_fastcheck(0, 0x3f000000u, 0x40000000u, 4097, &checked, &mism) == LDSP_OK && mism == 0);
    CHECK(ldsp_debug_math_fastcheck(1, 0x31800000u, 0x3eb17218u, 65537, &checked, &mism) == LDSP_OK && mism == 0);
    char buf[64];
    size_t len = 0;
    CHECK(ldsp_profile_only("k_pll_walk") == LDSP_OK && ldsp_profile_only(NULL) == LDSP_OK);
    CHECK(ldsp_profile_report(buf, sizeof(buf), &len) == LDSP_OK);
    size_t total = 0, idle = 0;
    CHECK(ldsp_debug_host_pools(&total, &idle) == LDSP_OK);
}

int main(void)
{
    misc();
    iir_designs();
    fir_designs();
    resamplers();
    loops();
    if (fails) {
        fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    printf("host driver: all checks passed\n");
    return 0;
}
