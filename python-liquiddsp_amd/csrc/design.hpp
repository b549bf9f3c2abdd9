// design.hpp -- host-side filter design used by libldsp objects at creation.
// Follows liquid-dsp's firdes.c / iirdes.c / window.c / math*.c definitions
// (the routines the reference reaches through firfilt_*_create_kaiser,
// firfilt_*_create_dc_blocker, resamp_*_create and iirfilt_*_create_prototype);
// see oracle/liquid_restate.c for the restatement these are checked against.
#pragma once
#include <complex>
#include <vector>

namespace ldsp {
namespace design {

float kaiser_beta_As(float as);
float kaiser(unsigned int i, unsigned int wlen, float beta);
// liquid_firdes_kaiser: windowed-sinc lowpass, n taps, cutoff fc, stop-band as, offset mu
std::vector<float> firdes_kaiser(unsigned int n, float fc, float as, float mu);
// liquid_firdes_notch(m, f0, as): 2m+1 taps
std::vector<float> firdes_notch(unsigned int m, float f0, float as);
// firhilbf_create(m, as): the 2m quadrature taps of the c2r Hilbert transform
std::vector<float> firhilb_taps(unsigned int m, float as);

struct SOS {
    std::vector<float> B, A;   // [nsos][3], a0 == 1
    unsigned int nsos = 0;
};
struct TF {
    std::vector<float> b, a;
};
// liquid_iirdes with LIQUID_IIRDES_SOS / LIQUID_IIRDES_TF.  Throws ldsp::Error
// (LDSP_EINVAL) for invalid parameters, LDSP_EUNSUP for ellip / bessel.
SOS iirdes_sos(int ftype, int btype, unsigned int order, float fc, float f0, float ap, float as);
TF iirdes_tf(int ftype, int btype, unsigned int order, float fc, float f0, float ap, float as);

} // namespace design
} // namespace ldsp
