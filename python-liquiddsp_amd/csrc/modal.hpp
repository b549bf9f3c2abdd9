// modal.hpp -- the modal (diagonal) form of an IIR filter's state-space
// recursion, built on the host when a filter is created, for the single-pass
// fast-mode kernel (k_iir_modal.hip).  Filters whose modal form fails the host
// check below keep the SOS-coordinate blocked scan (k_iir.hip).
#pragma once
#include <complex>
#include <string>
#include <vector>

#include "kernels.hpp"

namespace ldsp {

struct ModalForm {
    bool ok = false;
    std::string why;              // reason when !ok (diagnostics)
    int D = 0, M = 0, J = 0;
    double err = 0.0;             // host check: max |y_modal - y_ss| / max |y_ss| (impulse, noise, free response)
    k::IirModalCoef cf{};
    std::vector<double> tables;   // PS [6][M][4] | PL [64][M][4] | PB [J][M][4]  (k::IirModalPlan)
    // state conversions between the DF-II layout of the scans (s, D reals per
    // component) and the section states v (2 M reals: w_n, w_{n-1} per
    // section): v = to_v s ([2M][D]), s = from_v v ([D][2M])
    std::vector<double> to_v, from_v;
};

// s' = A s + B u, y = C s + Dd u (A row-major D x D); poles = the D eigenvalues of A
ModalForm modal_form(int D, const std::vector<long double>& A, const std::vector<long double>& B,
                     const std::vector<long double>& C, long double Dd,
                     const std::vector<std::complex<long double>>& poles);

// eigenvalues of the recursion: SOS sections 1 + a1 z^-1 + a2 z^-2 (a: [nsos][3])
std::vector<std::complex<long double>> sos_poles(const std::vector<float>& a, unsigned nsos);
// roots of z^D + a[1] z^(D-1) + ... + a[D] (a[i] = 0 for i >= na)
std::vector<std::complex<long double>> tf_poles(const std::vector<float>& a, int na, int D);

} // namespace ldsp
