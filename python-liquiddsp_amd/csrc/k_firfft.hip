// k_firfft.hip -- overlap-save FFT convolution for the complex FIR filter
// (firfilt_crcf with real taps: ComplexFIRFilter; the
// filter semantics are those of firfilt_crcf_execute_block behind
// src/firfilter.hpp:33 and demod.hpp:135-136).
//
// Direct form costs 4 L flop per complex sample (508 at L = 127), which makes
// it FP32-VALU bound at ~2x the HBM time.  Overlap-save moves it
// under the HBM roof: every wave owns windows of N points
//   w = x[b M - P .. b M + M - 1]      (P >= L-1 history samples, M = N - P)
//   y[b M + i - P] = IFFT(FFT(w) . H)[i]    for i in [P, N)
// with H = scale * FFT(h zero-padded) / N prepared on the host in float64;
// ~90 flop per output at L = 127 instead of 508.  Error vs the float64 truth is
// below the float32 direct form's own (tests/test_gpu_parity.py gates both).
//
// Layout: one window per wave, N/64 points per lane, Stockham autosort
// (N = 512: radices 8, 8, 8; N = 1024: 16, 16, 4).  The first pass works on the
// coalesced global load (lane l holds w[l + 64 r]); the last pass leaves lane
// l holding bins l + 64 s, exactly the input layout of the inverse's first
// pass, so the spectrum multiply needs no exchange.  The inverse is the
// forward transform of the conjugate.  The two exchanges per transform go
// through this wave's own padded LDS buffer (bank-conflict free for
// ds_*_b64) and need no workgroup barrier, so the load / transform / store
// phases of the 6 resident waves per SIMD overlap freely.  Waves own
// contiguous runs of windows: the P-sample overlap of consecutive windows is
// re-read from this CU's L1/L2, not HBM.
#include <type_traits>

#include "kernels.hpp"
#include "ldsp_common.hpp"

namespace ldsp {
namespace k {

namespace {

__device__ __forceinline__ int sl(int i) { return i + (i >> 3); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// a * w (complex), fused
__device__ __forceinline__ float2 cmul(float2 a, float2 w)
{
    return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}
// a * (-i)
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }

// forward 4-point DFT in place (sign -1)
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3)
{
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
    const float2 t2 = cadd(a1, a3), t3 = mul_mi(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

// forward 8-point DFT in place: v[k] = sum_r v[r] exp(-2 pi i r k / 8)
__device__ __forceinline__ void dft8(float2 (&v)[8])
{
    constexpr float r2 = 0.70710678118654752f;
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    // W8^1 = (1 - i)/sqrt2, W8^2 = -i, W8^3 = (-1 - i)/sqrt2
    const float2 w1 = make_float2((o1.x + o1.y) * r2, (o1.y - o1.x) * r2);
    const float2 w2 = mul_mi(o2);
    const float2 w3 = make_float2((o3.y - o3.x) * r2, -(o3.x + o3.y) * r2);
    v[0] = cadd(e0, o0);
    v[4] = csub(e0, o0);
    v[1] = cadd(e1, w1);
    v[5] = csub(e1, w1);
    v[2] = cadd(e2, w2);
    v[6] = csub(e2, w2);
    v[3] = cadd(e3, w3);
    v[7] = csub(e3, w3);
}

constexpr int kWN_ = 1024;

__device__ __forceinline__ int wsl(int i) { return i + (i >> 4); }

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ float2 cmulk(float2 a, float wr, float wi)
{
    return make_float2(fmaf(a.x, wr, -a.y * wi), fmaf(a.x, wi, a.y * wr));
}

// forward 16-point DFT (4 x 4): out[k + 4 m]
__device__ __forceinline__ void dft16(float2 (&v)[16])
{
    constexpr float c = 0.92387953251128674f, s = 0.38268343236508977f, r2 = 0.70710678118654752f;
#pragma unroll
    for (int j = 0; j < 4; j++) dft4(v[j], v[j + 4], v[j + 8], v[j + 12]);
    // b[j][k] = v[j + 4 k] *= W16^{jk}
    v[5] = cmulk(v[5], c, -s);                                   // j1 k1
    v[9] = make_float2((v[9].x + v[9].y) * r2, (v[9].y - v[9].x) * r2);   // j1 k2: W8
    v[13] = cmulk(v[13], s, -c);                                 // j1 k3
    v[6] = make_float2((v[6].x + v[6].y) * r2, (v[6].y - v[6].x) * r2);   // j2 k1: W8
    v[10] = mul_mi(v[10]);                                       // j2 k2: -i
    v[14] = make_float2((v[14].y - v[14].x) * r2, -(v[14].x + v[14].y) * r2);   // j2 k3: W16^6
    v[7] = cmulk(v[7], s, -c);                                   // j3 k1: W16^3
    v[11] = make_float2((v[11].y - v[11].x) * r2, -(v[11].x + v[11].y) * r2);   // j3 k2: W16^6
    v[15] = cmulk(v[15], -c, s);                                 // j3 k3: W16^9
    // DFT4 over j for each k: inputs v[4k + j]... (b[j][k] sits at v[j + 4k])
#pragma unroll
    for (int k = 0; k < 4; k++) dft4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    // now v[4k + m] = X[k + 4m]; transpose to v[i] = X[i]
    float2 o[16];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int m = 0; m < 4; m++) o[k + 4 * m] = v[4 * k + m];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = o[i];
}

// forward 1024-point FFT of one wave's window held as v[r] = data[lane + 64 r];
// on return v[s] = X[lane + 64 s].  d: this wave's padded LDS buffer.
__device__ __forceinline__ void fft1024(float2 (&v)[16], float2* d, const float2* tw, int lane)
{
    dft16(v);
#pragma unroll
    for (int r = 0; r < 16; r++) d[wsl(lane * 16 + r)] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = d[wsl(lane + 64 * r)];
    const int k = lane & 15;
#pragma unroll
    for (int r = 1; r < 16; r++) v[r] = cmul(v[r], tw[(r - 1) * 16 + k]);
    dft16(v);
    wave_lds_sync();
    const int o = (lane >> 4) * 256 + k;
#pragma unroll
    for (int r = 0; r < 16; r++) d[wsl(o + 16 * r)] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int jj = lane + 64 * q;
        float2 a0 = d[wsl(jj)], a1 = d[wsl(jj + 256)], a2 = d[wsl(jj + 512)], a3 = d[wsl(jj + 768)];
        a1 = cmul(a1, tw[240 + jj]);
        a2 = cmul(a2, tw[240 + 256 + jj]);
        a3 = cmul(a3, tw[240 + 512 + jj]);
        dft4(a0, a1, a2, a3);
        v[q] = a0;
        v[q + 4] = a1;
        v[q + 8] = a2;
        v[q + 12] = a3;
    }
    wave_lds_sync();
}

__device__ __forceinline__ void fft512(float2 (&v)[8], float2* d, const float2* tw, int lane)
{
    dft8(v);
#pragma unroll
    for (int r = 0; r < 8; r++) d[sl(lane * 8 + r)] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = d[sl(lane + 64 * r)];
    const int k = lane & 7;
#pragma unroll
    for (int r = 1; r < 8; r++) v[r] = cmul(v[r], tw[(r - 1) * 8 + k]);
    dft8(v);
    wave_lds_sync();
    const int o = (lane >> 3) * 64 + k;
#pragma unroll
    for (int r = 0; r < 8; r++) d[sl(o + 8 * r)] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = d[sl(lane + 64 * r)];
#pragma unroll
    for (int r = 1; r < 8; r++) v[r] = cmul(v[r], tw[56 + (r - 1) * 64 + lane]);
    dft8(v);
    // v[r] = X[lane + 64 r]
}


// Fused NCO mix (BASELINE config 3, NCO.mix_down -> ComplexFIRFilter): the raw
// sample x[i] enters the filter as x[i] e^{-+j theta_i}, theta_i = theta0 + i
// dtheta (mod 2^32), with the sine table and operation order of k_nco_mix
// (nco_crcf_mix_block_{down,up}), so the filter sees bit for bit what the
// separate mix kernel would have written.  The history holds mixed samples.
struct Mix {
    uint32_t theta0, dtheta;
    int down;
};
// tab: (sin, cos) pairs of the NCO table, tab[i] = (sintab[i], sintab[(i + 256) & 1023]),
// or the sine table itself (the cosine one quarter turn on: two reads, 4 KB of LDS);
// t = theta + 2^21 (the table index rounds theta to the nearest of 1024 cells)
__device__ __forceinline__ float2 nco_sc(const float2* tab, uint32_t t) { return tab[__builtin_amdgcn_ubfe(t, 22, 10)]; }
__device__ __forceinline__ float2 nco_sc(const float* tab, uint32_t t)
{
    return make_float2(tab[__builtin_amdgcn_ubfe(t, 22, 10)], tab[__builtin_amdgcn_ubfe(t + (1u << 30), 22, 10)]);
}
// x * (c + j s') with s' = -s for a down-mix: (a c - b s') + j (a s' + b c) --
// k_nco_mix's x * conj(c + js) = (a c - b (-s)) + j (a (-s) + b c) term for
// term (negation is exact), selected by a sign mask instead of a branch
__device__ __forceinline__ float2 nco_apply(float2 v, float2 sc, const Mix& mx)
{
    const float sn = __uint_as_float(__float_as_uint(sc.x) ^ (mx.down ? 0x80000000u : 0u)), cs = sc.y;
    return make_float2(v.x * cs - v.y * sn, v.x * sn + v.y * cs);
}
template <class T>
__device__ __forceinline__ float2 nco_mix1(float2 v, long i, const Mix& mx, const T* tab)
{
    return nco_apply(v, nco_sc(tab, mx.theta0 + (uint32_t)i * mx.dtheta + (1u << 21)), mx);
}

// Raw window loads (the P history samples before the call's start come from
// hist, which already holds mixed samples).  The NCO mix is applied separately
// (mix_win) once the data is needed: a mix next to its load would make the wave
// wait for the load there, which with PREF is before this window's transforms,
// i.e. no prefetch at all.
template <int PPL>
__device__ __forceinline__ void load_win(float2 (&v)[PPL], const float2* __restrict__ x,
                                         const float2* __restrict__ hist, long n, int halo, long g0, int lane)
{
    if (g0 >= 0 && g0 + 64 * PPL <= n) {          // interior window: 32-bit lane offsets, no checks
        const float2* __restrict__ xb = x + g0;
#pragma unroll
        for (int r = 0; r < PPL; r++) v[r] = xb[lane + 64 * r];
        return;
    }
#pragma unroll
    for (int r = 0; r < PPL; r++) {
        const long gi = g0 + lane + 64 * r;
        float2 e = make_float2(0.0f, 0.0f);
        if (gi >= 0) {
            if (gi < n) e = x[gi];
        } else if (gi >= -halo) {
            e = hist[gi + halo];
        }
        v[r] = e;
    }
}

// the NCO mix of the samples of window g0 that come from x (0 <= gi < n)
template <int PPL, class T>
__device__ __forceinline__ void mix_win(float2 (&v)[PPL], long n, long g0, int lane, const Mix& mx, const T* ntab)
{
    if (g0 >= 0 && g0 + 64 * PPL <= n) {
#pragma unroll
        for (int r = 0; r < PPL; r++) v[r] = nco_mix1(v[r], g0 + lane + 64 * r, mx, ntab);
        return;
    }
#pragma unroll
    for (int r = 0; r < PPL; r++) {
        const long gi = g0 + lane + 64 * r;
        if (gi >= 0 && gi < n) v[r] = nco_mix1(v[r], gi, mx, ntab);
    }
}

template <int PPL>
__device__ __forceinline__ void store_win(const float2 (&v)[PPL], float2* __restrict__ y, long n, int P, long g0,
                                          int lane)
{
    // v[s] = conj(y_block[lane + 64 s]);  y[b M + i - P] = y_block[i] for i >= P
    float2* __restrict__ yb = y + g0;
    if (g0 + 64 * PPL <= n) {
#pragma unroll
        for (int s = 0; s < PPL; s++) {
            const int i = lane + 64 * s;
            if (i >= P) yb[i] = make_float2(v[s].x, -v[s].y);
        }
    } else {
#pragma unroll
        for (int s = 0; s < PPL; s++) {
            const int i = lane + 64 * s;
            if (i >= P && g0 + i < n) yb[i] = make_float2(v[s].x, -v[s].y);
        }
    }
}

template <bool MIX, class T>
__device__ __forceinline__ void write_hist(const float2* __restrict__ x, const float2* __restrict__ hist,
                                           float2* __restrict__ hist_out, long n, int halo, int t, int nt,
                                           const Mix& mx, const T* ntab)
{
    for (int j = t; j < halo; j += nt) {
        const long gi = n - halo + j;
        hist_out[j] = gi >= 0 ? (MIX ? nco_mix1(x[gi], gi, mx, ntab) : x[gi]) : hist[gi + halo];
    }
}

// 512-point windows: 8 points per lane, 4 waves per workgroup; tables in LDS.
// PREF: the next window's loads are issued before this one's transforms (one
// window of HBM reads in flight per wave beside the compute; costs registers).
constexpr int kVN = 512;
constexpr int kVSlots = kVN + kVN / 8;
constexpr int kVWaves = 4;

template <bool MIX, bool PREF>
__global__ void __launch_bounds__(64 * kVWaves) k_fir_fft512(const float2* __restrict__ x,
                                                             const float2* __restrict__ hist,
                                                             float2* __restrict__ hist_out, long n, int L, int P,
                                                             long nwin, long per, const float2* __restrict__ H,
                                                             const float2* __restrict__ tw, float2* __restrict__ y,
                                                             Mix mx, const float* __restrict__ table)
{
    __shared__ float2 buf[kVWaves][kVSlots];
    __shared__ float2 ltw[kFft512Tw];
    __shared__ float2 lH[kVN];
    __shared__ float2 ntab[MIX ? 1024 : 1];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int M = kVN - P;
    const int halo = L - 1;
    if (MIX)
        for (int j = t; j < 1024; j += 64 * kVWaves) ntab[j] = make_float2(table[j], table[(j + 256) & 1023]);
    for (int j = t; j < kFft512Tw; j += 64 * kVWaves) ltw[j] = tw[j];
    for (int j = t; j < kVN; j += 64 * kVWaves) lH[j] = H[j];
    __syncthreads();
    if (blockIdx.x == 0) write_hist<MIX>(x, hist, hist_out, n, halo, t, 64 * kVWaves, mx, ntab);
    const long w0 = ((long)blockIdx.x * kVWaves + wave) * per;
    const long w1 = min(nwin, w0 + per);
    float2* d = buf[wave];
    float2 nx[8];
    if (PREF && w0 < w1) load_win<8>(nx, x, hist, n, halo, w0 * M - P, lane);
    for (long w = w0; w < w1; w++) {
        const long g0 = w * M - P;
        float2 v[8];
        if (PREF) {
#pragma unroll
            for (int r = 0; r < 8; r++) v[r] = nx[r];
            if (MIX) mix_win<8>(v, n, g0, lane, mx, ntab);
            if (w + 1 < w1) load_win<8>(nx, x, hist, n, halo, g0 + M, lane);
        } else {
            load_win<8>(v, x, hist, n, halo, g0, lane);
            if (MIX) mix_win<8>(v, n, g0, lane, mx, ntab);
        }
        fft512(v, d, ltw, lane);
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const float2 p = cmul(v[s], lH[lane + 64 * s]);
            v[s] = make_float2(p.x, -p.y);
        }
        wave_lds_sync();       // pass-3 reads of d are done before pass-1 writes
        fft512(v, d, ltw, lane);
        store_win<8>(v, y, n, P, g0, lane);
        wave_lds_sync();
    }
}

// 1024-point windows (P > 128): 16 points per lane, WAVES waves per workgroup
// (4: three workgroups share a CU at <= 168 registers; 8: one).
constexpr int kWSlots = kWN_ + kWN_ / 16;

template <bool MIX, int WAVES, bool PREF>
__global__ void __launch_bounds__(64 * WAVES) k_fir_fft1024(const float2* __restrict__ x,
                                                            const float2* __restrict__ hist,
                                                            float2* __restrict__ hist_out, long n, int L, int P,
                                                            long nwin, long per, const float2* __restrict__ H,
                                                            const float2* __restrict__ tw, float2* __restrict__ y,
                                                            Mix mx, const float* __restrict__ table)
{
    __shared__ float2 buf[WAVES][kWSlots];
    __shared__ float2 ltw[kFft1024Tw];
    __shared__ float2 ntab[MIX ? 1024 : 1];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int M = kWN_ - P;
    const int halo = L - 1;
    if (MIX)
        for (int j = t; j < 1024; j += 64 * WAVES) ntab[j] = make_float2(table[j], table[(j + 256) & 1023]);
    for (int j = t; j < kFft1024Tw; j += 64 * WAVES) ltw[j] = tw[j];
    __syncthreads();
    if (blockIdx.x == 0) write_hist<MIX>(x, hist, hist_out, n, halo, t, 64 * WAVES, mx, ntab);
    const long w0 = ((long)blockIdx.x * WAVES + wave) * per;
    const long w1 = min(nwin, w0 + per);
    float2* d = buf[wave];
    float2 nx[16];
    if (PREF && w0 < w1) load_win<16>(nx, x, hist, n, halo, w0 * M - P, lane);
    for (long w = w0; w < w1; w++) {
        asm volatile("" ::: "memory");    // keep H reads inside the loop (register budget)
        const long g0 = w * M - P;
        float2 v[16];
        if (PREF) {
#pragma unroll
            for (int r = 0; r < 16; r++) v[r] = nx[r];
            if (MIX) mix_win<16>(v, n, g0, lane, mx, ntab);
            if (w + 1 < w1) load_win<16>(nx, x, hist, n, halo, g0 + M, lane);
        } else {
            load_win<16>(v, x, hist, n, halo, g0, lane);
            if (MIX) mix_win<16>(v, n, g0, lane, mx, ntab);
        }
        fft1024(v, d, ltw, lane);
#pragma unroll
        for (int s = 0; s < 16; s++) {
            const float2 p = cmul(v[s], H[lane + 64 * s]);
            v[s] = make_float2(p.x, -p.y);
        }
        fft1024(v, d, ltw, lane);
        store_win<16>(v, y, n, P, g0, lane);
    }
}

// 1024-point windows, bank-conflict-free exchanges (k_fir_fft1024x).  The
// same three passes as fft1024, with the two exchanges laid out for the LDS
// lane groups of MI355X (MI355X_MICROARCH LDS table: ds_write_b64 serves 16
// contiguous lanes per cycle over 32 banks, ds_read_b64 32 lanes over 64):
//   pass 1 -> 2: element lane*16 + r at r*66 + lane   (stores: 16 contiguous
//                lanes; loads: lane reads k*66 + lh + 4r, banks 4k + 2lh + 8r
//                mod 64 -> all 32 lanes of a group distinct)
//   pass 2 -> 3: element e at e                        (stores: 16 contiguous,
//                loads: 32 contiguous)
// so every exchange access costs its minimum LDS cycles (fft1024's padding
// leaves a 2-way conflict in every pass-2/3 read group), and every address is a
// per-lane base plus an immediate offset.  The inverse transform is the
// forward one of the re/im-swapped spectrum (IFFT(Z) = swap(FFT(swap(Z))) / N,
// the 1/N folded into H), so neither conjugation costs an instruction.
constexpr int kXPad = 66;
constexpr int kXSlots = 16 * kXPad;

// One ds_read_b64 / ds_write_b64 per access.  Left alone the compiler pairs
// neighbouring accesses into ds_read2_b64 / ds_write2_b64, which the LDS serves
// in 16-lane groups over 32 banks (MI355X_MICROARCH LDS table): twice the
// cycles of two ds_read_b64, and 2-way bank conflicts in the pass-2 reads the
// layouts above make conflict-free.  Volatile accesses are not paired.
typedef float lds_f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) volatile lds_f2 lds_vf2;
__device__ __forceinline__ float2 lds_ld(const float2* p)
{
    const lds_f2 r = *(const lds_vf2*)p;
    return make_float2(r.x, r.y);
}
__device__ __forceinline__ void lds_st(float2* p, float2 v)
{
    lds_f2 t;
    t.x = v.x;
    t.y = v.y;
    *(lds_vf2*)p = t;
}

__device__ __forceinline__ void fft1024x(float2 (&v)[16], float2* d, const float2* tw, int lane)
{
    const int lh = lane >> 4, k = lane & 15;
    dft16(v);
    // Each pass issues all its LDS reads before the first use (twiddles ahead
    // of the exchange stores, then the exchanged data), so a wave waits for
    // one LDS round trip per pass, not one per twiddle.
    const float2* t2 = tw + k;
    float2 w[15];
#pragma unroll
    for (int r = 1; r < 16; r++) w[r - 1] = lds_ld(t2 + (r - 1) * 16);
    float2* d1 = d + lane;
#pragma unroll
    for (int r = 0; r < 16; r++) lds_st(d1 + r * kXPad, v[r]);
    wave_lds_sync();
    const float2* d2 = d + k * kXPad + lh;
#pragma unroll
    for (int r = 0; r < 16; r++) v[r] = lds_ld(d2 + 4 * r);
#pragma unroll
    for (int r = 1; r < 16; r++) v[r] = cmul(v[r], w[r - 1]);
    dft16(v);
    // pass 3: lane holds a_m = element lane + 64 q + 256 m in v[q + 4 m], and
    // its radix-4 outputs go back to the same registers
    const float2* t3 = tw + 240 + lane;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int m = 1; m < 4; m++) w[3 * q + m - 1] = lds_ld(t3 + 64 * q + 256 * (m - 1));
    float2* d3 = d + lh * 256 + k;
#pragma unroll
    for (int r = 0; r < 16; r++) lds_st(d3 + 16 * r, v[r]);
    wave_lds_sync();
    const float2* d4 = d + lane;
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = lds_ld(d4 + 64 * j);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        float2 a0 = v[q], a1 = cmul(v[q + 4], w[3 * q]), a2 = cmul(v[q + 8], w[3 * q + 1]),
               a3 = cmul(v[q + 12], w[3 * q + 2]);
        dft4(a0, a1, a2, a3);
        v[q] = a0;
        v[q + 4] = a1;
        v[q + 8] = a2;
        v[q + 12] = a3;
    }
}

__device__ __forceinline__ float2 swap_ri(float2 a) { return make_float2(a.y, a.x); }

// NCO mix of the 16 points of an interior window: sample g0 + lane + 64 r has
// phase theta0 + (g0 + lane + 64 r) dtheta; t carries the + 2^21 rounding of
// the table index (nco_mix1), so each point costs an add, a bit-field extract
// and the table read besides the 6 products of the mix itself.
template <int PPL, class T>
__device__ __forceinline__ void mix_interior(float2 (&v)[PPL], long g0, int lane, const Mix& mx, const T* tab)
{
    const uint32_t t0 = mx.theta0 + (uint32_t)(g0 + lane) * mx.dtheta + (1u << 21);
    const uint32_t d64 = mx.dtheta << 6;
    float2 sc[PPL];
#pragma unroll
    for (int r = 0; r < PPL; r++) sc[r] = nco_sc(tab, t0 + (uint32_t)r * d64);
#pragma unroll
    for (int r = 0; r < PPL; r++) v[r] = nco_apply(v[r], sc[r], mx);
}

template <bool MIX, bool PREF, int WAVES, bool ILV = false>
__global__ void __launch_bounds__(64 * WAVES) k_fir_fft1024x(const float2* __restrict__ x,
                                                          const float2* __restrict__ hist,
                                                          float2* __restrict__ hist_out, long n, int L, int P,
                                                          long nwin, long per, const float2* __restrict__ H,
                                                          const float2* __restrict__ tw, float2* __restrict__ y,
                                                          Mix mx, const float* __restrict__ table)
{
    // H stays on chip, so the window is the loop's only global traffic (a
    // global H read would share vmcnt with the window loads and make the
    // multiply wait for them): in registers with 4-wave workgroups (H[lane +
    // 64 s] is the same for every window of a lane; 32 VGPRs, and three
    // workgroups' LDS still fit a CU), in LDS with larger ones (128 VGPRs).
    constexpr bool kHReg = WAVES == 4;
    __shared__ float2 buf[WAVES][kXSlots];
    __shared__ float2 ltw[kFft1024Tw];
    __shared__ float2 lH[kHReg ? 1 : kWN_];
    __shared__ float2 ntab[MIX ? 1024 : 1];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int M = kWN_ - P;
    const int p64 = P >> 6;           // P is a multiple of 64 (IirObj::fft_P): outputs s < p64 are discarded
    const int halo = L - 1;
    if (MIX)
        for (int j = t; j < 1024; j += 64 * WAVES) ntab[j] = make_float2(table[j], table[(j + 256) & 1023]);
    for (int j = t; j < kFft1024Tw; j += 64 * WAVES) ltw[j] = tw[j];
    float2 hr[kHReg ? 16 : 1];
    if constexpr (kHReg) {
#pragma unroll
        for (int s = 0; s < 16; s++) hr[s] = H[lane + 64 * s];
    } else {
        for (int j = t; j < kWN_; j += 64 * WAVES) lH[j] = H[j];
    }
    __syncthreads();
    if (blockIdx.x == 0) write_hist<MIX>(x, hist, hist_out, n, halo, t, 64 * WAVES, mx, ntab);
    // ILV: the workgroup's windows interleaved over its waves (wave k takes
    // k, k + WAVES, ..), so the P-sample overlap a window shares with the next
    // is read by another wave at about the same time, from L2, instead of by
    // the same wave one window (~10 us) later, when it has often left L2
    const long wb = ILV ? (long)blockIdx.x * WAVES * per + wave : ((long)blockIdx.x * WAVES + wave) * per;
    const long we = ILV ? min(nwin, (long)(blockIdx.x + 1) * WAVES * per) : min(nwin, wb + per);
    const long step = ILV ? WAVES : 1;
    float2* d = buf[wave];
    const float2* Hl = lH + lane;
    float2 nx[16];
    if (PREF && wb < we) load_win<16>(nx, x, hist, n, halo, wb * M - P, lane);
    for (long w = wb; w < we; w += step) {
        const long g0 = w * M - P;
        const bool interior = g0 >= 0 && g0 + kWN_ <= n;
        float2 v[16];
        if (PREF) {
#pragma unroll
            for (int r = 0; r < 16; r++) v[r] = nx[r];
            if (w + step < we) load_win<16>(nx, x, hist, n, halo, g0 + step * M, lane);
        } else {
            load_win<16>(v, x, hist, n, halo, g0, lane);
        }
        if (MIX) {
            if (interior) mix_interior<16>(v, g0, lane, mx, ntab);
            else mix_win<16>(v, n, g0, lane, mx, ntab);
        }
        fft1024x(v, d, ltw, lane);
        float2 h[16];
#pragma unroll
        for (int s = 0; s < 16; s++) h[s] = kHReg ? hr[kHReg ? s : 0] : lds_ld(Hl + 64 * s);
#pragma unroll
        for (int s = 0; s < 16; s++) v[s] = swap_ri(cmul(v[s], h[s]));
        fft1024x(v, d, ltw, lane);
        float2* yb = y + g0 + lane;
        if (g0 + kWN_ <= n) {
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s >= p64) yb[64 * s] = swap_ri(v[s]);
        } else {
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s >= p64 && g0 + lane + 64 * s < n) yb[64 * s] = swap_ri(v[s]);
        }
    }
}

// 512-point windows, bank-conflict-free exchanges (k_fir_fft512x; the layout
// argument of fft1024x for radices 8, 8, 8):
//   pass 1 -> 2: element lane*8 + r at r*68 + lane   (loads: k*68 + l8 + 8r,
//                banks 8k + 2 l8 mod 64, l8 = lane >> 3: distinct in a group)
//   pass 2 -> 3: element e at e + 8 (e >> 6)        (stores: the two 8-lane
//                runs of a 16-lane group 16 banks apart; loads contiguous)
constexpr int kYPad = 68;
constexpr int kYSlots = 8 * 72;

__device__ __forceinline__ void fft512x(float2 (&v)[8], float2* d, const float2* tw, int lane)
{
    const int l8 = lane >> 3, k = lane & 7;
    dft8(v);
    // all of a pass's LDS reads in flight before the first use (fft1024x)
    const float2* t2 = tw + k;
    float2 w[7];
#pragma unroll
    for (int r = 1; r < 8; r++) w[r - 1] = lds_ld(t2 + (r - 1) * 8);
    float2* d1 = d + lane;
#pragma unroll
    for (int r = 0; r < 8; r++) lds_st(d1 + r * kYPad, v[r]);
    wave_lds_sync();
    const float2* d2 = d + k * kYPad + l8;
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = lds_ld(d2 + 8 * r);
#pragma unroll
    for (int r = 1; r < 8; r++) v[r] = cmul(v[r], w[r - 1]);
    dft8(v);
    const float2* t3 = tw + 56 + lane;
#pragma unroll
    for (int r = 1; r < 8; r++) w[r - 1] = lds_ld(t3 + (r - 1) * 64);
    float2* d3 = d + l8 * 72 + k;
#pragma unroll
    for (int r = 0; r < 8; r++) lds_st(d3 + 8 * r, v[r]);
    wave_lds_sync();
    const float2* d4 = d + lane;
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = lds_ld(d4 + 72 * r);
#pragma unroll
    for (int r = 1; r < 8; r++) v[r] = cmul(v[r], w[r - 1]);
    dft8(v);
}

template <bool MIX, bool ILV = false>
__global__ void __launch_bounds__(64 * kVWaves) k_fir_fft512x(const float2* __restrict__ x,
                                                              const float2* __restrict__ hist,
                                                              float2* __restrict__ hist_out, long n, int L, int P,
                                                              long nwin, long per, const float2* __restrict__ H,
                                                              const float2* __restrict__ tw, float2* __restrict__ y,
                                                              Mix mx, const float* __restrict__ table)
{
    __shared__ float2 buf[kVWaves][kYSlots];
    __shared__ float2 ltw[kFft512Tw];
    __shared__ float2 lH[kVN];
    __shared__ float2 ntab[MIX ? 1024 : 1];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int M = kVN - P;
    const int p64 = P >> 6;
    const int halo = L - 1;
    if (MIX)
        for (int j = t; j < 1024; j += 64 * kVWaves) ntab[j] = make_float2(table[j], table[(j + 256) & 1023]);
    for (int j = t; j < kFft512Tw; j += 64 * kVWaves) ltw[j] = tw[j];
    for (int j = t; j < kVN; j += 64 * kVWaves) lH[j] = H[j];
    __syncthreads();
    if (blockIdx.x == 0) write_hist<MIX>(x, hist, hist_out, n, halo, t, 64 * kVWaves, mx, ntab);
    const long wb = ILV ? (long)blockIdx.x * kVWaves * per + wave : ((long)blockIdx.x * kVWaves + wave) * per;
    const long we = ILV ? min(nwin, (long)(blockIdx.x + 1) * kVWaves * per) : min(nwin, wb + per);
    const long step = ILV ? kVWaves : 1;     // (k_fir_fft1024x)
    float2* d = buf[wave];
    const float2* Hl = lH + lane;
    for (long w = wb; w < we; w += step) {
        const long g0 = w * M - P;
        const bool interior = g0 >= 0 && g0 + kVN <= n;
        float2 v[8];
        load_win<8>(v, x, hist, n, halo, g0, lane);
        if (MIX) {
            if (interior) mix_interior<8>(v, g0, lane, mx, ntab);
            else mix_win<8>(v, n, g0, lane, mx, ntab);
        }
        fft512x(v, d, ltw, lane);
        float2 h[8];
#pragma unroll
        for (int s = 0; s < 8; s++) h[s] = lds_ld(Hl + 64 * s);
#pragma unroll
        for (int s = 0; s < 8; s++) v[s] = swap_ri(cmul(v[s], h[s]));
        fft512x(v, d, ltw, lane);
        float2* yb = y + g0 + lane;
        if (g0 + kVN <= n) {
#pragma unroll
            for (int s = 0; s < 8; s++)
                if (s >= p64) yb[64 * s] = swap_ri(v[s]);
        } else {
#pragma unroll
            for (int s = 0; s < 8; s++)
                if (s >= p64 && g0 + lane + 64 * s < n) yb[64 * s] = swap_ri(v[s]);
        }
    }
}

// Waves resident on the device for a kernel (CUs x blocks per CU x waves per block).
long resident_waves(const void* fn, int threads)
{
    int dev = 0, cus = 0, per_cu = 0;
    LDSP_HIP(hipGetDevice(&dev));
    LDSP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    LDSP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0));
    return (long)std::max(1, cus) * std::max(1, per_cu) * (threads / 64);
}

} // namespace

// Kernel variant: (512: prefetch) x (1024: prefetch, 4 or 8 waves); the
// defaults were measured on MI355X; tuning builds take
// LDSP_FFT_VARIANT = bit 0 prefetch-512, bit 1 prefetch-1024, bit 2 1024 with 8 waves
// (k_fir_fft1024x: 16, one workgroup per CU), bit 3 1024-point
// windows for short filters too, bit 4 the padded-exchange k_fir_fft1024, bit 5
// the padded-exchange k_fir_fft512.
constexpr int kFftVariantDefault = 256;   // conflict-free exchanges, windows interleaved over waves; 512: 6 waves / SIMD, 1024: 4-wave blocks, no prefetch
static int fft_variant()
{
    static const int var = LDSP_KNOB("LDSP_FFT_VARIANT", kFftVariantDefault);
    return var;
}
static bool fft_small(int P) { return P <= 128 && !(fft_variant() & 8); }

int fir_fft_points(int P) { return fft_small(P) ? kVN : kWN_; }

template <bool MIX>
static void fft_launch(bool small, int var, unsigned grid_of_waves_fn_unused, const float2* xc, const float2* hc,
                       float2* ho, long n, int L, int P, long nwin, const float2* Hc, const float2* tc, float2* yc,
                       const Mix& mx, const float* tab, hipStream_t s)
{
    (void)grid_of_waves_fn_unused;
    auto run = [&](const void* fn, int wpb, auto launch) {
        static long slots_cache[2][1024] = {};
        long& slots = slots_cache[MIX ? 1 : 0][(small ? 512 : 0) | (var & 511)];
        if (slots == 0) slots = resident_waves(fn, 64 * wpb);
        const long waves = std::min(nwin, slots);
        const long per = (nwin + waves - 1) / waves;       // contiguous windows per wave
        const long used = (nwin + per - 1) / per;
        const unsigned grid = (unsigned)((used + wpb - 1) / wpb);
        launch(grid, per);
    };
#define LDSP_FFT_LAUNCH(KERNEL, WPB)                                                                           \
    run((const void*)KERNEL, WPB, [&](unsigned grid, long per) {                                                \
        hipLaunchKernelGGL(KERNEL, dim3(grid), dim3(64 * (WPB)), 0, s, xc, hc, ho, n, L, P, nwin, per, Hc, tc, yc, \
                           mx, tab);                                                                           \
    })
    if (small && !(var & 32)) {
        if (var & 256) LDSP_FFT_LAUNCH((k_fir_fft512x<MIX, true>), kVWaves);
        else LDSP_FFT_LAUNCH((k_fir_fft512x<MIX, false>), kVWaves);
    } else if (small) {
        if (var & 1) LDSP_FFT_LAUNCH((k_fir_fft512<MIX, true>), kVWaves);
        else LDSP_FFT_LAUNCH((k_fir_fft512<MIX, false>), kVWaves);
    } else if (!(var & 16)) {
        switch ((var & 2) | (var >> 6 & 3) << 2 | (var & 256) >> 4) {
        case 16: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, false, 4, true>), 4); break;
        case 18: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, true, 4, true>), 4); break;
        case 28: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, false, 16, true>), 16); break;
        case 0: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, false, 4>), 4); break;
        case 2: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, true, 4>), 4); break;
        case 4: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, false, 6>), 6); break;
        case 6: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, true, 6>), 6); break;
        case 8: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, false, 8>), 8); break;
        case 10: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, true, 8>), 8); break;
        case 12: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, false, 16>), 16); break;
        default: LDSP_FFT_LAUNCH((k_fir_fft1024x<MIX, true, 16>), 16); break;
        }
    } else {
        switch (var & 6) {
        case 0: LDSP_FFT_LAUNCH((k_fir_fft1024<MIX, 4, false>), 4); break;
        case 2: LDSP_FFT_LAUNCH((k_fir_fft1024<MIX, 4, true>), 4); break;
        case 4: LDSP_FFT_LAUNCH((k_fir_fft1024<MIX, 8, false>), 8); break;
        default: LDSP_FFT_LAUNCH((k_fir_fft1024<MIX, 8, true>), 8); break;
        }
    }
#undef LDSP_FFT_LAUNCH
}

void fir_fft(const void* x, const void* hist, void* hist_out, size_t n, int L, int P, const void* H, const void* tw,
             void* y, hipStream_t s, const NcoFuse* nco)
{
    if (n == 0) return;
    const bool small = fft_small(P);
    const long N = small ? kVN : kWN_;
    const long M = N - P;
    const long nwin = (long)((n + M - 1) / M);
    const int var = fft_variant();
    Mix mx{0u, 0u, 0};
    const float* tab = nullptr;
    if (nco) {
        mx = Mix{nco->theta0, nco->dtheta, nco->down ? 1 : 0};
        tab = nco->table;
    }
    const float2 *xc = (const float2*)x, *hc = (const float2*)hist, *Hc = (const float2*)H, *tc = (const float2*)tw;
    float2 *ho = (float2*)hist_out, *yc = (float2*)y;
    if (nco) {
        LDSP_PROF(s, small ? "k_fir_fft512_nco" : "k_fir_fft1024_nco");
        fft_launch<true>(small, var, 0, xc, hc, ho, (long)n, L, P, nwin, Hc, tc, yc, mx, tab, s);
    } else {
        LDSP_PROF(s, small ? "k_fir_fft512" : "k_fir_fft1024");
        fft_launch<false>(small, var, 0, xc, hc, ho, (long)n, L, P, nwin, Hc, tc, yc, mx, tab, s);
    }
    LDSP_HIP(hipGetLastError());
}

} // namespace k
} // namespace ldsp
