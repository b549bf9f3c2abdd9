// capi.cpp -- the C ABI of libldsp (include/ldsp.h): object lifetime, host-side
// design and state bookkeeping, device staging, and dispatch to the gfx950
// kernels.  No CPU fallback exists: every execute runs on a HIP device and
// fails with LDSP_EHIP when none is present.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "batch.hpp"
#include "design.hpp"
#include "modal.hpp"
#include "kernels.hpp"
#include "ldsp_math.hpp"
#include "ldsp_common.hpp"

namespace ldsp {

static thread_local std::string g_last_error;

#ifdef LDSP_TUNING
long knob_env(const char* name, long dflt)
{
    const char* v = std::getenv(name);
    return v ? std::atol(v) : dflt;
}
double knob_env_f(const char* name, double dflt)
{
    const char* v = std::getenv(name);
    return v ? std::atof(v) : dflt;
}
const char* knob_env_s(const char* name) { return std::getenv(name); }
#endif
void set_last_error(const std::string& m) { g_last_error = m; }

// roctx through dlopen (ldsp_common.hpp RoctxRange): resolved once; absent library -> no-ops
namespace {
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    Roctx()
    {
        void* h = nullptr;
        for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"}) {
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        }
        if (!h) return;
        push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
        pop = (int (*)())dlsym(h, "roctxRangePop");
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
};
const Roctx& roctx()
{
    static const Roctx r;
    return r;
}
} // namespace
void roctx_push(const char* m)
{
    if (roctx().push) roctx().push(m);
}
void roctx_pop()
{
    if (roctx().pop) roctx().pop();
}

int current_device()
{
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) throw Error(LDSP_EHIP, "no HIP device available (libldsp has no CPU fallback)");
    int d = 0;
    LDSP_HIP(hipGetDevice(&d));
    return d;
}

hipStream_t library_stream(int device)
{
    static std::mutex mu;
    static std::vector<hipStream_t> streams;
    std::lock_guard<std::mutex> lk(mu);
    if ((int)streams.size() <= device) streams.resize(device + 1, nullptr);
    if (!streams[device]) {
        DeviceGuard g(device);
        LDSP_HIP(hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking));
    }
    return streams[device];
}

// Resolve where a call runs: host-memory calls use the library stream and stage
// through grow-only device buffers owned by the object.
struct Exec {
    int device;
    hipStream_t stream;
    bool host;
};

// The device a call's buffers live on.  A device-memory call runs on the
// device that holds its input (made current for the call, so an object's first
// call binds it there); a host-memory call on the current device.
struct BufDevice {
    int dev;
    DeviceGuard g;
    static int of(int mem, const void* x)
    {
        if (mem == LDSP_MEM_DEVICE && x) {
            hipPointerAttribute_t a;
            if (hipPointerGetAttributes(&a, x) == hipSuccess && a.type == hipMemoryTypeDevice) return a.device;
            (void)hipGetLastError();
        }
        return current_device();
    }
    BufDevice(int mem, const void* x) : dev(of(mem, x)), g(dev) {}
};

static Exec make_exec(int device, int mem, void* stream, const BufDevice& bd)
{
    LDSP_REQUIRE(mem == LDSP_MEM_HOST || mem == LDSP_MEM_DEVICE, "mem must be LDSP_MEM_HOST or LDSP_MEM_DEVICE");
    if (mem == LDSP_MEM_DEVICE && bd.dev != device)
        throw Error(LDSP_EINVAL, "buffer on device " + std::to_string(bd.dev) + " but the object lives on device " +
                                     std::to_string(device) + " (objects are bound to the device of their first call)");
    Exec e;
    e.device = device;
    e.host = (mem == LDSP_MEM_HOST);
    e.stream = e.host ? library_stream(device) : (hipStream_t)stream;
    return e;
}

template <typename T>
static T* upload(DevBuf& b, const std::vector<T>& v, int dev)
{
    b.ensure(std::max<size_t>(v.size(), 1) * sizeof(T), dev);
    if (!v.empty()) LDSP_HIP(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return b.as<T>();
}

// Zero device memory before any stream can read it: hipMemset runs on the
// null stream, which does not order against the non-blocking library stream or
// a caller's stream, so wait for it (create / reset paths only).
static void zero_now(void* p, int v, size_t bytes)
{
    LDSP_HIP(hipMemset(p, v, bytes));
    LDSP_HIP(hipDeviceSynchronize());
}

// Host <-> device staging for LDSP_MEM_HOST calls
// Host buffers pass through a pinned staging buffer (a copy from / to pageable
// memory is staged by the runtime at a fraction of the DMA rate, and it is the
// per-call overhead of the README's numpy callbacks); each host call ends with a
// stream synchronize, so the next call may reuse the buffer.  Above kPinMax the
// pageable copy is used directly (no pinned memory of that size per object).
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    void* ensure(size_t bytes) {
        if (bytes <= cap && p) return p;
        const size_t want = (std::max(bytes, cap + cap / 4) + 65535) & ~(size_t)65535;
        if (p) LDSP_HIP(hipHostFree(p));
        p = nullptr;
        cap = 0;
        LDSP_HIP(hipHostMalloc(&p, want, hipHostMallocDefault));
        cap = want;
        return p;
    }
};
// Host staging of the numpy (host-buffer) path: pinned buffers shared by every
// object a thread calls on one device (a host-buffer call is synchronous -- it
// returns only after its output copy -- so a thread's calls never overlap in
// them).  Grown on demand up to kPinMax each (larger transfers go unpinned), never
// shrunk.  A thread takes a pool from a process-wide free list on its first host
// call on a device and returns it there when it exits (thread_local holder), so
// short-lived threads (thread pools, DataLoader workers) reuse pools instead of
// leaking page-locked memory: the number of pools is bounded by the number of
// threads making host calls at the same time.  The free list itself is never
// destroyed (hipHostFree at process teardown can outlive the HIP runtime).
struct PinnedPool {
    PinnedBuf hin, hout;
    hipEvent_t hin_done = nullptr;    // the last copy out of hin (a call that threw may not have synchronized)
    hipEvent_t done()
    {
        if (!hin_done) LDSP_HIP(hipEventCreateWithFlags(&hin_done, hipEventDisableTiming));
        return hin_done;
    }
};
namespace {
struct PoolList {
    std::mutex mu;
    std::vector<std::vector<PinnedPool*>> free;    // per device
    size_t total = 0;                              // pools ever created
};
PoolList& pool_list()
{
    static PoolList* l = new PoolList();           // never destroyed (see above)
    return *l;
}
struct ThreadPools {
    std::vector<PinnedPool*> pools;                // this thread's, per device
    ~ThreadPools()
    {
        PoolList& l = pool_list();
        std::lock_guard<std::mutex> lk(l.mu);
        for (size_t d = 0; d < pools.size(); d++)
            if (pools[d]) {
                if (l.free.size() <= d) l.free.resize(d + 1);
                l.free[d].push_back(pools[d]);
            }
    }
};
} // namespace
static PinnedPool& pinned_pool(int device)
{
    thread_local ThreadPools tp;
    if ((int)tp.pools.size() <= device) tp.pools.resize(device + 1, nullptr);
    if (!tp.pools[device]) {
        PoolList& l = pool_list();
        std::lock_guard<std::mutex> lk(l.mu);
        if ((int)l.free.size() > device && !l.free[device].empty()) {
            tp.pools[device] = l.free[device].back();
            l.free[device].pop_back();
        } else {
            tp.pools[device] = new PinnedPool();
            l.total++;
        }
    }
    return *tp.pools[device];
}

// Is p page-locked host memory (ldsp_host_alloc, hipHostMalloc, hipHostRegister)?
// Such buffers are copied by DMA directly (no staging copy on the host).
static bool host_pinned(const void* p)
{
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) == hipSuccess) return a.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    return false;
}

struct Staging {
    static constexpr size_t kPinMax = (size_t)16 << 20;
    DevBuf in, out;                   // per object (device side)
    Staging() = default;
    Staging(const Staging&) = delete;
    Staging& operator=(const Staging&) = delete;
    const void* dev_in(const Exec& e, const void* x, size_t bytes)
    {
        if (!e.host) return x;
        in.ensure(bytes, e.device);
        if (bytes && host_pinned(x)) {
            // page-locked input: DMA from it directly (the call ends with a synchronize)
            LDSP_HIP(hipMemcpyAsync(in.p, x, bytes, hipMemcpyHostToDevice, e.stream));
        } else if (bytes && bytes <= kPinMax) {
            PinnedPool& pp = pinned_pool(e.device);
            LDSP_HIP(hipEventSynchronize(pp.done()));
            std::memcpy(pp.hin.ensure(bytes), x, bytes);
            LDSP_HIP(hipMemcpyAsync(in.p, pp.hin.p, bytes, hipMemcpyHostToDevice, e.stream));
            LDSP_HIP(hipEventRecord(pp.hin_done, e.stream));
        } else if (bytes) {
            LDSP_HIP(hipMemcpyAsync(in.p, x, bytes, hipMemcpyHostToDevice, e.stream));
        }
        return in.p;
    }
    void* dev_out(const Exec& e, void* y, size_t bytes)
    {
        if (!e.host) return y;
        return out.ensure(bytes, e.device);
    }
    void finish(const Exec& e, void* y, size_t bytes)
    {
        if (!e.host) return;
        if (bytes && host_pinned(y)) {
            LDSP_HIP(hipMemcpyAsync(y, out.p, bytes, hipMemcpyDeviceToHost, e.stream));
            PinnedPool& pp = pinned_pool(e.device);
            LDSP_HIP(hipEventRecord(pp.done(), e.stream));
            LDSP_HIP(hipEventSynchronize(pp.done()));
            return;
        }
        if (bytes && bytes <= kPinMax) {
            PinnedPool& pp = pinned_pool(e.device);
            LDSP_HIP(hipMemcpyAsync(pp.hout.ensure(bytes), out.p, bytes, hipMemcpyDeviceToHost, e.stream));
            // wait on an event (the host spins on it) rather than the stream, whose
            // synchronize may yield the thread: a README block makes five of these waits
            LDSP_HIP(hipEventRecord(pp.done(), e.stream));
            LDSP_HIP(hipEventSynchronize(pp.hin_done));
            std::memcpy(y, pp.hout.p, bytes);
            return;
        }
        if (bytes) LDSP_HIP(hipMemcpyAsync(y, out.p, bytes, hipMemcpyDeviceToHost, e.stream));
        LDSP_HIP(hipStreamSynchronize(e.stream));
    }
};

// ====================================================================== FIR
struct FirObj {
    std::vector<float> h;
    bool cplx = false;
    float scale = 1.0f;
    int mode = LDSP_MODE_FAST;
    int device = -1;
    DevBuf taps_pad, taps_rev, hist[2];
    DevBuf fft_H, fft_tw;             // overlap-save spectrum (for fft_scale) and twiddles
    DevBuf mixbuf;                    // ldsp_nco_mix_firfilt off the fused path: the mixed samples
    float fft_scale = 0.0f;
    bool fft_ready = false;
    int cur = 0;
    hipStream_t last = nullptr;
    StreamMark ord;                   // cross-stream call order (ldsp_common.hpp)
    Staging stg;
    size_t esz() const { return cplx ? 8 : 4; }
    // FAST on complex data with L in [kFirFftMinTaps, 1025] runs the overlap-save
    // FFT kernel (HBM-bound); shorter filters and DIRECT use the register-blocked
    // direct form (VALU-bound at 4 L flop / sample).
    static constexpr int kFirFftMinTaps = 48;
    int fft_P() const { return ((int)h.size() - 1 + 63) / 64 * 64; }
    bool use_fft() const
    {
        const int L = (int)h.size();
        return mode == LDSP_MODE_FAST && cplx && L >= kFirFftMinTaps && fft_P() <= 512;
    }
    void prepare_fft()
    {
        if (fft_ready && fft_scale == scale) return;
        const int L = (int)h.size();
        const int N = k::fir_fft_points(fft_P());
        std::vector<float> Hf(2 * (size_t)N);
        for (int f = 0; f < N; f++) {
            double re = 0.0, im = 0.0;
            for (int i = 0; i < L; i++) {
                const double a = -2.0 * M_PI * (double)(((long)f * i) % N) / N;
                re += (double)h[i] * cos(a);
                im += (double)h[i] * sin(a);
            }
            Hf[2 * f] = (float)(re * (double)scale / N);
            Hf[2 * f + 1] = (float)(im * (double)scale / N);
        }
        // Stockham twiddles exp(-2 pi i r k / (Ns R)), [pass][r-1][k] (kernels.hpp)
        std::vector<float> tw;
        const int p512[2][2] = {{8, 8}, {64, 8}}, p1024[2][2] = {{16, 16}, {256, 4}};
        for (const auto& pr : (N == 512 ? p512 : p1024))
            for (int r = 1; r < pr[1]; r++)
                for (int kk = 0; kk < pr[0]; kk++) {
                    const double a = -2.0 * M_PI * (double)(r * kk) / (double)(pr[0] * pr[1]);
                    tw.push_back((float)cos(a));
                    tw.push_back((float)sin(a));
                }
        upload(fft_H, Hf, device);
        upload(fft_tw, tw, device);
        fft_scale = scale;
        fft_ready = true;
    }
    void ensure_device()
    {
        if (device >= 0) return;
        const int dev = current_device();
        const int L = (int)h.size();
        std::vector<float> pad((L + 15) / 16 * 16, 0.0f), rev(L);
        for (int i = 0; i < L; i++) {
            pad[i] = h[i];
            rev[L - 1 - i] = h[i];
        }
        upload(taps_pad, pad, dev);
        upload(taps_rev, rev, dev);
        for (auto& b : hist) {
            b.ensure(std::max<size_t>(L - 1, 1) * esz(), dev);
            zero_now(b.p, 0, std::max<size_t>(L - 1, 1) * esz());
        }
        device = dev;
    }
};
} // namespace ldsp

struct ldsp_firfilt_s : ldsp::FirObj {};
struct ldsp_resamp_s;
struct ldsp_nco_s;
struct ldsp_iirfilt_s;
struct ldsp_agc_s;
struct ldsp_ampmodem_s;

namespace ldsp {

// ====================================================================== resampler
struct ResampObj {
    bool cplx = true;                 // complex samples
    bool real_taps = false;           // crcf: complex samples, real taps (CResampler)
    float rate = 1.0f;
    unsigned int m = 0, npfb = 0, sub_len = 0;
    int bits_index = 0;
    uint32_t step = 0;
    uint64_t phase = 0;
    float fc = 0, as = 0;
    std::vector<float> hproto, sub;   // sub: [npfb][sub_len] reversed (complex interleaved if cplx)
    int device = -1;
    DevBuf dsub, hist[2];
    int cur = 0;
    hipStream_t last = nullptr;
    StreamMark ord;                   // cross-stream call order (ldsp_common.hpp)
    Staging stg;
    size_t esz() const { return cplx ? 8 : 4; }
    void set_rate(float r)
    {
        LDSP_REQUIRE(r > 0, "resamp: resampling rate must be greater than zero");
        LDSP_REQUIRE(r >= 0.004f && r <= 250.0f, "resamp: resampling rate must be in [0.004, 250]");
        rate = r;
        step = (uint32_t)round((double)((float)(1 << 24) / rate));
    }
    size_t num_outputs(size_t n) const
    {
        if (n == 0) return 0;
        const long long num = (long long)(n - 1) * (1LL << 24) + 0xffffffLL - (long long)phase;
        return num < 0 ? 0 : (size_t)(num / step) + 1;
    }
    void ensure_device()
    {
        if (device >= 0) return;
        const int dev = current_device();
        upload(dsub, sub, dev);
        for (auto& b : hist) {
            b.ensure(std::max<size_t>(sub_len - 1, 1) * esz(), dev);
            zero_now(b.p, 0, std::max<size_t>(sub_len - 1, 1) * esz());
        }
        device = dev;
    }
};

// ====================================================================== NCO
struct NcoObj {
    int type = 0;
    uint32_t theta = 0, dtheta = 0;
    float alpha = 0.1f, beta = 0.0f;
    std::vector<float> table;
    int device = -1;
    DevBuf dtab;
    Staging stg;
    void ensure_device()
    {
        if (device >= 0) return;
        const int dev = current_device();
        upload(dtab, table, dev);
        device = dev;
    }
};

static std::vector<float> nco_table()
{
    // nco.proto.c: sintab[i] = sinf(2.0f*M_PI*(float)(i)/1024.0f)
    std::vector<float> t(1024);
    for (int i = 0; i < 1024; i++) t[i] = sinf((float)(2.0f * 3.14159265358979323846 * (float)i / 1024.0f));
    return t;
}

static uint32_t nco_constrain(float theta)
{
    const float p = (float)((double)theta * 0.159154943091895);
    float f = p - (float)(long long)p;
    if (f < 0.0f) f = (float)((double)f + 1.0);
    return (uint32_t)(long long)(f * 4294967296.0f);
}

// ====================================================================== IIR
struct IirObj {
    bool cplx = true;
    bool sos = true;
    unsigned int nsos = 0;
    std::vector<float> b, a;          // SOS: [nsos][3] each; TF: nb, na (normalised by a0)
    int nb = 0, na = 0, nv = 0, D = 0;
    int mode = LDSP_MODE_FAST;
    int spec_W = 0;                   // > 0: fast-decaying filter -> speculative exact chunks
    int device = -1;
    DevBuf db, da, st32, st64, sc1, sc2, mats;
    DevBuf bmats, bsc1, bsc2, bsc3;   // blocked scan (D <= 8): matrices and scratch
    int bplan_G = 0;
    // single-pass modal scan (k_iir_modal.hip): the modal form (ok == false:
    // the blocked scan), its tables, the per-unit published end states, the
    // call epoch, and the modal state in two buffers (a call reads its start
    // state from mst and writes its end state into mstb; swapped after the call)
    ModalForm mf;
    DevBuf mtab, magg, mst, mstb;
    long magg_units = 0;
    uint32_t m_epoch = 0;
    int path_force = 0;               // ldsp_debug_iir_path: 0 auto, 1 blocked scan, 2 modal
    DevBuf iq;                        // int16 IQ converted for the paths that do not read it themselves
    DevBuf rsside, rsbuf;             // ldsp_iirfilt_resamp_execute: unit edges (fused) / filter output (two calls)
    enum { kSt32 = 0, kSt64 = 1, kStModal = 2 };
    int state_at = kSt32;             // where the authoritative state lives
    int plan_C = 0;
    long plan_nch = 0;
    int plan_G = 0;
    hipStream_t last = nullptr;
    StreamMark ord;                   // cross-stream call order (ldsp_common.hpp)
    Staging stg;
    std::vector<double> A;            // D x D one-step state matrix (float64)

    int fsz() const { return sos ? 3 * (int)nsos : nv; }
    int ncomp() const { return cplx ? 2 : 1; }
    // Long look-backs: outside its one-XCD small-call mode (<= 16 J units) the
    // modal scan's 8 per-XCD unit ranges each start with J(J+1)/2 predecessor
    // recomputes (k_iir_modal.hip); a slowly decaying filter (J >= 16) whose
    // recomputes would exceed a quarter of the call's units takes the blocked scan.
    bool modal_pays(size_t n) const
    {
        const long units = k::iir_modal_units(n), J = mf.J;
        return J < 16 || units <= 16 * J || 4 * J * (J + 1) <= units / 4;
    }
    // which kernel path a call of n samples takes
    enum Path { kSpec, kSeq, kModal, kBlk, kScan };
    Path path_for(size_t n) const
    {
        // fast-decaying filters: speculative exact chunks (the sequential
        // loop's bits, so exact mode takes them too: FMStereo's de-emphasis)
        static const long spec_min = LDSP_KNOB("LDSP_IIR_SPEC_MIN", 0L);
        if (D == 0) return kSeq;
        if (path_force == 0 && spec_W > 0 && spec_W <= 16384 && (long)n >= spec_min) return kSpec;
        if (mode == LDSP_MODE_EXACT) return kSeq;
        if (mf.ok && path_force != 1 && (path_force >= 2 || modal_pays(n))) return kModal;
        return D <= k::kIirBlkMaxD ? kBlk : kScan;
    }

    // one step of the recursion on a state vector (the layout of the scan
    // kernels), in double or long double
    template <class R>
    R step_t(std::vector<R>& v, R x) const
    {
        if (sos) {
            R t = x;
            for (unsigned s = 0; s < nsos; s++) {
                const R v1 = v[2 * s], v2 = v[2 * s + 1];
                const R v0 = t - (R)a[3 * s + 1] * v1 - (R)a[3 * s + 2] * v2;
                t = (R)b[3 * s] * v0 + (R)b[3 * s + 1] * v1 + (R)b[3 * s + 2] * v2;
                v[2 * s + 1] = v1;
                v[2 * s] = v0;
            }
            return t;
        }
        R r = x;
        for (int i = 1; i < na; i++) r -= (R)a[i] * v[i - 1];
        R y = (R)b[0] * r;
        for (int i = 1; i < nb; i++) y += (R)b[i] * v[i - 1];
        for (int i = D - 1; i > 0; i--) v[i] = v[i - 1];
        if (D > 0) v[0] = r;
        return y;
    }
    double step_host(std::vector<double>& v, double x) const { return step_t<double>(v, x); }

    void finalize()
    {
        D = sos ? 2 * (int)nsos : nv - 1;
        A.assign((size_t)D * D, 0.0);
        for (int c = 0; c < D; c++) {
            std::vector<double> v(D, 0.0);
            v[c] = 1.0;
            step_host(v, 0.0);
            for (int r = 0; r < D; r++) A[(size_t)r * D + c] = v[r];
        }
        // modal form for the single-pass scan (long-double state space)
        mf = ModalForm{};
        if (D > 0) {
            using L = long double;
            std::vector<L> Al((size_t)D * D), Bl(D), Cl(D);
            for (int c = 0; c < D; c++) {
                std::vector<L> v(D, 0.0L);
                v[c] = 1.0L;
                Cl[c] = step_t<L>(v, 0.0L);
                for (int r = 0; r < D; r++) Al[(size_t)r * D + c] = v[r];
            }
            std::vector<L> v(D, 0.0L);
            const L Dd = step_t<L>(v, 1.0L);
            Bl = v;
            mf = modal_form(D, Al, Bl, Cl, Dd, sos ? sos_poles(a, nsos) : tf_poles(a, na, D));
        }
        // decay length: smallest 2^k with ||A^(2^k)||_inf < 2^-70
        spec_W = 0;
        if (D > 0) {
            std::vector<double> P = A;
            for (int k = 0; k <= 12; k++) {
                double nrm = 0;
                for (int r = 0; r < D; r++) {
                    double s = 0;
                    for (int q = 0; q < D; q++) s += fabs(P[(size_t)r * D + q]);
                    nrm = std::max(nrm, s);
                }
                if (nrm < 8.5e-22) {
                    spec_W = 2 << k;   // twice the decay length, as margin
                    break;
                }
                P = matmul(P, P);
            }
        }
    }
    std::vector<double> matmul(const std::vector<double>& X, const std::vector<double>& Y) const
    {
        std::vector<double> Z((size_t)D * D, 0.0);
        for (int r = 0; r < D; r++)
            for (int k = 0; k < D; k++) {
                const double x = X[(size_t)r * D + k];
                for (int c = 0; c < D; c++) Z[(size_t)r * D + c] += x * Y[(size_t)k * D + c];
            }
        return Z;
    }
    std::vector<double> matpow(std::vector<double> X, uint64_t e) const
    {
        std::vector<double> R((size_t)D * D, 0.0);
        for (int i = 0; i < D; i++) R[(size_t)i * D + i] = 1.0;
        while (e) {
            if (e & 1) R = matmul(R, X);
            X = matmul(X, X);
            e >>= 1;
        }
        return R;
    }
    void ensure_device()
    {
        if (device >= 0) return;
        const int dev = current_device();
        upload(db, b, dev);
        upload(da, a, dev);
        st32.ensure(sizeof(float) * 2 * std::max(fsz(), 1), dev);
        zero_now(st32.p, 0, sizeof(float) * 2 * std::max(fsz(), 1));
        st64.ensure(sizeof(double) * 2 * std::max(D, 1), dev);
        zero_now(st64.p, 0, sizeof(double) * 2 * std::max(D, 1));
        if (mf.ok) {
            const size_t mb = sizeof(double) * 2 * 2 * mf.M;
            zero_now(mst.ensure(mb, dev), 0, mb);
            mstb.ensure(mb, dev);
            upload(mtab, mf.tables, dev);
        }
        state_at = kSt32;
        device = dev;
    }
    k::IirDesc desc() const
    {
        k::IirDesc d;
        d.sos = sos ? 1 : 0;
        d.nsos = (int)nsos;
        d.nb = nb;
        d.na = na;
        d.nv = nv;
        d.D = D;
        d.b = db.as<float>();
        d.a = da.as<float>();
        return d;
    }
    // Move the authoritative state between the float32 DF-II layout (exact
    // paths), the float64 layout of the SOS-coordinate scans and the modal
    // coordinates (k_iir_modal), through the host (mode switches only).
    void state_to(int to, hipStream_t s)
    {
        if (state_at == to) return;
        const int nc = ncomp(), fs = fsz();
        std::vector<double> d(2 * std::max(D, 1), 0.0);
        LDSP_HIP(hipStreamSynchronize(s));
        // 1. current state -> float64 layout d
        if (state_at == kSt32) {
            std::vector<float> f(2 * std::max(fs, 1), 0.0f);
            LDSP_HIP(hipMemcpy(f.data(), st32.p, f.size() * 4, hipMemcpyDeviceToHost));
            for (int c = 0; c < nc; c++) {
                if (sos)
                    for (unsigned q = 0; q < nsos; q++) {
                        d[c * D + 2 * q] = f[c * fs + 3 * q];
                        d[c * D + 2 * q + 1] = f[c * fs + 3 * q + 1];
                    }
                else
                    for (int i = 0; i < D; i++) d[c * D + i] = f[c * fs + i];
            }
        } else if (state_at == kSt64) {
            LDSP_HIP(hipMemcpy(d.data(), st64.p, d.size() * 8, hipMemcpyDeviceToHost));
        } else {
            const int M = mf.M;
            std::vector<double> v(2 * 2 * M);
            LDSP_HIP(hipMemcpy(v.data(), mst.p, v.size() * 8, hipMemcpyDeviceToHost));
            for (int c = 0; c < nc; c++)
                for (int i = 0; i < D; i++) {
                    double t = 0;
                    for (int q = 0; q < 2 * M; q++) t += mf.from_v[(size_t)i * 2 * M + q] * v[c * 2 * M + q];
                    d[c * D + i] = t;
                }
        }
        // 2. float64 layout -> target
        if (to == kSt32) {
            std::vector<float> f(2 * std::max(fs, 1), 0.0f);
            for (int c = 0; c < nc; c++) {
                if (sos)
                    for (unsigned q = 0; q < nsos; q++) {
                        f[c * fs + 3 * q] = (float)d[c * D + 2 * q];
                        f[c * fs + 3 * q + 1] = (float)d[c * D + 2 * q + 1];
                        f[c * fs + 3 * q + 2] = 0.0f;
                    }
                else
                    for (int i = 0; i < fs; i++) f[c * fs + i] = i < D ? (float)d[c * D + i] : 0.0f;
            }
            LDSP_HIP(hipMemcpy(st32.p, f.data(), f.size() * 4, hipMemcpyHostToDevice));
        } else if (to == kSt64) {
            LDSP_HIP(hipMemcpy(st64.p, d.data(), d.size() * 8, hipMemcpyHostToDevice));
        } else {
            const int M = mf.M;
            std::vector<double> v(2 * 2 * M, 0.0);
            for (int c = 0; c < nc; c++)
                for (int q = 0; q < 2 * M; q++) {
                    double t = 0;
                    for (int i = 0; i < D; i++) t += mf.to_v[(size_t)q * D + i] * d[c * D + i];
                    v[c * 2 * M + q] = t;
                }
            LDSP_HIP(hipMemcpy(mst.p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
        }
        state_at = to;
    }
    // Blocked scan plan (k_iir_blk): 256-sample chunks, 256 chunks per block.
    k::IirBlkPlan blk_plan(size_t n)
    {
        const long C = k::kIirBlkChunk, CB = C * k::kIirBlkChunks;
        const long nch = (long)((n + C - 1) / C);
        const long nblk = (long)((n + CB - 1) / CB);
        const int G = (int)((nblk + 1023) / 1024);
        const size_t DD = (size_t)D * D;
        if (G != bplan_G) {
            std::vector<double> all;
            std::vector<double> M = matpow(A, (uint64_t)C);
            for (int l = 0; l < 8; l++) {                     // A^{C 2^l}
                all.insert(all.end(), M.begin(), M.end());
                M = matmul(M, M);
            }
            const std::vector<double> AB = matpow(A, (uint64_t)CB);
            all.insert(all.end(), AB.begin(), AB.end());
            M = matpow(AB, (uint64_t)G);
            for (int l = 0; l < 10; l++) {                    // A^{CB G 2^l}
                all.insert(all.end(), M.begin(), M.end());
                M = matmul(M, M);
            }
            upload(bmats, all, device);
            bplan_G = G;
        }
        k::IirBlkPlan p;
        p.nchunks = nch;
        p.nblk = nblk;
        p.G = G;
        p.AL = bmats.as<double>();
        p.AB = p.AL + 8 * DD;
        p.AG = p.AB + DD;
        p.local = (double*)bsc1.ensure((size_t)nch * ncomp() * D * sizeof(double), device);
        p.blocal = (double*)bsc2.ensure((size_t)nblk * ncomp() * D * sizeof(double), device);
        p.bstart = (double*)bsc3.ensure((size_t)nblk * ncomp() * D * sizeof(double), device);
        return p;
    }
    // Modal scan plan: the tables (uploaded with the state), the per-unit
    // granules (zero when allocated: below every epoch) and this call's epoch.
    k::IirModalPlan modal_plan(size_t n)
    {
        const long units = k::iir_modal_units(n);
        const size_t per = (size_t)ncomp() * mf.M * 4 * sizeof(uint64_t);
        if (units > magg_units) {
            magg.ensure((size_t)units * per, device);
            zero_now(magg.p, 0, magg.cap);
            magg_units = (long)(magg.cap / per);
        }
        if (++m_epoch == 0) {                         // wrapped: restart the granules
            zero_now(magg.p, 0, magg.cap);
            m_epoch = 1;
        }
        k::IirModalPlan p;
        p.J = mf.J;
        p.PS = mtab.as<double>();
        p.PL = p.PS + 6 * mf.M * 4;
        p.PB = p.PL + 64 * mf.M * 4;
        p.agg = magg.as<uint64_t>();
        p.epoch = m_epoch;
        p.recompute = path_force == 3 ? 1 : 0;
        // one XCD while its 32 CUs stream the call faster than a range start
        // recomputes its J predecessors (~2.5 us each): up to 16 J units
        static const int onex = LDSP_KNOB("LDSP_IIR_ONEXCD", -1);
        p.one_xcd = onex >= 0 ? onex : (units <= 16L * mf.J ? 1 : 0);
        p.variant = LDSP_KNOB("LDSP_IIR_VARIANT", 0);
        return p;
    }
    k::IirScanPlan scan_plan(size_t n)
    {
        int C = 64;
        while (C < 1024 && (size_t)C * 65536 < n) C <<= 1;
        const long nch = (long)((n + C - 1) / C);
        const int G = (int)((nch + 1023) / 1024);
        if (C != plan_C || G != plan_G) {
            const std::vector<double> AC = matpow(A, (uint64_t)C);
            std::vector<double> M = matpow(AC, (uint64_t)G);
            std::vector<double> all(AC);
            for (int l = 0; l < 10; l++) {
                all.insert(all.end(), M.begin(), M.end());
                M = matmul(M, M);
            }
            upload(mats, all, device);
            plan_C = C;
            plan_G = G;
        }
        plan_nch = nch;
        const size_t need = (size_t)nch * ncomp() * D * sizeof(double);
        sc1.ensure(need, device);
        sc2.ensure(need, device);
        k::IirScanPlan p;
        p.C = C;
        p.nchunks = nch;
        p.G = G;
        p.levels = 10;
        p.AC = mats.as<double>();
        p.AG = mats.as<double>() + (size_t)D * D;
        p.local = sc1.as<double>();
        p.carry = sc2.as<double>();
        return p;
    }
};

// ====================================================================== AGC
struct AgcObj {
    k::AgcState h{};                  // host mirror
    float bandwidth = 0.01f;
    int device = -1;
    DevBuf dst, status;
    // Per-call scratch in two slots (call parity) and the input history the
    // speculative warm-ups read (the last hist_len samples before the call, in
    // a ring of three: call k reads hist[k % 3] and writes hist[(k + 1) % 3], so
    // call k + 1's front may start while call k's chunks still read theirs;
    // call k + 2, which overwrites it, first waits for call k's back half).
    DevBuf scr[2], hist[3];
    long hist_len = 0, hist_valid = 0;
    uint64_t ncall = 0;
    bool dev_newer = false;           // device state advanced past the mirror
    bool upload_pending = true;
    hipStream_t last = nullptr;
    // Cross-stream order (ldsp_common.hpp): ord = back halves (the true
    // state), front = front halves (history), slot[s] = scratch slot s free.
    StreamMark ord, front, slot[2];
    Staging stg;
    int tsa_perturb = 0;              // ldsp_debug_agc_tsa_perturb (test hook)
    int perturb = 0;                  // ldsp_debug_agc_perturb (test hook, chunk-parallel calls)
    int rounds_force = -1;            // ldsp_debug_agc_rounds (test hook; -1: the default)
    void init()
    {
        // agc_crcf_create: bandwidth 0.01, reset (g=1, y2'=1), squelch disabled,
        // threshold 0, timeout 100, scale 1
        bandwidth = 0.01f;
        h.alpha = bandwidth;
        h.g = 1.0f;
        h.y2p = 1.0f;
        h.locked = 0;
        h.mode = 7;
        h.threshold = 0.0f;
        h.timeout = 100;
        h.timer = 0;
        h.scale = 1.0f;
    }
    void pull()
    {
        if (!dev_newer) return;
        LDSP_HIP(hipStreamSynchronize(last));
        DeviceGuard g(device);
        LDSP_HIP(hipMemcpy(&h, dst.p, sizeof(h), hipMemcpyDeviceToHost));
        dev_newer = false;
    }
    void modified() { upload_pending = true; }
    void ensure_device()
    {
        if (device >= 0) return;
        const int dev = current_device();
        dst.ensure(sizeof(k::AgcState), dev);
        device = dev;
        upload_pending = true;
    }
};

// ====================================================================== AmpModem
// Live PLL objects (AmpModem, BroadcastAM) per device: a walker may be launched
// before its predecessor has finished (amp_pll_stage), holding a CU while it
// waits.  Waiting walkers and the walkers they wait for number at most twice the
// live objects on the device, so the early path is taken only while those stay
// within half the device's CUs (amp_early_max: CUs / 4 objects, 64 on MI355X; a
// CPX-partitioned device gets its own, smaller bound).  Other processes sharing
// the GPU are not counted: their walkers can only delay a hand-off, which the
// walker's bounded wait turns into LDSP_EHIP at the next call (amp_check_err),
// never into a silent result.
static constexpr int kAmpMaxDev = 64;
static std::atomic<int> g_amp_live[kAmpMaxDev];
static int amp_early_max(int dev)
{
    static std::atomic<int> cache[kAmpMaxDev];
    if (dev < 0 || dev >= kAmpMaxDev) return 0;
    int v = cache[dev].load();
    if (v == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
        v = cus / 4 > 0 ? cus / 4 : -1;
        cache[dev] = v;
    }
    return v;
}
struct AmpLive {
    int dev = -1;
    void set(int d)
    {
        if (dev < 0 && d >= 0 && d < kAmpMaxDev) {
            dev = d;
            g_amp_live[d]++;
        }
    }
    bool early_ok() const { return dev >= 0 && g_amp_live[dev].load() <= amp_early_max(dev); }
    AmpLive() = default;
    ~AmpLive()
    {
        if (dev >= 0) g_amp_live[dev]--;
    }
    AmpLive(const AmpLive&) = delete;
    AmpLive& operator=(const AmpLive&) = delete;
};
// Host-mapped error flags (one word per PLL object, taken from page-sized
// blocks that are never freed: hipHostFree at teardown can outlive the runtime).
// A walker whose hand-off wait times out sets its object's flag; every call
// checks it on entry (amp_check_err), so a bad walk is reported at the latest by
// the object's next call even when no call synchronises in between.
struct ErrFlags {
    std::mutex mu;
    std::vector<uint32_t*> free_list;
    uint32_t* take()
    {
        std::lock_guard<std::mutex> lk(mu);
        if (free_list.empty()) {
            void* p = nullptr;
            LDSP_HIP(hipHostMalloc(&p, 4096, hipHostMallocMapped | hipHostMallocCoherent));
            for (int i = 1023; i >= 0; i--) free_list.push_back((uint32_t*)p + i);
        }
        uint32_t* f = free_list.back();
        free_list.pop_back();
        *(volatile uint32_t*)f = 0;
        return f;
    }
    void give(uint32_t* f)
    {
        std::lock_guard<std::mutex> lk(mu);
        free_list.push_back(f);
    }
};
static ErrFlags& err_flags()
{
    static ErrFlags* e = new ErrFlags();   // never destroyed (see above)
    return *e;
}
static constexpr unsigned long long kWalkWaitTicks = 100000000ull;   // 1 s of s_memrealtime (100 MHz)
// ldsp_debug_walk_early: -1 default (early hand-off on), 0 / 1 forced
static std::atomic<int> g_walk_early{-1};
struct AmpObj {
    AmpLive live;
    uint32_t* herr = nullptr;             // host-mapped walker timeout flag (ErrFlags)
    float mod_index = 0.75f;
    int type = 0;
    int suppressed = 1;
    unsigned int m = 25;
    std::vector<float> lp, dc, hq, table;     // hq: the usb / lsb Hilbert transform's 2m quadrature taps
    k::AmpState st{};
    int device = -1;
    DevBuf dlp, ddc, dtab, dst, lph[2], dch[2];
    // usb / lsb: Hilbert taps, its input history (4m - 1 samples, ping-pong) and per-slot v1 scratch
    DevBuf dhq, hbh[2], v1[2];
    int hcur = 0;
    // Per-call scratch in two slots (call parity) and the delay-line history in
    // three (call index mod 3), so that call k's front half (lowpass, history,
    // candidates) can run while call k-1's walker still reads its own slot.
    DevBuf x0[2], mb[2], pll[2], dlh[3];
    unsigned long long ncall = 0;
    uint32_t wexp = 0;                    // launches issued that write the PLL state (AmpState::wepoch)
    size_t last_pll_n = 0;                // samples of the last call's PLL launch
    const void* last_stats = nullptr;     // walker counters of the last parallel call (in its scratch slot)
    int cur = 0;
    bool dev_newer = false;
    hipStream_t last = nullptr;
    // Cross-stream order (ldsp_common.hpp): `front` = end of a call's front half
    // (lowpass + delay histories, candidate guess state), `ord` = end of a call's
    // walk (true PLL state), `post` = end of its DC blocker (history),
    // `slot[i]` = end of the last call that used scratch slot i.
    StreamMark front, ord, post, slot[2];
    Staging stg;
    void reset_host()
    {
        st.theta = 0;
        st.dtheta = 0;
        st.alpha = 0.001f;
        st.beta = sqrtf(st.alpha);
        for (int i = 0; i < 2; i++) {
            st.gth[i] = st.theta;
            st.gd[i] = st.dtheta;
        }
    }
    void sync_all()
    {
        ord.sync();
        post.sync();
        front.sync();
        for (auto& sm : slot) sm.sync();
    }
    void ensure_device()
    {
        if (device >= 0) return;
        const int dev = current_device();
        std::vector<float> lr(lp.rbegin(), lp.rend()), dr(dc.rbegin(), dc.rend());
        upload(dlp, lr, dev);
        upload(ddc, dr, dev);
        upload(dtab, table, dev);
        dst.ensure(sizeof(k::AmpState), dev);
        st.wepoch = wexp;
        if (!herr) herr = err_flags().take();
        void* hdev = nullptr;
        LDSP_HIP(hipHostGetDevicePointer(&hdev, herr, 0));
        st.herr = (uint32_t*)hdev;
        if (!st.wait_ticks) st.wait_ticks = kWalkWaitTicks;
        LDSP_HIP(hipMemcpy(dst.p, &st, sizeof(st), hipMemcpyHostToDevice));
        live.set(dev);
        for (int i = 0; i < 2; i++) {
            lph[i].ensure((2 * m) * 8, dev);
            zero_now(lph[i].p, 0, (2 * m) * 8);
            dch[i].ensure((2 * m) * 4, dev);
            zero_now(dch[i].p, 0, (2 * m) * 4);
        }
        for (auto& b : dlh) {
            b.ensure(m * 8, dev);
            zero_now(b.p, 0, m * 8);
        }
        if (!hq.empty()) {
            upload(dhq, hq, dev);
            for (auto& b : hbh) {
                b.ensure((4 * m - 1) * 8, dev);
                zero_now(b.p, 0, (4 * m - 1) * 8);
            }
        }
        device = dev;
    }
    AmpObj() = default;
    AmpObj(const AmpObj&) = delete;
    AmpObj& operator=(const AmpObj&) = delete;
    ~AmpObj()
    {
        if (herr) err_flags().give(herr);
    }
};

} // namespace ldsp

struct ldsp_resamp_s : ldsp::ResampObj {};
struct ldsp_nco_s : ldsp::NcoObj {};
struct ldsp_iirfilt_s : ldsp::IirObj {};
struct ldsp_agc_s : ldsp::AgcObj {};
struct ldsp_ampmodem_s : ldsp::AmpObj {};

// BroadcastAM: the AmpModem carrier-PLL stage with mod_index 1 (re(v1) / 1
// == re(v1)) followed by an owned SOS IIR DC blocker instead of the FIR one.
struct ldsp_bcastam_s : ldsp::AmpObj {
    ldsp_iirfilt_t dcb = nullptr;
};

// Streaming state of the per-sample kernels lives on the device, ping-ponged
// between two buffers so a call never reads what it writes.
struct ldsp_freqdem_s {
    float kf = 0.0f, ref = 0.0f;
    int device = -1, cur = 0;
    ldsp::DevBuf prev[2];
    hipStream_t last = nullptr;
    ldsp::StreamMark ord;                   // cross-stream call order (ldsp_common.hpp)
    ldsp::Staging stg;
};

// FMStereo (demod.hpp:4-85): freqdem(4) + mixer loop + two TF de-emphasis
// filters (exact) + two resamp_rrrf_create_default resamplers.
struct ldsp_fmstereo_s {
    float iq_rate = 0, pcm_rate = 0;
    ldsp_freqdem_t dem = nullptr;
    ldsp_iirfilt_t emph[2] = {nullptr, nullptr};
    ldsp_resamp_t aud[2] = {nullptr, nullptr};
    std::vector<float> table;
    ldsp::k::FmState st{};
    int device = -1;
    ldsp::DevBuf dst, dtab, sbuf, lr[2], le[2], out[2];
    hipStream_t last = nullptr;
    ldsp::StreamMark ord;                  // cross-stream call order (ldsp_common.hpp)
    ldsp::Staging stg;
};

struct ldsp_delay_s {
    unsigned int nd = 1;
    int device = -1, cr = 0, cc = 0;
    ldsp::DevBuf hr[2], hc[2];     // real / complex lines of nd + 1 samples
    hipStream_t last = nullptr;
    ldsp::StreamMark ord;                  // cross-stream call order (ldsp_common.hpp)
    ldsp::Staging stg;
    void zero()
    {
        for (int i = 0; i < 2; i++) {
            ldsp::zero_now(hr[i].ensure((nd + 1) * 4, device), 0, (nd + 1) * 4);
            ldsp::zero_now(hc[i].ensure((nd + 1) * 8, device), 0, (nd + 1) * 8);
        }
        cr = cc = 0;
    }
};

using namespace ldsp;

// Run `fn` translating exceptions into status codes
template <typename F>
static int guard(F&& fn)
{
    try {
        fn();
        return LDSP_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("out of host memory");
        return LDSP_ENOMEM;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return LDSP_EHIP;
    }
}

#define NONNULL(p) LDSP_REQUIRE((p) != nullptr, #p " must not be NULL")

// ---------------------------------------------------------------- per-kernel timing
namespace ldsp {
namespace prof {
namespace {
std::atomic<bool> g_on{false};
std::mutex g_mu;
struct Pending {
    const char* name;
    hipEvent_t a, b;
    hipStream_t s;
};
std::vector<Pending> g_pending;
std::vector<std::pair<std::string, std::pair<long, double>>> g_done;   // name -> (calls, total ms)

// LDSP_PROF_TIMELINE=<file>: also append every profiled launch as
// "name stream start_ms end_ms" relative to the first launch since the last
// reset (overlap and gaps between streams; diagnostics only).
hipEvent_t g_t0 = nullptr;
void drain_locked()
{
    static const char* tl_path = LDSP_KNOB_S("LDSP_PROF_TIMELINE");
    FILE* tl = tl_path ? std::fopen(tl_path, "a") : nullptr;
    for (auto& r : g_pending) {
        float ms = 0.0f;
        if (hipEventSynchronize(r.b) == hipSuccess) (void)hipEventElapsedTime(&ms, r.a, r.b);
        if (tl) {
            if (!g_t0) g_t0 = r.a;
            float t0 = 0.0f;
            (void)hipEventElapsedTime(&t0, g_t0, r.a);
            std::fprintf(tl, "%s %p %.4f %.4f\n", r.name, (void*)r.s, t0, t0 + ms);
        }
        if (r.a != g_t0) (void)hipEventDestroy(r.a);     // the origin lives until the next reset
        (void)hipEventDestroy(r.b);
        auto it = std::find_if(g_done.begin(), g_done.end(), [&](const auto& e) { return e.first == r.name; });
        if (it == g_done.end()) g_done.push_back({r.name, {1, (double)ms}});
        else {
            it->second.first++;
            it->second.second += ms;
        }
    }
    g_pending.clear();
    if (tl) std::fclose(tl);
}
} // namespace

bool enabled() { return g_on.load(std::memory_order_relaxed); }

// ldsp_profile_only: time only the launches of one kernel (the bench's timed
// steps record the dominant kernel alone: two events per launch of it instead
// of two per launch of every kernel)
// The filter points into an interned, never-freed set of names, so a Scope that
// compares against it while another thread changes the filter never reads freed
// memory (the set's nodes do not move).
std::atomic<const char*> g_only{nullptr};
std::set<std::string>* g_only_names = new std::set<std::string>();

Scope::Scope(hipStream_t s_, const char* n) : s(s_), name(n)
{
    // a launcher that issues its kernel directly while a many-call records (batch.hpp)
    // would run it out of order: refuse before the launch
    if (batch_active()) throw Error(LDSP_EUNSUP, std::string("kernel not batchable in a many-call: ") + n);
    if (!enabled()) return;
    const char* only = g_only.load(std::memory_order_relaxed);
    if (only && std::strcmp(only, n) != 0) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventRecord(a, s) != hipSuccess) a = nullptr;
}

Scope::~Scope()
{
    if (!a) return;
    hipEvent_t b = nullptr;
    if (hipEventCreate(&b) != hipSuccess || hipEventRecord(b, s) != hipSuccess) {
        (void)hipEventDestroy(a);
        return;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_pending.push_back({name, a, b, s});
    if (g_pending.size() > 4096) drain_locked();
}
} // namespace prof
} // namespace ldsp

extern "C" {

int ldsp_profile_enable(int on)
{
    ldsp::prof::g_on.store(on != 0);
    return LDSP_OK;
}

int ldsp_profile_only(const char* kernel)
{
    return guard([&] {
        std::lock_guard<std::mutex> lk{ldsp::prof::g_mu};
        if (kernel && *kernel)
            ldsp::prof::g_only.store(ldsp::prof::g_only_names->insert(kernel).first->c_str());
        else
            ldsp::prof::g_only.store(nullptr);
    });
}

int ldsp_profile_reset(void)
{
    return guard([&] {
        std::lock_guard<std::mutex> lk{ldsp::prof::g_mu};
        ldsp::prof::drain_locked();
        ldsp::prof::g_done.clear();
        if (ldsp::prof::g_t0) (void)hipEventDestroy(ldsp::prof::g_t0);
        ldsp::prof::g_t0 = nullptr;
    });
}

int ldsp_profile_report(char* buf, size_t cap, size_t* len)
{
    return guard([&] {
        NONNULL(len);
        std::string out;
        {
            std::lock_guard<std::mutex> lk{ldsp::prof::g_mu};
            ldsp::prof::drain_locked();
            char line[256];
            for (const auto& e : ldsp::prof::g_done) {
                std::snprintf(line, sizeof(line), "%s %ld %.6f\n", e.first.c_str(), e.second.first, e.second.second);
                out += line;
            }
        }
        *len = out.size();
        if (buf && cap > 0) {
            const size_t m = std::min(cap - 1, out.size());
            std::memcpy(buf, out.data(), m);
            buf[m] = 0;
        }
    });
}

const char* ldsp_last_error(void) { return g_last_error.c_str(); }
int ldsp_version(void) { return 100; }

int ldsp_device_count(int* n)
{
    return guard([&] {
        NONNULL(n);
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
        *n = c;
    });
}

int ldsp_stream_synchronize(void* stream)
{
    return guard([&] { LDSP_HIP(hipStreamSynchronize((hipStream_t)stream)); });
}

int ldsp_debug_math_eval(int fn, const float* a, const float* b, float* y, size_t n, void* stream)
{
    return guard([&] {
        LDSP_REQUIRE(fn >= 0 && fn <= 8, "math_eval: unknown function");
        (void)current_device();
        k::math_eval(fn, a, b ? b : a, y, n, (hipStream_t)stream);
    });
}

int ldsp_debug_math_fastcheck(int fn, uint32_t begin, uint32_t end, uint32_t stride, uint64_t* checked,
                              uint64_t* mismatches)
{
    return guard([&] {
        LDSP_REQUIRE(fn >= 0 && fn <= 1 && stride > 0 && checked && mismatches, "math_fastcheck: bad arguments");
        uint64_t c = 0, bad = 0;
        for (uint64_t u = begin; u < end; u += stride) {
            const float a = bitsf((uint32_t)u);
            if (fn == 0) {
                if (lm_logf_fast_ok(a)) {
                    c++;
                    bad += fbits(lm_logf_fast(a)) != fbits(lm_logf(a));
                }
            } else if (fn == 1) {
                if (lm_expf_fast_ok(a)) {
                    c++;
                    bad += fbits(lm_expf_fast(a)) != fbits(lm_expf(a));
                }
            }
        }
        *checked = c;
        *mismatches = bad;
    });
}

// ---------------------------------------------------------------- FIR
static int fir_make(std::vector<float> h, int cplx, ldsp_firfilt_t* q)
{
    LDSP_REQUIRE(!h.empty(), "firfilt: filter length must be > 0");
    LDSP_REQUIRE((int)h.size() <= k::kFirMaxTaps, "firfilt: filter length exceeds 8192 taps");
    auto* o = new ldsp_firfilt_s();
    o->h = std::move(h);
    o->cplx = cplx != 0;
    *q = o;
    return LDSP_OK;
}

int ldsp_firfilt_create(const float* h, unsigned int n, int cplx, ldsp_firfilt_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(h != nullptr || n == 0, "firfilt: taps must not be NULL");
        fir_make(std::vector<float>(h, h + n), cplx, q);
    });
}

int ldsp_firfilt_create_kaiser(unsigned int n, float fc, float as, float mu, int cplx, ldsp_firfilt_t* q)
{
    return guard([&] {
        NONNULL(q);
        fir_make(design::firdes_kaiser(n, fc, as, mu), cplx, q);
    });
}

int ldsp_firfilt_create_dc_blocker(unsigned int m, float as, int cplx, ldsp_firfilt_t* q)
{
    return guard([&] {
        NONNULL(q);
        fir_make(design::firdes_notch(m, 0.0f, as), cplx, q);
    });
}

int ldsp_firfilt_destroy(ldsp_firfilt_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}

int ldsp_firfilt_reset(ldsp_firfilt_t q)
{
    return guard([&] {
        NONNULL(q);
        if (q->device < 0) return;
        DeviceGuard g(q->device);
        const size_t bytes = std::max<size_t>(q->h.size() - 1, 1) * q->esz();
        for (auto& b : q->hist) LDSP_HIP(hipMemsetAsync(b.p, 0, bytes, q->last));
        q->ord.mark(q->last);              // a call on another stream waits for the zeroing
    });
}

int ldsp_firfilt_set_scale(ldsp_firfilt_t q, float s) { return guard([&] { NONNULL(q); q->scale = s; }); }
int ldsp_firfilt_get_scale(ldsp_firfilt_t q, float* s) { return guard([&] { NONNULL(q); NONNULL(s); *s = q->scale; }); }
int ldsp_firfilt_get_length(ldsp_firfilt_t q, unsigned int* n)
{
    return guard([&] { NONNULL(q); NONNULL(n); *n = (unsigned)q->h.size(); });
}
int ldsp_firfilt_get_taps(ldsp_firfilt_t q, float* h)
{
    return guard([&] { NONNULL(q); NONNULL(h); std::copy(q->h.begin(), q->h.end(), h); });
}
int ldsp_firfilt_set_mode(ldsp_firfilt_t q, int mode)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(mode == LDSP_MODE_FAST || mode == LDSP_MODE_EXACT || mode == LDSP_MODE_DIRECT, "unknown mode");
        q->mode = mode;
    });
}

int ldsp_firfilt_get_mode(ldsp_firfilt_t q, int* mode)
{
    return guard([&] { NONNULL(q); NONNULL(mode); *mode = q->mode; });
}

// liquid firfilt_freqresponse: H = scale * sum_i hrev[i] exp(+j 2 pi f i)
int ldsp_firfilt_freqresponse(ldsp_firfilt_t q, float f, float* re, float* im)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(re);
        NONNULL(im);
        const size_t L = q->h.size();
        std::complex<float> H(0.0f, 0.0f);
        for (size_t i = 0; i < L; i++) {
            const float hr = q->h[L - 1 - i];
            const float ang = (float)(2 * 3.14159265358979323846 * (double)f * (double)i);
            H += hr * std::exp(std::complex<float>(0.0f, ang));
        }
        H *= q->scale;
        *re = H.real();
        *im = H.imag();
    });
}

// One filter call on device buffers, in stream order after the object's
// previous call; `fuse` applies an NCO mix to the samples as the overlap-save
// kernel loads them (only on that path: the caller checks fir_can_fuse).
static void fir_dispatch(ldsp_firfilt_s* q, const void* dx, size_t n, void* dy, hipStream_t s, const k::NcoFuse* fuse)
{
    const int L = (int)q->h.size();
    void* hin = q->hist[q->cur].p;
    void* hout = q->hist[1 - q->cur].p;
    if (L <= 1 && n == 0) return;
    if (q->mode == LDSP_MODE_EXACT)
        k::fir_exact(q->cplx, dx, hin, hout, n, q->taps_rev.as<float>(), L, q->scale, dy, s);
    else if (q->use_fft() && n > 0) {
        if (!q->fft_ready || q->fft_scale != q->scale) {
            LDSP_HIP(hipStreamSynchronize(s));   // tables may be in use by queued work
            q->prepare_fft();
        }
        k::fir_fft(dx, hin, hout, n, L, q->fft_P(), q->fft_H.p, q->fft_tw.p, dy, s, fuse);
    } else
        k::fir_fast(q->cplx, dx, hin, hout, n, q->taps_pad.as<float>(), L, q->scale, dy, s);
    if (L > 1) q->cur = 1 - q->cur;
}

int ldsp_firfilt_execute(ldsp_firfilt_t q, const void* x, size_t n, void* y, int mem, void* stream)
{
    LDSP_RANGE("ldsp_firfilt_execute");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "firfilt_execute: NULL buffer");
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const size_t bytes = n * q->esz();
        const void* dx = q->stg.dev_in(e, x, bytes);
        void* dy = q->stg.dev_out(e, y, bytes);
        fir_dispatch(q, dx, n, dy, e.stream, nullptr);
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, bytes);
    });
}

// ---------------------------------------------------------------- resampler
int ldsp_resamp_create(float rate, unsigned int m, float fc, float as, unsigned int npfb, int cplx, ldsp_resamp_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(m > 0, "resamp: filter semi-length must be greater than zero");
        LDSP_REQUIRE(fc > 0.0f && fc < 0.5f, "resamp: filter cutoff must be in (0, 0.5)");
        LDSP_REQUIRE(as > 0.0f, "resamp: filter stop-band suppression must be greater than zero");
        LDSP_REQUIRE(npfb > 0, "resamp: number of filters must be greater than zero");
        LDSP_REQUIRE(cplx >= 0 && cplx <= 2, "resamp: kind must be 0 (rrrf), 1 (cccf) or 2 (crcf)");
        std::unique_ptr<ldsp_resamp_s> o(new ldsp_resamp_s());
        o->cplx = cplx != 0;
        o->real_taps = cplx == 2;
        o->set_rate(rate);
        o->m = m;
        o->fc = fc;
        o->as = as;
        unsigned int bits = 0;
        for (unsigned int v = npfb - 1; v; v >>= 1) bits++;   // liquid_nextpow2
        LDSP_REQUIRE(bits <= 16, "resamp: too many filters");
        o->npfb = 1u << bits;
        o->bits_index = 24 - (int)bits;
        const unsigned int n = 2 * m * o->npfb + 1;
        std::vector<float> hf = design::firdes_kaiser(n, fc / ((float)o->npfb), as, 0.0f);
        float gain = 0.0f;
        for (float v : hf) gain += v;
        gain = (float)o->npfb / gain;
        o->hproto.resize(n);
        for (unsigned int i = 0; i < n; i++) o->hproto[i] = hf[i] * gain;
        o->sub_len = (n - 1) / o->npfb;
        const unsigned c = (o->cplx && !o->real_taps) ? 2 : 1;
        o->sub.assign((size_t)o->npfb * o->sub_len * c, 0.0f);
        for (unsigned int b = 0; b < o->npfb; b++)
            for (unsigned int k = 0; k < o->sub_len; k++)
                o->sub[((size_t)b * o->sub_len + (o->sub_len - k - 1)) * c] = o->hproto[b + k * o->npfb];
        *q = o.release();
    });
}

int ldsp_resamp_create_default(float rate, int kind, ldsp_resamp_t* q)
{
    // resamp_*_create_default (liquid resamp.proto.c, recalled): m 7, fc 0.25, As 60, npfb 256
    return ldsp_resamp_create(rate, 7, 0.25f, 60.0f, 256, kind, q);
}

int ldsp_resamp_destroy(ldsp_resamp_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}

int ldsp_resamp_reset(ldsp_resamp_t q)
{
    return guard([&] {
        NONNULL(q);
        q->phase = 0;
        if (q->device < 0) return;
        DeviceGuard g(q->device);
        const size_t bytes = std::max<size_t>(q->sub_len - 1, 1) * q->esz();
        for (auto& b : q->hist) LDSP_HIP(hipMemsetAsync(b.p, 0, bytes, q->last));
        q->ord.mark(q->last);              // a call on another stream waits for the zeroing
    });
}

int ldsp_resamp_set_rate(ldsp_resamp_t q, float rate) { return guard([&] { NONNULL(q); q->set_rate(rate); }); }
int ldsp_resamp_get_rate(ldsp_resamp_t q, float* r) { return guard([&] { NONNULL(q); NONNULL(r); *r = q->rate; }); }
int ldsp_resamp_get_info(ldsp_resamp_t q, unsigned int* npfb, uint32_t* step, uint32_t* phase, unsigned int* sub_len)
{
    return guard([&] {
        NONNULL(q);
        if (npfb) *npfb = q->npfb;
        if (step) *step = q->step;
        if (phase) *phase = (uint32_t)q->phase;
        if (sub_len) *sub_len = q->sub_len;
    });
}
int ldsp_resamp_get_taps(ldsp_resamp_t q, float* h, unsigned int cap, unsigned int* n)
{
    return guard([&] {
        NONNULL(q);
        if (n) *n = (unsigned)q->hproto.size();
        if (h) {
            LDSP_REQUIRE(cap >= q->hproto.size(), "resamp_get_taps: capacity too small");
            std::copy(q->hproto.begin(), q->hproto.end(), h);
        }
    });
}
int ldsp_resamp_num_outputs(ldsp_resamp_t q, size_t n, size_t* nout)
{
    return guard([&] { NONNULL(q); NONNULL(nout); *nout = q->num_outputs(n); });
}

int ldsp_resamp_execute(ldsp_resamp_t q, const void* x, size_t n, void* y, size_t cap, size_t* nout, int mem,
                        void* stream)
{
    LDSP_RANGE("ldsp_resamp_execute");
    return guard([&] {
        NONNULL(q);
        const size_t K = q->num_outputs(n);
        if (nout) *nout = K;
        if (K > cap) throw Error(LDSP_ERANGE, "resamp_execute: output capacity too small");
        LDSP_REQUIRE(n == 0 || x, "resamp_execute: NULL input");
        LDSP_REQUIRE(K == 0 || y, "resamp_execute: NULL output");
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const void* dx = q->stg.dev_in(e, x, n * q->esz());
        void* dy = q->stg.dev_out(e, y, K * q->esz());
        if (n > 0) {
            k::ResampPlan p;
            p.P0 = q->phase;
            p.step = q->step;
            p.bits_index = q->bits_index;
            p.sub_len = (int)q->sub_len;
            p.npfb = (int)q->npfb;
            p.K = K;
            int KB = 64;
            auto span_for = [&](int kb) {
                return (int)(((uint64_t)(kb - 1) * q->step >> 24) + 3 + q->sub_len);
            };
            while (KB > 1 && (size_t)span_for(KB) * q->esz() > 48 * 1024) KB >>= 1;
            p.KB = KB;
            p.span_max = span_for(KB);
            const int tkb = k::resamp_tile_outputs(q->step, (int)q->sub_len, (int)q->npfb, q->cplx, q->real_taps);
            if (tkb > 0) {
                p.KB = tkb;
                p.tile = 1;
            }
            k::resamp(q->cplx, q->real_taps, dx, q->hist[q->cur].p, q->hist[1 - q->cur].p, n, q->dsub.as<float>(), p, dy,
                      e.stream);
            if (q->sub_len > 1) q->cur = 1 - q->cur;
            q->phase = (uint64_t)((long long)q->phase + (long long)K * q->step - (long long)n * (1LL << 24));
        }
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, K * q->esz());
    });
}

// ---------------------------------------------------------------- NCO
int ldsp_nco_create(int type, ldsp_nco_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(type == 0 || type == 1, "nco: type must be 0 (nco) or 1 (vco)");
        auto* o = new ldsp_nco_s();
        o->type = type;
        o->table = nco_table();
        o->alpha = 0.1f;                     // nco_crcf_pll_set_bandwidth(q, 0.1f) at create
        o->beta = sqrtf(o->alpha);
        *q = o;
    });
}
int ldsp_nco_destroy(ldsp_nco_t q) { return guard([&] { delete q; }); }
int ldsp_nco_reset(ldsp_nco_t q) { return guard([&] { NONNULL(q); q->theta = 0; q->dtheta = 0; }); }
int ldsp_nco_set_frequency(ldsp_nco_t q, float f) { return guard([&] { NONNULL(q); q->dtheta = nco_constrain(f); }); }
int ldsp_nco_adjust_frequency(ldsp_nco_t q, float df)
{
    return guard([&] { NONNULL(q); q->dtheta += nco_constrain(df); });
}
int ldsp_nco_set_phase(ldsp_nco_t q, float p) { return guard([&] { NONNULL(q); q->theta = nco_constrain(p); }); }
int ldsp_nco_adjust_phase(ldsp_nco_t q, float dp) { return guard([&] { NONNULL(q); q->theta += nco_constrain(dp); }); }
int ldsp_nco_get_frequency(ldsp_nco_t q, float* f)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(f);
        const double kPi = 3.14159265358979323846;
        const float d = (float)(2.0f * kPi * (double)(float)q->dtheta / (double)(float)(1ULL << 32));
        *f = d > kPi ? (float)(d - 2 * kPi) : d;
    });
}
int ldsp_nco_get_phase(ldsp_nco_t q, float* p)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(p);
        const double kPi = 3.14159265358979323846;
        const float t = (float)(2.0f * kPi * (double)(float)q->theta / (double)(float)(1ULL << 32));
        *p = t > kPi ? (float)(t - 2 * kPi) : t;
    });
}
int ldsp_nco_pll_set_bandwidth(ldsp_nco_t q, float bw)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(bw >= 0.0f, "nco_pll_set_bandwidth: bandwidth must be positive");
        q->alpha = bw;
        q->beta = sqrtf(q->alpha);
    });
}
int ldsp_nco_pll_step(ldsp_nco_t q, float dphi)
{
    return guard([&] {
        NONNULL(q);
        q->dtheta += nco_constrain(dphi * q->alpha);
        q->theta += nco_constrain(dphi * q->beta);
    });
}
int ldsp_nco_get_state(ldsp_nco_t q, uint32_t* t, uint32_t* d)
{
    return guard([&] { NONNULL(q); if (t) *t = q->theta; if (d) *d = q->dtheta; });
}
int ldsp_nco_set_state(ldsp_nco_t q, uint32_t t, uint32_t d)
{
    return guard([&] { NONNULL(q); q->theta = t; q->dtheta = d; });
}

int ldsp_nco_mix(ldsp_nco_t q, const void* x, size_t n, void* y, int down, int mem, void* stream)
{
    LDSP_RANGE("ldsp_nco_mix");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "nco_mix: NULL buffer");
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        const void* dx = q->stg.dev_in(e, x, n * 8);
        void* dy = q->stg.dev_out(e, y, n * 8);
        k::nco_mix(dx, dy, n, q->theta, q->dtheta, q->dtab.as<float>(), down != 0, q->type, e.stream);
        q->theta += (uint32_t)((uint64_t)n * q->dtheta);
        q->stg.finish(e, y, n * 8);
    });
}

// NCO mix fused into the complex FIR (BASELINE config 3): y = fir(nco.mix(x)).
int ldsp_nco_mix_firfilt(ldsp_nco_t nco, ldsp_firfilt_t q, const void* x, size_t n, void* y, int down, int mem,
                         void* stream)
{
    LDSP_RANGE("ldsp_nco_mix_firfilt");
    return guard([&] {
        NONNULL(nco);
        NONNULL(q);
        LDSP_REQUIRE(q->cplx, "nco_mix_firfilt: the filter must be complex (firfilt_crcf / ComplexFIRFilter)");
        LDSP_REQUIRE(n == 0 || (x && y), "nco_mix_firfilt: NULL buffer");
        const BufDevice bd(mem, x);
        q->ensure_device();
        nco->ensure_device();
        LDSP_REQUIRE(nco->device == q->device, "nco_mix_firfilt: the NCO and the filter live on different devices");
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const size_t bytes = n * 8;
        const void* dx = q->stg.dev_in(e, x, bytes);
        void* dy = q->stg.dev_out(e, y, bytes);
        if (n > 0 && q->use_fft() && nco->type == 0) {
            const k::NcoFuse f{nco->theta, nco->dtheta, down != 0, nco->dtab.as<float>()};
            fir_dispatch(q, dx, n, dy, e.stream, &f);          // the mixed samples never reach HBM
        } else if (n > 0) {
            // other filter modes / the VCO: mix into scratch, then filter (same results)
            void* mb = q->mixbuf.ensure(bytes, q->device);
            k::nco_mix(dx, mb, n, nco->theta, nco->dtheta, nco->dtab.as<float>(), down != 0, nco->type, e.stream);
            fir_dispatch(q, mb, n, dy, e.stream, nullptr);
        } else {
            fir_dispatch(q, dx, 0, dy, e.stream, nullptr);
        }
        nco->theta += (uint32_t)((uint64_t)n * nco->dtheta);
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, bytes);
    });
}

// ---------------------------------------------------------------- IIR
static void iir_finalize_sos(ldsp_iirfilt_s* o, const float* B, const float* A, unsigned nsos)
{
    LDSP_REQUIRE(nsos > 0 && nsos <= 8, "iirfilt: 1..8 second-order sections supported");
    o->sos = true;
    o->nsos = nsos;
    o->b.resize(3 * nsos);
    o->a.resize(3 * nsos);
    for (unsigned s = 0; s < nsos; s++) {
        const float a0 = A[3 * s];          // iirfiltsos_set_coefficients
        LDSP_REQUIRE(a0 != 0.0f, "iirfilt: a0 must be non-zero");
        for (int k = 0; k < 3; k++) {
            o->b[3 * s + k] = B[3 * s + k] / a0;
            o->a[3 * s + k] = A[3 * s + k] / a0;
        }
    }
    o->finalize();
}

int ldsp_iirfilt_create_sos(const float* B, const float* A, unsigned int nsos, int cplx, ldsp_iirfilt_t* q)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(B);
        NONNULL(A);
        std::unique_ptr<ldsp_iirfilt_s> o(new ldsp_iirfilt_s());
        o->cplx = cplx != 0;
        iir_finalize_sos(o.get(), B, A, nsos);
        *q = o.release();
    });
}

int ldsp_iirfilt_create_tf(const float* b, unsigned int nb, const float* a, unsigned int na, int cplx,
                           ldsp_iirfilt_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(b && a && nb > 0 && na > 0, "iirfilt: coefficient arrays must be non-empty");
        LDSP_REQUIRE(nb <= 17 && na <= 17, "iirfilt: transfer functions up to order 16 supported");
        LDSP_REQUIRE(a[0] != 0.0f, "iirfilt: a[0] must be non-zero");
        std::unique_ptr<ldsp_iirfilt_s> o(new ldsp_iirfilt_s());
        o->cplx = cplx != 0;
        o->sos = false;
        o->nb = (int)nb;
        o->na = (int)na;
        o->nv = (int)std::max(nb, na);
        const float a0 = a[0];              // iirfilt_create: normalise by a[0]
        o->b.resize(nb);
        o->a.resize(na);
        for (unsigned i = 0; i < nb; i++) o->b[i] = b[i] / a0;
        for (unsigned i = 0; i < na; i++) o->a[i] = a[i] / a0;
        o->finalize();
        *q = o.release();
    });
}

int ldsp_iirfilt_create_prototype(int ftype, int btype, unsigned int order, float fc, float f0, float ap, float as,
                                  int cplx, ldsp_iirfilt_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(ftype >= 0 && ftype <= 4, "iirfilt: unknown filter type");
        LDSP_REQUIRE(btype >= 0 && btype <= 3, "iirfilt: unknown band type");
        design::SOS s = design::iirdes_sos(ftype, btype, order, fc, f0, ap, as);
        std::unique_ptr<ldsp_iirfilt_s> o(new ldsp_iirfilt_s());
        o->cplx = cplx != 0;
        iir_finalize_sos(o.get(), s.B.data(), s.A.data(), s.nsos);
        *q = o.release();
    });
}

int ldsp_iirfilt_destroy(ldsp_iirfilt_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}

int ldsp_iirfilt_reset(ldsp_iirfilt_t q)
{
    return guard([&] {
        NONNULL(q);
        if (q->device < 0) return;
        DeviceGuard g(q->device);
        LDSP_HIP(hipMemsetAsync(q->st32.p, 0, q->st32.cap, q->last));
        LDSP_HIP(hipMemsetAsync(q->st64.p, 0, q->st64.cap, q->last));
        if (q->mst.p) LDSP_HIP(hipMemsetAsync(q->mst.p, 0, q->mst.cap, q->last));
        q->ord.mark(q->last);              // a call on another stream waits for the zeroing
    });
}

int ldsp_iirfilt_set_mode(ldsp_iirfilt_t q, int mode)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(mode == LDSP_MODE_FAST || mode == LDSP_MODE_EXACT, "unknown mode");
        q->mode = mode;
    });
}
int ldsp_iirfilt_get_nsos(ldsp_iirfilt_t q, unsigned int* n)
{
    return guard([&] { NONNULL(q); NONNULL(n); *n = q->sos ? q->nsos : 0; });
}
int ldsp_debug_iir_path(ldsp_iirfilt_t q, int path)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(path >= 0 && path <= 3,
                     "iirfilt: path must be 0 (automatic), 1 (blocked scan), 2 (modal) or 3 (modal, look-back recomputed)");
        LDSP_REQUIRE(path < 2 || q->mf.ok, "iirfilt: this filter has no valid modal form");
        q->path_force = path;
    });
}
int ldsp_debug_agc_tsa_perturb(ldsp_agc_t q, int on)
{
    return guard([&] {
        NONNULL(q);
        q->tsa_perturb = on ? 1 : 0;
    });
}
int ldsp_debug_agc_perturb(ldsp_agc_t q, int on)
{
    return guard([&] {
        NONNULL(q);
        q->perturb = on ? 1 : 0;
    });
}
int ldsp_debug_agc_rounds(ldsp_agc_t q, int rounds)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(rounds >= -1 && rounds <= 6, "agc: rounds must be -1 (default) or 0..6");
        q->rounds_force = rounds;
    });
}
int ldsp_debug_agc_reruns(ldsp_agc_t q, unsigned int* runfix, unsigned int* verify)
{
    return guard([&] {
        NONNULL(q);
        q->pull();
        if (runfix) *runfix = (unsigned)q->h.pad[2];
        if (verify) *verify = (unsigned)q->h.pad[1];
    });
}
int ldsp_debug_agc_tsa_reruns(ldsp_agc_t q, unsigned int* count)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(count);
        q->pull();
        *count = (unsigned)q->h.pad[0];
    });
}
int ldsp_debug_iir_modal_info(ldsp_iirfilt_t q, int* ok, int* modes, int* lookback, double* err)
{
    return guard([&] {
        NONNULL(q);
        if (ok) *ok = q->mf.ok ? 1 : 0;
        if (modes) *modes = q->mf.M;
        if (lookback) *lookback = q->mf.J;
        if (err) *err = q->mf.err;
    });
}
int ldsp_iirfilt_get_sos(ldsp_iirfilt_t q, float* B, float* A)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(q->sos, "iirfilt_get_sos: filter is in transfer-function form");
        if (B) std::copy(q->b.begin(), q->b.end(), B);
        if (A) std::copy(q->a.begin(), q->a.end(), A);
    });
}

// liquid iirfilt_freqresponse (evaluates with exp(+j 2 pi f k))
int ldsp_iirfilt_freqresponse(ldsp_iirfilt_t q, float f, float* re, float* im)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(re);
        NONNULL(im);
        using cf = std::complex<float>;
        const double kPi = 3.14159265358979323846;
        auto ex = [&](int k) { return std::exp(cf(0.0f, (float)(2 * kPi * (double)f * (double)k))); };
        cf H;
        if (!q->sos) {
            cf Ha(0.0f, 0.0f), Hb(0.0f, 0.0f);
            for (int i = 0; i < q->nb; i++) Hb += q->b[i] * ex(i);
            for (int i = 0; i < q->na; i++) Ha += q->a[i] * ex(i);
            H = Hb / Ha;
        } else {
            H = cf(1.0f, 0.0f);
            for (unsigned s = 0; s < q->nsos; s++) {
                const cf Hb = q->b[3 * s] * ex(0) + q->b[3 * s + 1] * ex(1) + q->b[3 * s + 2] * ex(2);
                const cf Ha = q->a[3 * s] * ex(0) + q->a[3 * s + 1] * ex(1) + q->a[3 * s + 2] * ex(2);
                H *= Hb / Ha;
            }
        }
        *re = H.real();
        *im = H.imag();
    });
}

// iq16: x is n int16 (I, Q) pairs (bytes_to_iq's input); the blocked float64
// scan converts them on load, the other paths after a k_bytes_to_iq pass.
static int iirfilt_execute(ldsp_iirfilt_t q, const void* x, size_t n, void* y, int mem, void* stream, bool iq16)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "iirfilt_execute: NULL buffer");
        LDSP_REQUIRE(!iq16 || q->cplx, "iirfilt_execute_iq16: the filter is real; int16 IQ input needs a complex one");
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const size_t bytes = n * (q->cplx ? 8 : 4);
        const void* dx = q->stg.dev_in(e, x, iq16 ? n * 4 : bytes);
        void* dy = q->stg.dev_out(e, y, bytes);
        if (n > 0) {
            const k::IirDesc d = q->desc();
            using P = IirObj::Path;
            const P path = q->path_for(n);
            enum { kSpec = P::kSpec, kSeq = P::kSeq, kModal = P::kModal, kBlk = P::kBlk, kScan = P::kScan };
            if (iq16 && path != kModal && path != kBlk) {   // not fused: convert first
                void* cx = q->iq.ensure(n * 8, q->device);
                k::bytes_to_iq(dx, cx, n, e.stream);
                dx = cx;
                iq16 = false;
            }
            switch (path) {
            case kSpec: {   // speculative exact chunks (same bits as sequential)
                q->state_to(IirObj::kSt32, e.stream);
                k::SpecPlan p;
                p.W = q->spec_W;
                p.C = std::max(128, q->spec_W / 32);   // W + C steps per lane, <= 1/32 redundancy growth
                p.nchunks = (long)((n + p.C - 1) / p.C);
                const size_t need = k::spec_scratch_bytes(p.nchunks, q->ncomp(), q->fsz());
                p.scratch = q->sc1.ensure(need, q->device);
                k::iir_spec(q->cplx, d, dx, n, q->st32.as<float>(), p, dy, e.stream);
                break;
            }
            case kSeq:
                q->state_to(IirObj::kSt32, e.stream);
                k::iir_seq(q->cplx, d, dx, n, q->st32.as<float>(), dy, e.stream);
                break;
            case kModal: {  // one pass: reads mst (the call's start), writes mstb (its end); then swap
                q->state_to(IirObj::kStModal, e.stream);
                const k::IirModalPlan p = q->modal_plan(n);
                k::iir_modal(q->cplx, q->mf.cf, dx, n, q->mst.as<double>(), q->mstb.as<double>(), p, dy, e.stream,
                             iq16);
                std::swap(q->mst.p, q->mstb.p);
                std::swap(q->mst.cap, q->mstb.cap);
                break;
            }
            case kBlk: {
                q->state_to(IirObj::kSt64, e.stream);
                const k::IirBlkPlan p = q->blk_plan(n);
                k::iir_blk(q->cplx, d, q->b.data(), q->a.data(), dx, n, q->st64.as<double>(), p, dy, e.stream, iq16);
                break;
            }
            case kScan: {
                q->state_to(IirObj::kSt64, e.stream);
                const k::IirScanPlan p = q->scan_plan(n);
                k::iir_scan(q->cplx, d, dx, n, q->st64.as<double>(), p, dy, e.stream);
                break;
            }
            }
        }
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, bytes);
    });
}
int ldsp_iirfilt_execute(ldsp_iirfilt_t q, const void* x, size_t n, void* y, int mem, void* stream)
{
    LDSP_RANGE("ldsp_iirfilt_execute");
    return iirfilt_execute(q, x, n, y, mem, stream, false);
}
int ldsp_iirfilt_execute_iq16(ldsp_iirfilt_t q, const void* x, size_t n, void* y, int mem, void* stream)
{
    LDSP_RANGE("ldsp_iirfilt_execute_iq16");
    return iirfilt_execute(q, x, n, y, mem, stream, true);
}

// IIR -> resampler (resamp(iirfilt(x))) in one pass when the filter takes the
// modal scan: the filter outputs stay on chip (k_iir_modal<RS>), the resampler
// outputs are the resampler kernels' bits, and both objects' states advance as
// after the two calls.  Any other configuration runs the two calls.
int ldsp_iirfilt_resamp_execute(ldsp_iirfilt_t q, ldsp_resamp_t rs, const void* x, size_t n, void* y, size_t cap,
                                size_t* nout, int mem, void* stream)
{
    LDSP_RANGE("ldsp_iirfilt_resamp_execute");
    return guard([&] {
        NONNULL(q);
        NONNULL(rs);
        LDSP_REQUIRE(q->cplx == rs->cplx, "iirfilt_resamp_execute: the filter and the resampler must both be complex "
                                          "or both real");
        const size_t K = rs->num_outputs(n);
        if (nout) *nout = K;
        if (K > cap) throw Error(LDSP_ERANGE, "iirfilt_resamp_execute: output capacity too small");
        LDSP_REQUIRE(n == 0 || x, "iirfilt_resamp_execute: NULL input");
        LDSP_REQUIRE(K == 0 || y, "iirfilt_resamp_execute: NULL output");
        const BufDevice bd(mem, x);
        q->ensure_device();
        rs->ensure_device();
        LDSP_REQUIRE(q->device == rs->device, "iirfilt_resamp_execute: the filter and the resampler live on different "
                                              "devices");
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        const size_t es = q->cplx ? 8 : 4;
        const bool fuse = n > 0 && q->path_for(n) == IirObj::kModal && rs->sub_len >= 2 &&
                          rs->sub_len - 1 <= 1024u;
        if (!fuse) {
            auto ok = [](int rc) {
                if (rc != LDSP_OK) throw Error(rc, ldsp_last_error());
            };
            if (e.host) {
                // the hand-over in page-locked memory when the pool has it (the two
                // calls then DMA it directly), pageable otherwise; the caller's stream
                const size_t tb = std::max<size_t>(n, 1) * es;
                void* tp = nullptr;
                std::vector<char> tv;
                if (ldsp_host_alloc(tb, &tp) != LDSP_OK) {
                    tp = nullptr;
                    tv.resize(tb);
                }
                struct Free {
                    void* p;
                    ~Free() { if (p) (void)ldsp_host_free(p); }
                } fr{tp};
                void* t = tp ? tp : tv.data();
                ok(ldsp_iirfilt_execute(q, x, n, t, LDSP_MEM_HOST, stream));
                ok(ldsp_resamp_execute(rs, t, n, y, cap, nout, LDSP_MEM_HOST, stream));
            } else {
                void* t = q->rsbuf.ensure(std::max<size_t>(n, 1) * es, q->device);
                ok(ldsp_iirfilt_execute(q, x, n, t, LDSP_MEM_DEVICE, stream));
                ok(ldsp_resamp_execute(rs, t, n, y, cap, nout, LDSP_MEM_DEVICE, stream));
                q->ord.mark(e.stream);            // the next filter call rewrites t only after the resampler read it
            }
            return;
        }
        q->ord.wait(e.stream);
        rs->ord.wait(e.stream);
        const void* dx = q->stg.dev_in(e, x, n * es);
        void* dy = rs->stg.dev_out(e, y, K * es);
        q->state_to(IirObj::kStModal, e.stream);
        const k::IirModalPlan p = q->modal_plan(n);
        k::IirResampFuse f;
        f.sub = rs->dsub.as<float>();
        f.P0 = rs->phase;
        f.step = rs->step;
        f.bits_index = rs->bits_index;
        f.sub_len = (int)rs->sub_len;
        f.ctaps = (rs->cplx && !rs->real_taps) ? 1 : 0;
        f.K = (long)K;
        f.side = (float*)q->rsside.ensure(k::iir_resamp_side_bytes(n, (int)rs->sub_len, q->cplx), q->device);
        f.y = (float*)dy;
        k::iir_modal_resamp(q->cplx, q->mf.cf, dx, n, q->mst.as<double>(), q->mstb.as<double>(), p, f,
                            rs->hist[rs->cur].p, rs->hist[1 - rs->cur].p, e.stream);
        std::swap(q->mst.p, q->mstb.p);
        std::swap(q->mst.cap, q->mstb.cap);
        rs->cur = 1 - rs->cur;
        rs->phase = (uint64_t)((long long)rs->phase + (long long)K * rs->step - (long long)n * (1LL << 24));
        q->ord.mark(e.stream);
        rs->ord.mark(e.stream);
        q->last = e.stream;
        rs->last = e.stream;
        rs->stg.finish(e, y, K * es);
    });
}

// ---------------------------------------------------------------- AGC
int ldsp_agc_create(ldsp_agc_t* q)
{
    return guard([&] {
        NONNULL(q);
        auto* o = new ldsp_agc_s();
        o->init();
        *q = o;
    });
}
int ldsp_agc_destroy(ldsp_agc_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}

// agc_crcf_reset: g = 1, y2' = 1, unlock, squelch ENABLED unless disabled
int ldsp_agc_reset(ldsp_agc_t q)
{
    return guard([&] {
        NONNULL(q);
        q->pull();
        q->h.g = 1.0f;
        q->h.y2p = 1.0f;
        q->h.locked = 0;
        q->h.mode = (q->h.mode == 7) ? 7 : 1;
        q->modified();
    });
}
int ldsp_agc_set_bandwidth(ldsp_agc_t q, float bw)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(bw >= 0.0f && bw <= 1.0f, "agc_set_bandwidth: bandwidth must be in [0, 1]");
        q->pull();
        q->bandwidth = bw;
        q->h.alpha = bw;
        q->modified();
    });
}
int ldsp_agc_get_bandwidth(ldsp_agc_t q, float* bw) { return guard([&] { NONNULL(q); NONNULL(bw); *bw = q->bandwidth; }); }
int ldsp_agc_lock(ldsp_agc_t q, int on)
{
    return guard([&] { NONNULL(q); q->pull(); q->h.locked = on ? 1 : 0; q->modified(); });
}
int ldsp_agc_squelch_enable(ldsp_agc_t q, int on)
{
    return guard([&] { NONNULL(q); q->pull(); q->h.mode = on ? 1 : 7; q->modified(); });
}
int ldsp_agc_squelch_set_threshold(ldsp_agc_t q, float t)
{
    return guard([&] { NONNULL(q); q->pull(); q->h.threshold = t; q->modified(); });
}
int ldsp_agc_squelch_get_threshold(ldsp_agc_t q, float* t)
{
    return guard([&] { NONNULL(q); NONNULL(t); *t = q->h.threshold; });
}
int ldsp_agc_squelch_set_timeout(ldsp_agc_t q, unsigned int t)
{
    return guard([&] { NONNULL(q); q->pull(); q->h.timeout = t; q->modified(); });
}
int ldsp_agc_squelch_get_status(ldsp_agc_t q, int* s)
{
    return guard([&] { NONNULL(q); NONNULL(s); q->pull(); *s = q->h.mode; });
}
int ldsp_agc_get_gain(ldsp_agc_t q, float* g) { return guard([&] { NONNULL(q); NONNULL(g); q->pull(); *g = q->h.g; }); }
int ldsp_agc_set_gain(ldsp_agc_t q, float g)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(g > 0.0f, "agc_set_gain: gain must be greater than zero");
        q->pull();
        q->h.g = g;
        q->modified();
    });
}
int ldsp_agc_get_scale(ldsp_agc_t q, float* s) { return guard([&] { NONNULL(q); NONNULL(s); *s = q->h.scale; }); }
int ldsp_agc_set_scale(ldsp_agc_t q, float s)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(s > 0.0f, "agc_set_scale: scale must be greater than zero");
        q->pull();
        q->h.scale = s;
        q->modified();
    });
}
int ldsp_agc_get_signal_level(ldsp_agc_t q, float* x)
{
    return guard([&] { NONNULL(q); NONNULL(x); q->pull(); *x = (float)(1.0 / (double)q->h.g); });
}
int ldsp_agc_set_signal_level(ldsp_agc_t q, float x)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(x > 0.0f, "agc_set_signal_level: level must be greater than zero");
        q->pull();
        q->h.g = (float)(1.0 / (double)x);
        q->h.y2p = 1.0f;
        q->modified();
    });
}
int ldsp_agc_get_rssi(ldsp_agc_t q, float* r)
{
    return guard([&] { NONNULL(q); NONNULL(r); q->pull(); *r = (float)(-20 * log10((double)q->h.g)); });
}
int ldsp_agc_set_rssi(ldsp_agc_t q, float r)
{
    return guard([&] {
        NONNULL(q);
        q->pull();
        q->h.g = powf(10.0f, -r / 20.0f);
        if (q->h.g < 1e-16f) q->h.g = 1e-16f;
        q->h.y2p = 1.0f;
        q->modified();
    });
}
int ldsp_agc_set_mode(ldsp_agc_t q, int mode)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(mode == LDSP_MODE_FAST || mode == LDSP_MODE_EXACT, "unknown mode");
    });
}

// Two halves per call (k_agc.hip): the front runs the speculative chunks --
// from the input history alone once it holds hist_len samples, so call k + 1's
// front overlaps call k's back half on another stream -- and the back half
// checks chunk 0 against the true state, repairs and verifies, and advances it.
int ldsp_agc_execute(ldsp_agc_t q, const void* x, size_t n, void* y, uint8_t* status, int mem, void* stream)
{
    LDSP_RANGE("ldsp_agc_execute");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "agc_execute: NULL buffer");
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        const int sl = (int)(q->ncall & 1), h3 = (int)(q->ncall % 3);
        q->slot[sl].wait(e.stream);
        q->front.wait(e.stream);
        if (q->upload_pending) {
            q->ord.wait(e.stream);
            LDSP_HIP(hipStreamSynchronize(e.stream));
            LDSP_HIP(hipMemcpy(q->dst.p, &q->h, sizeof(q->h), hipMemcpyHostToDevice));
            q->upload_pending = false;
        }
        const void* dx = q->stg.dev_in(e, x, n * 8);
        void* dy = q->stg.dev_out(e, y, n * 8);
        uint8_t* dstat = status ? (uint8_t*)q->status.ensure(std::max<size_t>(n, 1), q->device) : nullptr;
        // exact warm-up W = 5/bandwidth after an approximate one of Wa = 40/bandwidth
        // (k_agc.hip); measured on the AM chain at bandwidth 0.01 the exact loop then
        // coalesces within ~110 samples on average, 2834 at worst.  The chunks that
        // have not by then (~70 of 1 573 per 64 Mi call at W = 5/bw, 7 at 20/bw) go
        // to the windowed one-wave run-fix, which stops at the first checkpoint that
        // meets the stored trajectory: single call 3.72 -> 3.42 ms against W = 20/bw
        // (W = 3/bw: 3.71, more runs), 20-step and batched channels unchanged
        // (gpurun_out r05zo).
        const float a = q->h.alpha > 1e-6f ? q->h.alpha : 1e-6f;
        static const float wmul = LDSP_KNOB_F("LDSP_AGC_WMUL", 5.0f);
        static const float wamul = LDSP_KNOB_F("LDSP_AGC_WAMUL", 40.0f);
        // repair rounds (flag + run-by-run re-run launches) before the one-wave
        // verifier, which re-runs whatever a round left: on the bench chain every
        // repair lands in round 1 (rounds 2-3 found nothing), and with 8 channels
        // per GPU each launch on a chain waits 0.1-0.2 ms for a slot, so one round
        // (8 channels 5.62-5.78 vs 5.83-6.24 ms per step, profiles/r04v_channels.txt)
        static const int rounds = LDSP_KNOB("LDSP_AGC_ROUNDS", 1);
        static const bool nospec = LDSP_KNOB("LDSP_AGC_NOSPEC", 0) != 0;   // A/B: every call from the true state
        const int W = (int)std::min(1 << 18, std::max(256, (int)(wmul / a)));
        const int Wa = (int)std::min(1 << 20, std::max(1024, (int)(wamul / a)));
        const long hl = (long)W + Wa + k::kAgcPow;
        if (hl != q->hist_len) {             // bandwidth changed: history restarts
            q->hist_len = hl;
            q->hist_valid = 0;
            for (int i = 0; i < 3; i++) q->hist[i].ensure((size_t)hl * 8, q->device);
        }
        // Latency per step on one lane (scripts/ubench/loop_lat.hip): approximate
        // 0.06 us, exact 0.25 us.  Chunk-parallel from guesses (every chunk Wa
        // approximate + W + 256 exact steps, ~0.8 us at bandwidth 0.01, overlapping
        // the previous call) once a call is long enough that the true-start chunks
        // below would take more than half of that.
        static const size_t parmin = (size_t)LDSP_KNOB("LDSP_AGC_PARMIN", 0L);
        const bool par = n >= (parmin ? parmin : std::max<size_t>(2048, (size_t)(0.5 * (0.06 * Wa + 0.25 * (W + 256)) / 0.06)));
        // below that, from ~300 samples: chunks approximating from the true state
        // (latency 0.06 us per sample before the last chunk + 256 exact steps)
        static const size_t tsamin = (size_t)LDSP_KNOB("LDSP_AGC_TSAMIN", 320L);
        const bool tsa = !par && n >= tsamin;
        const bool spec = !nospec && !tsa && q->hist_valid >= hl;
        k::SpecPlan p;
        if (n > 0 && (par || tsa)) {
            p.W = tsa ? 0 : W;                 // tsa: every chunk from 1 on is checked against its predecessor
            p.Wa = Wa;
            p.rounds = tsa ? 1 : std::max(0, std::min(q->rounds_force >= 0 ? q->rounds_force : rounds, 6));
            // (tsa: one run covers the rare deviation)
            // chunk length: every chunk re-runs Wa + W warm-up steps (6 000 at
            // bandwidth 0.01) for its C outputs, so C = 1024 does a quarter of the
            // front's work of C = 256 at ~20 % more latency (hidden under the PLL
            // walk in a streamed chain); measured on 8 channels per GPU 6.6 -> 6.3
            // ms per step (scripts/agc_chunk_sweep.sh).  Small calls (tsa): the
            // one wave runs the approximate loop up to the last chunk's start and
            // then C exact steps, so the shortest chunks that still fit 64 lanes
            // (C >= 32) cut the exact tail: a README call (1 573 samples) 256 -> 32
            // exact steps after the same approximate run.  Multi-wave tsa calls keep 256.
            static const int agc_c = LDSP_KNOB("LDSP_AGC_C", 1024);
            static const int tsa_cmin = LDSP_KNOB("LDSP_AGC_TSA_CMIN", 32);
            const int c64 = (int)(((n + 63) / 64 + 31) / 32 * 32);      // 64 chunks of a multiple of 32
            p.C = tsa ? (c64 <= 256 ? std::max(tsa_cmin, c64) : 256) : agc_c;
            p.nchunks = (long)((n + p.C - 1) / p.C);
            p.scratch = q->scr[sl].ensure(k::agc_scratch_bytes(p.nchunks, p.C), q->device);
            p.hist = q->hist[h3].p;
            p.H = spec ? (int)hl : 0;
            // a small call's chunks in one wave check and repair themselves (tsa 2:
            // no flag / repair / verify launches on the call's critical path)
            static const bool tsa_sep = LDSP_KNOB("LDSP_AGC_TSA_SEPARATE", 0) != 0;
            p.tsa = tsa ? (p.nchunks <= 64 && !tsa_sep && !LDSP_KNOB("LDSP_DEBUG_AGC", 0) ? 2 : 1) : 0;
            if (p.tsa == 2 && q->tsa_perturb) p.tsa |= 4;
            if (!tsa && q->perturb) p.tsa |= 8;          // test hook: odd chunks start 1 ulp off
        }
        // the next call's history first: its front then waits for this copy only
        if (n > 0) k::delay_hist(dx, q->hist[h3].p, q->hist[(h3 + 1) % 3].p, n, (int)hl, e.stream);
        q->front.mark(e.stream);
        static const bool dbg = LDSP_KNOB("LDSP_DEBUG_AGC", 0) != 0;    // per-round re-run counters
        if (n > 0 && (par || tsa)) {
            if (dbg) {
                p.dbg = (unsigned*)p.scratch + (size_t)p.nchunks * 8;
                LDSP_HIP(hipMemsetAsync(p.dbg, 0, 8 * sizeof(unsigned), e.stream));
            }
            if (!spec) q->ord.wait(e.stream);         // chunks near the start read the true state
            k::agc_spec_front(dx, n, q->dst.as<k::AgcState>(), p, dy, dstat, e.stream);
            // speculative call: the repair rounds need no true state (off the chain between calls)
            if (spec) k::agc_spec_repair(dx, n, q->dst.as<k::AgcState>(), p, dy, dstat, e.stream);
        }
        q->ord.wait(e.stream);
        if (n > 0) {
            if (par || tsa) {
                if (spec) k::agc_spec_verify(dx, n, q->dst.as<k::AgcState>(), p, dy, dstat, e.stream);
                else if (!(p.tsa & 2)) k::agc_spec_back(dx, n, q->dst.as<k::AgcState>(), p, dy, dstat, e.stream);
                if (dbg) {
                    unsigned c[8];
                    LDSP_HIP(hipMemcpyAsync(c, p.dbg, sizeof(c), hipMemcpyDeviceToHost, e.stream));
                    LDSP_HIP(hipStreamSynchronize(e.stream));
                    std::fprintf(stderr, "[ldsp agc] n=%zu chunks=%ld W=%d Wa=%d spec=%d rounds=%d reruns per round:", n,
                                 p.nchunks, p.W, p.Wa, spec ? 1 : 0, p.rounds);
                    for (int r = 0; r <= p.rounds; r++) std::fprintf(stderr, " %u", c[r]);
                    std::fprintf(stderr, " (last = verifier)\n");
                }
            } else {
                k::agc_seq(dx, n, q->dst.as<k::AgcState>(), dy, dstat, e.stream);
            }
            q->dev_newer = true;
            q->hist_valid = std::min<long>(hl, q->hist_valid + (long)n);
        }
        q->ord.mark(e.stream);
        q->slot[sl].mark(e.stream);
        q->ncall++;
        q->last = e.stream;
        if (status && n > 0) {
            LDSP_HIP(hipMemcpyAsync(status, dstat, n, hipMemcpyDeviceToHost, e.stream));
            LDSP_HIP(hipStreamSynchronize(e.stream));
        }
        q->stg.finish(e, y, n * 8);
    });
}

// ---------------------------------------------------------------- AmpModem
int ldsp_ampmodem_create(float mod_index, int type, int suppressed_carrier, ldsp_ampmodem_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(type >= 0 && type <= 2, "ampmodem: type must be 0 (dsb), 1 (usb) or 2 (lsb)");
        std::unique_ptr<ldsp_ampmodem_s> o(new ldsp_ampmodem_s());
        o->mod_index = mod_index;
        o->type = type;
        o->suppressed = suppressed_carrier != 0;
        o->m = 25;
        o->lp = design::firdes_kaiser(2 * o->m + 1, 0.01f, 40.0f, 0.0f);   // carrier lowpass
        o->dc = design::firdes_notch(o->m, 0.0f, 20.0f);                     // DC blocker
        if (type != 0) o->hq = design::firhilb_taps(o->m, 60.0f);            // firhilbf_create(m, 60)
        o->table = nco_table();
        o->reset_host();
        *q = o.release();
    });
}
int ldsp_ampmodem_destroy(ldsp_ampmodem_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}
static void amp_reset(AmpObj* q)
{
    q->reset_host();
    q->dev_newer = false;
    if (q->device < 0) return;
    DeviceGuard g(q->device);
    q->sync_all();
    q->st.wepoch = q->wexp;               // every issued launch has published: the epoch stands
    q->st.werr = 0;
    if (q->herr) __atomic_store_n(q->herr, 0u, __ATOMIC_RELEASE);
    LDSP_HIP(hipMemcpy(q->dst.p, &q->st, sizeof(q->st), hipMemcpyHostToDevice));
    for (int i = 0; i < 2; i++) {
        for (DevBuf* b : {&q->lph[i], &q->dch[i]})
            if (b->p) zero_now(b->p, 0, b->cap);
    }
    for (auto& b : q->dlh)
        if (b.p) zero_now(b.p, 0, b.cap);
    for (auto& b : q->hbh)
        if (b.p) zero_now(b.p, 0, b.cap);
    q->hcur = 0;
}
int ldsp_ampmodem_reset(ldsp_ampmodem_t q)
{
    return guard([&] {
        NONNULL(q);
        amp_reset(q);
    });
}
int ldsp_ampmodem_get_taps(ldsp_ampmodem_t q, float* lowpass, float* dcblock, float* hilbert)
{
    return guard([&] {
        NONNULL(q);
        if (lowpass) std::copy(q->lp.begin(), q->lp.end(), lowpass);
        if (dcblock) std::copy(q->dc.begin(), q->dc.end(), dcblock);
        if (hilbert) {
            const std::vector<float> hq = q->hq.empty() ? design::firhilb_taps(q->m, 60.0f) : q->hq;
            std::copy(hq.begin(), hq.end(), hilbert);
        }
    });
}
// A walker whose wait for the previous call's state timed out has walked from a
// stale state: its call's output is invalid.  Raised at every entry point of the
// object (and after the host path's synchronisation) until ldsp_ampmodem_reset.
static void amp_check_err(const AmpObj* q)
{
    const bool dev_flag = q->herr && __atomic_load_n(q->herr, __ATOMIC_ACQUIRE) != 0;
    if (q->st.werr || dev_flag)
        throw Error(LDSP_EHIP, "ampmodem: a PLL walker's wait for the previous call's state timed out; "
                               "the output of that call is not valid (reset the object)");
}
int ldsp_ampmodem_get_pll_state(ldsp_ampmodem_t q, uint32_t* t, uint32_t* d)
{
    return guard([&] {
        NONNULL(q);
        if (q->dev_newer) {
            DeviceGuard g(q->device);
            q->sync_all();
            LDSP_HIP(hipMemcpy(&q->st, q->dst.p, sizeof(q->st), hipMemcpyDeviceToHost));
            q->dev_newer = false;
            amp_check_err(q);
        }
        if (t) *t = q->st.theta;
        if (d) *d = q->st.dtheta;
    });
}

int ldsp_debug_walk_early(int on)
{
    return g_walk_early.exchange(on < 0 ? -1 : (on != 0));
}

int ldsp_debug_iir_sect_trace(void* dev_buf)
{
    return k::iir_sect_trace(dev_buf);
}

int ldsp_debug_pll_margin(int log2_b)
{
    return k::pll_margin_override(log2_b);
}

int ldsp_ampmodem_walk_stats(ldsp_ampmodem_t q, uint64_t* entries, uint64_t* repairs, uint64_t* fallbacks)
{
    return guard([&] {
        NONNULL(q);
        unsigned long long stt[5] = {0, 0, 0, 0, 0};
        if (q->last_stats) {
            DeviceGuard g(q->device);
            q->sync_all();
            LDSP_HIP(hipMemcpy(stt, q->last_stats, sizeof(stt), hipMemcpyDeviceToHost));
        }
        if (entries) *entries = stt[4];
        if (repairs) *repairs = stt[0];
        if (fallbacks) *fallbacks = stt[1];
    });
}

int ldsp_ampmodem_walk_active(ldsp_ampmodem_t q, uint64_t* ticks, uint64_t* count)
{
    return guard([&] {
        NONNULL(q);
        k::AmpState st{};
        if (q->dst.p) {
            DeviceGuard g(q->device);
            q->sync_all();
            LDSP_HIP(hipMemcpy(&st, q->dst.p, sizeof(st), hipMemcpyDeviceToHost));
            q->st.werr = st.werr;
            amp_check_err(q);
        }
        if (ticks) *ticks = st.wact;
        if (count) *count = st.wact_n;
    });
}
int ldsp_ampmodem_walk_clocks(ldsp_ampmodem_t q, uint64_t* walk, uint64_t* wait)
{
    return guard([&] {
        NONNULL(q);
        unsigned long long stt[4] = {0, 0, 0, 0};
        if (q->last_stats) {
            DeviceGuard g(q->device);
            q->sync_all();
            LDSP_HIP(hipMemcpy(stt, q->last_stats, sizeof(stt), hipMemcpyDeviceToHost));
        }
        if (walk) *walk = stt[2];
        if (wait) *wait = stt[3];
    });
}

int ldsp_ampmodem_seq_stats(ldsp_ampmodem_t q, uint64_t* batches, uint64_t* redone)
{
    return guard([&] {
        NONNULL(q);
        k::AmpState st{};
        if (q->dst.p) {
            DeviceGuard g(q->device);
            q->sync_all();
            LDSP_HIP(hipMemcpy(&st, q->dst.p, sizeof(st), hipMemcpyDeviceToHost));
        }
        if (batches) *batches = st.sq_batches;
        if (redone) *redone = st.sq_redone;
    });
}

// Carrier lowpass + delay + PLL walk of AmpModem / BroadcastAM: writes
// re(v1) / mod_index (costas 0) or the Costas-loop output (costas 1) to mbuf
// (slot scratch when mbuf is null).  Returns the buffer written.  The caller
// enqueues its post-filter and then amp_call_end().  Stream order (see AmpObj):
//   wait slot[s] (call k-2 done with slot s) and front (call k-1's histories and guess)
//   lowpass, delay history, candidates            -> mark front
//   wait ord (call k-1's walk; ord is marked before its DC blocker) -> walker
// Costas: the candidates start from the true state (the loop's two stable
// points half a turn apart make a guess ambiguous), so its front also waits for
// call k-1's walk.
// Calls above kAmpPieceMax samples run as consecutive sub-calls of at most that
// many (same bits: every stage streams its state across calls): the walker stores
// repaired outputs through 32-bit byte offsets (k_pll.hip), so one launch covers < 2^30.
static constexpr size_t kAmpPieceMax = size_t(1) << 29;

static float* amp_pll_stage(AmpObj* q, const Exec& e, const void* dx, size_t n, float mod_index, int costas, float* mbuf,
                            int out_idx = 0)
{
    const int L = 2 * (int)q->m + 1;
    const int sl = (int)(q->ncall & 1);
    const int h3 = (int)(q->ncall % 3);
    q->slot[sl].wait(e.stream);
    q->front.wait(e.stream);
    if (costas) q->ord.wait(e.stream);
    if (!mbuf) mbuf = (float*)q->mb[sl].ensure(n * 4, q->device);
    void* x0 = q->x0[sl].ensure(n * 8, q->device);
    k::fir_exact(true, dx, q->lph[q->cur].p, q->lph[1 - q->cur].p, n, q->dlp.as<float>(), L, 1.0f, x0, e.stream);
    k::PllCall c;
    c.x0 = x0;
    c.x = dx;
    c.hist = q->dlh[h3].p;
    c.hist_out = q->dlh[(h3 + 1) % 3].p;
    c.m = (int)q->m;
    c.n = n;
    c.st = q->dst.as<k::AmpState>();
    c.gcur = (int)(q->ncall & 1);
    c.table = q->dtab.as<float>();
    c.mod_index = mod_index;
    c.costas = costas;
    c.out_idx = out_idx;
    c.alpha_host = q->st.alpha;
    c.y = mbuf;
    c.scratch = k::pll_parallel(n, costas) ? q->pll[sl].ensure(k::pll_scratch_bytes(n), q->device) : nullptr;
    c.wexp = q->wexp;
    q->last_stats = c.scratch ? (const char*)c.scratch + k::pll_stats_offset(n) : nullptr;
    k::pll_front(c, e.stream);
    const bool par = k::pll_parallel(n, costas);
    if (par) q->front.mark(e.stream);     // the sequential loop writes the guess itself: mark after it
    // (A dedicated high-priority walker queue was measured: the ~25 us between
    // walks stayed -- it is the dispatcher waiting for a whole CU to drain for the
    // walker's 135 KiB of LDS, not the cross-queue event -- and the chain slowed.)
    // Early hand-off: the carrier walker does not wait for the previous call's
    // walk on the stream; it is dispatched as soon as its candidates are ready and
    // waits on the device for the state's epoch (k_pll_walk_body), so the CU it
    // needs is taken while the previous walk still runs.  The sequential loops and
    // Costas keep the stream order.
    static const bool early_knob = LDSP_KNOB("LDSP_WALK_EARLY", 1) != 0;
    const int ov = g_walk_early.load(std::memory_order_relaxed);
    const bool early_on = ov < 0 ? early_knob : ov != 0;
    // (calls up to 2^26 samples, after one of at most that: the previous walk then
    // takes < 0.1 s, far inside the walker's 1 s bound on its wait)
    const bool early = early_on && par && !costas && q->live.early_ok() &&
                       n <= (size_t(1) << 26) && q->last_pll_n <= (size_t(1) << 26);
    if (!early) q->ord.wait(e.stream);
    k::pll_back(c, e.stream);
    if (n > 0) {
        q->wexp++;
        q->last_pll_n = n;
    }
    q->ord.mark(e.stream);                // the true PLL state: the next call's walk may start
    if (!par) q->front.mark(e.stream);
    static const bool dbg_pll = LDSP_KNOB("LDSP_DEBUG_PLL", 0) != 0;
    if (par && dbg_pll) {
        unsigned long long stt[7];
        LDSP_HIP(hipMemcpyAsync(stt, (char*)c.scratch + k::pll_stats_offset(n), sizeof(stt), hipMemcpyDeviceToHost,
                                e.stream));
        LDSP_HIP(hipStreamSynchronize(e.stream));
        std::fprintf(stderr, "[ldsp pll] n=%zu entries=%llu repairs=%llu fallback_lane_blocks=%llu walk_clk=%llu "
                     "wait_clk=%llu lane_blocks_repaired=%llu first_pass_set_final=%llu\n", n, stt[4], stt[0], stt[1],
                     stt[2], stt[3], stt[5], stt[6]);
    }
    return mbuf;
}

static void amp_call_end(AmpObj* q, const Exec& e)
{
    q->slot[q->ncall & 1].mark(e.stream);
    q->ncall++;
    q->cur = 1 - q->cur;
    q->dev_newer = true;
}

// usb / lsb (liquid ampmodem_demod_ssb_pll_carrier / ampmodem_demod_ssb, see
// oracle/liquid_restate.c).  Carrier: the DSB carrier PLL stage writes each
// sample's table index, k_ssb_v1 recomputes v1 = delay(x) mixed down by it, the
// Hilbert c2r keeps the sideband (0.5 * . / mod_index) and the DC blocker
// follows.  Suppressed carrier: the Hilbert c2r of x alone.  The Hilbert history
// is ordered across streams by `post` (like the DC blocker's).
static void amp_ssb(AmpObj* q, const Exec& e, const void* dx, size_t n, float* dy)
{
    const int M = (int)q->m, H = 4 * M - 1, usb = q->type == 1 ? 1 : 0;
    if (q->suppressed) {
        q->post.wait(e.stream);
        k::ssb_c2r(dx, q->hbh[q->hcur].p, n, q->dhq.as<float>(), M, usb, q->mod_index, dy, e.stream);
        k::delay_hist(dx, q->hbh[q->hcur].p, q->hbh[1 - q->hcur].p, n, H, e.stream);
        q->post.mark(e.stream);
        q->hcur = 1 - q->hcur;
        return;
    }
    const int L = 2 * M + 1;
    const int sl = (int)(q->ncall & 1);
    const void* dhist = q->dlh[q->ncall % 3].p;           // this call's delay-line history (read by the PLL stage too)
    float* mbuf = amp_pll_stage(q, e, dx, n, q->mod_index, 0, nullptr, 1);
    void* v1 = q->v1[sl].ensure(n * 8, q->device);
    q->post.wait(e.stream);
    k::ssb_v1(mbuf, dx, dhist, M, q->dtab.as<float>(), n, v1, e.stream);
    k::ssb_c2r(v1, q->hbh[q->hcur].p, n, q->dhq.as<float>(), M, usb, q->mod_index, mbuf, e.stream);
    k::delay_hist(v1, q->hbh[q->hcur].p, q->hbh[1 - q->hcur].p, n, H, e.stream);
    k::fir_exact(false, mbuf, q->dch[q->cur].p, q->dch[1 - q->cur].p, n, q->ddc.as<float>(), L, 1.0f, dy, e.stream);
    q->post.mark(e.stream);
    q->hcur = 1 - q->hcur;
    amp_call_end(q, e);
}

int ldsp_ampmodem_demodulate(ldsp_ampmodem_t q, const void* x, size_t n, void* y, int mem, void* stream)
{
    LDSP_RANGE("ldsp_ampmodem_demodulate");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "ampmodem_demodulate: NULL buffer");
        if (n > kAmpPieceMax) {              // the walker's 32-bit store offsets: consecutive sub-calls
            for (size_t off = 0; off < n; off += kAmpPieceMax) {
                const int rc = ldsp_ampmodem_demodulate(q, (const char*)x + off * 8, std::min(kAmpPieceMax, n - off),
                                                        (char*)y + off * 4, mem, stream);
                if (rc != LDSP_OK) throw Error(rc, g_last_error);
            }
            return;
        }
        amp_check_err(q);
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        const void* dx = q->stg.dev_in(e, x, n * 8);
        float* dy = (float*)q->stg.dev_out(e, y, n * 4);
        if (n > 0 && q->type != 0) {
            amp_ssb(q, e, dx, n, dy);
        } else if (n > 0) {
            const int L = 2 * (int)q->m + 1;
            float* mbuf = amp_pll_stage(q, e, dx, n, q->mod_index, q->suppressed ? 1 : 0, q->suppressed ? dy : nullptr);
            if (!q->suppressed) {
                // the DC blocker is off the walker's chain: the next call's walk
                // waits for this walk only (ord), the next DC blocker for this one
                q->post.wait(e.stream);
                k::fir_exact(false, mbuf, q->dch[q->cur].p, q->dch[1 - q->cur].p, n, q->ddc.as<float>(), L, 1.0f,
                             dy, e.stream);
                q->post.mark(e.stream);
            }
            amp_call_end(q, e);
        }
        q->last = e.stream;
        q->stg.finish(e, y, n * 4);
        if (e.host) amp_check_err(q);         // synchronised: this call's own walk is done
    });
}

int ldsp_debug_ampmodem_handoff(ldsp_ampmodem_t q, uint64_t wait_ticks, int epoch_skew)
{
    return guard([&] {
        NONNULL(q);
        q->ensure_device();
        DeviceGuard g(q->device);
        q->sync_all();
        q->st.wait_ticks = wait_ticks ? (unsigned long long)wait_ticks : kWalkWaitTicks;
        LDSP_HIP(hipMemcpy((char*)q->dst.p + offsetof(k::AmpState, wait_ticks), &q->st.wait_ticks,
                           sizeof(q->st.wait_ticks), hipMemcpyHostToDevice));
        q->wexp += (uint32_t)epoch_skew;
    });
}

// ---------------------------------------------------------------- BroadcastAM
int ldsp_bcastam_create(unsigned int m, ldsp_bcastam_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(m >= 1 && m <= 4096, "bcastam: m must be in [1, 4096]");
        std::unique_ptr<ldsp_bcastam_s> o(new ldsp_bcastam_s());
        o->mod_index = 1.0f;
        o->type = 0;
        o->suppressed = 0;
        o->m = m;
        o->lp = design::firdes_kaiser(2 * m + 1, 0.01f, 40.0f, 0.0f);
        o->table = nco_table();
        o->reset_host();
        // cheby2 highpass, SOS, order 3, fc 20/48000, f0 0, Ap 0.5, As 20 (demod.hpp:104)
        int rc = ldsp_iirfilt_create_prototype(2, 1, 3, 20.0f / 48000.0f, 0.0f, 0.5f, 20.0f, 0, &o->dcb);
        if (rc != LDSP_OK) throw Error(rc, g_last_error);
        *q = o.release();
    });
}
int ldsp_bcastam_destroy(ldsp_bcastam_t q)
{
    return guard([&] {
        if (!q) return;
        if (q->last) (void)hipStreamSynchronize(q->last);
        ldsp_iirfilt_destroy(q->dcb);
        delete q;
    });
}
int ldsp_bcastam_reset(ldsp_bcastam_t q)
{
    return guard([&] {
        NONNULL(q);
        amp_reset(q);
        const int rc = ldsp_iirfilt_reset(q->dcb);
        if (rc != LDSP_OK) throw Error(rc, g_last_error);
    });
}
int ldsp_bcastam_set_mode(ldsp_bcastam_t q, int mode)
{
    return guard([&] {
        NONNULL(q);
        const int rc = ldsp_iirfilt_set_mode(q->dcb, mode);
        if (rc != LDSP_OK) throw Error(rc, g_last_error);
    });
}
int ldsp_bcastam_get_mode(ldsp_bcastam_t q, int* mode)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(mode);
        *mode = q->dcb->mode;
    });
}
int ldsp_bcastam_demodulate(ldsp_bcastam_t q, const void* x, size_t n, void* y, void* pre, int mem, void* stream)
{
    LDSP_RANGE("ldsp_bcastam_demodulate");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "bcastam_demodulate: NULL buffer");
        if (n > kAmpPieceMax) {              // as ldsp_ampmodem_demodulate
            for (size_t off = 0; off < n; off += kAmpPieceMax) {
                const size_t m = std::min(kAmpPieceMax, n - off);
                const int rc = ldsp_bcastam_demodulate(q, (const char*)x + off * 8, m, (char*)y + off * 4,
                                                       pre ? (char*)pre + off * 4 : nullptr, mem, stream);
                if (rc != LDSP_OK) throw Error(rc, g_last_error);
            }
            return;
        }
        amp_check_err(q);
        const BufDevice bd(mem, x);
        q->ensure_device();
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        const void* dx = q->stg.dev_in(e, x, n * 8);
        float* dy = (float*)q->stg.dev_out(e, y, n * 4);
        if (n > 0) {
            float* mbuf = amp_pll_stage(q, e, dx, n, 1.0f, 0, nullptr);
            const int rc = ldsp_iirfilt_execute(q->dcb, mbuf, n, dy, LDSP_MEM_DEVICE, e.stream);
            if (rc != LDSP_OK) throw Error(rc, g_last_error);
            if (pre) {
                LDSP_HIP(hipMemcpyAsync(pre, mbuf, n * 4, e.host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice,
                                        e.stream));
            }
            amp_call_end(q, e);
        }
        q->last = e.stream;
        q->stg.finish(e, y, n * 4);
        if (e.host) amp_check_err(q);
    });
}

// ---------------------------------------------------------------- FreqDem
int ldsp_freqdem_create(float kf, ldsp_freqdem_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(kf > 0.0f, "freqdem: kf must be > 0");
        std::unique_ptr<ldsp_freqdem_s> o(new ldsp_freqdem_s());
        o->kf = kf;
        o->ref = (float)(1.0 / (2 * M_PI * (double)kf));   // freqdem.c: 1/(2*M_PI*kf) in double, stored float
        *q = o.release();
    });
}
int ldsp_freqdem_destroy(ldsp_freqdem_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}
int ldsp_freqdem_reset(ldsp_freqdem_t q)
{
    return guard([&] {
        NONNULL(q);
        if (q->device < 0) return;
        DeviceGuard g(q->device);
        if (q->last) LDSP_HIP(hipStreamSynchronize(q->last));
        for (int i = 0; i < 2; i++) zero_now(q->prev[i].p, 0, 8);
    });
}
int ldsp_freqdem_get_kf(ldsp_freqdem_t q, float* kf)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(kf);
        *kf = q->kf;
    });
}
int ldsp_freqdem_demodulate(ldsp_freqdem_t q, const void* x, size_t n, void* y, int mem, void* stream)
{
    LDSP_RANGE("ldsp_freqdem_demodulate");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "freqdem_demodulate: NULL buffer");
        const BufDevice bd(mem, x);
        if (q->device < 0) {
            const int dev = current_device();
            for (int i = 0; i < 2; i++) zero_now(q->prev[i].ensure(8, dev), 0, 8);
            q->device = dev;
        }
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const void* dx = q->stg.dev_in(e, x, n * 8);
        float* dy = (float*)q->stg.dev_out(e, y, n * 4);
        if (n > 0) {
            k::freqdem(dx, q->prev[q->cur].p, q->prev[1 - q->cur].p, n, q->ref, dy, e.stream);
            q->cur = 1 - q->cur;
        }
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, n * 4);
    });
}

// ---------------------------------------------------------------- Delay
int ldsp_delay_create(unsigned int nd, ldsp_delay_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(nd <= (1u << 26), "delay: nd too large");
        std::unique_ptr<ldsp_delay_s> o(new ldsp_delay_s());
        o->nd = nd;
        *q = o.release();
    });
}
int ldsp_delay_destroy(ldsp_delay_t q)
{
    return guard([&] {
        if (q && q->last) (void)hipStreamSynchronize(q->last);
        delete q;
    });
}
int ldsp_delay_set_delay(ldsp_delay_t q, unsigned int nd)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(nd <= (1u << 26), "delay: nd too large");
        q->nd = nd;
        if (q->device < 0) return;
        DeviceGuard g(q->device);
        if (q->last) LDSP_HIP(hipStreamSynchronize(q->last));
        q->zero();
    });
}
int ldsp_delay_get_delay(ldsp_delay_t q, unsigned int* nd)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(nd);
        *nd = q->nd;
    });
}
int ldsp_delay_execute(ldsp_delay_t q, const void* x, size_t n, int cplx, void* y, int mem, void* stream)
{
    LDSP_RANGE("ldsp_delay_execute");
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(n == 0 || (x && y), "delay_execute: NULL buffer");
        const BufDevice bd(mem, x);
        if (q->device < 0) {
            q->device = current_device();
            DeviceGuard g(q->device);
            q->zero();
        }
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const size_t es = cplx ? 8 : 4;
        const void* dx = q->stg.dev_in(e, x, n * es);
        void* dy = q->stg.dev_out(e, y, n * es);
        if (n > 0) {
            const int D = (int)q->nd + 1;
            int& c = cplx ? q->cc : q->cr;
            ldsp::DevBuf* h = cplx ? q->hc : q->hr;
            k::delay(cplx != 0, dx, h[c].p, h[1 - c].p, n, D, dy, e.stream);
            c = 1 - c;
        }
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, n * es);
    });
}

// ---------------------------------------------------------------- FMStereo
int ldsp_fmstereo_create(float iq_rate, float pcm_rate, ldsp_fmstereo_t* q)
{
    return guard([&] {
        NONNULL(q);
        LDSP_REQUIRE(iq_rate > 0.0f && pcm_rate > 0.0f, "fmstereo: rates must be > 0");
        const float rate = pcm_rate / iq_rate;
        if (rate > 1.0f)
            throw Error(LDSP_EUNSUP, "fmstereo: pcm_rate > iq_rate (the reference drops the samples of inputs that "
                                     "produce two outputs, demod.hpp:45-47; not reproduced)");
        std::unique_ptr<ldsp_fmstereo_s> o(new ldsp_fmstereo_s());
        o->iq_rate = iq_rate;
        o->pcm_rate = pcm_rate;
        // demod.hpp:19-31: 75 us de-emphasis (double arithmetic stored as float)
        float a[2], b[1];
        a[0] = 1.0;
        a[1] = -exp(-1.0 / (75.0E-6 * iq_rate));
        b[0] = 1.0 + a[1];
        auto ok = [](int rc) {
            if (rc != LDSP_OK) throw Error(rc, g_last_error);
        };
        ok(ldsp_freqdem_create(4.0f, &o->dem));
        for (int c = 0; c < 2; c++) {
            ok(ldsp_iirfilt_create_tf(b, 1, a, 2, 0, &o->emph[c]));
            ok(ldsp_iirfilt_set_mode(o->emph[c], LDSP_MODE_EXACT));
            ok(ldsp_resamp_create_default(rate, 0, &o->aud[c]));
        }
        o->table = nco_table();
        o->st.theta = 0;
        o->st.dtheta = 0;
        o->st.pe = 0.0f;           // uninitialised member in the reference (demod.hpp:13)
        o->st.alpha = 0.1f;        // nco_crcf_create: PLL bandwidth 0.1
        o->st.beta = sqrtf(0.1f);
        *q = o.release();
    });
}
int ldsp_fmstereo_destroy(ldsp_fmstereo_t q)
{
    return guard([&] {
        if (!q) return;
        if (q->last) (void)hipStreamSynchronize(q->last);
        ldsp_freqdem_destroy(q->dem);
        for (int c = 0; c < 2; c++) {
            ldsp_iirfilt_destroy(q->emph[c]);
            ldsp_resamp_destroy(q->aud[c]);
        }
        delete q;
    });
}
int ldsp_fmstereo_reset(ldsp_fmstereo_t q)
{
    return guard([&] {
        NONNULL(q);
        for (int c = 0; c < 2; c++) {   // demod.hpp:34-37: only the resamplers
            const int rc = ldsp_resamp_reset(q->aud[c]);
            if (rc != LDSP_OK) throw Error(rc, g_last_error);
        }
    });
}
int ldsp_fmstereo_num_outputs(ldsp_fmstereo_t q, size_t n, size_t* nout)
{
    return guard([&] {
        NONNULL(q);
        NONNULL(nout);
        size_t k = 0;
        const int rc = ldsp_resamp_num_outputs(q->aud[0], n, &k);
        if (rc != LDSP_OK) throw Error(rc, g_last_error);
        *nout = 2 * k;
    });
}
int ldsp_fmstereo_get_state(ldsp_fmstereo_t q, uint32_t* theta, uint32_t* dtheta, float* pe)
{
    return guard([&] {
        NONNULL(q);
        if (q->device >= 0) {
            DeviceGuard g(q->device);
            if (q->last) LDSP_HIP(hipStreamSynchronize(q->last));
            LDSP_HIP(hipMemcpy(&q->st, q->dst.p, sizeof(q->st), hipMemcpyDeviceToHost));
        }
        if (theta) *theta = q->st.theta;
        if (dtheta) *dtheta = q->st.dtheta;
        if (pe) *pe = q->st.pe;
    });
}
int ldsp_fmstereo_execute(ldsp_fmstereo_t q, const void* x, size_t n, void* y, size_t cap, size_t* nout, int mem,
                          void* stream)
{
    LDSP_RANGE("ldsp_fmstereo_execute");
    return guard([&] {
        NONNULL(q);
        size_t k = 0;
        int rc = ldsp_resamp_num_outputs(q->aud[0], n, &k);
        if (rc != LDSP_OK) throw Error(rc, g_last_error);
        if (nout) *nout = 2 * k;
        if (2 * k > cap) throw Error(LDSP_ERANGE, "fmstereo_execute: output capacity too small");
        LDSP_REQUIRE(n == 0 || x, "fmstereo_execute: NULL input");
        LDSP_REQUIRE(k == 0 || y, "fmstereo_execute: NULL output");
        const BufDevice bd(mem, x);
        if (q->device < 0) {
            const int dev = current_device();
            q->dst.ensure(sizeof(k::FmState), dev);
            LDSP_HIP(hipMemcpy(q->dst.p, &q->st, sizeof(q->st), hipMemcpyHostToDevice));
            upload(q->dtab, q->table, dev);
            q->device = dev;
        }
        DeviceGuard g(q->device);
        const Exec e = make_exec(q->device, mem, stream, bd);
        q->ord.wait(e.stream);
        const void* dx = q->stg.dev_in(e, x, n * 8);
        float* dy = (float*)q->stg.dev_out(e, y, 2 * k * 4);
        if (n > 0) {
            auto ok = [](int r) {
                if (r != LDSP_OK) throw Error(r, g_last_error);
            };
            float* sd = (float*)q->sbuf.ensure(n * 4, q->device);
            ok(ldsp_freqdem_demodulate(q->dem, dx, n, sd, LDSP_MEM_DEVICE, e.stream));
            float* l = (float*)q->lr[0].ensure(n * 4, q->device);
            float* r = (float*)q->lr[1].ensure(n * 4, q->device);
            k::fm_pll(sd, n, q->dst.as<k::FmState>(), q->dtab.as<float>(), l, r, e.stream);
            float* outs[2];
            for (int c = 0; c < 2; c++) {
                float* de = (float*)q->le[c].ensure(n * 4, q->device);
                ok(ldsp_iirfilt_execute(q->emph[c], c ? r : l, n, de, LDSP_MEM_DEVICE, e.stream));
                outs[c] = (float*)q->out[c].ensure(std::max<size_t>(k, 1) * 4, q->device);
                size_t kc = 0;
                ok(ldsp_resamp_execute(q->aud[c], de, n, outs[c], k, &kc, LDSP_MEM_DEVICE, e.stream));
                LDSP_REQUIRE(kc == k, "fmstereo: resampler output counts diverged");
            }
            k::interleave2(outs[0], outs[1], k, dy, e.stream);
        }
        q->ord.mark(e.stream);
        q->last = e.stream;
        q->stg.finish(e, y, 2 * k * 4);
    });
}

// ------------------------------------------------------- many-calls (batch.hpp)
// C independent objects of one class, one call each on the same stream, with
// one launch per kernel for all of them: every object's execute runs with the
// recorder active (its host bookkeeping exactly as for a single call), then the
// recorded work is issued with the launches of objects that run the same
// kernel on the same grid merged (blockIdx.y = object).  Device memory only;
// the objects must be distinct.
// `batchable(c)`: object c's call takes a path whose every kernel has a merged
// form; otherwise the objects run one after another (the same bits, C times the
// launches) -- e.g. exact-mode transfer-function IIR filters, single-sideband AmpModems.
extern "C++" {
template <class T, class B, class F>
static int run_many(T* const* q, int C, void* stream, B&& batchable, F&& one)
{
    return guard([&] {
        LDSP_REQUIRE(q != nullptr && C >= 1 && C <= 4096, "many: 1 .. 4096 objects");
        for (int c = 0; c < C; c++) {
            LDSP_REQUIRE(q[c] != nullptr, "many: NULL object");
            for (int c2 = 0; c2 < c; c2++) LDSP_REQUIRE(q[c2] != q[c], "many: the objects must be distinct");
        }
        bool all = true;
        for (int c = 0; c < C; c++) all = all && batchable(c);
        if (!all) {
            for (int c = 0; c < C; c++) {
                const int rc = one(c);
                if (rc != LDSP_OK) throw Error(rc, g_last_error);
            }
            return;
        }
        BatchRecorder rec(C, (hipStream_t)stream);
        int rc = LDSP_OK;
        std::string err;
        for (int c = 0; c < C && rc == LDSP_OK; c++) {
            rec.channel(c);
            rc = one(c);
            if (rc != LDSP_OK) err = g_last_error;
        }
        rec.flush();                         // every object whose host state advanced gets its device work
        if (rc != LDSP_OK) throw Error(rc, err);
    });
}
} // extern "C++"

int ldsp_agc_execute_many(ldsp_agc_t* q, const void* const* x, size_t n, void* const* y, int C, void* stream)
{
    LDSP_RANGE("ldsp_agc_execute_many");
    return run_many(q, C, stream, [](int) { return true; }, [&](int c) {
        return ldsp_agc_execute(q[c], x[c], n, y[c], nullptr, LDSP_MEM_DEVICE, stream);
    });
}

int ldsp_ampmodem_demodulate_many(ldsp_ampmodem_t* q, const void* const* x, size_t n, void* const* y, int C,
                                  void* stream)
{
    LDSP_RANGE("ldsp_ampmodem_demodulate_many");
    return run_many(q, C, stream, [&](int c) { return q[c]->type == 0; }, [&](int c) {
        return ldsp_ampmodem_demodulate(q[c], x[c], n, y[c], LDSP_MEM_DEVICE, stream);
    });
}

int ldsp_iirfilt_execute_many(ldsp_iirfilt_t* q, const void* const* x, size_t n, void* const* y, int C, void* stream)
{
    LDSP_RANGE("ldsp_iirfilt_execute_many");
    return run_many(q, C, stream, [&](int c) {
        const IirObj::Path p = q[c]->path_for(n);
        // exact SOS cascades: k_iir_sect, one workgroup per (object, component)
        const bool sect = p == IirObj::kSeq && q[c]->sos && q[c]->D > 0 && q[c]->nsos >= 1 &&
                          q[c]->nsos <= (unsigned)k::kIirSectMaxSos;
        return p == IirObj::kSpec || p == IirObj::kModal || sect;
    }, [&](int c) {
        return ldsp_iirfilt_execute(q[c], x[c], n, y[c], LDSP_MEM_DEVICE, stream);
    });
}

int ldsp_iirfilt_resamp_execute_many(ldsp_iirfilt_t* q, ldsp_resamp_t* rs, const void* const* x, size_t n,
                                     void* const* y, size_t cap, size_t* nout, int C, void* stream)
{
    LDSP_RANGE("ldsp_iirfilt_resamp_execute_many");
    if (q == nullptr || rs == nullptr || C < 1 || C > 4096) {
        set_last_error("many: 1 .. 4096 objects, filters and resamplers both given");
        return LDSP_EINVAL;
    }
    for (int c = 0; c < C; c++)
        if (rs[c] == nullptr) {
            set_last_error("many: NULL resampler");
            return LDSP_EINVAL;
        }
    for (int c = 0; c < C; c++)                  // the resamplers must be distinct too
        for (int c2 = 0; c2 < c; c2++)
            if (rs[c] == rs[c2]) {
                set_last_error("many: the objects must be distinct");
                return LDSP_EINVAL;
            }
    return run_many(q, C, stream, [&](int c) {       // the fused pass (ldsp_iirfilt_resamp_execute)
        return rs && rs[c] && q[c]->cplx == rs[c]->cplx && q[c]->path_for(n) == IirObj::kModal &&
               rs[c]->sub_len >= 2 && rs[c]->sub_len - 1 <= 1024u;
    }, [&](int c) {
        return ldsp_iirfilt_resamp_execute(q[c], rs[c], x[c], n, y[c], cap, nout ? nout + c : nullptr,
                                           LDSP_MEM_DEVICE, stream);
    });
}

// ------------------------------------------------------- page-locked host pool
// Blocks are whole 64 KB multiples; a request takes the smallest free block that
// fits and is at most twice its size.  Freed blocks are cached up to kCacheMax
// (hipHostFree beyond it); at most kLiveMax is handed out at a time.
namespace {
struct HostPool {
    static constexpr size_t kCacheMax = (size_t)256 << 20, kLiveMax = (size_t)1 << 30;
    std::mutex mu;
    std::multimap<size_t, void*> free;
    std::map<void*, size_t> live;
    size_t cached = 0, out = 0;
};
HostPool& host_pool()
{
    static HostPool* p = new HostPool();    // never destroyed: frees can come at interpreter teardown
    return *p;
}
} // namespace

int ldsp_host_alloc(size_t bytes, void** p)
{
    return guard([&] {
        LDSP_REQUIRE(p != nullptr, "host_alloc: NULL output pointer");
        *p = nullptr;
        const size_t want = (std::max<size_t>(bytes, 1) + 65535) & ~(size_t)65535;
        HostPool& hp = host_pool();
        void* b = nullptr;
        size_t sz = want;
        {
            std::lock_guard<std::mutex> lk(hp.mu);
            auto it = hp.free.lower_bound(want);
            // the limit counts the block actually handed out (a cached block may be up to 2x want)
            if (it != hp.free.end() && it->first <= 2 * want && hp.out + it->first <= HostPool::kLiveMax) {
                b = it->second;
                sz = it->first;
                hp.cached -= sz;
                hp.free.erase(it);
                hp.live[b] = sz;
                hp.out += sz;
                *p = b;
                return;
            }
            if (hp.out + want > HostPool::kLiveMax) throw Error(LDSP_ENOMEM, "host_alloc: page-locked pool exhausted");
            hp.out += want;                  // reserved while the allocation runs outside the lock
        }
        if (hipHostMalloc(&b, want, hipHostMallocPortable) != hipSuccess || !b) {
            (void)hipGetLastError();
            std::lock_guard<std::mutex> lk(hp.mu);
            hp.out -= want;
            throw Error(LDSP_ENOMEM, "host_alloc: hipHostMalloc failed");
        }
        std::lock_guard<std::mutex> lk(hp.mu);
        hp.live[b] = sz;
        *p = b;
    });
}

int ldsp_host_free(void* p)
{
    return guard([&] {
        if (!p) return;
        HostPool& hp = host_pool();
        std::vector<void*> evict;            // hipHostFree may synchronise the device: never under the lock
        {
            std::lock_guard<std::mutex> lk(hp.mu);
            auto it = hp.live.find(p);
            LDSP_REQUIRE(it != hp.live.end(), "host_free: not a block of ldsp_host_alloc");
            const size_t sz = it->second;
            hp.live.erase(it);
            hp.out -= sz;
            hp.free.emplace(sz, p);
            hp.cached += sz;
            while (hp.cached > HostPool::kCacheMax && !hp.free.empty()) {
                auto big = std::prev(hp.free.end());
                hp.cached -= big->first;
                evict.push_back(big->second);
                hp.free.erase(big);
            }
        }
        for (void* b : evict) (void)hipHostFree(b);
    });
}

int ldsp_debug_host_pools(size_t* total, size_t* idle)
{
    return guard([&] {
        PoolList& l = pool_list();
        std::lock_guard<std::mutex> lk(l.mu);
        size_t f = 0;
        for (const auto& v : l.free) f += v.size();
        if (total) *total = l.total;
        if (idle) *idle = f;
    });
}

// ---------------------------------------------------------------- bytes_to_iq
int ldsp_bytes_to_iq(const void* in, size_t nbytes, void* y, int mem, void* stream)
{
    static std::mutex mu;
    static std::vector<std::unique_ptr<Staging>> stgs;   // per device, host-memory calls only
    return guard([&] {
        const size_t n = nbytes / 4;
        LDSP_REQUIRE(n == 0 || (in && y), "bytes_to_iq: NULL buffer");
        const BufDevice bd(mem, in);
        const int dev = bd.dev;
        const Exec e = make_exec(dev, mem, stream, bd);
        std::unique_lock<std::mutex> lk(mu, std::defer_lock);
        if (e.host) lk.lock();   // the staging buffers are shared by host-memory calls
        if ((int)stgs.size() <= dev) stgs.resize(dev + 1);
        if (!stgs[dev]) stgs[dev].reset(new Staging());
        Staging& stg = *stgs[dev];
        const void* dx = stg.dev_in(e, in, n * 4);
        void* dy = stg.dev_out(e, y, n * 8);
        k::bytes_to_iq(dx, dy, n, e.stream);
        stg.finish(e, y, n * 8);
    });
}

} // extern "C"
