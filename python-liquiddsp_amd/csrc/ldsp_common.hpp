// ldsp_common.hpp -- shared host-side plumbing for libldsp: error reporting,
// HIP checks, grow-only device buffers, stream selection.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "../../include/ldsp.h"

namespace ldsp {

// Error carried from the implementation to the C ABI boundary (-> ldsp_last_error()).
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define LDSP_HIP(call)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess)                                                              \
            throw ::ldsp::Error(LDSP_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Per-kernel timing (ldsp_profile_enable): a Scope records a HIP event pair on
// the launch stream around one kernel launch; ldsp_profile_report() resolves
// them into per-kernel call counts and total device time.  Disabled: one
// relaxed atomic load per launch.
namespace prof {
bool enabled();
struct Scope {
    hipEvent_t a = nullptr;
    hipStream_t s;
    const char* name;
    Scope(hipStream_t s_, const char* n);
    ~Scope();
};
} // namespace prof
#define LDSP_PROF_CAT2(a, b) a##b
#define LDSP_PROF_CAT(a, b) LDSP_PROF_CAT2(a, b)
#define LDSP_PROF(stream, name) ::ldsp::prof::Scope LDSP_PROF_CAT(ldsp_prof_, __LINE__)((stream), (name))

// roctx range around a C-ABI call (SURVEY section 5 tracing): visible in
// `rocprofv3 --marker-trace`.  librocprofiler-sdk-roctx is resolved with dlopen
// on first use (capi.cpp), so the library loads and runs without it (the ranges
// are then no-ops).
void roctx_push(const char* m);
void roctx_pop();
struct RoctxRange {
    explicit RoctxRange(const char* m) { roctx_push(m); }
    ~RoctxRange() { roctx_pop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};
#define LDSP_RANGE(name) ::ldsp::RoctxRange LDSP_PROF_CAT(ldsp_range_, __LINE__)(name)

#define LDSP_REQUIRE(cond, msg)                                                            \
    do {                                                                                   \
        if (!(cond)) throw ::ldsp::Error(LDSP_EINVAL, (msg));                              \
    } while (0)

// Grow-only device allocation owned by one object (allocation happens lazily,
// outside any timed/captured region once warmed up).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int device = -1;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) {
            int cur = 0;
            if (hipGetDevice(&cur) == hipSuccess && cur != device) (void)hipSetDevice(device);
            (void)hipFree(p);
            if (cur != device) (void)hipSetDevice(cur);
        }
        p = nullptr;
        cap = 0;
    }
    // Grows only: geometric (x1.25) and rounded up to 64 KiB, because every
    // regrowth frees the old buffer and hipFree waits for the whole device --
    // a block size that varies by one sample between calls (resampler output)
    // must not stall the host in steady state.
    void* ensure(size_t bytes, int dev) {
        if (bytes <= cap && p) return p;
        release();
        device = dev;
        size_t want = std::max(bytes, cap + cap / 4);
        want = (std::max<size_t>(want, 16) + 65535) & ~(size_t)65535;
        LDSP_HIP(hipMalloc(&p, want));
        cap = want;
        return p;
    }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

// Select the device an object lives on and make it current for the call.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        LDSP_HIP(hipGetDevice(&prev));
        if (prev != dev) LDSP_HIP(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
    }
};

// Many-calls (batch.hpp): while a recorder is active on this thread, stream
// waits and event records are recorded in call order instead of issued.
class BatchRecorder;
BatchRecorder* batch_active();
void batch_record_wait(hipEvent_t ev);
void batch_record_mark(hipEvent_t ev);

// Cross-stream order of one object's device state.  An execute marks the point
// on its stream where the object's state (and the scratch it reuses) is final;
// an execute enqueued on a different stream first waits for that point, so
// calls made on several streams still run in call order per object while
// different objects (or independent parts of one object) overlap.  Calls on one
// stream need nothing beyond stream order.
struct StreamMark {
    hipEvent_t ev = nullptr;
    hipStream_t s = nullptr;
    bool set = false;
    StreamMark() = default;
    StreamMark(const StreamMark&) = delete;
    StreamMark& operator=(const StreamMark&) = delete;
    ~StreamMark() {
        if (ev) (void)hipEventDestroy(ev);
    }
    void wait(hipStream_t t) const {
        if (!(set && s != t)) return;
        if (batch_active()) batch_record_wait(ev);
        else LDSP_HIP(hipStreamWaitEvent(t, ev, 0));
    }
    void mark(hipStream_t t) {
        if (!ev) LDSP_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (batch_active()) batch_record_mark(ev);
        else LDSP_HIP(hipEventRecord(ev, t));
        s = t;
        set = true;
    }
    void sync() const {
        if (set) LDSP_HIP(hipEventSynchronize(ev));
    }
};

// Tuning and diagnostic environment knobs (warm-up lengths, walker margin,
// debug counters, timeline dumps) are read only by a tuning build
// (`make EXTRA=-DLDSP_TUNING`); the product library reads no environment
// and always uses the default.
#ifdef LDSP_TUNING
long knob_env(const char* name, long dflt);
double knob_env_f(const char* name, double dflt);
const char* knob_env_s(const char* name);
#define LDSP_KNOB(name, dflt) ((decltype(dflt))::ldsp::knob_env(name, (long)(dflt)))
#define LDSP_KNOB_F(name, dflt) ((decltype(dflt))::ldsp::knob_env_f(name, (double)(dflt)))
#define LDSP_KNOB_S(name) (::ldsp::knob_env_s(name))
#else
#define LDSP_KNOB(name, dflt) (dflt)
#define LDSP_KNOB_F(name, dflt) (dflt)
#define LDSP_KNOB_S(name) ((const char*)nullptr)
#endif

// Serial-latency kernels (the one-lane loops, chunk warm-ups, the PLL walk,
// single-workgroup scans) share SIMDs with the streaming kernels of other
// calls in flight; the highest wave priority lets their dependent chains issue
// first instead of by wave age (MI355X_MICROARCH.md, two waves per SIMD, item 2).
#define LDSP_LATENCY_CRITICAL() __builtin_amdgcn_s_setprio(3)

int current_device();                       // throws LDSP_EHIP when no GPU is present
hipStream_t library_stream(int device);     // per-device non-blocking stream for host-memory calls

} // namespace ldsp
