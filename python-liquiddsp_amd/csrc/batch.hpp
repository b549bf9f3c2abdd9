// batch.hpp -- one launch per kernel for C independent objects
// (ldsp_*_execute_many; SURVEY 7 H5 "batch channels", 8(e)).
//
// A many-call runs each object's ordinary execute path with a thread-local
// recorder active: kernel launches, cross-stream waits and event records are
// appended to that object's op list instead of being issued, while all host
// bookkeeping (phases, slots, histories, plans) advances exactly as for a
// single call.  flush() then issues the lists round-robin by op index: the
// index-i launches of all objects that run the same kernel with the same grid
// become ONE launch whose blockIdx.y selects the object (its arguments from a
// Many<A> array), everything else is issued per object in object order.  Per
// object the ops keep their order, so every object computes what its own
// execute would have, bit for bit; different objects never depend on each other.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <vector>

#include "ldsp_common.hpp"

namespace ldsp {

constexpr size_t kManyArgBytes = 3584;   // argument bytes of a merged launch (the kernarg limit is 4 KB)

// Per-object arguments of a merged launch: entry blockIdx.y.
template <class A>
struct Many {
    static constexpr int kCap = (int)(kManyArgBytes / sizeof(A) < 16 ? kManyArgBytes / sizeof(A) : 16);
    static_assert(kCap >= 1, "kernel arguments too large to batch");
    A a[kCap];
};

struct BatchOp {
    int kind = 0;                     // 0 launch, 1 wait for an event, 2 record an event
    const void* many = nullptr;       // merged kernel (nullptr: never merged)
    dim3 g, b;
    size_t shm = 0;
    bool xcd = false;                 // unit-to-XCD mapping matters: merge only when g.x % 8 == 0
    std::vector<unsigned char> args;
    std::function<void(hipStream_t)> one;                                        // issue this op alone
    std::function<void(hipStream_t, const std::vector<const BatchOp*>&)> merged;  // issue a group in one launch
    hipEvent_t ev = nullptr;
};

class BatchRecorder {
public:
    BatchRecorder(int nch, hipStream_t s);
    ~BatchRecorder();
    BatchRecorder(const BatchRecorder&) = delete;
    BatchRecorder& operator=(const BatchRecorder&) = delete;
    void channel(int c) { cur_ = c; }
    void add(BatchOp&& op) { ops_[cur_].push_back(std::move(op)); }
    hipStream_t stream() const { return s_; }
    void flush();                     // issue everything recorded (once)
    int merged_launches() const { return merged_; }

private:
    hipStream_t s_;
    int cur_ = 0, merged_ = 0;
    bool done_ = false;
    std::vector<std::vector<BatchOp>> ops_;
    BatchRecorder* prev_ = nullptr;
};

BatchRecorder* batch_active();

// Launch kernel `one` (argument A), or record it when a many-call is recording;
// `many` (argument Many<A>, blockIdx.y = object) may be null.
template <class A>
void launch(const char* name, void (*one)(A), void (*many)(Many<A>), dim3 g, dim3 b, size_t shm, hipStream_t s,
            const A& a, bool xcd = false)
{
    if (BatchRecorder* r = batch_active()) {
        BatchOp op;
        op.kind = 0;
        op.many = (const void*)many;
        op.g = g;
        op.b = b;
        op.shm = shm;
        op.xcd = xcd;
        op.args.resize(sizeof(A));
        std::memcpy(op.args.data(), &a, sizeof(A));
        op.one = [=](hipStream_t st) {
            LDSP_PROF(st, name);
            A aa = a;
            void* kp[] = {&aa};
            LDSP_HIP(hipLaunchKernel((const void*)one, g, b, kp, shm, st));
        };
        if (many)
            op.merged = [=](hipStream_t st, const std::vector<const BatchOp*>& grp) {
                for (size_t i = 0; i < grp.size(); i += Many<A>::kCap) {
                    const int cnt = (int)std::min<size_t>(Many<A>::kCap, grp.size() - i);
                    Many<A> m;
                    for (int j = 0; j < cnt; j++) std::memcpy(&m.a[j], grp[i + j]->args.data(), sizeof(A));
                    LDSP_PROF(st, name);
                    void* kp[] = {&m};
                    LDSP_HIP(hipLaunchKernel((const void*)many, dim3(g.x, (unsigned)cnt, 1), b, kp, shm, st));
                }
            };
        r->add(std::move(op));
        return;
    }
    LDSP_PROF(s, name);
    A aa = a;
    void* kp[] = {&aa};
    LDSP_HIP(hipLaunchKernel((const void*)one, g, b, kp, shm, s));
}

// A one-object kernel and its merged form around a __device__ body run(const A&)
// that reads blockIdx.x / threadIdx.x only (blockIdx.y is the object).
#define LDSP_KERNEL_PAIR(NAME, A, RUN, ...)                                                          \
    __global__ void __launch_bounds__(__VA_ARGS__) NAME(A a) { RUN(a); }                              \
    __global__ void __launch_bounds__(__VA_ARGS__) NAME##_many(::ldsp::Many<A> m) { RUN(m.a[blockIdx.y]); }

} // namespace ldsp
