// batch.cpp -- the many-call recorder (batch.hpp).
#include "batch.hpp"

namespace ldsp {

namespace {
thread_local BatchRecorder* g_active = nullptr;
}

BatchRecorder* batch_active() { return g_active; }

BatchRecorder::BatchRecorder(int nch, hipStream_t s) : s_(s), ops_((size_t)std::max(nch, 1))
{
    prev_ = g_active;
    g_active = this;
}

BatchRecorder::~BatchRecorder()
{
    if (g_active == this) g_active = prev_;
}

void batch_record_wait(hipEvent_t ev)
{
    BatchOp op;
    op.kind = 1;
    op.ev = ev;
    g_active->add(std::move(op));
}

void batch_record_mark(hipEvent_t ev)
{
    BatchOp op;
    op.kind = 2;
    op.ev = ev;
    g_active->add(std::move(op));
}

void BatchRecorder::flush()
{
    if (done_) return;
    done_ = true;
    if (g_active == this) g_active = prev_;      // issuing, not recording
    size_t len = 0;
    for (const auto& v : ops_) len = std::max(len, v.size());
    const int C = (int)ops_.size();
    std::vector<char> used((size_t)C);
    std::vector<const BatchOp*> grp;
    for (size_t i = 0; i < len; i++) {
        std::fill(used.begin(), used.end(), 0);
        for (int c = 0; c < C; c++) {
            if (i >= ops_[c].size() || used[c]) continue;
            const BatchOp& op = ops_[c][i];
            used[c] = 1;
            if (op.kind == 1) {
                LDSP_HIP(hipStreamWaitEvent(s_, op.ev, 0));
                continue;
            }
            if (op.kind == 2) {
                LDSP_HIP(hipEventRecord(op.ev, s_));
                continue;
            }
            grp.clear();
            grp.push_back(&op);
            if (op.many && op.g.y == 1 && op.g.z == 1 && (!op.xcd || op.g.x % 8 == 0)) {
                for (int c2 = c + 1; c2 < C; c2++) {
                    if (i >= ops_[c2].size() || used[c2]) continue;
                    const BatchOp& o2 = ops_[c2][i];
                    if (o2.kind == 0 && o2.many == op.many && o2.g.x == op.g.x && o2.g.y == op.g.y &&
                        o2.g.z == op.g.z && o2.b.x == op.b.x && o2.b.y == op.b.y && o2.b.z == op.b.z &&
                        o2.shm == op.shm) {
                        grp.push_back(&o2);
                        used[c2] = 1;
                    }
                }
            }
            if (grp.size() > 1) {
                op.merged(s_, grp);
                merged_++;
            } else {
                op.one(s_);
            }
        }
    }
}

} // namespace ldsp
