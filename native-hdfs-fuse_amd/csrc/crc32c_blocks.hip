// crc32c_blocks.hip -- concurrent block writes coalesced into one launch
// (include/hdfs_crc32c.h section 3b).
//
// libfuse runs hadoop_fuse_write_block on many worker threads at once
// (src/fuse.c:1771 starts fuse_main without -s; fuse.c:336-449 writes one
// block per call, hadoop_rpc_send_packets cuts it into packets,
// hadooprpc.c:815-860).  One launch per 4 MiB block is bound by HIP's launch
// path (~3.5-4 us per block), while one launch over 16
// blocks takes ~0.94 us per block.  A crc32c_blocks queue collects the
// blocks several threads submit within a short window and sends them out as
// ONE multi-block launch of the block's plan (crc32c_plan_exec_blocks: the
// block table rides in the kernel arguments, so a flush builds and uploads
// nothing).
//
// Group commit: a submit that fills the queue (max_blocks) flushes it; a
// thread waiting for a block still queued flushes when the window since the
// queue's first block has passed, else sleeps until then or until another
// thread's flush took its block.  Every flush records an event on the
// queue's stream; a waiter waits for the event of the flush that carried its
// block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "hdfs_crc32c.h"
#include "runtime_internal.h"

using namespace hdfs_crc;
using Clock = std::chrono::steady_clock;

struct crc32c_blocks {
    crc32c_plan *plan = nullptr;
    int device = 0;
    uint32_t max_blocks = 16;
    std::chrono::microseconds window{20};
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<const void *> pend_payload;
    std::vector<uint32_t *> pend_out;
    Clock::time_point first_pending;
    uint64_t next_ticket = 0;   // tickets handed out
    uint64_t flushed_upto = 0;  // tickets below this have been launched
    uint64_t done_upto = 0;     // ... and are known complete
    struct Flush {
        uint64_t hi;  // tickets below hi
        hipEvent_t ev;
    };
    std::deque<Flush> inflight;
    std::vector<hipEvent_t> spare;
    uint64_t flushes = 0, blocks = 0;
};

namespace {

// Completed flushes off the front of the queue (non-blocking).  Caller holds q->mu.
void reap(crc32c_blocks *q) {
    while (!q->inflight.empty()) {
        const hipError_t e = hipEventQuery(q->inflight.front().ev);
        if (e == hipErrorNotReady) return;
        if (e != hipSuccess) (void)hipGetLastError();
        q->done_upto = q->inflight.front().hi;
        q->spare.push_back(q->inflight.front().ev);
        q->inflight.pop_front();
    }
}

// One multi-block launch of everything queued.  Caller holds q->mu.
int flush_locked(crc32c_blocks *q) {
    if (q->pend_payload.empty()) return 0;
    DeviceGuard guard(q->device);
    reap(q);
    hipEvent_t ev = nullptr;
    if (!q->spare.empty()) {
        ev = q->spare.back();
        q->spare.pop_back();
    } else {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    int rc = crc32c_plan_exec_blocks(q->plan, q->pend_payload.data(), q->pend_out.data(), q->pend_payload.size(),
                                     q->stream);
    if (!rc && hipEventRecord(ev, q->stream) != hipSuccess) rc = fail(-EIO, "hipEventRecord failed");
    if (rc) {
        q->spare.push_back(ev);
        return rc;
    }
    q->inflight.push_back({q->next_ticket, ev});
    q->flushes++;
    q->blocks += q->pend_payload.size();
    q->flushed_upto = q->next_ticket;
    q->pend_payload.clear();
    q->pend_out.clear();
    q->cv.notify_all();
    return 0;
}

}  // namespace

extern "C" {

int crc32c_blocks_create(crc32c_plan *plan, uint32_t max_blocks, uint32_t window_us, crc32c_blocks **out) {
    if (!plan || !out) return fail(-EINVAL, "plan/out == NULL");
    *out = nullptr;
    std::unique_ptr<crc32c_blocks, int (*)(crc32c_blocks *)> q(new crc32c_blocks, crc32c_blocks_destroy);
    q->plan = plan;
    q->device = plan->ctx->device;
    q->max_blocks = max_blocks ? std::min<uint32_t>(max_blocks, 1024u) : 16u;
    q->window = std::chrono::microseconds(window_us);
    q->pend_payload.reserve(q->max_blocks);
    q->pend_out.reserve(q->max_blocks);
    DeviceGuard guard(q->device);
    HIP_TRY(hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking));
    *out = q.release();
    return 0;
}

int crc32c_block_submit(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket) {
    if (!q || !dev_out) return fail(-EINVAL, "queue/out == NULL");
    std::lock_guard<std::mutex> lock(q->mu);
    if (q->pend_payload.empty()) q->first_pending = Clock::now();
    if (ticket) *ticket = q->next_ticket;
    q->next_ticket++;
    q->pend_payload.push_back(dev_payload);
    q->pend_out.push_back(dev_out);
    if (q->pend_payload.size() >= q->max_blocks) return flush_locked(q);
    return 0;
}

int crc32c_block_flush(crc32c_blocks *q) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    std::lock_guard<std::mutex> lock(q->mu);
    return flush_locked(q);
}

int crc32c_block_wait(crc32c_blocks *q, uint64_t ticket) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    std::unique_lock<std::mutex> lock(q->mu);
    if (ticket >= q->next_ticket) return fail(-EINVAL, "ticket %llu was never handed out", (unsigned long long)ticket);
    while (ticket >= q->flushed_upto) {  // still queued: flush when full or when the window has passed
        const Clock::time_point due = q->first_pending + q->window;
        if (q->pend_payload.size() >= q->max_blocks || Clock::now() >= due) {
            if (int rc = flush_locked(q)) return rc;
            break;
        }
        q->cv.wait_until(lock, due);
    }
    if (ticket < q->done_upto) return 0;
    reap(q);
    if (ticket < q->done_upto) return 0;
    hipEvent_t ev = nullptr;
    for (const auto &f : q->inflight)
        if (ticket < f.hi) {
            ev = f.ev;
            break;
        }
    lock.unlock();
    // (if the event is recycled for a later flush meanwhile, this waits for
    // that one: later on the same stream, so still after this block)
    if (ev) {
        DeviceGuard guard(q->device);
        HIP_TRY(hipEventSynchronize(ev));
    }
    return 0;
}

int crc32c_block_checksums(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out) {
    uint64_t t = 0;
    if (int rc = crc32c_block_submit(q, dev_payload, dev_out, &t)) return rc;
    return crc32c_block_wait(q, t);
}

int crc32c_blocks_stats(const crc32c_blocks *q, uint64_t *flushes, uint64_t *blocks) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    crc32c_blocks *m = const_cast<crc32c_blocks *>(q);
    std::lock_guard<std::mutex> lock(m->mu);
    if (flushes) *flushes = q->flushes;
    if (blocks) *blocks = q->blocks;
    return 0;
}

int crc32c_blocks_destroy(crc32c_blocks *q) {
    if (!q) return 0;
    {
        std::lock_guard<std::mutex> lock(q->mu);
        (void)flush_locked(q);
    }
    DeviceGuard guard(q->device);
    if (q->stream) {
        (void)hipStreamSynchronize(q->stream);
        (void)hipStreamDestroy(q->stream);
    }
    for (const auto &f : q->inflight) (void)hipEventDestroy(f.ev);
    for (hipEvent_t e : q->spare) (void)hipEventDestroy(e);
    delete q;
    return 0;
}

}  // extern "C"
