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
// queue's first block has passed (so does the queue's completion thread).
// A flush's completion event is its last launch's own stop event
// (hipExtLaunchKernel; an hipEventRecord after the launch costs more,
// tools/launch_stop_probe).  Completion: one thread per queue (the
// completer) polls the oldest flush's event, publishes its end (done_upto)
// and wakes the waiters, which spin on done_upto briefly and then sleep on
// the condition variable.  Only the completer queries the events: round 3's
// first form made the first waiter of each flush poll its event, so several
// threads polled HIP at once while others launched.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
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
    std::condition_variable cv;       // waiters: done_upto moved
    std::condition_variable work_cv;  // completer: a flush or a pending block appeared, or stop
    std::vector<const void *> pend_payload;
    std::vector<uint32_t *> pend_out;
    Clock::time_point first_pending;
    uint64_t next_ticket = 0;               // tickets handed out
    uint64_t flushed_upto = 0;              // tickets below this have been launched
    std::atomic<uint64_t> done_upto{0};     // ... and are known complete
    struct Flush {
        uint64_t hi;  // tickets below hi
        hipEvent_t ev;
    };
    std::deque<Flush> inflight;
    std::vector<hipEvent_t> spare;
    uint64_t flushes = 0, blocks = 0;
    std::atomic<int> error{0};            // a failed flush or event: every waiter returns it
    std::atomic<bool> has_pending{false};  // pend_payload non-empty (read without the lock)
    bool stop = false;
    bool record_events = false;  // A/B (HDFS_CRC32C_QUEUE_RECORD=1): an hipEventRecord after each flush
    std::thread completer;
};

namespace {

// Waiters spin this long on done_upto before sleeping (HDFS_CRC32C_QUEUE_SPIN_US: A/B).
std::chrono::microseconds spin_time() {
    static const std::chrono::microseconds t = [] {
        const char *e = std::getenv("HDFS_CRC32C_QUEUE_SPIN_US");
        return std::chrono::microseconds(e ? std::atoi(e) : 50);
    }();
    return t;
}

// One multi-block launch of everything queued.  Caller holds q->mu.
int flush_locked(crc32c_blocks *q) {
    if (q->pend_payload.empty()) return 0;
    DeviceGuard guard(q->device);
    hipEvent_t ev = nullptr;
    if (!q->spare.empty()) {
        ev = q->spare.back();
        q->spare.pop_back();
    } else {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDefault));
    }
    // the flush's event is the last launch's own stop event
    int rc = q->record_events
                 ? crc32c_plan_exec_blocks(q->plan, q->pend_payload.data(), q->pend_out.data(), q->pend_payload.size(),
                                           q->stream)
                 : exec_blocks(q->plan, q->pend_payload.data(), q->pend_out.data(), q->pend_payload.size(), q->stream,
                               ev);
    if (!rc && q->record_events && hipEventRecord(ev, q->stream) != hipSuccess) rc = fail(-EIO, "hipEventRecord failed");
    if (rc) {
        q->spare.push_back(ev);
        return rc;
    }
    const bool was_idle = q->inflight.empty();
    q->inflight.push_back({q->next_ticket, ev});
    q->flushes++;
    q->blocks += q->pend_payload.size();
    q->flushed_upto = q->next_ticket;
    q->pend_payload.clear();
    q->pend_out.clear();
    q->has_pending.store(false, std::memory_order_relaxed);
    q->cv.notify_all();  // (waiters of these blocks stop flushing)
    if (was_idle) q->work_cv.notify_one();
    return 0;
}

// The queue's one HIP waiter: completes flushes in launch order (polling the
// front flush's event -- the only thread that queries the queue's events, so
// the threads that submit and launch never contend with it in the runtime),
// publishes done_upto, and flushes a partial queue once its window passed.
void completer_loop(crc32c_blocks *q) {
    DeviceGuard guard(q->device);
    std::unique_lock<std::mutex> lock(q->mu);
    for (;;) {
        if (!q->pend_payload.empty() && Clock::now() >= q->first_pending + q->window) {
            if (int rc = flush_locked(q)) {  // (the blocks are dropped: their waiters get the error)
                q->error = rc;
                q->pend_payload.clear();
                q->pend_out.clear();
                q->has_pending.store(false, std::memory_order_relaxed);
                q->flushed_upto = q->next_ticket;
                if (q->inflight.empty()) q->done_upto.store(q->next_ticket, std::memory_order_release);
                q->cv.notify_all();
            }
        }
        if (q->inflight.empty()) {
            if (q->stop) return;
            if (q->pend_payload.empty())
                q->work_cv.wait(lock);
            else
                q->work_cv.wait_until(lock, q->first_pending + q->window);
            continue;
        }
        const crc32c_blocks::Flush f = q->inflight.front();
        lock.unlock();
        hipError_t e;
        int polls = 0;
        while ((e = hipEventQuery(f.ev)) == hipErrorNotReady) {
            // (a flush is ~15 us: poll; a partial queue's window may pass meanwhile)
            if ((++polls & 63) == 0 && q->has_pending.load(std::memory_order_relaxed)) break;
            std::this_thread::yield();
        }
        lock.lock();
        if (e == hipErrorNotReady) continue;  // (back to check the window)
        if (e != hipSuccess) q->error = fail(-EIO, "block flush: %s", hipGetErrorString(e));
        q->inflight.pop_front();
        q->spare.push_back(f.ev);
        // (after a dropped partial queue, the last flush also completes its tickets)
        q->done_upto.store(q->inflight.empty() && q->error ? q->flushed_upto : f.hi, std::memory_order_release);
        q->cv.notify_all();
    }
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
    const char *rec = std::getenv("HDFS_CRC32C_QUEUE_RECORD");
    q->record_events = rec && rec[0] == '1';
    q->pend_payload.reserve(q->max_blocks);
    q->pend_out.reserve(q->max_blocks);
    DeviceGuard guard(q->device);
    HIP_TRY(hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking));
    try {
        q->completer = std::thread(completer_loop, q.get());
    } catch (...) {
        return fail(-ENOMEM, "cannot start the queue's completion thread");
    }
    *out = q.release();
    return 0;
}

int crc32c_block_submit(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket) {
    if (!q || !dev_out) return fail(-EINVAL, "queue/out == NULL");
    std::lock_guard<std::mutex> lock(q->mu);
    const bool first = q->pend_payload.empty();
    if (first) q->first_pending = Clock::now();
    if (ticket) *ticket = q->next_ticket;
    q->next_ticket++;
    q->pend_payload.push_back(dev_payload);
    q->pend_out.push_back(dev_out);
    if (q->pend_payload.size() >= q->max_blocks) return flush_locked(q);
    if (first) {
        q->has_pending.store(true, std::memory_order_relaxed);
        q->work_cv.notify_one();  // (the completer flushes it when the window passes)
    }
    return 0;
}

int crc32c_block_flush(crc32c_blocks *q) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    std::lock_guard<std::mutex> lock(q->mu);
    return flush_locked(q);
}

int crc32c_block_wait(crc32c_blocks *q, uint64_t ticket) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (ticket < q->done_upto.load(std::memory_order_acquire)) return q->error;
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
    lock.unlock();
    const Clock::time_point spin_end = Clock::now() + spin_time();
    while (Clock::now() < spin_end) {
        if (ticket < q->done_upto.load(std::memory_order_acquire)) return q->error;
        std::this_thread::yield();
    }
    lock.lock();
    q->cv.wait(lock, [&] { return ticket < q->done_upto.load(std::memory_order_acquire); });
    return q->error;
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
        if (q->stream) (void)flush_locked(q);
        q->stop = true;
        q->work_cv.notify_all();
    }
    if (q->completer.joinable()) q->completer.join();  // (returns once every flush completed)
    DeviceGuard guard(q->device);
    if (q->stream) {
        (void)hipStreamSynchronize(q->stream);
        plan_forget_stream(q->plan, q->stream);  // (idle now; the plan must not touch it once destroyed)
        (void)hipStreamDestroy(q->stream);
    }
    for (const auto &f : q->inflight) (void)hipEventDestroy(f.ev);
    for (hipEvent_t e : q->spare) (void)hipEventDestroy(e);
    delete q;
    return 0;
}

}  // extern "C"
