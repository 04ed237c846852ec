// crc32c_blocks.hip -- concurrent block writes coalesced into one launch
// (include/hdfs_crc32c.h section 3b).
//
// libfuse runs hadoop_fuse_write_block on many worker threads at once
// (src/fuse.c:1771 starts fuse_main without -s; fuse.c:336-449 writes one
// block per call, hadoop_rpc_send_packets cuts it into packets,
// hadooprpc.c:815-860).  One launch per 4 MiB block is bound by HIP's launch
// path (~3.5-4 us per block), while one launch over 16
// blocks takes ~1.0 us per block from HBM.  A crc32c_blocks queue collects
// the blocks several threads submit within a short window and sends them
// out as ONE multi-block launch of the block's plan
// (crc32c_plan_exec_blocks: the block table rides in the kernel arguments,
// so a flush builds and uploads nothing).
//
// One worker thread per queue makes every HIP call of the queue: it
// launches a batch when it holds max_blocks blocks, on crc32c_block_flush,
// or when window_us have passed since its first block (group commit), and
// completes the launches in order by polling their events (a flush's event
// is its last launch's own stop event, hipExtLaunchKernel).  Submitting and
// waiting threads only touch the queue's lock and its done_upto counter
// (waiters spin on it briefly, then sleep on a condition variable).
// Round 3 first launched from the submitting threads and had every waiter
// -- then one watcher per flush, then one poller -- query events: HIP's
// launch path and its event queries contend, and with two or three flushes
// outstanding a launch call took ~27 us instead of ~5 (tools/block_rate,
// HDFS_CRC32C_QUEUE_TRACE).
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
#include <string>
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
    std::condition_variable work_cv;  // worker: a batch is due, or stop
    std::vector<const void *> pend_payload;
    std::vector<uint32_t *> pend_out;
    Clock::time_point first_pending;
    uint64_t next_ticket = 0;            // tickets handed out
    std::atomic<uint64_t> done_upto{0};  // tickets below this are complete
    std::atomic<bool> due{false};        // a batch is full or a flush was asked for
    bool flush_req = false;
    bool stop = false;
    bool worker_sleeping = false;
    struct Flush {
        uint64_t hi;  // tickets below hi
        hipEvent_t ev;
        size_t trace_idx;
    };
    std::deque<Flush> inflight;  // worker only
    std::vector<hipEvent_t> spare;  // worker only
    uint64_t flushes = 0, blocks = 0;
    std::atomic<int> error{0};  // a failed flush or event: every later wait returns it
    bool record_events = false;  // A/B (HDFS_CRC32C_QUEUE_RECORD=1): an hipEventRecord after each flush
    unsigned event_flags = hipEventDisableTiming;  // A/B (HDFS_CRC32C_QUEUE_TIMING=1: timing events)
    std::thread worker;
    // Diagnostic (HDFS_CRC32C_QUEUE_TRACE=<file>): per flush, steady-clock
    // ns of its first submit, issue start / end, completion seen; written
    // as JSON lines at destroy.
    struct TraceRec {
        int64_t first, issue0, issue1, done;
        uint32_t nblocks, inflight_before;
    };
    std::vector<TraceRec> trace;
    std::string trace_path;
};

namespace {

std::chrono::microseconds env_us(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return std::chrono::microseconds(e ? std::atoi(e) : dflt);
}
// Waiters spin this long on done_upto before sleeping (HDFS_CRC32C_QUEUE_SPIN_US: A/B).
std::chrono::microseconds spin_time() {
    static const std::chrono::microseconds t = env_us("HDFS_CRC32C_QUEUE_SPIN_US", 50);
    return t;
}
// The worker's time between event polls (HDFS_CRC32C_QUEUE_POLL_US: A/B).
std::chrono::microseconds poll_gap() {
    static const std::chrono::microseconds t = env_us("HDFS_CRC32C_QUEUE_POLL_US", 2);
    return t;
}

int64_t ns(Clock::time_point t) {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count();
}

// Launches the batch (worker thread; `lock` held on entry and exit, released
// around the launch).
void launch_batch(crc32c_blocks *q, std::unique_lock<std::mutex> &lock, std::vector<const void *> &pays,
                  std::vector<uint32_t *> &outs) {
    // (at most max_blocks: blocks submitted while the worker was busy wait
    // for the next launch)
    const size_t n = std::min<size_t>(q->pend_payload.size(), q->max_blocks);
    pays.assign(q->pend_payload.begin(), q->pend_payload.begin() + n);
    outs.assign(q->pend_out.begin(), q->pend_out.begin() + n);
    q->pend_payload.erase(q->pend_payload.begin(), q->pend_payload.begin() + n);
    q->pend_out.erase(q->pend_out.begin(), q->pend_out.begin() + n);
    const uint64_t hi = q->next_ticket - q->pend_payload.size();
    const int64_t first = ns(q->first_pending);
    if (q->pend_payload.empty()) {
        q->flush_req = false;
        q->due.store(false, std::memory_order_relaxed);
    } else {
        q->first_pending = Clock::now();
        q->due.store(q->flush_req || q->pend_payload.size() >= q->max_blocks, std::memory_order_relaxed);
    }
    lock.unlock();
    hipEvent_t ev = nullptr;
    if (!q->spare.empty()) {
        ev = q->spare.back();
        q->spare.pop_back();
    }
    int rc = 0;
    if (!ev && hipEventCreateWithFlags(&ev, q->event_flags) != hipSuccess) {
        ev = nullptr;
        rc = fail(-EIO, "hipEventCreate failed");
    }
    const Clock::time_point issue0 = Clock::now();
    // the flush's event is the last launch's own stop event
    if (!rc)
        rc = q->record_events ? crc32c_plan_exec_blocks(q->plan, pays.data(), outs.data(), pays.size(), q->stream)
                              : exec_blocks(q->plan, pays.data(), outs.data(), pays.size(), q->stream, ev);
    if (!rc && q->record_events && hipEventRecord(ev, q->stream) != hipSuccess) rc = fail(-EIO, "hipEventRecord failed");
    const Clock::time_point issue1 = Clock::now();
    size_t tidx = SIZE_MAX;
    if (!q->trace_path.empty()) {
        tidx = q->trace.size();
        q->trace.push_back({first, ns(issue0), ns(issue1), 0, uint32_t(pays.size()), uint32_t(q->inflight.size())});
    }
    lock.lock();
    q->flushes++;
    q->blocks += pays.size();
    if (rc) {  // nothing to wait for: its tickets complete (with the error) once those before them have
        q->error = rc;
        if (ev) q->spare.push_back(ev);
        ev = nullptr;
    }
    q->inflight.push_back({hi, ev, tidx});
}

// Completes the front flush if its event has (worker; lock NOT held).
// Returns true when it did.
bool complete_front(crc32c_blocks *q) {
    const crc32c_blocks::Flush f = q->inflight.front();
    if (f.ev) {
        const hipError_t e = hipEventQuery(f.ev);
        if (e == hipErrorNotReady) return false;
        if (e != hipSuccess) q->error = fail(-EIO, "block flush: %s", hipGetErrorString(e));
        q->spare.push_back(f.ev);
    }
    q->inflight.pop_front();
    if (f.trace_idx != SIZE_MAX) q->trace[f.trace_idx].done = ns(Clock::now());
    {
        std::lock_guard<std::mutex> lock(q->mu);
        q->done_upto.store(f.hi, std::memory_order_release);
    }
    q->cv.notify_all();
    return true;
}

void worker_loop(crc32c_blocks *q) {
    DeviceGuard guard(q->device);
    std::vector<const void *> pays;
    std::vector<uint32_t *> outs;
    pays.reserve(q->max_blocks);
    outs.reserve(q->max_blocks);
    std::unique_lock<std::mutex> lock(q->mu);
    for (;;) {
        const bool pending = !q->pend_payload.empty();
        if (pending && (q->pend_payload.size() >= q->max_blocks || q->flush_req || q->stop ||
                        Clock::now() >= q->first_pending + q->window)) {
            launch_batch(q, lock, pays, outs);
            continue;
        }
        if (q->inflight.empty()) {
            if (q->stop) return;
            q->worker_sleeping = true;
            if (pending)
                q->work_cv.wait_until(lock, q->first_pending + q->window);
            else
                q->work_cv.wait(lock);
            q->worker_sleeping = false;
            continue;
        }
        // a flush in flight: poll it (no lock held), watching for a due batch
        lock.unlock();
        while (!complete_front(q)) {
            const Clock::time_point until = Clock::now() + poll_gap();
            while (Clock::now() < until && !q->due.load(std::memory_order_relaxed)) __builtin_ia32_pause();
            if (q->due.load(std::memory_order_relaxed)) break;
            if (pending) break;  // (re-check the window)
        }
        lock.lock();
    }
}

// Caller holds q->mu: wakes the worker for a due batch.
void mark_due(crc32c_blocks *q) {
    q->due.store(true, std::memory_order_relaxed);
    if (q->worker_sleeping) q->work_cv.notify_one();
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
    if (const char *tp = std::getenv("HDFS_CRC32C_QUEUE_TRACE")) {
        q->trace_path = tp;
        q->trace.reserve(1 << 16);
    }
    const char *rec = std::getenv("HDFS_CRC32C_QUEUE_RECORD");
    q->record_events = rec && rec[0] == '1';
    const char *tim = std::getenv("HDFS_CRC32C_QUEUE_TIMING");
    if (tim && tim[0] == '1') q->event_flags = hipEventDefault;
    q->pend_payload.reserve(q->max_blocks);
    q->pend_out.reserve(q->max_blocks);
    DeviceGuard guard(q->device);
    HIP_TRY(hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking));
    try {
        q->worker = std::thread(worker_loop, q.get());
    } catch (...) {
        return fail(-ENOMEM, "cannot start the queue's worker thread");
    }
    *out = q.release();
    return 0;
}

int crc32c_block_submit(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket) {
    if (!q || !dev_out) return fail(-EINVAL, "queue/out == NULL");
    std::lock_guard<std::mutex> lock(q->mu);
    if (q->stop) return fail(-EINVAL, "queue is being destroyed");
    const bool first = q->pend_payload.empty();
    if (first) q->first_pending = Clock::now();
    if (ticket) *ticket = q->next_ticket;
    q->next_ticket++;
    q->pend_payload.push_back(dev_payload);
    q->pend_out.push_back(dev_out);
    if (q->pend_payload.size() >= q->max_blocks)
        mark_due(q);
    else if (first && q->worker_sleeping)
        q->work_cv.notify_one();  // (it flushes the batch when the window passes)
    return 0;
}

int crc32c_block_flush(crc32c_blocks *q) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    std::lock_guard<std::mutex> lock(q->mu);
    if (!q->pend_payload.empty()) {
        q->flush_req = true;
        mark_due(q);
    }
    return 0;
}

int crc32c_block_wait(crc32c_blocks *q, uint64_t ticket) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (ticket < q->done_upto.load(std::memory_order_acquire)) return q->error;
    {
        std::lock_guard<std::mutex> lock(q->mu);
        if (ticket >= q->next_ticket)
            return fail(-EINVAL, "ticket %llu was never handed out", (unsigned long long)ticket);
    }
    const Clock::time_point spin_end = Clock::now() + spin_time();
    while (Clock::now() < spin_end) {
        if (ticket < q->done_upto.load(std::memory_order_acquire)) return q->error;
        std::this_thread::yield();
    }
    std::unique_lock<std::mutex> lock(q->mu);
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
        q->stop = true;  // (the worker launches what is queued, completes everything, returns)
        mark_due(q);
    }
    if (q->worker.joinable()) q->worker.join();
    DeviceGuard guard(q->device);
    if (q->stream) {
        (void)hipStreamSynchronize(q->stream);
        plan_forget_stream(q->plan, q->stream);  // (idle now; the plan must not touch it once destroyed)
        (void)hipStreamDestroy(q->stream);
    }
    for (const auto &f : q->inflight)
        if (f.ev) (void)hipEventDestroy(f.ev);
    for (hipEvent_t e : q->spare) (void)hipEventDestroy(e);
    if (!q->trace_path.empty())
        if (FILE *f = std::fopen(q->trace_path.c_str(), "a")) {
            for (const auto &r : q->trace)
                std::fprintf(f, "{\"first\": %lld, \"issue0\": %lld, \"issue1\": %lld, \"done\": %lld, \"nblocks\": %u, \"inflight_before\": %u}\n",
                             (long long)r.first, (long long)r.issue0, (long long)r.issue1, (long long)r.done, r.nblocks,
                             r.inflight_before);
            std::fprintf(f, "{\"end\": 1}\n");
            std::fclose(f);
        }
    delete q;
    return 0;
}

}  // extern "C"
