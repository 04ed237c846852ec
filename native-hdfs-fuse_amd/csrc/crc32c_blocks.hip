// crc32c_blocks.hip -- concurrent block writes coalesced into one launch
// (include/hdfs_crc32c.h section 3b).
//
// libfuse runs hadoop_fuse_write_block on many worker threads at once
// (src/fuse.c:1771 starts fuse_main without -s; fuse.c:336-449 writes one
// block per call, hadoop_rpc_send_packets cuts it into packets,
// hadooprpc.c:815-860).  One launch per 4 MiB block is bound by HIP's launch
// path (~3.5-4 us per block), while one launch over 16
// blocks takes ~0.9 us per block from HBM.  A crc32c_blocks queue collects
// the blocks several threads submit within a short window and sends them
// out as ONE multi-block launch of the block's plan
// (crc32c_plan_exec_blocks: the block table rides in the kernel arguments,
// so a flush builds and uploads nothing).
//
// One worker thread per queue makes every HIP call of the queue: it
// launches a batch when it holds max_blocks blocks, on crc32c_block_flush,
// or when window_us have passed since it saw the batch's first block (group
// commit), and completes the launches in order by polling their events (a
// flush's event is its last launch's own stop event, hipExtLaunchKernel).
//
// Submitting and waiting threads take no lock on the fast path: a ticket is
// one atomic add, the block goes into the ring slot of its ticket, published
// by the slot's sequence word; waiters spin on the completed-ticket counter
// and only sleep (condition variable) after spin_time.  Round 3's first
// queue kept the pending blocks under one mutex: 16 threads resubmitting
// after a flush queued on it (a futex hand-off each), and a batch took ~40
// us to fill against ~15 us of GPU time per flush (HDFS_CRC32C_QUEUE_TRACE,
// DESIGN.md section 5).
//
// Resident mode (crc32c_blocks_create_resident, opt-in): the same calls are
// served by a resident kernel instead (crc32c_resident.hip /
// resident_engine.h) -- no launch per flush, no worker thread; the kernel
// holds every CU while it runs and exits idle_us after the last block.
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
#include <pthread.h>
#include <time.h>
#include <thread>
#include <vector>

#include "hdfs_crc32c.h"
#include "hdfs_crc32c_debug.h"
#include "runtime_internal.h"

using namespace hdfs_crc;
using Clock = std::chrono::steady_clock;

namespace {
struct alignas(64) Slot {
    std::atomic<uint64_t> seq{0};  // ticket + 1 once payload/out hold ticket's block
    const void *payload = nullptr;
    uint32_t *out = nullptr;
    crc32c_plan *plan = nullptr;  // the block's shape (crc32c_block_submit_plan; else the queue's)
};
}  // namespace

struct crc32c_blocks {
    crc32c_plan *plan = nullptr;
    ResidentEngine *res = nullptr;  // resident mode: every call goes to it
    int device = 0;
    uint32_t max_blocks = 16;
    std::chrono::microseconds window{20};
    hipStream_t stream = nullptr;
    // the ring: ticket t's block in slots[t & mask] (reusable once t is launched)
    std::unique_ptr<Slot[]> slots;
    uint64_t mask = 0;
    alignas(64) std::atomic<uint64_t> next_ticket{0};   // tickets handed out (| kStopBit once destroy began)
    alignas(64) std::atomic<uint64_t> launched_upto{0}; // tickets below this are in a launch
    alignas(64) std::atomic<uint64_t> done_upto{0};     // tickets below this are complete
    alignas(64) std::atomic<uint64_t> flush_upto{0};    // crc32c_block_flush: launch tickets below this now
    std::atomic<bool> stop{false};
    std::atomic<bool> worker_sleeping{false};
    std::atomic<int> sleepers{0};  // waiters asleep on cv
    // Failed flushes (rare): each one's ticket range and error, so a wait
    // returns the error of its own flush only -- tickets before and after it
    // succeed as their flushes do.  Flushes complete in ticket order, so the
    // ranges are sorted; consecutive failed flushes with the same error are
    // merged into one range (a device that keeps failing keeps one entry).
    std::mutex err_mu;
    std::vector<std::pair<std::pair<uint64_t, uint64_t>, int>> failed;
    std::atomic<int> nfailed{0};
    std::mutex mu;                  // only for the two condition variables
    std::condition_variable cv;       // waiters: done_upto moved
    std::condition_variable work_cv;  // worker: a ticket was handed out, or stop
    struct Flush {
        uint64_t lo, hi;  // tickets [lo, hi)
        hipEvent_t ev;
        int err;  // its issue failed (nothing to wait for)
        size_t trace_idx;
        crc32c_plan *plan;  // its blocks' shape
    };
    std::deque<Flush> inflight;     // worker only
    std::vector<hipEvent_t> spare;  // worker only
    std::atomic<uint64_t> flushes{0}, blocks{0};
    std::atomic<uint32_t> inject_fail{0};  // crc32c_debug_blocks_fail_flushes
    bool record_events = false;  // A/B (HDFS_CRC32C_QUEUE_RECORD=1): an hipEventRecord after each flush
    unsigned event_flags = hipEventDisableTiming;  // A/B (HDFS_CRC32C_QUEUE_TIMING=1: timing events)
    // A/B (HDFS_CRC32C_QUEUE_BLOCKING=1): with max_inflight() flushes in
    // flight (nothing more may be launched), the worker sleeps in
    // hipEventSynchronize on the oldest one's blocking-sync event instead of
    // polling it.
    bool blocking = false;
    std::thread worker;
    // Diagnostic (HDFS_CRC32C_QUEUE_TRACE=<file>): per flush, steady-clock
    // ns of its first block seen by the worker, issue start / end,
    // completion seen; written as JSON lines at destroy.
    struct TraceRec {
        int64_t first, issue0, issue1, done;
        uint32_t nblocks, inflight_before;
    };
    std::vector<TraceRec> trace;
    std::string trace_path;
};

namespace {

// Set in next_ticket by crc32c_blocks_destroy: a submit sees it in the same
// atomic word it takes its ticket from, so no ticket is handed out after the
// worker may have seen the last one.
constexpr uint64_t kStopBit = 1ull << 63;

uint64_t tickets_out(const crc32c_blocks *q, std::memory_order o = std::memory_order_acquire) {
    return q->next_ticket.load(o) & ~kStopBit;
}

void record_failure(crc32c_blocks *q, uint64_t lo, uint64_t hi, int err) {
    std::lock_guard<std::mutex> lock(q->err_mu);
    if (!q->failed.empty() && q->failed.back().first.second == lo && q->failed.back().second == err)
        q->failed.back().first.second = hi;
    else
        q->failed.push_back({{lo, hi}, err});
    q->nfailed.store(int(q->failed.size()), std::memory_order_release);
}

// The error of the flush ticket t went out in (0 when it succeeded): a
// binary search over the sorted failed ranges.
int ticket_error(crc32c_blocks *q, uint64_t t) {
    if (!q->nfailed.load(std::memory_order_acquire)) return 0;
    std::lock_guard<std::mutex> lock(q->err_mu);
    auto it = std::upper_bound(q->failed.begin(), q->failed.end(), t,
                               [](uint64_t v, const auto &f) { return v < f.first.first; });
    if (it == q->failed.begin()) return 0;
    --it;
    return t < it->first.second ? it->second : 0;
}

std::chrono::microseconds env_us(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return std::chrono::microseconds(e ? std::atoi(e) : dflt);
}
// Waiters spin this long on done_upto before sleeping (HDFS_CRC32C_QUEUE_SPIN_US: A/B).
std::chrono::microseconds spin_time() {
    static const std::chrono::microseconds t = env_us("HDFS_CRC32C_QUEUE_SPIN_US", 50);
    return t;
}
// The worker spins this long with nothing queued or in flight before it
// sleeps (HDFS_CRC32C_QUEUE_IDLE_US: A/B).
std::chrono::microseconds idle_spin() {
    static const std::chrono::microseconds t = env_us("HDFS_CRC32C_QUEUE_IDLE_US", 200);
    return t;
}

// Launches the worker keeps in flight at most (HDFS_CRC32C_QUEUE_INFLIGHT:
// A/B).  Two keep the GPU busy (one running, one queued behind it); with
// three to six queued, HIP's launch call itself slowed from ~4 to 16-20 us
// (tools/block_rate depth 4, HDFS_CRC32C_QUEUE_TRACE), so blocks wait in the
// ring instead and go out in fuller launches.
size_t max_inflight() {
    static const size_t n = [] {
        const char *e = std::getenv("HDFS_CRC32C_QUEUE_INFLIGHT");
        const int v = e ? std::atoi(e) : 2;
        return size_t(v > 0 ? v : 2);
    }();
    return n;
}

int64_t ns(Clock::time_point t) {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count();
}

void relax() {
    for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
}

// Tickets from `from` whose blocks are published, contiguous, of one plan
// (one launch runs one block shape), at most `cap`; *cut: the run ended at
// a published block of another plan (nothing more can join this batch).
uint32_t ready_from(const crc32c_blocks *q, uint64_t from, uint32_t cap, bool *cut) {
    uint32_t n = 0;
    const crc32c_plan *plan = nullptr;
    *cut = false;
    while (n < cap && q->slots[(from + n) & q->mask].seq.load(std::memory_order_acquire) == from + n + 1) {
        const crc32c_plan *p = q->slots[(from + n) & q->mask].plan;
        if (n && p != plan) {
            *cut = true;
            break;
        }
        plan = p;
        ++n;
    }
    return n;
}

// Launches tickets [from, from + n) (worker).
void launch_batch(crc32c_blocks *q, uint64_t from, uint32_t n, Clock::time_point first,
                  std::vector<const void *> &pays, std::vector<uint32_t *> &outs) {
    pays.resize(n);
    outs.resize(n);
    crc32c_plan *const plan = q->slots[from & q->mask].plan;  // (one plan: ready_from)
    for (uint32_t i = 0; i < n; ++i) {
        const Slot &s = q->slots[(from + i) & q->mask];
        pays[i] = s.payload;
        outs[i] = s.out;
    }
    // (the kernel arguments hold copies: the slots may be reused from here)
    q->launched_upto.store(from + n, std::memory_order_release);
    hipEvent_t ev = nullptr;
    if (!q->spare.empty()) {
        ev = q->spare.back();
        q->spare.pop_back();
    }
    int rc = 0;
    for (uint32_t k = q->inject_fail.load(std::memory_order_relaxed); k && !rc;)
        if (q->inject_fail.compare_exchange_weak(k, k - 1, std::memory_order_relaxed)) rc = fail(-EIO, "injected flush failure");
    if (!rc && !ev && hipEventCreateWithFlags(&ev, q->event_flags) != hipSuccess) {
        ev = nullptr;
        rc = fail(-EIO, "hipEventCreate failed");
    }
    const Clock::time_point issue0 = Clock::now();
    // the flush's event is the last launch's own stop event
    if (!rc)
        rc = q->record_events ? crc32c_plan_exec_blocks(plan, pays.data(), outs.data(), n, q->stream)
                              : exec_blocks(plan, pays.data(), outs.data(), n, q->stream, ev);
    if (!rc && q->record_events && hipEventRecord(ev, q->stream) != hipSuccess) rc = fail(-EIO, "hipEventRecord failed");
    const Clock::time_point issue1 = Clock::now();
    size_t tidx = SIZE_MAX;
    if (!q->trace_path.empty()) {
        tidx = q->trace.size();
        q->trace.push_back({ns(first), ns(issue0), ns(issue1), 0, n, uint32_t(q->inflight.size())});
    }
    q->flushes.fetch_add(1, std::memory_order_relaxed);
    q->blocks.fetch_add(n, std::memory_order_relaxed);
    if (rc) {  // nothing to wait for: its tickets complete (with the error) once those before them have
        if (ev) q->spare.push_back(ev);
        ev = nullptr;
    }
    q->inflight.push_back({from, from + n, ev, rc, tidx, plan});
}

// Wakes waiters asleep on done_upto (worker).  Called after the launch
// that a completion makes possible, never between them: a futex wake of
// many sleepers takes the worker tens of us, which the GPU then idles
// (16 threads x 4 blocks in flight, before this order: 2.2-2.8 us per block).
void wake_sleepers(crc32c_blocks *q) {
    if (q->sleepers.load(std::memory_order_seq_cst) > 0) {
        { std::lock_guard<std::mutex> lock(q->mu); }
        q->cv.notify_all();
    }
}

// Completes the front flush if its event has (worker): publishes
// done_upto (spinning waiters see it at once; sleepers are woken by the
// caller's wake_sleepers).  Returns true when it did.
bool complete_front(crc32c_blocks *q) {
    const crc32c_blocks::Flush f = q->inflight.front();
    int err = f.err;
    if (f.ev) {
        const hipError_t e = hipEventQuery(f.ev);
        if (e == hipErrorNotReady) return false;
        if (e != hipSuccess) err = fail(-EIO, "block flush: %s", hipGetErrorString(e));
        q->spare.push_back(f.ev);
    }
    if (err) record_failure(q, f.lo, f.hi, err);  // (before done_upto: a waiter that sees it sees this)
    q->inflight.pop_front();
    // A block of another plan (crc32c_block_submit_plan): once its last
    // flush in flight is complete, the plan no longer needs the queue's
    // stream at its release -- it may be destroyed as soon as its waits
    // return, and the queue's stream may go before it.
    if (f.plan != q->plan && std::none_of(q->inflight.begin(), q->inflight.end(),
                                          [&](const crc32c_blocks::Flush &o) { return o.plan == f.plan; }))
        plan_forget_stream(f.plan, q->stream);
    if (f.trace_idx != SIZE_MAX) q->trace[f.trace_idx].done = ns(Clock::now());
    q->done_upto.store(f.hi, std::memory_order_seq_cst);
    return true;
}

void worker_loop(crc32c_blocks *q) {
    DeviceGuard guard(q->device);
    std::vector<const void *> pays;
    std::vector<uint32_t *> outs;
    pays.reserve(q->max_blocks);
    outs.reserve(q->max_blocks);
    uint64_t launched = 0;
    bool wake = false;        // done_upto moved: sleepers to wake once nothing is to launch
    bool have_first = false;  // a ready block seen since the last launch
    Clock::time_point first, idle_since = Clock::now();
    for (;;) {
        bool cut = false;
        const uint32_t n = q->inflight.size() < max_inflight() ? ready_from(q, launched, q->max_blocks, &cut) : 0u;
        if (n) {
            const Clock::time_point now = Clock::now();
            if (!have_first) first = now, have_first = true;
            const bool stopping = q->stop.load(std::memory_order_acquire);
            if (n >= q->max_blocks || cut || q->flush_upto.load(std::memory_order_acquire) > launched || stopping ||
                now >= first + q->window) {
                launch_batch(q, launched, n, first, pays, outs);
                launched += n;
                have_first = false;
                idle_since = Clock::now();
                continue;
            }
        }
        if (wake) {
            wake_sleepers(q);
            wake = false;
        }
        if (!q->inflight.empty()) {
            if (complete_front(q)) {
                wake = true;
                idle_since = Clock::now();
            } else if (q->blocking && q->inflight.size() >= max_inflight() && q->inflight.front().ev) {
                (void)hipEventSynchronize(q->inflight.front().ev);  // (its status: complete_front's query)
            } else {
                relax();
            }
            continue;
        }
        if (tickets_out(q) != launched) {  // a submit in progress, or a window open
            relax();
            continue;
        }
        if (q->stop.load(std::memory_order_acquire)) return;
        if (Clock::now() < idle_since + idle_spin()) {
            relax();
            continue;
        }
        // idle: sleep until a ticket is handed out (Dekker with crc32c_block_submit)
        q->worker_sleeping.store(true, std::memory_order_seq_cst);
        {
            std::unique_lock<std::mutex> lock(q->mu);
            q->work_cv.wait(lock, [&] {
                return tickets_out(q, std::memory_order_seq_cst) != launched ||
                       q->stop.load(std::memory_order_seq_cst);
            });
        }
        q->worker_sleeping.store(false, std::memory_order_relaxed);
        idle_since = Clock::now();
    }
}

void wake_worker(crc32c_blocks *q) {
    if (q->worker_sleeping.load(std::memory_order_seq_cst)) {
        { std::lock_guard<std::mutex> lock(q->mu); }
        q->work_cv.notify_one();
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
    uint64_t cap = 1024;
    while (cap < 4ull * q->max_blocks) cap <<= 1;
    q->slots.reset(new Slot[cap]);
    q->mask = cap - 1;
    if (const char *tp = std::getenv("HDFS_CRC32C_QUEUE_TRACE")) {
        q->trace_path = tp;
        q->trace.reserve(1 << 16);
    }
    const char *rec = std::getenv("HDFS_CRC32C_QUEUE_RECORD");
    q->record_events = rec && rec[0] == '1';
    const char *tim = std::getenv("HDFS_CRC32C_QUEUE_TIMING");
    if (tim && tim[0] == '1') q->event_flags = hipEventDefault;
    const char *blk = std::getenv("HDFS_CRC32C_QUEUE_BLOCKING");
    if (blk && blk[0] == '1') {
        q->blocking = true;
        q->event_flags |= hipEventBlockingSync;
    }
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

int crc32c_blocks_create_resident(crc32c_plan *plan, uint32_t idle_us, crc32c_blocks **out) {
    if (!plan || !out) return fail(-EINVAL, "plan/out == NULL");
    *out = nullptr;
    std::unique_ptr<crc32c_blocks> q(new crc32c_blocks);
    q->plan = plan;
    q->device = plan->ctx->device;
    {
        DeviceGuard guard(q->device);
        HIP_TRY(resident_preload_product());
    }
    if (int rc = resident_create(plan, idle_us, resident_launch_product, false, &q->res, resident_launch_product_general))
        return rc;
    *out = q.release();
    return 0;
}

int crc32c_block_submit(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket) {
    return crc32c_block_submit_plan(q, nullptr, dev_payload, dev_out, ticket);
}

int crc32c_block_submit_plan(crc32c_blocks *q, crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out,
                             uint64_t *ticket) {
    if (!q || !dev_out) return fail(-EINVAL, "queue/out == NULL");
    if (q->res) return resident_submit(q->res, plan, dev_payload, dev_out, ticket);
    if (!plan) plan = q->plan;
    if (plan != q->plan && (plan->ctx->device != q->device || plan->absolute))
        return fail(-EINVAL, "the plan must be one block's shape (offsets from the block start) on the queue's device");
    // the stop check and the ticket are one atomic step (kStopBit)
    uint64_t t = q->next_ticket.load(std::memory_order_relaxed);
    do {
        if (t & kStopBit) return fail(-EINVAL, "queue is being destroyed");
    } while (!q->next_ticket.compare_exchange_weak(t, t + 1, std::memory_order_seq_cst, std::memory_order_relaxed));
    // the ring is full only with mask + 1 blocks queued and none launched yet
    while (t - q->launched_upto.load(std::memory_order_acquire) > q->mask) std::this_thread::yield();
    Slot &s = q->slots[t & q->mask];
    s.payload = dev_payload;
    s.out = dev_out;
    s.plan = plan;
    s.seq.store(t + 1, std::memory_order_release);
    if (ticket) *ticket = t;
    wake_worker(q);
    return 0;
}

int crc32c_block_flush(crc32c_blocks *q) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (q->res) return 0;  // (the resident kernel takes every block as it is submitted)
    const uint64_t hi = tickets_out(q);
    uint64_t cur = q->flush_upto.load(std::memory_order_relaxed);
    while (cur < hi && !q->flush_upto.compare_exchange_weak(cur, hi, std::memory_order_acq_rel)) {
    }
    wake_worker(q);
    return 0;
}

int crc32c_block_wait(crc32c_blocks *q, uint64_t ticket) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (q->res) return resident_wait(q->res, ticket);
    if (ticket < q->done_upto.load(std::memory_order_acquire)) return ticket_error(q, ticket);
    if (ticket >= tickets_out(q))
        return fail(-EINVAL, "ticket %llu was never handed out", (unsigned long long)ticket);
    const Clock::time_point spin_end = Clock::now() + spin_time();
    for (int i = 0;; ++i) {
        if (ticket < q->done_upto.load(std::memory_order_acquire)) return ticket_error(q, ticket);
        if ((i & 63) == 63 && Clock::now() >= spin_end) break;
        if ((i & 7) == 7)
            std::this_thread::yield();
        else
            relax();
    }
    q->sleepers.fetch_add(1, std::memory_order_seq_cst);
    {
        std::unique_lock<std::mutex> lock(q->mu);
        q->cv.wait(lock, [&] { return ticket < q->done_upto.load(std::memory_order_seq_cst); });
    }
    q->sleepers.fetch_sub(1, std::memory_order_relaxed);
    return ticket_error(q, ticket);
}

int crc32c_block_checksums(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out) {
    uint64_t t = 0;
    if (int rc = crc32c_block_submit(q, dev_payload, dev_out, &t)) return rc;
    return crc32c_block_wait(q, t);
}

int crc32c_blocks_stats(const crc32c_blocks *q, uint64_t *flushes, uint64_t *blocks) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (q->res) {  // (launches of the resident kernel; blocks handed to it)
        if (flushes) *flushes = resident_launches(q->res);
        if (blocks) *blocks = resident_tickets(q->res);
        return 0;
    }
    if (flushes) *flushes = q->flushes.load(std::memory_order_relaxed);
    if (blocks) *blocks = q->blocks.load(std::memory_order_relaxed);
    return 0;
}

int crc32c_debug_blocks_fail_flushes(crc32c_blocks *q, uint32_t n) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (q->res) return fail(-EINVAL, "a resident queue has no flushes");
    q->inject_fail.store(n, std::memory_order_relaxed);
    return 0;
}

int crc32c_debug_blocks_resident_inject(crc32c_blocks *q, int hold, uint32_t fail_waits) {
    if (!q) return fail(-EINVAL, "queue == NULL");
    if (!q->res) return fail(-EINVAL, "not a resident queue");
    return resident_inject(q->res, hold != 0, fail_waits);
}

int crc32c_debug_blocks_worker_cpu_ns(crc32c_blocks *q, uint64_t *ns) {
    if (!q || !ns) return fail(-EINVAL, "queue/ns == NULL");
    if (q->res) {  // (no worker thread)
        *ns = 0;
        return 0;
    }
    clockid_t cid;
    timespec ts{};
    if (pthread_getcpuclockid(q->worker.native_handle(), &cid) != 0 || clock_gettime(cid, &ts) != 0)
        return fail(-EIO, "worker thread CPU clock unavailable");
    *ns = uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
    return 0;
}

int crc32c_blocks_destroy(crc32c_blocks *q) {
    if (!q) return 0;
    if (q->res) {  // (every queued block completes, then the kernel stops)
        const int rc = resident_destroy(q->res, true);
        delete q;
        return rc;
    }
    // (no ticket is handed out from here; the worker launches what is
    // queued, completes everything, returns)
    q->next_ticket.fetch_or(kStopBit, std::memory_order_seq_cst);
    q->stop.store(true, std::memory_order_seq_cst);
    {
        std::lock_guard<std::mutex> lock(q->mu);
    }
    q->work_cv.notify_one();
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
