// crc32c_resident.hip -- the resident-kernel mode of the block queue
// (crc32c_blocks_create_resident, include/hdfs_crc32c.h section 3b): the
// host side of resident_engine.h's kernel, and the product's one shape of it
// (16 waves per workgroup, 7 blocks in flight, 2 waves per block and
// workgroup: the best 16-writers x 1-block shape of round 4's A/B,
// DESIGN.md section 5 "One block per writer").
//
// The host side: a ticket is one atomic add on a counter that also carries
// the stop bit (a submit after destroy began is refused in the same atomic
// step); the ticket's slot in the pinned, device-mapped host ring is written
// with two tagged words; the kernel is launched on demand (a submit finding
// every launch exited, or a waiter that has waited 100 us) and never while
// one runs; a waiter polls the slot's `done` word (host memory the kernel
// writes at system scope).  Destroy drains: every ticket handed out
// completes first, then the stop word ends the launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "resident_engine.h"
#include "runtime_internal.h"

using namespace hdfs_crc_res;

namespace hdfs_crc {

struct ResidentEngine {
    crc32c_plan *plan = nullptr;
    int device = 0;
    uint32_t grid = 0;
    uint64_t idle_ticks = 0;
    ResidentLaunch launch = nullptr;
    HostRing *h = nullptr;      // host view
    HostRing *h_dev = nullptr;  // the same memory, device view
    DevRing *d = nullptr;
    hipStream_t stream = nullptr;
    std::atomic<uint64_t> next{0};  // tickets handed out (| kStop once destroy began)
    std::mutex mu;                  // launches
    bool running = false;           // a launch may be on the GPU (under mu)
    std::atomic<uint64_t> launches{0};
    uint64_t *stamps = nullptr;  // trace (debug A/B only)
};

namespace {

constexpr uint64_t kStop = 1ull << 63;
// A wait gives up after this long without its block completing (the kernel
// itself gives up after kStuckMs without progress).
constexpr auto kWaitDeadline = std::chrono::seconds(5);

uint64_t handed_out(const ResidentEngine *r) { return r->next.load(std::memory_order_acquire) & ~kStop; }

// Launches the kernel unless one is running (caller holds r->mu).  A launch
// that has exited shows as an idle stream.
int ensure_running(ResidentEngine *r) {
    if (r->running) {
        const hipError_t q = hipStreamQuery(r->stream);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return fail(-EIO, "resident kernel: %s", hipGetErrorString(q));
        r->running = false;
    }
    const uint64_t col = __atomic_load_n(&r->h->exit_col, __ATOMIC_ACQUIRE);
    if (col >= handed_out(r)) return 0;  // nothing queued
    KParams kp = plan_params(r->plan, nullptr, nullptr);
    RParams p{};
    p.h = r->h_dev;
    p.d = r->d;
    p.tiles = kp.tiles;
    p.table_s4 = kp.table_s4;
    p.ntiles = kp.ntiles;
    p.flags = kp.flags;
    for (int i = 0; i < 5; ++i) p.c_lg[i] = kp.c_lg[i];
    p.first = col;
    p.idle_ticks = r->idle_ticks;
    p.stamps = r->stamps;
    DeviceGuard guard(r->device);
    // (fresh control words; the device slots keep their tags: a tag names its ticket)
    const uint64_t ctl[3] = {col, col, 0};
    HIP_TRY(hipMemcpyAsync(&r->d->fwd, ctl, sizeof ctl, hipMemcpyHostToDevice, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));  // (ctl is on this stack)
    HIP_TRY(r->launch(p, r->grid, r->stream));
    r->running = true;
    r->launches.fetch_add(1, std::memory_order_release);
    return 0;
}

}  // namespace

hipError_t resident_launch_product(const RParams &p, uint32_t grid, hipStream_t stream) {
    hipLaunchKernelGGL((resident_kernel<16, 7, 2>), dim3(grid), dim3(16 * 64), 0, stream, p);
    return hipGetLastError();
}

int resident_create(crc32c_plan *plan, uint32_t idle_us, ResidentLaunch launch, bool stamps, ResidentEngine **out) {
    if (!plan || !out || !launch) return fail(-EINVAL, "plan/out/launch == NULL");
    *out = nullptr;
    const DevicePlan &dp = plan->dp;
    if (dp.ngen || dp.nseg || dp.nconst || dp.general || dp.misaligned || !dp.ntiles || plan->absolute)
        return fail(-EINVAL, "the resident kernel runs plans of aligned power-of-two tiles only");
    std::unique_ptr<ResidentEngine, void (*)(ResidentEngine *)> r(new ResidentEngine, [](ResidentEngine *e) {
        (void)resident_destroy(e, false);
    });
    r->plan = plan;
    r->device = plan->ctx->device;
    r->grid = uint32_t(std::min(plan->ctx->num_cu, int(kMaxWg)));
    r->idle_ticks = uint64_t(idle_us ? idle_us : 2000) * kTicksPerUs;
    r->launch = launch;
    DeviceGuard guard(r->device);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&r->h), sizeof(HostRing), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(static_cast<void *>(r->h), 0, sizeof(HostRing));
    void *hd = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&hd, r->h, 0));
    r->h_dev = static_cast<HostRing *>(hd);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&r->d), sizeof(DevRing)));
    HIP_TRY(hipMemset(r->d, 0, sizeof(DevRing)));
    HIP_TRY(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
    if (stamps) {
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&r->stamps), sizeof(uint64_t) * 4 * kStampRing));
        HIP_TRY(hipMemset(r->stamps, 0, sizeof(uint64_t) * 4 * kStampRing));
    }
    // (the plan's descriptors are uploaded on the context's upload stream)
    if (plan->dp.uploaded) HIP_TRY(hipStreamWaitEvent(r->stream, plan->dp.uploaded, 0));
    *out = r.release();
    return 0;
}

int resident_submit(ResidentEngine *r, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket) {
    if (!r || !dev_payload || !dev_out) return fail(-EINVAL, "bad arguments");
    const uint64_t pa = reinterpret_cast<uint64_t>(dev_payload), oa = reinterpret_cast<uint64_t>(dev_out);
    if (pa & 15u) return fail(-EINVAL, "payload must be 16-byte aligned");
    if (oa & 3u) return fail(-EINVAL, "dev_out must be 4-byte aligned");
    if ((pa | oa) & ~kAddrMask) return fail(-EINVAL, "address above 2^48: does not fit a ring slot");
    // The ticket is taken only once its slot is free (block t - kRing
    // complete), so no error can leave a ticket without its slot written: a
    // hole would stop the forwarder (it forwards consecutive tickets) and
    // with it every later ticket.  The stop check and the ticket are one
    // atomic step (kStop); a lost race re-checks the next ticket's slot.
    uint64_t t = r->next.load(std::memory_order_relaxed);
    for (;;) {
        if (t & kStop) return fail(-EINVAL, "queue is being destroyed");
        if (t >= kRing && __atomic_load_n(&r->h->done[t % kRing], __ATOMIC_ACQUIRE) < t - kRing + 1) {
            if (int rc = resident_wait(r, t - kRing)) return rc;  // (no ticket taken: the queue is intact)
            t = r->next.load(std::memory_order_relaxed);
            continue;
        }
        if (r->next.compare_exchange_weak(t, t + 1, std::memory_order_acq_rel, std::memory_order_relaxed)) break;
    }
    const uint32_t sl = uint32_t(t % kRing);
    __atomic_store_n(&r->h->slot[sl][0], pa | tag_of(t), __ATOMIC_RELAXED);
    __atomic_store_n(&r->h->slot[sl][1], oa | tag_of(t), __ATOMIC_RELEASE);
    if (ticket) *ticket = t;
    // every launch so far has exited (or is exiting): start one (a launch
    // still running forwards this ticket; one that exits before seeing it is
    // relaunched by the waiter)
    if (__atomic_load_n(&r->h->exits, __ATOMIC_ACQUIRE) >= r->launches.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lock(r->mu);
        return ensure_running(r);
    }
    return 0;
}

int resident_wait(ResidentEngine *r, uint64_t ticket) {
    if (!r) return fail(-EINVAL, "queue == NULL");
    if (ticket >= handed_out(r)) return fail(-EINVAL, "ticket %llu was never handed out", (unsigned long long)ticket);
    const uint32_t sl = uint32_t(ticket % kRing);
    auto t0 = std::chrono::steady_clock::now();
    const auto deadline = t0 + kWaitDeadline;
    for (uint32_t i = 0;; ++i) {
        const uint64_t v = __atomic_load_n(&r->h->done[sl], __ATOMIC_ACQUIRE);
        if (v >= ticket + 1) return 0;  // (a later ticket in the slot implies this one completed)
        if ((i & 255u) == 255u) {
            const auto t = std::chrono::steady_clock::now();
            if (t > deadline) return fail(-ETIMEDOUT, "resident kernel: block %llu not done", (unsigned long long)ticket);
            if (t - t0 > std::chrono::microseconds(100)) {  // the kernel may have exited: relaunch it
                std::lock_guard<std::mutex> lock(r->mu);
                if (int rc = ensure_running(r)) return rc;
                t0 = t;
            }
            std::this_thread::yield();
        } else {
            __builtin_ia32_pause();
        }
    }
}

uint64_t resident_launches(const ResidentEngine *r) { return r ? r->launches.load() : 0; }
uint64_t resident_tickets(const ResidentEngine *r) { return r ? handed_out(r) : 0; }

int resident_trace(ResidentEngine *r, uint64_t *stamps, uint64_t *rtt_ticks, uint64_t *rtt_polls) {
    if (!r || !stamps || !rtt_ticks || !rtt_polls) return fail(-EINVAL, "bad arguments");
    if (!r->stamps) return fail(-EINVAL, "no trace: the runner was created without stamps");
    DeviceGuard guard(r->device);
    std::lock_guard<std::mutex> lock(r->mu);
    // (the launch ends first: the forwarder's round-trip sums are written at its exit)
    __atomic_store_n(&r->h->stop, 1u, __ATOMIC_RELEASE);
    HIP_TRY(hipStreamSynchronize(r->stream));
    __atomic_store_n(&r->h->stop, 0u, __ATOMIC_RELEASE);
    r->running = false;
    HIP_TRY(hipMemcpy(stamps, r->stamps, sizeof(uint64_t) * 4 * kStampRing, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(rtt_ticks, &r->d->rtt_sum, sizeof(uint64_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(rtt_polls, &r->d->rtt_n, sizeof(uint64_t), hipMemcpyDeviceToHost));
    return 0;
}

int resident_destroy(ResidentEngine *r, bool drain) {
    if (!r) return 0;
    // (no ticket is handed out from here)
    const uint64_t n = r->next.fetch_or(kStop, std::memory_order_acq_rel) & ~kStop;
    int rc = 0;
    if (drain && n && r->h) rc = resident_wait(r, n - 1);  // (blocks complete in ticket order)
    if (r->h) __atomic_store_n(&r->h->stop, 1u, __ATOMIC_RELEASE);
    DeviceGuard guard(r->device);
    if (r->stream) {
        (void)hipStreamSynchronize(r->stream);  // (the kernel exits on the stop word)
        (void)hipStreamDestroy(r->stream);
    }
    if (r->d) (void)hipFree(r->d);
    if (r->stamps) (void)hipFree(r->stamps);
    if (r->h) (void)hipHostFree(r->h);
    delete r;
    return rc;
}

}  // namespace hdfs_crc
