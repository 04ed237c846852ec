// crc32c_resident.hip -- the resident-kernel mode of the block queue
// (crc32c_blocks_create_resident, include/hdfs_crc32c.h section 3b): the
// host side of resident_engine.h's kernel, and the product's one shape of it
// (16 waves per workgroup, 7 blocks in flight, 2 waves per block and
// workgroup: the best 16-writers x 1-block shape of round 4's A/B,
// DESIGN.md section 5 "One block per writer").
//
// The host side: a ticket is one atomic add on a counter that also carries
// the stop bit (a submit after destroy began is refused in the same atomic
// step), taken only once its slot is free; the ticket's slot in the pinned,
// device-mapped host ring is written with three tagged words (payload, out,
// the block's plan's shape record); the kernel is launched on demand (a submit finding
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
    ResidentLaunch launch = nullptr;          // the aligned-only build
    ResidentLaunch launch_general = nullptr;  // the general build (null: blocks that need it are refused)
    bool plan_simple = false;                 // the queue's plan runs in the aligned-only build
    std::atomic<bool> general{false};         // a block needed the general build: every launch from then on is
    HostRing *h = nullptr;      // host view
    HostRing *h_dev = nullptr;  // the same memory, device view
    DevRing *d = nullptr;
    hipStream_t stream = nullptr;
    std::atomic<uint64_t> next{0};  // tickets handed out (| kStop once destroy began)
    std::mutex mu;                  // launches
    bool running = false;           // a launch may be on the GPU (under mu)
    bool running_general = false;   // ... of the general build
    std::atomic<uint64_t> launches{0};
    uint64_t *stamps = nullptr;  // trace (debug A/B only)
    // crc32c_debug_blocks_resident_inject: no launch while held; the next
    // fail_waits waits give up at once (-ETIMEDOUT)
    std::atomic<bool> hold{false};
    std::atomic<uint32_t> fail_waits{0};
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
    if (r->hold.load(std::memory_order_acquire)) return 0;
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
    p.table_s4 = kp.table_s4;
    p.flags = kp.flags;
    const DevicePlan &dp = r->plan->dp;
    p.def = Shape{kp.tiles, kp.gen, dp.ntiles, dp.ngen, (!dp.ngen && !dp.misaligned && !dp.general) ? 1u : 0u};
    for (int i = 0; i < 5; ++i) p.c_lg[i] = kp.c_lg[i];
    for (int i = 0; i < 4; ++i) p.c_small[i] = kp.c_small[i];
    p.first = col;
    p.idle_ticks = r->idle_ticks;
    p.stamps = r->stamps;
    DeviceGuard guard(r->device);
    // (fresh control words; the device slots keep their tags: a tag names its ticket)
    const uint64_t ctl[3] = {col, col, 0};
    HIP_TRY(hipMemcpyAsync(&r->d->fwd, ctl, sizeof ctl, hipMemcpyHostToDevice, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));  // (ctl is on this stack)
    const bool gen = r->general.load(std::memory_order_acquire);
    HIP_TRY((gen ? r->launch_general : r->launch)(p, r->grid, r->stream));
    r->running = true;
    r->running_general = gen;
    r->launches.fetch_add(1, std::memory_order_release);
    return 0;
}

// A plan whose blocks the resident kernel runs: bytesPerChecksum 512 << k --
// power-of-two tiles, general tiles of 2^k-block chunks (a packet's tail
// behind its full chunks) and GenItems --, offsets from the block's payload
// (no buffer lists), same device and same checksum type / byte order as the
// queue's.
int shape_ok(const ResidentEngine *r, const crc32c_plan *plan) {
    const DevicePlan &dp = plan->dp;
    if (dp.nseg || dp.nconst || dp.half || dp.padtiles || !dp.gen_pow2 || plan->absolute)
        return fail(-EINVAL, "the resident kernel runs blocks of bytesPerChecksum 512 << k (power-of-two tiles, "
                             "packet tails and trimmed first packets), payload offsets from the block start: no half, "
                             "padded or general tiles of other chunk lengths, no buffer lists");
    if (!dp.ntiles && !dp.ngen) return fail(-EINVAL, "the plan has no checksum");
    if (r && (plan->ctx->device != r->device ||
              ((plan->flags ^ r->plan->flags) & (CRC32C_BIG_ENDIAN | CRC32C_TYPE_CRC32))))
        return fail(-EINVAL, "the plan's device, checksum type or byte order differs from the queue's");
    return 0;
}

// The kernel reads the plan's shape record and items: its upload must be
// complete (once per plan; a host wait on its upload event).
int shape_uploaded(crc32c_plan *plan) {
    DevicePlan &dp = plan->dp;
    if (dp.ready.load(std::memory_order_acquire)) return 0;
    RelaxedCapture relaxed;  // (another thread may be capturing a graph)
    if (dp.uploaded) HIP_TRY(hipEventSynchronize(dp.uploaded));
    dp.ready.store(true, std::memory_order_release);
    return 0;
}

}  // namespace

hipError_t resident_launch_product(const RParams &p, uint32_t grid, hipStream_t stream) {
    hipLaunchKernelGGL((resident_kernel<16, 7, 2, false>), dim3(grid), dim3(16 * 64), 0, stream, p);
    return hipGetLastError();
}
hipError_t resident_launch_product_general(const RParams &p, uint32_t grid, hipStream_t stream) {
    hipLaunchKernelGGL((resident_kernel<16, 7, 2, true>), dim3(grid), dim3(16 * 64), 0, stream, p);
    return hipGetLastError();
}
// Loads both builds' code onto the current device now (HIP loads a code
// object at its first use), so the queue's first blocks do not pay for it.
hipError_t resident_preload_product() {
    hipFuncAttributes a;
    hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&resident_kernel<16, 7, 2, false>));
    if (e == hipSuccess)
        e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&resident_kernel<16, 7, 2, true>));
    return e;
}

namespace {

// A block that needs the general build was just queued: from here every
// launch is the general build.  A running aligned-only launch ends at that
// block (its forwarder stops there); once it has, the general build starts.
int switch_to_general(ResidentEngine *r) {
    std::lock_guard<std::mutex> lock(r->mu);
    if (r->running && !r->running_general) {
        DeviceGuard guard(r->device);
        const auto deadline = std::chrono::steady_clock::now() + kWaitDeadline;
        for (;;) {
            const hipError_t q = hipStreamQuery(r->stream);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return fail(-EIO, "resident kernel: %s", hipGetErrorString(q));
            if (std::chrono::steady_clock::now() > deadline)
                return fail(-ETIMEDOUT, "resident kernel: the aligned-only launch did not end");
            std::this_thread::yield();
        }
        r->running = false;
    }
    return ensure_running(r);
}

}  // namespace

int resident_create(crc32c_plan *plan, uint32_t idle_us, ResidentLaunch launch, bool stamps, ResidentEngine **out,
                    ResidentLaunch launch_general) {
    if (!plan || !out || !launch) return fail(-EINVAL, "plan/out/launch == NULL");
    *out = nullptr;
    if (int rc = shape_ok(nullptr, plan)) return rc;
    std::unique_ptr<ResidentEngine, void (*)(ResidentEngine *)> r(new ResidentEngine, [](ResidentEngine *e) {
        (void)resident_destroy(e, false);
    });
    r->plan = plan;
    r->device = plan->ctx->device;
    r->grid = uint32_t(std::min(plan->ctx->num_cu, int(kMaxWg)));
    r->idle_ticks = uint64_t(idle_us ? idle_us : 2000) * kTicksPerUs;
    r->launch = launch;
    r->launch_general = launch_general;
    r->plan_simple = !plan->dp.ngen && !plan->dp.misaligned && !plan->dp.general;
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

int resident_submit(ResidentEngine *r, crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out,
                    uint64_t *ticket) {
    if (!r || !dev_payload || !dev_out) return fail(-EINVAL, "bad arguments");
    if (!plan) plan = r->plan;
    if (plan != r->plan)
        if (int rc = shape_ok(r, plan)) return rc;
    if (int rc = shape_uploaded(plan)) return rc;
    const uint64_t pa = reinterpret_cast<uint64_t>(dev_payload), oa = reinterpret_cast<uint64_t>(dev_out);
    const uint64_t sa = reinterpret_cast<uint64_t>(plan->dp.d + kResShapeOff);
    if (oa & 3u) return fail(-EINVAL, "dev_out must be 4-byte aligned");
    if ((pa | oa | sa) & ~kAddrMask) return fail(-EINVAL, "address above 2^48: does not fit a ring slot");
    // (the aligned-only build runs the queue's plan when it is simple, on a
    // 16-byte aligned payload; any other block needs the general build)
    const bool needs_general = plan != r->plan || !r->plan_simple || (pa & 15u);
    if (needs_general && !r->launch_general)
        return fail(-EINVAL, "this queue runs aligned blocks of its own plan only");
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
    if (needs_general) __atomic_store_n(&r->h->shape[sl], sa | tag_of(t), __ATOMIC_RELAXED);
    __atomic_store_n(&r->h->slot[sl][0], pa | tag_of(t), __ATOMIC_RELAXED);
    __atomic_store_n(&r->h->slot[sl][1], oa | tag_of(t) | (needs_general ? kShapeFlag : 0), __ATOMIC_RELEASE);
    if (ticket) *ticket = t;
    if (needs_general && !r->general.exchange(true, std::memory_order_acq_rel)) return switch_to_general(r);
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
    for (uint32_t k = r->fail_waits.load(std::memory_order_relaxed); k;)
        if (r->fail_waits.compare_exchange_weak(k, k - 1, std::memory_order_relaxed))
            return fail(-ETIMEDOUT, "resident kernel: block %llu not done (injected)", (unsigned long long)ticket);
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

int resident_inject(ResidentEngine *r, bool hold, uint32_t fail_waits) {
    if (!r) return fail(-EINVAL, "queue == NULL");
    r->fail_waits.store(fail_waits, std::memory_order_relaxed);
    r->hold.store(hold, std::memory_order_release);
    if (!hold) {  // (what was submitted while held goes out now)
        std::lock_guard<std::mutex> lock(r->mu);
        return ensure_running(r);
    }
    return 0;
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
