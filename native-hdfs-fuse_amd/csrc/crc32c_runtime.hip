// crc32c_runtime.hip -- host side of the C ABI (include/hdfs_crc32c.h):
// device contexts, batch plans (packet batches and Hadoop_Fuse_Buffer write
// plans) and the host-resident staging pipeline.  The multi-GPU driver is in
// crc32c_multi.hip.  Every GPU entry point returns 0 or -errno; only the
// per-packet host calls given CRC32C_CPU_FALLBACK substitute the CPU path
// (crc32c_chunks_cpu), and they report it (crc32c_last_path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "crc_math.h"
#include "hdfs_crc32c.h"
#include "hdfs_crc32c_debug.h"
#include "kernel_abi.h"
#include "plan.h"
#include "host_copy.h"
#include "runtime_internal.h"

namespace {
thread_local int g_last_path = CRC32C_PATH_NONE;
}  // namespace

using namespace hdfs_crc;

namespace {

constexpr size_t kSliceBytes = 64ull << 20;  // host pipeline slice (whole packets), default
// Scattered packets from pinned memory are copied run by run when the runs
// average at least this much (each copy costs ~15 us on the copy engine).
constexpr uint64_t kMinRunBytes = 1ull << 20;
// The first slice of a pageable batch is staged and copied in pieces of this
// size, so that the copy engine starts after one piece instead of a slice.
constexpr size_t kFirstPieceBytes = 8ull << 20;
constexpr size_t kZeroCopyBytes = 1ull << 20;  // (zero_copy_bytes)

// Batches up to this many bytes (pinned: a quarter of it) skip the copy
// command: the CPU copies them into pinned, device-MAPPED staging and the
// kernel reads them there (a copy command costs ~15 us of latency per call
// before the kernel can start; DESIGN.md section 5, host-resident per call).
// The caller's own pinned memory is not read in place: hipHostMalloc's
// default allocation is not guaranteed to be mapped for the device.
// $HDFS_CRC32C_ZERO_COPY_KB overrides the threshold (A/B only; 0 = never).
size_t zero_copy_bytes() {
    static const size_t v = [] {
        const char *e = std::getenv("HDFS_CRC32C_ZERO_COPY_KB");
        const long kb = e ? std::atol(e) : -1;
        return kb >= 0 && kb <= (1 << 20) ? size_t(kb) << 10 : kZeroCopyBytes;
    }();
    return v;
}

// Host pipeline slice size: kSliceBytes, or $HDFS_CRC32C_SLICE_MB (A/B only).
size_t slice_bytes() {
    static const size_t v = [] {
        const char *e = std::getenv("HDFS_CRC32C_SLICE_MB");
        const long mb = e ? std::atol(e) : 0;
        return mb > 0 && mb <= 1024 ? size_t(mb) << 20 : kSliceBytes;
    }();
    return v;
}

}  // namespace

namespace hdfs_crc {

static KParams base_params(const crc32c_ctx *ctx, const void *payload, uint32_t *out, uint32_t flags) {
    KParams p;
    std::memset(&p, 0, sizeof p);
    p.payload = static_cast<const uint8_t *>(payload);
    p.out = out;
    const int ty = (flags & CRC32C_TYPE_CRC32) ? 1 : 0;
    p.table = ctx->d_table[ty];
    p.table_s4 = ctx->d_table_s4[ty];
    p.flags = flags;
    std::memcpy(p.c_lg, ctx->c_lg[ty], sizeof p.c_lg);
    std::memcpy(p.c_small, ctx->c_small[ty], sizeof p.c_small);
    return p;
}

// General tiles or padded power-of-two tiles: both run in the builds with
// the general-tile code (kGeneralItems).
static bool has_general(const HostPlan &hp) {
    for (const FastTile &t : hp.tiles)
        if ((t.meta & (kGeneralTile | kHalfTile)) || tile_pad_bits(t.meta)) return true;
    return false;
}

// Some work item shifts block results by Z^(512 s): power-of-two tiles of
// bpc > 512 (lg > 0), general tiles and the general / spanning items.  A
// batch of bpc-512 tiles only (configs 2, 3, 4) stages the image without
// its Z section: 144 of 152 KiB (full image), 20 of 28 KiB (compact).
static bool needs_z(const HostPlan &hp) {
    if (!hp.gen.empty() || !hp.seg.empty()) return true;
    for (const FastTile &t : hp.tiles)
        if ((t.meta & kGeneralTile) || ((t.meta >> 8) & 0xffu)) return true;
    return false;
}

// Some general tile's full chunks are padded (bpc not a multiple of 512), or
// some tile is a padded power-of-two one.  Such batches run the general build
// with both paths even without shifted tiles: the general-tiles-only build,
// which helps unpadded general tiles (412-byte tails: 48.2 -> 46.2 us), was
// measured slower for padded ones (bpc 1000: 62.8 -> 64.3 us, same box, 3
// rounds; padded power-of-two tiles of bpc 2000, kbench: 48.46 against
// 46.77 us, round 5).
static bool has_padded_general(const HostPlan &hp) {
    static const bool off = [] {  // (A/B: HDFS_CRC32C_PADDED_FULL=0 sends them to the general-tiles-only build)
        const char *e = std::getenv("HDFS_CRC32C_PADDED_FULL");
        return e && e[0] == '0';
    }();
    if (off) return false;
    for (const FastTile &t : hp.tiles)
        if (tile_pad_bits(t.meta) && !(t.meta & kHalfTile)) return true;  // (general or padded power-of-two tiles)
    return false;
}

static bool has_padded_tiles(const HostPlan &hp) {
    for (const FastTile &t : hp.tiles)
        if (!(t.meta & (kGeneralTile | kHalfTile)) && tile_pad_bits(t.meta)) return true;
    return false;
}

static bool has_half(const HostPlan &hp) {
    for (const FastTile &t : hp.tiles)
        if ((t.meta & (kGeneralTile | kHalfTile)) == kHalfTile) return true;
    return false;
}

// Some power-of-two tile starts off 16-byte alignment (the general build's
// shifted loads read it from the aligned address below).
static bool has_misaligned(const HostPlan &hp) {
    for (const FastTile &t : hp.tiles)
        if (!(t.meta & (kGeneralTile | kHalfTile)) && !tile_pad_bits(t.meta) && (t.src & 15u)) return true;
    return false;
}

KParams plan_params(const crc32c_plan *plan, const void *payload, uint32_t *out) {
    KParams p = base_params(plan->ctx, payload, out, plan->flags);
    const DevicePlan &dp = plan->dp;
    p.tiles = reinterpret_cast<const FastTile *>(dp.d + dp.tiles_off);
    p.gen = reinterpret_cast<const GenItem *>(dp.d + dp.gen_off);
    p.seg = reinterpret_cast<const SegItem *>(dp.d + dp.seg_off);
    p.pieces = reinterpret_cast<const GenPiece *>(dp.d + dp.pieces_off);
    p.consts = reinterpret_cast<const ConstRun *>(dp.d + dp.consts_off);
    p.ntiles = dp.ntiles;
    p.ngen = dp.ngen;
    p.nseg = dp.nseg;
    p.nconst = dp.nconst;
    // the general builds: general tiles (bit 0), shifted loads of tiles off 16-byte alignment (bit 1)
    p.general = (dp.general ? kGeneralItems : 0u) |
                ((dp.misaligned || (dp.padded && !dp.half) || (reinterpret_cast<uintptr_t>(p.payload) & 15u))
                     ? kGeneralShift
                     : 0u) |
                (dp.half ? kGeneralHalf : 0u) | (dp.padtiles ? kGeneralPadded : 0u);
    p.skip_z = dp.needs_z ? 0u : 1u;
    p.done_ctr = plan->counted ? reinterpret_cast<unsigned long long *>(dp.d + kDoneCtrOff) : nullptr;
    return p;
}

namespace {

size_t pool_class(size_t bytes) {
    size_t c = 4096;
    while (c < bytes) c <<= 1;
    return c;
}

hipEvent_t take_event(crc32c_ctx *ctx) {  // caller holds ctx->pool_mu
    if (ctx->spare_events.empty()) return nullptr;
    hipEvent_t e = ctx->spare_events.back();
    ctx->spare_events.pop_back();
    return e;
}

void drop_block(BlockPool &pool, uint8_t *p) {
    for (size_t i = 0; i < pool.all.size(); ++i)
        if (pool.all[i].first == p) {
            pool.all[i] = pool.all.back();
            pool.all.pop_back();
            return;
        }
}

// Moves every release whose events have all completed back into the pools
// (non-blocking queries), then trims the free lists to kFreeBlocksMax.
// Caller holds ctx->pool_mu.
// The launches of a release's plan have all completed: its completion
// counters, read back into its pinned staging block on the upload stream by
// the previous call (a read is issued here when none is in flight), sum to
// the workgroups launched.  Non-blocking.  Caller holds ctx->pool_mu.
bool launches_done(crc32c_ctx *ctx, Release &r) {
    if (!r.d || !r.expected) return true;
    if (r.reading) {
        const hipError_t q = hipEventQuery(r.read_ev);
        if (q == hipErrorNotReady) return false;
        r.reading = false;
        if (q != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        uint64_t sum = 0;
        for (uint32_t k = 0; k < kDoneCtrs; ++k) {
            uint64_t v;
            std::memcpy(&v, r.h + kDoneCtrOff + k * kDoneCtrStride, sizeof v);
            sum += v;
        }
        if (sum >= r.expected) return true;
    }
    if (!r.read_ev && !(r.read_ev = take_event(ctx)) &&
        hipEventCreateWithFlags(&r.read_ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        r.read_ev = nullptr;
        return false;
    }
    if (hipMemcpyAsync(r.h + kDoneCtrOff, r.d + kDoneCtrOff, kDoneCtrs * kDoneCtrStride, hipMemcpyDeviceToHost,
                       ctx->upload_stream) != hipSuccess ||
        hipEventRecord(r.read_ev, ctx->upload_stream) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    r.reading = true;
    return false;
}

void reap_releases(crc32c_ctx *ctx) {
    for (size_t i = 0; i < ctx->releases.size();) {
        Release &r = ctx->releases[i];
        bool done = true;
        for (hipEvent_t e : r.events) {
            const hipError_t q = hipEventQuery(e);
            if (q == hipSuccess) continue;
            if (q != hipErrorNotReady) (void)hipGetLastError();
            done = false;
            break;
        }
        if (!done || !launches_done(ctx, r)) {
            ++i;
            continue;
        }
        if (r.d) ctx->dev_pool.free.emplace_back(r.d, r.dcap);
        if (r.h) ctx->host_pool.free.emplace_back(r.h, r.hcap);
        ctx->spare_events.insert(ctx->spare_events.end(), r.events.begin(), r.events.end());
        if (r.read_ev) ctx->spare_events.push_back(r.read_ev);
        ctx->releases[i] = std::move(ctx->releases.back());
        ctx->releases.pop_back();
    }
    while (ctx->dev_pool.free.size() > kFreeBlocksMax) {  // stream-ordered: no device synchronisation
        uint8_t *p = ctx->dev_pool.free.front().first;
        ctx->dev_pool.free.erase(ctx->dev_pool.free.begin());
        drop_block(ctx->dev_pool, p);
        (void)hipFreeAsync(p, ctx->upload_stream);
    }
    while (ctx->host_pool.free.size() > kFreeBlocksMax) {
        uint8_t *p = ctx->host_pool.free.front().first;
        ctx->host_pool.free.erase(ctx->host_pool.free.begin());
        drop_block(ctx->host_pool, p);
        (void)hipHostFree(p);
    }
}

// A block of at least `bytes` from the pool (caller holds ctx->pool_mu and
// has reaped the releases).  New device blocks come from the stream-ordered
// allocator on the upload stream (the upload that fills them follows on the
// same stream; every launch waits for that upload).
int pool_get(crc32c_ctx *ctx, BlockPool &pool, size_t bytes, uint8_t **out, size_t *cap) {
    const size_t c = pool_class(bytes);
    for (size_t i = 0; i < pool.free.size(); ++i)
        if (pool.free[i].second == c) {
            *out = pool.free[i].first;
            *cap = c;
            pool.free[i] = pool.free.back();
            pool.free.pop_back();
            return 0;
        }
    uint8_t *p = nullptr;
    if (pool.pinned)
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&p), c, hipHostMallocDefault));
    else
        HIP_TRY(hipMallocAsync(reinterpret_cast<void **>(&p), c, ctx->upload_stream));
    pool.all.emplace_back(p, c);
    *out = p;
    *cap = c;
    return 0;
}

}  // namespace

int upload_plan(crc32c_ctx *ctx, const HostPlan &hp, DevicePlan *dp) {
    if (hp.tiles.size() > UINT32_MAX || hp.gen.size() > UINT32_MAX || hp.seg.size() > UINT32_MAX ||
        hp.consts.size() > UINT32_MAX)
        return fail(-E2BIG, "batch too large");
    dp->ntiles = uint32_t(hp.tiles.size());
    dp->ngen = uint32_t(hp.gen.size());
    dp->nseg = uint32_t(hp.seg.size());
    dp->nconst = uint32_t(hp.consts.size());
    dp->general = has_general(hp);
    dp->misaligned = has_misaligned(hp);
    dp->padded = has_padded_general(hp);
    dp->half = has_half(hp);
    dp->padtiles = has_padded_tiles(hp);
    dp->needs_z = needs_z(hp);
    dp->gen_pow2 = true;
    for (const FastTile &t : hp.tiles)
        if ((t.meta & (kGeneralTile | kHalfTile)) == kGeneralTile) {
            const uint32_t k = (t.meta >> 8) & 31u, pad = (t.meta >> 18) & 511u;  // (crc32c_general.h gshape)
            if (pad || !k || (k & (k - 1u))) dp->gen_pow2 = false;
        }
    dp->slots_off = 0;  // the verify slot first, the completion counters, then the work items
    static_assert(kSlotWords * sizeof(uint32_t) <= kDoneCtrOff, "the verify slot precedes the counters");
    dp->tiles_off = kPlanHeadBytes;
    dp->gen_off = dp->tiles_off + hp.tiles.size() * sizeof(FastTile);
    dp->seg_off = dp->gen_off + hp.gen.size() * sizeof(GenItem);
    dp->pieces_off = dp->seg_off + hp.seg.size() * sizeof(SegItem);
    dp->consts_off = dp->pieces_off + hp.pieces.size() * sizeof(GenPiece);
    const size_t bytes = dp->consts_off + hp.consts.size() * sizeof(ConstRun);
    RelaxedCapture relaxed;  // (another thread may be capturing a graph)
    {
        std::lock_guard<std::mutex> lock(ctx->pool_mu);
        reap_releases(ctx);
        if (int rc = pool_get(ctx, ctx->dev_pool, bytes, &dp->d, &dp->cap)) return rc;
        if (int rc = pool_get(ctx, ctx->host_pool, bytes, &dp->h, &dp->hcap)) return rc;
        dp->uploaded = take_event(ctx);
    }
    if (!dp->uploaded) HIP_TRY(hipEventCreateWithFlags(&dp->uploaded, hipEventDisableTiming));
    uint8_t *img = dp->h;
    init_sched_slots(reinterpret_cast<uint32_t *>(img + dp->slots_off));
    std::memset(img + kDoneCtrOff, 0, kDoneCtrs * kDoneCtrStride);
    ResShape rs{};
    rs.tiles = reinterpret_cast<const FastTile *>(dp->d + dp->tiles_off);
    rs.gen = reinterpret_cast<const GenItem *>(dp->d + dp->gen_off);
    rs.ntiles = dp->ntiles;
    rs.ngen = dp->ngen;
    rs.simple = (!dp->ngen && !dp->misaligned && !dp->general) ? 1u : 0u;
    std::memcpy(img + kResShapeOff, &rs, sizeof rs);
    std::memcpy(img + dp->tiles_off, hp.tiles.data(), hp.tiles.size() * sizeof(FastTile));
    std::memcpy(img + dp->gen_off, hp.gen.data(), hp.gen.size() * sizeof(GenItem));
    std::memcpy(img + dp->seg_off, hp.seg.data(), hp.seg.size() * sizeof(SegItem));
    std::memcpy(img + dp->pieces_off, hp.pieces.data(), hp.pieces.size() * sizeof(GenPiece));
    std::memcpy(img + dp->consts_off, hp.consts.data(), hp.consts.size() * sizeof(ConstRun));
    HIP_TRY(hipMemcpyAsync(dp->d, img, bytes, hipMemcpyHostToDevice, ctx->upload_stream));
    HIP_TRY(hipEventRecord(dp->uploaded, ctx->upload_stream));
    dp->ready.store(false, std::memory_order_release);
    return 0;
}

// Orders a launch on `stream` after the plan's upload: nothing once the
// upload is known complete; else a stream wait on its event (or, while the
// stream is being captured into a graph, a host wait: a capture cannot wait
// on work outside it).
int prepare_launch(crc32c_plan *plan, hipStream_t stream, bool *capturing_out) {
    RelaxedCapture relaxed;  // (the queries below while another thread captures a graph)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(stream, &cs));
    const bool capturing = cs != hipStreamCaptureStatusNone;
    if (capturing) plan->captured = true;
    if (capturing_out) *capturing_out = capturing;
    if (!plan->counted &&
        std::find(plan->launch_streams.begin(), plan->launch_streams.end(), stream) == plan->launch_streams.end())
        plan->launch_streams.push_back(stream);
    DevicePlan *dp = &plan->dp;
    if (!dp->ready.load(std::memory_order_acquire) && dp->uploaded) {
        const hipError_t q = hipEventQuery(dp->uploaded);
        if (q == hipSuccess) {
            dp->ready.store(true, std::memory_order_release);
        } else {
            if (q != hipErrorNotReady) HIP_TRY(q);
            if (capturing) {
                HIP_TRY(hipEventSynchronize(dp->uploaded));
                dp->ready.store(true, std::memory_order_release);
            } else {
                HIP_TRY(hipStreamWaitEvent(stream, dp->uploaded, 0));
            }
        }
    }
    return 0;
}

void plan_forget_stream(crc32c_plan *plan, hipStream_t stream) {
    std::lock_guard<std::mutex> lock(plan->mu);
    auto &v = plan->launch_streams;
    v.erase(std::remove(v.begin(), v.end(), stream), v.end());
}

void release_plan_blocks(crc32c_plan *plan) {
    crc32c_ctx *ctx = plan->ctx;
    DevicePlan *dp = &plan->dp;
    RelaxedCapture relaxed;
    Release r;
    r.d = dp->d;
    r.dcap = dp->cap;
    r.h = dp->h;
    r.hcap = dp->hcap;
    bool held = plan->captured || plan->unaccounted;
    if (plan->counted) {
        // (no stream of the plan's launches is touched: the completion
        // counters tell when they are done, reap_releases)
        r.expected = plan->wgs_issued;
        held = held || (r.expected && !r.h);
    }
    // Per launch stream: nothing when it is idle (its launches of the plan
    // are done -- the usual case: exec, synchronise, destroy), else an event
    // recorded now (it completes after them).  The streams must still exist:
    // a plan without CRC32C_COUNT_COMPLETION is destroyed before the streams
    // it was launched on.
    for (hipStream_t s : plan->launch_streams) {
        if (held) break;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
            (void)hipGetLastError();
            held = true;  // (a capture in progress on it may hold the plan's launches)
            break;
        }
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) continue;
        if (q != hipErrorNotReady) {
            (void)hipGetLastError();
            held = true;
            break;
        }
        hipEvent_t e = nullptr;
        {
            std::lock_guard<std::mutex> lock(ctx->pool_mu);
            e = take_event(ctx);
        }
        if ((!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) || hipEventRecord(e, s) != hipSuccess) {
            (void)hipGetLastError();
            if (e) {
                std::lock_guard<std::mutex> lock(ctx->pool_mu);
                ctx->spare_events.push_back(e);
            }
            held = true;
            break;
        }
        r.events.push_back(e);
    }
    plan->launch_streams.clear();
    if (dp->uploaded) r.events.push_back(dp->uploaded);
    std::lock_guard<std::mutex> lock(ctx->pool_mu);
    if (held && r.d) {
        ctx->held.emplace_back(r.d, r.dcap);
        drop_block(ctx->dev_pool, r.d);
        r.d = nullptr;
    }
    ctx->releases.push_back(std::move(r));
    dp->d = dp->h = nullptr;
    dp->cap = dp->hcap = 0;
    dp->uploaded = nullptr;
}

// Context teardown (every plan destroyed): waits for the releases, then
// frees every pooled block and spare event.
void release_pools(crc32c_ctx *ctx) {
    std::lock_guard<std::mutex> lock(ctx->pool_mu);
    for (Release &r : ctx->releases)
        for (hipEvent_t e : r.events) (void)hipEventSynchronize(e);
    // the destroyed plans' launches: their counters read back until they are
    // complete (bounded: after 10 s the device is synchronised instead)
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    for (;;) {
        reap_releases(ctx);
        if (ctx->releases.empty()) break;
        if (std::chrono::steady_clock::now() > deadline) {
            (void)hipDeviceSynchronize();
            for (Release &r : ctx->releases) {
                if (r.reading) (void)hipEventSynchronize(r.read_ev);
                r.reading = false;
                r.expected = 0;
            }
            reap_releases(ctx);
            break;
        }
        (void)hipStreamSynchronize(ctx->upload_stream);  // (the read-backs)
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (!ctx->held.empty()) (void)hipDeviceSynchronize();  // (blocks graphs captured; graphs outlived by the context)
    for (auto &b : ctx->dev_pool.all) (void)hipFreeAsync(b.first, ctx->upload_stream);
    for (auto &b : ctx->held) (void)hipFreeAsync(b.first, ctx->upload_stream);
    (void)hipStreamSynchronize(ctx->upload_stream);
    for (auto &b : ctx->host_pool.all) (void)hipHostFree(b.first);
    for (hipEvent_t e : ctx->spare_events) (void)hipEventDestroy(e);
    ctx->dev_pool = BlockPool();
    ctx->host_pool = BlockPool();
    ctx->host_pool.pinned = true;
    ctx->releases.clear();
    ctx->held.clear();
    ctx->spare_events.clear();
}

}  // namespace hdfs_crc

namespace {

int alloc_slots(SchedSlots &s) {
    if (s.d) return 0;
    std::vector<uint32_t> init(kSlotWords);
    init_sched_slots(init.data());
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&s.d), init.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(s.d, init.data(), init.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return 0;
}

// Launches p on `stream`.  Verification launches use the sequence's slot
// (left reset by the previous one); the caller keeps launches on `slots`
// in GPU order.  *grid: the workgroups launched (0: none).
int launch(const crc32c_ctx *ctx, KParams p, SchedSlots &slots, hipStream_t stream, hipEvent_t stop = nullptr,
           uint32_t *grid = nullptr) {
    if (grid) *grid = 0;
    const uint64_t items = uint64_t(p.ntiles) + p.ngen + p.nseg + p.nconst;
    if (!items) {
        if (stop) HIP_TRY(hipEventRecord(stop, stream));
        return 0;
    }
    const bool sched = p.expect != nullptr;
    if (sched) {
        int rc = alloc_slots(slots);
        if (rc) return rc;
        p.sched = slots.d;
    }
    // (A/B knob HDFS_CRC32C_CU_CAP=n: launches size their grid for at most n
    // CUs, leaving the rest to kernels beside them -- an RCCL group
    // overlapping a pipelined multi-plan step; measured no gain)
    static const int cap = [] {
        const char *e = std::getenv("HDFS_CRC32C_CU_CAP");
        return e ? std::atoi(e) : 0;
    }();
    const uint32_t ncu = uint32_t(cap > 0 && cap < ctx->num_cu ? cap : ctx->num_cu);
    HIP_TRY(launch_plan_kernel(p, ncu, stream, stop, grid));
    return 0;
}

// Orders the plan's next verify launch on `stream` after its previous ones:
// when the stream changes, an event recorded on the previous stream now (it
// covers that stream's launches so far) is waited on.  Same stream: nothing
// to do (stream order).  Caller holds plan->mu.
int order_plan_launch(crc32c_plan *plan, hipStream_t stream) {
    if (plan->launched && plan->last_stream != stream) {
        if (!plan->last_done) HIP_TRY(hipEventCreateWithFlags(&plan->last_done, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(plan->last_done, plan->last_stream));
        HIP_TRY(hipStreamWaitEvent(stream, plan->last_done, 0));
    }
    plan->last_stream = stream;
    plan->launched = true;
    return 0;
}

int launch_plan(crc32c_plan *plan, const KParams &p, hipStream_t stream, hipEvent_t stop = nullptr) {
    std::lock_guard<std::mutex> lock(plan->mu);
    bool capturing = false;
    if (int rc = prepare_launch(plan, stream, &capturing)) return rc;
    if (p.expect) {  // only verify launches use the plan's scheduler slots
        int rc = order_plan_launch(plan, stream);
        if (rc) return rc;
        // (the mismatch bitmap is cleared by the launch itself, after that
        // wait: a previous verify still setting bits in it has finished)
    }
    uint32_t grid = 0;
    const int rc = launch(plan->ctx, p, plan->sched, stream, stop, &grid);
    // (its workgroups count themselves into the plan's completion counters;
    // a captured launch's plan block is never reused anyway)
    if (!rc && !capturing) plan->wgs_issued += grid;
    return rc;
}

constexpr uint32_t kKnownFlags =
    CRC32C_BIG_ENDIAN | CRC32C_TYPE_CRC32 | CRC32C_DEVICE_ADDRESSES | CRC32C_CPU_FALLBACK | CRC32C_COUNT_COMPLETION;

int check_flags(uint32_t flags) {
    if (flags & ~kKnownFlags) return fail(-EINVAL, "unknown flags 0x%x", flags & ~kKnownFlags);
    return 0;
}

int check_packets(const crc32c_packet *pkts, size_t npkts) {
    if (npkts && !pkts) return fail(-EINVAL, "packets == NULL");
    for (size_t i = 0; i < npkts; ++i)
        if (pkts[i].len && pkts[i].bpc == 0) return fail(-EINVAL, "packet %zu: bytesPerChecksum == 0", i);
    return 0;
}

// Device buffer of at least `need` bytes.
int grow_device(uint8_t **d, size_t *cap, size_t need) {
    if (*cap >= need) return 0;
    if (*d) (void)hipFree(*d);
    *d = nullptr;
    *cap = 0;
    const size_t c = std::max(need, size_t(4096));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(d), c));
    *cap = c;
    return 0;
}

// Pinned host buffer of at least `need` bytes.
int grow_pinned(uint8_t **h, size_t *cap, size_t need) {
    if (*cap >= need) return 0;
    if (*h) (void)hipHostFree(*h);
    *h = nullptr;
    *cap = 0;
    const size_t c = std::max(need, size_t(4096));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(h), c, hipHostMallocDefault));
    *cap = c;
    return 0;
}

// Pinned, device-mapped host buffer of at least `need` bytes.
template <typename T>
int grow_mapped(T **h, T **d, size_t *cap, size_t need) {
    if (*cap >= need) return 0;
    if (*h) (void)hipHostFree(*h);
    *h = nullptr;
    *d = nullptr;
    *cap = 0;
    const size_t c = std::max(need, size_t(4096));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(h), c * sizeof(T), hipHostMallocMapped));
    void *dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, *h, 0));
    *d = static_cast<T *>(dp);
    *cap = c;
    return 0;
}

void free_stage(Stage &s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.h_payload) (void)hipHostFree(s.h_payload);
    if (s.h_zc) (void)hipHostFree(s.h_zc);  // d_zc is its mapping
    if (s.d_payload) (void)hipFree(s.d_payload);
    if (s.h_desc) (void)hipHostFree(s.h_desc);  // d_desc is its mapping
    if (s.h_out) (void)hipHostFree(s.h_out);  // d_out is its mapping
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.sched.d) (void)hipFree(s.sched.d);
    s = Stage();
}

// Completes the slice in flight on `s`: wait (polled: the caller blocks
// anyway, and a polled wait returns as soon as the kernel ends), then
// scatter its checksums.
int drain_stage(Stage &s, uint32_t *out) {
    if (!s.pending) return 0;
    s.pending = false;
    hipError_t e;
    while ((e = hipEventQuery(s.done)) == hipErrorNotReady) std::this_thread::yield();
    HIP_TRY(e);
    for (size_t i = 0; i + 2 < s.scatter.size(); i += 3)
        std::memcpy(out + s.scatter[i], s.h_out + s.scatter[i + 1], s.scatter[i + 2] * sizeof(uint32_t));
    s.scatter.clear();
    return 0;
}

bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Host-resident batch on one context (caller holds ctx->mu).
int batch_host_locked(crc32c_ctx *ctx, const uint8_t *payload, const crc32c_packet *pkts, size_t npkts,
                      uint32_t *out, uint32_t flags) {
    DeviceGuard guard(ctx->device);
    if (!ctx->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    for (Stage &s : ctx->stage) {
        if (!s.stream) {
            HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
        }
    }
    const bool pinned = npkts && is_pinned(payload);
    size_t i = 0;
    int which = 0;
    std::vector<crc32c_packet> local;
    std::vector<std::pair<uint64_t, uint64_t>> runs;  // [begin, end) payload ranges copied one by one
    std::vector<uint32_t> run_of;                     // run of each packet of the slice
    std::vector<uint64_t> run_dst;                    // device offset of each run
    std::vector<uint64_t> src_off;                    // gather: source offset of each packet
    HostPlan plan;
    while (i < npkts) {
        // Slice = consecutive packets totalling about slice_bytes().
        size_t j = i;
        uint64_t bytes = 0, lo = UINT64_MAX, hi = 0;
        while (j < npkts && (j == i || bytes + pkts[j].len <= slice_bytes())) {
            bytes += pkts[j].len;
            if (pkts[j].len) {
                lo = std::min<uint64_t>(lo, pkts[j].payload_off);
                hi = std::max<uint64_t>(hi, pkts[j].payload_off + pkts[j].len);
            }
            ++j;
        }
        Stage &s = ctx->stage[which];
        int rc = drain_stage(s, out);
        if (rc) return rc;
        if (lo == UINT64_MAX) lo = hi = 0;
        lo &= ~uint64_t(15);  // keep every packet's 16-byte phase (fast-path alignment)
        // Contiguous-enough slices move as one range (direct from pinned
        // memory, else through the pinned staging buffer).  Scattered
        // packets from pinned memory move as one copy per contiguous run when
        // the runs are long (an HDFS block per run, e.g. crc32c_multi's
        // round-robin shards); otherwise they are gathered packet by packet
        // into the staging buffer by the CPU.
        const bool ranged = (hi - lo) <= bytes + bytes / 4 + 4096;
        runs.clear();
        run_of.assign(j - i, 0);
        if (!ranged && pinned) {
            for (size_t k = i; k < j; ++k) {
                if (!pkts[k].len) continue;
                const uint64_t b0 = pkts[k].payload_off, b1 = b0 + pkts[k].len;
                if (!runs.empty() && b0 >= runs.back().second && b0 <= runs.back().second + 4096)
                    runs.back().second = b1;
                else
                    runs.emplace_back(b0, b1);
                run_of[k - i] = uint32_t(runs.size() - 1);
            }
            if (runs.empty() || bytes / runs.size() < kMinRunBytes) runs.clear();
        }
        const bool by_runs = !runs.empty();
        size_t stage_bytes = ranged ? size_t(hi - lo) : size_t(bytes + 16 * (j - i));
        if (by_runs) {
            stage_bytes = 0;
            for (const auto &r : runs) stage_bytes += size_t(r.second - (r.first & ~uint64_t(15))) + 16;
        }
        // 1. The payload copy goes first: it needs no plan, and the copy
        //    stream runs the slices' copies back to back.  (This stage's
        //    previous kernel is done: drain_stage waited for it.)
        //    A small batch (one slice) is not copied: the kernel reads it in
        //    host memory (zero copy), and no device or pinned staging is
        //    grown for it.
        // (pinned input: only small batches -- a CPU copy of 1 MiB already
        // costs what the copy command saves; 64 KiB: 22 vs 40 us per call)
        const bool zero_copy = ranged && i == 0 && j == npkts &&
                               (hi - lo) <= (pinned ? zero_copy_bytes() / 4 : zero_copy_bytes());
        if (!zero_copy) {
            rc = grow_device(&s.d_payload, &s.payload_cap, stage_bytes + 16);
            if (!rc && !(pinned && (ranged || by_runs)))
                rc = grow_pinned(&s.h_payload, &s.staging_cap, stage_bytes + 16);
            if (rc) return rc;
        }
        local.assign(pkts + i, pkts + j);
        const uint8_t *kpayload = s.d_payload;
        if (zero_copy) {  // (into mapped staging, which the kernel reads in place)
            rc = grow_mapped(&s.h_zc, &s.d_zc, &s.zc_cap, stage_bytes + 16);
            if (rc) return rc;
            copy_range(s.h_zc, payload + lo, stage_bytes);
            kpayload = s.d_zc;
        }
        if (zero_copy) {
            for (crc32c_packet &pk : local) pk.payload_off -= lo;
        } else if (ranged) {
            for (crc32c_packet &pk : local) pk.payload_off -= lo;
            if (pinned) {
                HIP_TRY(hipMemcpyAsync(s.d_payload, payload + lo, stage_bytes, hipMemcpyHostToDevice,
                                       ctx->copy_stream));
            } else if (i == 0) {
                // nothing to overlap the first slice's staging with: copy it
                // H2D piece by piece as the pieces are staged
                hipError_t err = hipSuccess;
                copy_range_pipelined(s.h_payload, payload + lo, stage_bytes, kFirstPieceBytes,
                                     [&](size_t o, size_t n) {
                                         if (err == hipSuccess)
                                             err = hipMemcpyAsync(s.d_payload + o, s.h_payload + o, n,
                                                                  hipMemcpyHostToDevice, ctx->copy_stream);
                                     });
                HIP_TRY(err);
            } else {
                copy_range(s.h_payload, payload + lo, stage_bytes);
                HIP_TRY(hipMemcpyAsync(s.d_payload, s.h_payload, stage_bytes, hipMemcpyHostToDevice,
                                       ctx->copy_stream));
            }
        } else if (by_runs) {
            // run r (from a0 = its start rounded down to 16) lands at
            // run_dst[r], keeping its 16-byte phase (fast-path alignment)
            run_dst.resize(runs.size());
            uint64_t dst = 0;
            for (size_t r = 0; r < runs.size(); ++r) {
                const uint64_t a0 = runs[r].first & ~uint64_t(15);
                HIP_TRY(hipMemcpyAsync(s.d_payload + dst, payload + a0, size_t(runs[r].second - a0),
                                       hipMemcpyHostToDevice, ctx->copy_stream));
                run_dst[r] = dst;
                dst += (runs[r].second - a0 + 15) & ~uint64_t(15);
            }
            for (size_t k = 0; k < local.size(); ++k) {
                crc32c_packet &pk = local[k];
                const uint32_t r = run_of[k];
                pk.payload_off = pk.len ? run_dst[r] + (pk.payload_off - (runs[r].first & ~uint64_t(15))) : 0;
            }
        } else {
            uint64_t gather_off = 0;
            src_off.resize(local.size());
            for (size_t k = 0; k < local.size(); ++k) {
                src_off[k] = local[k].payload_off;
                local[k].payload_off = gather_off;
                gather_off = (gather_off + local[k].len + 15) & ~uint64_t(15);
            }
            parallel_copy(local.size(), size_t(bytes), [&](size_t b, size_t e) {
                for (size_t k = b; k < e; ++k)
                    std::memcpy(s.h_payload + local[k].payload_off, payload + src_off[k], local[k].len);
            });
            HIP_TRY(hipMemcpyAsync(s.d_payload, s.h_payload, stage_bytes, hipMemcpyHostToDevice, ctx->copy_stream));
        }
        if (!zero_copy) HIP_TRY(hipEventRecord(s.copied, ctx->copy_stream));
        // 2. Plan and descriptors while the copy runs.
        uint64_t nout = 0;
        s.scatter.clear();
        for (size_t k = 0; k < local.size(); ++k) {
            const uint64_t n = crc32c_nchunks(local[k].len, local[k].bpc);
            s.scatter.push_back(pkts[i + k].out_idx);
            s.scatter.push_back(nout);
            s.scatter.push_back(n);
            local[k].out_idx = nout;
            nout += n;
        }
        rc = build_plan(local.data(), local.size(), &plan);
        if (rc) return fail(rc, "invalid packet in batch");
        const size_t desc_bytes = (plan.tiles.size() + plan.gen.size()) * 16;
        rc = grow_mapped(&s.h_desc, &s.d_desc, &s.desc_cap, desc_bytes + 16);
        if (rc) return rc;
        rc = grow_mapped(&s.h_out, &s.d_out, &s.out_cap, size_t(nout) + 1);
        if (rc) return rc;
        std::memcpy(s.h_desc, plan.tiles.data(), plan.tiles.size() * 16);
        std::memcpy(s.h_desc + plan.tiles.size() * 16, plan.gen.data(), plan.gen.size() * 16);
        // 3. Kernel and checksums on the stage's stream, after the copy.
        if (!zero_copy) HIP_TRY(hipStreamWaitEvent(s.stream, s.copied, 0));
        KParams p = base_params(ctx, kpayload, s.d_out, flags);
        p.tiles = reinterpret_cast<const FastTile *>(s.d_desc);
        p.gen = reinterpret_cast<const GenItem *>(s.d_desc + plan.tiles.size() * 16);
        p.ntiles = uint32_t(plan.tiles.size());
        p.ngen = uint32_t(plan.gen.size());
        // (the staged slices keep every packet's 16-byte phase: tiles off
        // alignment take the general build's shifted loads, as in plans)
        p.general = (has_general(plan) ? kGeneralItems : 0u) |
                    ((has_misaligned(plan) || (has_padded_general(plan) && !has_half(plan))) ? kGeneralShift : 0u) |
                    (has_half(plan) ? kGeneralHalf : 0u) | (has_padded_tiles(plan) ? kGeneralPadded : 0u);
        p.skip_z = needs_z(plan) ? 0u : 1u;
        rc = launch(ctx, p, s.sched, s.stream);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(s.done, s.stream));
        s.pending = true;
        which ^= 1;
        i = j;
    }
    for (Stage &s : ctx->stage) {
        int rc = drain_stage(s, out);
        if (rc) return rc;
    }
    return 0;
}

std::once_flag g_default_once;
crc32c_ctx *g_default_ctx = nullptr;
int g_default_rc = 0;

// Host-resident batch with the context lock held and the stages reset on failure.
int batch_host(crc32c_ctx *ctx, const void *payload, const crc32c_packet *pkts, size_t npkts, uint32_t *out,
               uint32_t flags) {
    std::lock_guard<std::mutex> lock(ctx->mu);
    int rc = batch_host_locked(ctx, static_cast<const uint8_t *>(payload), pkts, npkts, out, flags);
    if (rc) {
        if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
        for (Stage &s : ctx->stage) {
            s.pending = false;
            s.scatter.clear();
            if (s.stream) (void)hipStreamSynchronize(s.stream);
        }
    }
    return rc;
}

// CRC32C_CPU_FALLBACK: the host CPU path over the same packets (the
// product's crc32c_chunks_cpu, never the test oracle).
int batch_cpu(const void *payload, const crc32c_packet *pkts, size_t npkts, uint32_t *out, uint32_t flags) {
    const uint32_t f = flags & (CRC32C_BIG_ENDIAN | CRC32C_TYPE_CRC32);
    for (size_t i = 0; i < npkts; ++i) {
        if (!pkts[i].len) continue;
        const int rc = crc32c_chunks_cpu(static_cast<const uint8_t *>(payload) + pkts[i].payload_off, pkts[i].len,
                                         pkts[i].bpc, out + pkts[i].out_idx, f);
        if (rc) return rc;
    }
    g_last_path = CRC32C_PATH_CPU;
    return 0;
}

}  // namespace

namespace hdfs_crc {

int make_plan(crc32c_ctx *ctx, const HostPlan &hp, uint32_t flags, bool absolute, uint64_t abs_base,
              crc32c_plan **out) {
    std::unique_ptr<crc32c_plan, int (*)(crc32c_plan *)> p(new crc32c_plan, crc32c_plan_destroy);
    p->ctx = ctx;
    ctx->refs.fetch_add(1, std::memory_order_relaxed);  // (released by crc32c_plan_destroy)
    p->nchecksums = hp.nchecksums;
    p->payload_bytes = hp.payload_bytes;
    p->flags = flags & (CRC32C_BIG_ENDIAN | CRC32C_TYPE_CRC32);
    p->counted = (flags & CRC32C_COUNT_COMPLETION) != 0;
    p->abs_base = abs_base;
    p->absolute = absolute;
    DeviceGuard guard(ctx->device);
    if (int rc = upload_plan(ctx, hp, &p->dp)) return rc;
    p->sched.d = reinterpret_cast<uint32_t *>(p->dp.d + p->dp.slots_off);  // uploaded initialised with the items
    *out = p.release();
    return 0;
}

}  // namespace hdfs_crc

extern "C" {

int crc32c_last_path(void) { return g_last_path; }

int crc32c_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

}  // extern "C"

namespace {
void reap_zombies(bool block);
}  // namespace

extern "C" {

int crc32c_ctx_create(int device, crc32c_ctx **out) {
    if (!out) return fail(-EINVAL, "out == NULL");
    *out = nullptr;
    reap_zombies(false);  // (contexts a plan's destroy left for later, whose work is done)
    const int ndev = crc32c_device_count();
    if (ndev <= 0) return fail(-ENODEV, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(-ENODEV, "device %d out of range (%d visible)", device, ndev);
    // A failure part-way releases what was already allocated.
    std::unique_ptr<crc32c_ctx, int (*)(crc32c_ctx *)> c(new crc32c_ctx, crc32c_ctx_destroy);
    c->device = device;
    DeviceGuard guard(device);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(-ENODEV, "device %d is %s; this library is built for gfx950 (MI355X)", device, prop.gcnArchName);
    c->num_cu = prop.multiProcessorCount;
    HIP_TRY(preload_plan_kernels());
    c->host_pool.pinned = true;
    HIP_TRY(hipStreamCreateWithFlags(&c->upload_stream, hipStreamNonBlocking));
    for (int ty = 0; ty < 2; ++ty) {
        const uint32_t poly = ty ? kPolyIeee : kPoly;
        std::vector<uint8_t> img(kTableAlloc, 0);
        build_lds_image(img.data(), poly);
        affine_constants(c->c_lg[ty], c->c_small[ty], poly);
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&c->d_table[ty]), kTableAlloc));
        HIP_TRY(hipMemcpy(c->d_table[ty], img.data(), kTableAlloc, hipMemcpyHostToDevice));
        std::vector<uint8_t> img4(kTableAllocS4Full, 0);
        build_lds_image_s4(img4.data(), poly);
        compact_s4_image(img4.data(), img4.data() + kS4COff);  // small batches
        zero_crc_table(reinterpret_cast<uint32_t *>(img4.data() + kZeroCrcOff), poly);  // general items
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&c->d_table_s4[ty]), kTableAllocS4Full));
        HIP_TRY(hipMemcpy(c->d_table_s4[ty], img4.data(), kTableAllocS4Full, hipMemcpyHostToDevice));
    }
    *out = c.release();
    return 0;
}

}  // extern "C"

namespace {

// The context's teardown, when its last reference goes.
void ctx_teardown(crc32c_ctx *ctx) {
    {
        DeviceGuard guard(ctx->device);
        for (Stage &s : ctx->stage) free_stage(s);
        if (ctx->copy_stream) {
            (void)hipStreamSynchronize(ctx->copy_stream);
            (void)hipStreamDestroy(ctx->copy_stream);
        }
        if (ctx->upload_stream) {
            release_pools(ctx);  // (waits for the destroyed plans' launches)
            (void)hipStreamDestroy(ctx->upload_stream);
        }
        for (int ty = 0; ty < 2; ++ty) {
            if (ctx->d_table[ty]) (void)hipFree(ctx->d_table[ty]);
            if (ctx->d_table_s4[ty]) (void)hipFree(ctx->d_table_s4[ty]);
        }
    }
    delete ctx;
}

// Contexts whose last reference went with a plan's destroy: torn down by
// the next crc32c_ctx_destroy, or by the next crc32c_ctx_create once their
// destroyed plans' launches are known complete (a non-blocking check, so a
// create never waits for another context's work), or left to process exit
// (plan destroy never synchronises, frees device memory or destroys a
// stream: it may run while another thread captures a graph).
std::mutex g_zombie_mu;
std::vector<crc32c_ctx *> g_zombies;

// Nothing of a zombie's destroyed plans can still be running (non-blocking:
// the release events are queried, counter read-backs issued, not awaited).
bool zombie_idle(crc32c_ctx *ctx) {
    std::lock_guard<std::mutex> lock(ctx->pool_mu);
    reap_releases(ctx);
    return ctx->releases.empty() && ctx->held.empty();
}

void reap_zombies(bool block) {
    std::vector<crc32c_ctx *> z;
    {
        std::lock_guard<std::mutex> lock(g_zombie_mu);
        if (block) {
            z.swap(g_zombies);
        } else {
            for (size_t i = 0; i < g_zombies.size();)
                if (zombie_idle(g_zombies[i])) {
                    z.push_back(g_zombies[i]);
                    g_zombies[i] = g_zombies.back();
                    g_zombies.pop_back();
                } else {
                    ++i;
                }
        }
    }
    for (crc32c_ctx *c : z) ctx_teardown(c);
}

void ctx_release(crc32c_ctx *ctx, bool defer) {
    if (ctx->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    if (defer) {
        std::lock_guard<std::mutex> lock(g_zombie_mu);
        g_zombies.push_back(ctx);
        return;
    }
    ctx_teardown(ctx);
}

}  // namespace

extern "C" {

int crc32c_ctx_destroy(crc32c_ctx *ctx) {
    reap_zombies(true);
    if (!ctx) return 0;
    ctx_release(ctx, false);
    return 0;
}

int crc32c_plan_create(crc32c_ctx *ctx, const crc32c_packet *pkts, size_t npkts, uint32_t flags,
                       crc32c_plan **out) {
    if (!ctx || !out) return fail(-EINVAL, "ctx/out == NULL");
    *out = nullptr;
    int rc = check_flags(flags);
    if (!rc) rc = check_packets(pkts, npkts);
    if (rc) return rc;
    const bool absolute = (flags & CRC32C_DEVICE_ADDRESSES) != 0;
    HostPlan hp;
    rc = build_plan(pkts, npkts, &hp, absolute);
    if (rc) return fail(rc, "invalid packet batch");
    uint64_t base = 0;
    if (absolute) rebase_plan(&hp, &base);  // offsets from the lowest address (16-byte phase kept)
    return make_plan(ctx, hp, flags, absolute, base, out);
}

int crc32c_plan_create_buffers(crc32c_ctx *ctx, const crc32c_buffer *buffers, uint32_t n_buffers,
                               uint64_t bufferoffset, uint64_t len, uint64_t blockoffset, uint32_t packetsize,
                               uint32_t bpc, uint32_t flags, crc32c_plan **out) {
    if (!ctx || !out) return fail(-EINVAL, "ctx/out == NULL");
    *out = nullptr;
    if (int rc = check_flags(flags)) return rc;
    HostPlan hp;
    const uint32_t poly = (flags & CRC32C_TYPE_CRC32) ? kPolyIeee : kPoly;
    int rc = build_write_plan(buffers, n_buffers, bufferoffset, len, blockoffset, packetsize, bpc, poly, &hp);
    if (rc) return fail(rc, "invalid buffer list / write range");
    uint64_t base = 0;
    rebase_plan(&hp, &base);
    return make_plan(ctx, hp, flags, true, base, out);
}

// The payload base a launch passes: the caller's buffer, or for an absolute
// plan its own base (the caller passes NULL).
static int plan_payload(const crc32c_plan *plan, const void **dev_payload) {
    if (!plan->absolute) return 0;
    if (*dev_payload) return fail(-EINVAL, "a device-address plan takes dev_payload = NULL");
    *dev_payload = reinterpret_cast<const void *>(uintptr_t(plan->abs_base));
    return 0;
}

static bool plan_reads_payload(const crc32c_plan *plan) {
    return plan->dp.ntiles || plan->dp.ngen || plan->dp.nseg;
}

int crc32c_plan_exec(crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out, void *stream) {
    if (!plan) return fail(-EINVAL, "plan == NULL");
    if (plan->nchecksums == 0) return 0;
    if (int rc = plan_payload(plan, &dev_payload)) return rc;
    if ((!dev_payload && plan_reads_payload(plan)) || !dev_out) return fail(-EINVAL, "payload/out == NULL");
    DeviceGuard guard(plan->ctx->device);
    return launch_plan(plan, plan_params(plan, dev_payload, dev_out), static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace hdfs_crc {

int exec_blocks(crc32c_plan *plan, const void *const *dev_payloads, uint32_t *const *dev_outs, size_t nblocks,
                hipStream_t s, hipEvent_t stop) {
    if (!plan) return fail(-EINVAL, "plan == NULL");
    if (plan->absolute) return fail(-EINVAL, "a multi-block launch takes a plan of one block's shape, not device addresses");
    if (nblocks && (!dev_payloads || !dev_outs)) return fail(-EINVAL, "payloads/outs == NULL");
    if (plan->nchecksums == 0 || nblocks == 0) {
        if (stop) HIP_TRY(hipEventRecord(stop, s));
        return 0;
    }
    for (size_t i = 0; i < nblocks; ++i)
        if ((!dev_payloads[i] && plan_reads_payload(plan)) || !dev_outs[i] || (uintptr_t(dev_outs[i]) & 3u))
            return fail(-EINVAL, "block %zu: payload NULL, or out NULL / not 4-byte aligned", i);
    DeviceGuard guard(plan->ctx->device);
    const DevicePlan &dp = plan->dp;
    if (dp.ngen || dp.nseg || dp.nconst || dp.ntiles == 0) {
        // (items other than tiles -- tails under 4 bytes, bpc outside [4, 8192]
        // -- have no multi-block form: one launch per block)
        for (size_t i = 0; i < nblocks; ++i)
            if (int rc = launch_plan(plan, plan_params(plan, dev_payloads[i], dev_outs[i]), s,
                                     i + 1 == nblocks ? stop : nullptr))
                return rc;
        return 0;
    }
    const uint64_t max_launch_tiles = UINT32_MAX;
    size_t i = 0;
    while (i < nblocks) {
        // Up to kMaxLaunchBlocks blocks whose payloads and outputs are within
        // reach of the launch's bases: payload deltas below 2^47 (tile
        // offsets keep a tail length in bits 48-63), output indices below 2^32.
        uintptr_t plo = UINTPTR_MAX, olo = UINTPTR_MAX, ohi = 0, phi = 0;
        size_t j = i;
        for (; j < nblocks && j - i < kMaxLaunchBlocks && uint64_t(j - i + 1) * dp.ntiles <= max_launch_tiles; ++j) {
            const uintptr_t pp = uintptr_t(dev_payloads[j]) & ~uintptr_t(15), oo = uintptr_t(dev_outs[j]);
            const uintptr_t nplo = std::min(plo, pp), nphi = std::max(phi, pp);
            const uintptr_t nolo = std::min(olo, oo), nohi = std::max(ohi, oo);
            if (j > i && (nphi - nplo >= (uintptr_t(1) << 47) || (nohi - nolo) / 4 + plan->nchecksums > (1ull << 32)))
                break;
            plo = nplo, phi = nphi, olo = nolo, ohi = nohi;
        }
        KParams p = plan_params(plan, reinterpret_cast<const void *>(plo), reinterpret_cast<uint32_t *>(olo));
        p.nblocks = uint32_t(j - i);
        p.block_tiles = dp.ntiles;
        p.ntiles = uint32_t(uint64_t(j - i) * dp.ntiles);
        for (size_t k = i; k < j; ++k) {
            BlockRef &b = p.blocks[k - i];
            b.payload_delta = uint64_t(uintptr_t(dev_payloads[k]) - plo);
            b.out_delta = uint32_t((uintptr_t(dev_outs[k]) - olo) / 4);
            b.reserved = 0;
            if (b.payload_delta & 15u) p.general |= kGeneralShift;  // (shifted loads for blocks off 16-byte alignment)
        }
        if (int rc = launch_plan(plan, p, s, j == nblocks ? stop : nullptr)) return rc;
        i = j;
    }
    return 0;
}

}  // namespace hdfs_crc

extern "C" {

int crc32c_plan_exec_blocks(crc32c_plan *plan, const void *const *dev_payloads, uint32_t *const *dev_outs,
                            size_t nblocks, void *stream) {
    return exec_blocks(plan, dev_payloads, dev_outs, nblocks, static_cast<hipStream_t>(stream), nullptr);
}

int crc32c_plan_verify(crc32c_plan *plan, const void *dev_payload, const uint32_t *dev_expected,
                       uint32_t *dev_result, void *stream) {
    return crc32c_plan_verify_bitmap(plan, dev_payload, dev_expected, dev_result, nullptr, stream);
}

int crc32c_plan_verify_bitmap(crc32c_plan *plan, const void *dev_payload, const uint32_t *dev_expected,
                              uint32_t *dev_result, uint32_t *dev_bad_bits, void *stream) {
    if (!plan) return fail(-EINVAL, "plan == NULL");
    if (!dev_result) return fail(-EINVAL, "result == NULL");
    DeviceGuard guard(plan->ctx->device);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const DevicePlan &dp = plan->dp;
    if (uint64_t(dp.ntiles) + dp.ngen + dp.nseg + dp.nconst == 0) {  // nothing to compare: set the result directly
        HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(dev_result), 0, 1, s));
        HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(dev_result + 1), 0xffffffff, 1, s));
        return 0;
    }
    if (int rc = plan_payload(plan, &dev_payload)) return rc;
    if ((!dev_payload && plan_reads_payload(plan)) || !dev_expected)
        return fail(-EINVAL, "payload/expected == NULL");
    KParams p = plan_params(plan, dev_payload, nullptr);
    p.expect = dev_expected;
    p.result = dev_result;
    p.bad_bits = dev_bad_bits;
    p.bad_words = dev_bad_bits ? uint32_t((plan->nchecksums + 31) / 32) : 0;
    return launch_plan(plan, p, s);
}

int64_t crc32c_verify_host(crc32c_ctx *ctx, const void *payload, const crc32c_packet *pkts, size_t npkts,
                           const uint32_t *expected, uint32_t flags, uint64_t *first_bad) {
    if (first_bad) *first_bad = UINT64_MAX;
    // (ctx == NULL is a missing GPU: with CRC32C_CPU_FALLBACK crc32c_batch_host
    // then computes on the host CPU)
    if (!ctx && !(flags & CRC32C_CPU_FALLBACK)) return fail(-EINVAL, "ctx == NULL");
    uint64_t n = 0;
    for (size_t i = 0; i < npkts; ++i)
        if (pkts && pkts[i].bpc) n = std::max<uint64_t>(n, pkts[i].out_idx + crc32c_nchunks(pkts[i].len, pkts[i].bpc));
    if (n && !expected) return fail(-EINVAL, "expected == NULL");
    std::vector<uint32_t> got(std::max<uint64_t>(n, 1));
    int rc = crc32c_batch_host(ctx, payload, pkts, npkts, got.data(), flags);
    if (rc) return rc;
    // Only the indices the packets cover are compared (gaps between packets are not checksums).
    int64_t bad = 0;
    uint64_t first = UINT64_MAX;
    for (size_t i = 0; i < npkts; ++i) {
        const uint64_t k0 = pkts[i].out_idx, k1 = k0 + crc32c_nchunks(pkts[i].len, pkts[i].bpc);
        for (uint64_t k = k0; k < k1; ++k)
            if (got[k] != expected[k]) {
                ++bad;
                first = std::min(first, k);
            }
    }
    if (first_bad) *first_bad = first;
    return bad;
}

int crc32c_plan_destroy(crc32c_plan *plan) {
    if (!plan) return 0;
    crc32c_ctx *ctx = plan->ctx;
    {
        DeviceGuard guard(ctx->device);
        release_plan_blocks(plan);  // (the verify slots live in the same block)
        if (plan->last_done) (void)hipEventDestroy(plan->last_done);
    }
    delete plan;
    ctx_release(ctx, true);
    return 0;
}

uint64_t crc32c_plan_nchecksums(const crc32c_plan *plan) { return plan ? plan->nchecksums : 0; }
uint64_t crc32c_debug_plan_block(const crc32c_plan *plan) {
    return plan ? uint64_t(reinterpret_cast<uintptr_t>(plan->dp.d)) : 0;
}
uint64_t crc32c_plan_payload_bytes(const crc32c_plan *plan) { return plan ? plan->payload_bytes : 0; }

int crc32c_chunks_dev(crc32c_ctx *ctx, const crc32c_packet *pkts, size_t npkts, const void *dev_payload,
                      uint32_t *dev_out, uint32_t flags, void *stream) {
    crc32c_plan *plan = nullptr;
    int rc = crc32c_plan_create(ctx, pkts, npkts, flags, &plan);
    if (rc) return rc;
    rc = crc32c_plan_exec(plan, dev_payload, dev_out, stream);
    if (!rc) {
        DeviceGuard guard(ctx->device);
        hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
        if (e != hipSuccess) rc = fail(-EIO, "hipStreamSynchronize: %s", hipGetErrorString(e));
    }
    crc32c_plan_destroy(plan);
    return rc;
}

int crc32c_batch_host(crc32c_ctx *ctx, const void *payload, const crc32c_packet *pkts, size_t npkts,
                      uint32_t *out, uint32_t flags) {
    g_last_path = CRC32C_PATH_NONE;
    int rc = check_flags(flags);
    if (!rc) rc = check_packets(pkts, npkts);
    if (rc) return rc;
    if (flags & CRC32C_DEVICE_ADDRESSES) return fail(-EINVAL, "CRC32C_DEVICE_ADDRESSES is for device-resident plans");
    if (npkts && (!payload || !out)) return fail(-EINVAL, "payload/out == NULL");
    rc = ctx ? batch_host(ctx, payload, pkts, npkts, out, flags) : fail(-ENODEV, "ctx == NULL");
    if (!rc) {
        g_last_path = CRC32C_PATH_GPU;
        return 0;
    }
    if (!(flags & CRC32C_CPU_FALLBACK) || rc == -EINVAL) return rc;
    return batch_cpu(payload, pkts, npkts, out, flags);
}

int crc32c_chunks(const void *packet, size_t len, uint32_t bpc, uint32_t *out, uint32_t flags) {
    g_last_path = CRC32C_PATH_NONE;
    if (bpc == 0) return fail(-EINVAL, "bytesPerChecksum == 0");
    if (int rc = check_flags(flags)) return rc;
    if (len == 0) return 0;
    if (len > UINT32_MAX) return fail(-EINVAL, "packet too large");
    std::call_once(g_default_once, [] {
        const char *env = std::getenv("HDFS_CRC32C_DEVICE");
        g_default_rc = crc32c_ctx_create(env ? std::atoi(env) : 0, &g_default_ctx);
    });
    crc32c_packet p;
    p.payload_off = 0;
    p.out_idx = 0;
    p.len = uint32_t(len);
    p.bpc = bpc;
    if (g_default_rc) {
        const int rc = fail(g_default_rc, "default GPU context unavailable");
        return (flags & CRC32C_CPU_FALLBACK) ? batch_cpu(packet, &p, 1, out, flags) : rc;
    }
    return crc32c_batch_host(g_default_ctx, packet, &p, 1, out, flags);
}

}  // extern "C"
