// runtime_internal.h -- the host runtime's object layouts, shared by the
// product library's runtime files and by the debug library (which links
// against libhdfs_crc32c.so).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <atomic>
#include <mutex>
#include <vector>

#include "errors.h"
#include "hdfs_crc32c.h"
#include "kernel_abi.h"
#include "plan.h"

namespace hdfs_crc_res {
struct RParams;  // resident_engine.h
}

namespace hdfs_crc {

// (fail(): errors.h)

#define HIP_TRY(expr)                                                                                          \
    do {                                                                                                       \
        hipError_t e_ = (expr);                                                                                \
        if (e_ != hipSuccess)                                                                                  \
            return ::hdfs_crc::fail(-EIO, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

// Restores the caller's current device (torch and other libraries keep their own).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// The device verification slot (kernel_abi.h) of one launch sequence that
// the GPU runs in order: a plan, or a host-pipeline stage.
struct SchedSlots {
    uint32_t *d = nullptr;  // kSlotWords u32
};

struct Stage {
    hipStream_t stream = nullptr;
    hipEvent_t copied = nullptr;  // the slice's H2D payload copy (on the context's copy stream) is done
    hipEvent_t done = nullptr;
    uint8_t *d_payload = nullptr;
    size_t payload_cap = 0;
    uint8_t *h_payload = nullptr;  // pinned staging, only for pageable or gathered payloads
    size_t staging_cap = 0;
    // Small pageable batches: pinned, device-MAPPED staging the kernel reads
    // in place (zero copy; d_zc is h_zc's mapping).
    uint8_t *h_zc = nullptr, *d_zc = nullptr;
    size_t zc_cap = 0;
    // Work descriptors: pinned host memory the kernel reads in place (d_desc
    // is its device mapping).  A slice's 64 KiB of descriptors are not worth
    // a copy of their own: on the copy stream each copy costs ~25 us (9 us
    // of transfer plus the ~15 us gap between copy commands).
    uint8_t *h_desc = nullptr, *d_desc = nullptr;
    size_t desc_cap = 0;
    // Checksums: written by the kernel straight into pinned host memory
    // (d_out is h_out's mapping), which saves a D2H copy on the tail.
    uint32_t *h_out = nullptr, *d_out = nullptr;
    size_t out_cap = 0;
    bool pending = false;
    // packets of the slice in flight: (global out_idx, local out index, count)
    std::vector<uint64_t> scatter;
    SchedSlots sched;  // this stage's launches are serialised on its stream
};

// Device copy of a HostPlan's work items and its verify scheduler slots, one
// block of the context's descriptor pool, uploaded asynchronously from a
// pinned staging block on the context's upload stream (`uploaded`).
struct DevicePlan {
    uint8_t *d = nullptr;
    size_t cap = 0;
    uint8_t *h = nullptr;  // pinned staging of the same image
    size_t hcap = 0;
    hipEvent_t uploaded = nullptr;
    std::atomic<bool> ready{false};  // the upload is known complete: launches need no wait
    uint32_t ntiles = 0, ngen = 0, nseg = 0, nconst = 0;
    bool general = false;     // some tile is a general tile
    bool misaligned = false;  // some power-of-two tile's offset is not a multiple of 16
    bool padded = false;      // some general tile's full chunks are padded (bpc not 512 k)
    bool half = false;        // some tile is a half tile (their own builds)
    bool padtiles = false;    // some tile is a padded power-of-two tile (full-image general builds)
    bool needs_z = true;      // some item shifts by Z^(512 s) (the image's last 7.5 KiB)
    bool gen_pow2 = true;     // every general tile's full chunks are 2^lg unpadded blocks (the resident kernel's)
    size_t tiles_off = 0, gen_off = 0, seg_off = 0, pieces_off = 0, consts_off = 0, slots_off = 0;
};

// Blocks of descriptor memory (device) or of its pinned staging (host),
// recycled instead of freed: hipFree costs ~12 us and hipMemcpy from pageable
// memory ~15 us, several times a short plan's whole launch.
struct BlockPool {
    bool pinned = false;
    std::vector<std::pair<uint8_t *, size_t>> free, all;
};
// Free blocks a pool keeps; more are returned (device blocks stream-ordered,
// hipFreeAsync on the upload stream, so no device-wide synchronisation).
constexpr size_t kFreeBlocksMax = 48;

// A destroyed plan's blocks, waiting for the GPU work that may still read
// them: an event recorded at destroy time on every stream the plan was
// launched on that was still busy, and its upload's event -- or, for a
// CRC32C_COUNT_COMPLETION plan, its upload's event and its launches'
// workgroups: the plan's completion counters (kernel_abi.h kDoneCtrOff) must
// sum to `expected`, read back (into the plan's pinned staging block) on the
// context's upload stream, so nothing touches the streams the plan was
// launched on.  Reusable once all of it has completed (queried without
// blocking when a block is next needed) -- no device-wide synchronisation,
// so other streams, other libraries' work and graph captures on other
// threads are never waited on or disturbed.
struct Release {
    uint8_t *d = nullptr, *h = nullptr;  // device block / pinned staging block (either may be null)
    size_t dcap = 0, hcap = 0;
    std::vector<hipEvent_t> events;
    uint64_t expected = 0;          // workgroups launched
    hipEvent_t read_ev = nullptr;   // the counters' read-back
    bool reading = false;           // a read-back is in flight
};

// Makes the calling thread's potentially-unsafe HIP calls (allocation, event
// records) legal while another thread captures a stream in global mode
// (torch.cuda.graph's default); restores the thread's mode on exit.
struct RelaxedCapture {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&mode); }
    ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&mode); }
};

}  // namespace hdfs_crc

struct crc32c_ctx {
    int device = 0;
    int num_cu = 0;
    // The context handle and every live plan hold one reference; the
    // context is torn down when the last goes (a plan destroyed after
    // crc32c_ctx_destroy -- e.g. one a garbage collector frees late -- still
    // returns its block to a live pool instead of a freed one).
    std::atomic<int> refs{1};
    // per checksum type (0 = CRC32C, 1 = CRC32 / CRC32C_TYPE_CRC32)
    uint8_t *d_table[2] = {nullptr, nullptr};
    uint8_t *d_table_s4[2] = {nullptr, nullptr};
    uint32_t c_lg[2][5];
    uint32_t c_small[2][4];
    std::mutex mu;
    // Host pipeline: every stage's H2D copies go on one copy stream, so they
    // run back to back at the full link rate while the other stage's kernel
    // runs on its own stream.  Two copies on two streams would share the
    // link, finish together and leave it idle while both stages drain.
    hipStream_t copy_stream = nullptr;
    hdfs_crc::Stage stage[2];
    // Plan descriptors: pooled device / pinned blocks, the stream their
    // uploads go on, and spare events (all under pool_mu).
    std::mutex pool_mu;
    hdfs_crc::BlockPool dev_pool, host_pool;
    std::vector<hdfs_crc::Release> releases;
    // device blocks of destroyed plans whose launches were captured into a
    // graph: the graph may replay them at any time, so they are never
    // reused (freed with the context)
    std::vector<std::pair<uint8_t *, size_t>> held;
    hipStream_t upload_stream = nullptr;
    std::vector<hipEvent_t> spare_events;
};

struct crc32c_plan {
    crc32c_ctx *ctx = nullptr;
    // Verify launches of a plan share its scheduler slots, so they are kept
    // in GPU order: one on another stream than the previous one first waits
    // for it (last_done).  Exec launches are not ordered.
    std::mutex mu;
    hdfs_crc::SchedSlots sched;
    hipStream_t last_stream = nullptr;
    hipEvent_t last_done = nullptr;
    bool launched = false;
    // Every stream a launch of the plan went on (at destroy time: nothing to
    // do for an idle one, else an event recorded on it gates the block's
    // reuse), and whether a launch went into a graph capture (then the block
    // is never reused).  (Round 3 first gave every launch a stop event to
    // complete instead; that cost every launch)
    std::vector<hipStream_t> launch_streams;
    bool captured = false;
    // CRC32C_COUNT_COMPLETION plans: the workgroups their launches were
    // issued with; their completion counters (kernel_abi.h kDoneCtrOff) gate
    // the block's reuse instead of the streams, so such a plan may be
    // destroyed after its streams.  unaccounted: a launch bypassed the count
    // (debug variants): the block is never reused.
    bool counted = false;
    uint64_t wgs_issued = 0;
    bool unaccounted = false;
    hdfs_crc::DevicePlan dp;
    uint64_t nchecksums = 0, payload_bytes = 0;
    uint32_t flags = 0;
    // Absolute plans (CRC32C_DEVICE_ADDRESSES, crc32c_plan_create_buffers):
    // offsets are relative to this device address (the lowest address read,
    // rounded down to 16), which the launches pass as the payload base.
    uint64_t abs_base = 0;
    bool absolute = false;
};

namespace hdfs_crc {

// Kernel parameters of a plan's launch on (payload, out); checks nothing.
KParams plan_params(const crc32c_plan *plan, const void *payload, uint32_t *out);
// Uploads a HostPlan's items (and fresh verify slots) to the context's
// device (into *dp), asynchronously; plan_ready orders a launch after it.
int upload_plan(crc32c_ctx *ctx, const HostPlan &hp, DevicePlan *dp);
// Before a launch of `plan` on `stream` (caller holds plan->mu): orders it
// after the plan's upload and notes the stream for the plan's release
// (unless the plan counts its completion); *capturing: the stream is being
// captured (the plan is then marked captured: its block is never reused).
int prepare_launch(crc32c_plan *plan, hipStream_t stream, bool *capturing = nullptr);
// `stream` (idle, about to be destroyed by the library itself: a block
// queue's) no longer needs an event at the plan's release.
void plan_forget_stream(crc32c_plan *plan, hipStream_t stream);
// crc32c_plan_exec_blocks; `stop` (optional) is completed by the last launch.
int exec_blocks(crc32c_plan *plan, const void *const *dev_payloads, uint32_t *const *dev_outs, size_t nblocks,
                hipStream_t stream, hipEvent_t stop);
// A destroyed plan's blocks back to the pools once its launches are done.
void release_plan_blocks(crc32c_plan *plan);
// Context teardown: waits for the releases, frees every pooled block.
void release_pools(crc32c_ctx *ctx);
// Creates a plan object from a built HostPlan (absolute: rebased, base given).
int make_plan(crc32c_ctx *ctx, const HostPlan &hp, uint32_t flags, bool absolute, uint64_t abs_base,
              crc32c_plan **out);

// ---- the resident kernel's host side (crc32c_resident.hip; kernel:
// resident_engine.h).  A launcher starts one instance of resident_kernel
// (its shape) with `grid` workgroups on `stream`.
using ResidentLaunch = hipError_t (*)(const hdfs_crc_res::RParams &p, uint32_t grid, hipStream_t stream);
struct ResidentEngine;
// Plans of power-of-two tiles and GenItems (one block's shape: the queue's
// default); idle_us = 0: 2000.  stamps: per-ticket trace (debug A/B).
// launch: the aligned-only build; launch_general: the general build (null:
// blocks that need it are refused).
int resident_create(crc32c_plan *plan, uint32_t idle_us, ResidentLaunch launch, bool stamps, ResidentEngine **out,
                    ResidentLaunch launch_general = nullptr);
// plan == NULL: the queue's plan.  Any payload alignment.
int resident_submit(ResidentEngine *r, crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out,
                    uint64_t *ticket);
int resident_wait(ResidentEngine *r, uint64_t ticket);
// Test hooks: hold = no launch (submits queue up); the next fail_waits
// waits return -ETIMEDOUT at once.
int resident_inject(ResidentEngine *r, bool hold, uint32_t fail_waits);
uint64_t resident_launches(const ResidentEngine *r);
uint64_t resident_tickets(const ResidentEngine *r);
// Ends the running launch (stop word), then copies the trace out.
int resident_trace(ResidentEngine *r, uint64_t *stamps, uint64_t *rtt_ticks, uint64_t *rtt_polls);
// drain: every ticket handed out completes first (a bounded wait each);
// then the stop word, the stream drained, everything freed.  Submits from
// the moment destroy begins are refused.
int resident_destroy(ResidentEngine *r, bool drain);
// The product's shape (16 waves, 7 phases, 2 waves per phase and workgroup):
// its aligned-only and general builds.
hipError_t resident_launch_product(const hdfs_crc_res::RParams &p, uint32_t grid, hipStream_t stream);
hipError_t resident_launch_product_general(const hdfs_crc_res::RParams &p, uint32_t grid, hipStream_t stream);
hipError_t resident_preload_product();

}  // namespace hdfs_crc
