// resident.hip -- A/B shapes of the resident checksum kernel
// (libhdfs_crc32c_debug.so only).  The kernel and its host side are the
// product's (resident_engine.h, crc32c_resident.hip: the block queue's
// resident mode runs the 16 / 7 / 2 shape); this file instantiates the other
// shapes round 4 measured and selects one by environment, with an optional
// per-ticket trace -- neither of which the product library reads:
//   HDFS_CRC32C_RESIDENT_WAVES   12 (12 / 5 / 2, default here), 16 (16 / 7 / 2,
//                                the product's), 12x11 (12 / 11 / 1) or 16x15
//                                (16 / 15 / 1): waves per workgroup / blocks
//                                in flight / worker waves per block
//   HDFS_CRC32C_RESIDENT_STAMPS  1: s_memrealtime per ticket at each hop
//                                (crc32c_debug_resident_trace)
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdlib>
#include <string>

#include "../resident_engine.h"
#include "../runtime_internal.h"
#include "hdfs_crc32c_debug.h"

using namespace hdfs_crc_res;

namespace {

template <uint32_t W, uint32_t P, uint32_t K>
hipError_t launch_shape(const RParams &p, uint32_t grid, hipStream_t stream) {
    hipLaunchKernelGGL((resident_kernel<W, P, K>), dim3(grid), dim3(W * 64), 0, stream, p);
    return hipGetLastError();
}

}  // namespace

struct crc32c_resident {
    hdfs_crc::ResidentEngine *e = nullptr;
};

extern "C" {

int crc32c_debug_resident_create(crc32c_plan *plan, uint32_t idle_us, crc32c_resident **out) {
    if (!out) return hdfs_crc::fail(-EINVAL, "out == NULL");
    *out = nullptr;
    hdfs_crc::ResidentLaunch launch = launch_shape<12, 5, 2>;
    if (const char *w = std::getenv("HDFS_CRC32C_RESIDENT_WAVES")) {
        const std::string s(w);
        if (s == "16") launch = hdfs_crc::resident_launch_product;
        if (s == "12x11") launch = launch_shape<12, 11, 1>;
        if (s == "16x15") launch = launch_shape<16, 15, 1>;
    }
    const char *st = std::getenv("HDFS_CRC32C_RESIDENT_STAMPS");
    crc32c_resident *r = new crc32c_resident;
    if (int rc = hdfs_crc::resident_create(plan, idle_us, launch, st && st[0] == '1', &r->e)) {
        delete r;
        return rc;
    }
    *out = r;
    return 0;
}

int crc32c_debug_resident_submit(crc32c_resident *r, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket) {
    if (!r) return hdfs_crc::fail(-EINVAL, "resident == NULL");
    return hdfs_crc::resident_submit(r->e, nullptr, dev_payload, dev_out, ticket);
}

int crc32c_debug_resident_wait(crc32c_resident *r, uint64_t ticket) {
    if (!r) return hdfs_crc::fail(-EINVAL, "resident == NULL");
    return hdfs_crc::resident_wait(r->e, ticket);
}

int crc32c_debug_resident_stats(const crc32c_resident *r, uint64_t *launches) {
    if (!r) return hdfs_crc::fail(-EINVAL, "resident == NULL");
    if (launches) *launches = hdfs_crc::resident_launches(r->e);
    return 0;
}

int crc32c_debug_resident_trace(crc32c_resident *r, uint64_t *stamps, uint64_t *rtt_ticks, uint64_t *rtt_polls) {
    if (!r) return hdfs_crc::fail(-EINVAL, "resident == NULL");
    return hdfs_crc::resident_trace(r->e, stamps, rtt_ticks, rtt_polls);
}

// (round 4's semantics: the stop word at once, queued blocks may be dropped)
int crc32c_debug_resident_destroy(crc32c_resident *r) {
    if (!r) return 0;
    (void)hdfs_crc::resident_destroy(r->e, false);
    delete r;
    return 0;
}

}  // extern "C"
