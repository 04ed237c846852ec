// crc32c_kernel.hip -- the production instantiations of the CDNA4 (gfx950)
// CRC32C chunk kernel (device code and design notes: crc32c_device.h).
//
// Exactly four kernels ship in libhdfs_crc32c.so: the slicing-by-4 kernel
// with non-temporal payload loads, 12 waves (768 threads) per workgroup and
// one workgroup per CU, storing checksums (crc32c_plan_exec) or comparing
// them (crc32c_plan_verify), each with or without the general-tile code (a
// batch without bpc outside 512 * 2^k runs the kernel that lacks it).  A/B and diagnostic variants are built only
// into libhdfs_crc32c_debug.so (debug/crc32c_variants.hip).
#include "crc32c_device.h"

namespace hdfs_crc {

hipError_t launch_plan_kernel(const KParams &p, uint32_t num_cu, hipStream_t stream) {
    using namespace hdfs_crc_dev;
    constexpr int kProd = kModeS4 | kModeNt;
    const dim3 g{production_grid(p, num_cu), 1, 1}, b{768, 1, 1};
    constexpr int kGen = kModeGeneral;
    if (p.expect) {
        if (!p.result || !p.sched || !p.sched_next) return hipErrorInvalidValue;
        if (p.general)
            hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeVerify>), g, b, 0, stream, p);
        else
            hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<768, 3, kProd | kModeVerify>), g, b, 0, stream, p);
    } else {
        if (p.general)
            hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen>), g, b, 0, stream, p);
        else
            hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<768, 3, kProd>), g, b, 0, stream, p);
    }
    return hipGetLastError();
}

}  // namespace hdfs_crc
