// kernel_abi.h -- what the host runtime hands the CRC32C kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_math.h"
#include "plan.h"

namespace hdfs_crc {

constexpr uint32_t kKernelThreads = 512;  // 8 waves per workgroup
constexpr uint32_t kKernelLdsBytes = uint32_t(kLdsBytes);
constexpr uint32_t kKernelShiftOff = uint32_t(kLdsShiftOff);
constexpr uint32_t kKernelWgPerCu = 2;  // 2 x 73 KiB of LDS per CU

struct KParams {
    const FastTile *tiles;
    const GenItem *gen;
    const uint8_t *payload;
    uint32_t *out;
    const uint8_t *table;  // kLdsBytes, staged into LDS by every workgroup
    uint32_t ntiles;
    uint32_t ngen;
    uint32_t flags;
    uint32_t c_lg[5];
    uint32_t c_small[4];
};

hipError_t launch_plan_kernel(const KParams &p, uint32_t grid, hipStream_t stream);

}  // namespace hdfs_crc
