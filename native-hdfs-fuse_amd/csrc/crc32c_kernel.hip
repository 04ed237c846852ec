// crc32c_kernel.hip -- the production instantiations of the CDNA4 (gfx950)
// CRC32C chunk kernel (device code and design notes: crc32c_device.h).
//
// libhdfs_crc32c.so ships the slicing-by-4 kernel with non-temporal payload
// loads, 12 waves (768 threads) per workgroup and one workgroup per CU, in
// these builds, each storing checksums (crc32c_plan_exec) or comparing them
// (crc32c_plan_verify):
//   * full image, power-of-two tiles only: the bulk path (config 2);
//   * full image with the general-tile code (bpc outside 512 * 2^k, packet
//     tails) and the shifted loads of tiles off 16-byte alignment, in three
//     forms: both paths, general tiles only, shifted tiles only (a build
//     without the path a batch does not need has its registers and schedule
//     to the other path); the both-paths form, which padded chunks run,
//     computes a general item's next subtile facts ahead (kModeGHoist);
//   * compact image (28 KiB staged instead of 152 KiB, with the general-tile
//     code): batches of at most kSmallBatchItemsPerCu work items per CU,
//     where the table staging is most of a launch (one 4 MiB block: 5.8 ->
//     5.2 us);
//   * the same with quarter units (each tile split over 4 waves, 2 pieces
//     per lane): batches of at most kQuarterTilesPerCu tiles per CU, where
//     one wave's load -> lookups chain is the launch (one 4 MiB block,
//     graph-replayed: 4.36 -> 3.71 us); up to kEarlyTilesPerCu tiles per
//     CU with the first unit's loads issued before the table staging (their
//     latencies overlap: one 4 MiB block 3.71-3.74 -> 3.57 us; at 3 tiles
//     per CU the staging queues behind them, 4.16-4.22 -> 4.41-4.46, round 6);
//     a batch with no general tiles and no tile off 16-byte alignment (a
//     whole aligned block) runs that form without the general-tile code and
//     with 8 waves per workgroup, one per unit (one 4 MiB block 3.57 ->
//     3.42 us without the code, -> 3.35 us with 8 waves, round 6);
//   * the same with half units (each tile over 2 waves): batches of more
//     than kQuarterTilesPerCu and at most kHalvesTilesPerCu tiles per CU
//     (2-3 blocks: 896 tiles 5.23-5.27 -> 4.69-4.73 us, 1024 tiles
//     5.29-5.35 -> 4.76-4.82, 1536 tiles 6.09-6.16 -> 5.73-5.79, round 6);
//   * full image with the general-tile code and half tiles (bpc <= 256,
//     513..768 and 1025..1280), with and without the shifted loads, for any batch holding
//     half tiles (compiled into the builds above, their code cost those
//     3-8 %).
// A/B and diagnostic variants are built only into libhdfs_crc32c_debug.so
// (debug/crc32c_variants.hip).
#include <hip/hip_ext.h>

#include "crc32c_device.h"

namespace hdfs_crc {

namespace {
// Work items per CU up to which the compact image wins: its T lookups are
// not conflict-free (one copy of each table instead of 32 lane columns), so
// once every CU has many tiles the full image's faster lookups pay back its
// staging (small batches; graph-replayed, 3072 tiles:
// 7.89 vs 8.24 us, 4096: 9.05 vs 9.39, 8192: full image ahead,
// profiles/r02/launch_probe_units_crossover.json).
constexpr uint64_t kSmallBatchItemsPerCu = 16;
// Tiles per CU up to which quarter units win (tools/launch_probe.py,
// profiles/r02/launch_probe_crossover.json: 512 tiles 3.71 vs 4.36 us, 768
// tiles 4.24 vs 4.72, 1024 tiles 5.56 vs 4.95).
constexpr uint64_t kQuarterTilesPerCu = 3;
// Tiles per CU up to which the quarter-unit build issues the first unit's
// loads before the table staging (tools/launch_probe.py, debug variants 82 /
// 83, profiles/r06/early/: 512 tiles 3.57 vs 3.71-3.74 us, 768 tiles
// 4.41-4.46 vs 4.16-4.22).
constexpr uint64_t kEarlyTilesPerCu = 2;
// Tiles per CU up to which half units win over whole tiles (debug variant
// 86 against production, tools/launch_probe.py, profiles/r06/halves/: 1280
// tiles 5.50-5.55 vs 5.95-5.98 us, 1536 5.73-5.79 vs 6.09-6.16, 1792
// 6.80-6.84 vs 6.56-6.58, 2048 7.02-7.13 vs 6.79-6.94).  (Round 2 measured
// halves only with the padded-tile code in the build: 2-5 %.)
constexpr uint64_t kHalvesTilesPerCu = 6;
}  // namespace

hipError_t launch_plan_kernel(const KParams &p, uint32_t num_cu, hipStream_t stream, hipEvent_t stop,
                              uint32_t *grid) {
    using namespace hdfs_crc_dev;
    constexpr int kProd = kModeS4 | kModeNt;
    constexpr int kGen = kModeGeneral;
    constexpr int kSmall = kModeS4C | kModeGeneral | kModeNoPadT;
    constexpr int kQuarter = kSmall | kModeQuarter;
    const uint64_t items = uint64_t(p.ntiles) + (uint64_t(p.ngen) + 1) / 2 + (uint64_t(p.nseg) + 1) / 2 + p.nconst;
    const bool half = (p.general & kGeneralHalf) != 0;  // (half tiles: builds of their own, full image)
    // (padded power-of-two tiles and half tiles only run in full-image
    // builds: their code in the small-batch builds cost config 3 ~4 %)
    const bool small = !half && !(p.general & kGeneralPadded) && items <= kSmallBatchItemsPerCu * num_cu;
    const bool quarter = small && p.ntiles <= kQuarterTilesPerCu * num_cu;
    const bool early = quarter && p.ntiles <= kEarlyTilesPerCu * num_cu;
    const bool halves = small && !quarter && p.ntiles <= kHalvesTilesPerCu * num_cu;
    const dim3 g{production_grid(p, num_cu, quarter ? 4u : halves ? 2u : 1u), 1, 1}, b{768, 1, 1};
    if (grid) *grid = g.x;
#define LAUNCH_B(K, B)                                                             \
    do {                                                                           \
        if (stop)                                                                  \
            hipExtLaunchKernelGGL(K, g, B, 0, stream, nullptr, stop, 0u, p);       \
        else                                                                       \
            hipLaunchKernelGGL(K, g, B, 0, stream, p);                             \
    } while (0)
#define LAUNCH(K) LAUNCH_B(K, b)
    const dim3 b8{512, 1, 1};  // (the aligned one-block form: 8 waves)
    // Half tiles run in builds of their own, any batch size (the full image):
    // with the shifted loads only where some tile is off 16-byte alignment
    // (padded general items -- a packet's tail -- do not need them there).
    const bool half_shift = half && (p.general & kGeneralShift) != 0;
    if (p.expect) {
        if (!p.result || !p.sched) return hipErrorInvalidValue;
        if (half_shift)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeGHoist | kModeHalfT | kModeVerify>));
        else if (half)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeNoShift | kModeHalfT | kModeVerify>));
        else if (early && !p.general)
            LAUNCH_B((hdfs_crc32c_plan_kernel<512, 2, kProd | kModeS4C | kModeQuarter | kModeEarly | kModeVerify>), b8);
        else if (early)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kQuarter | kModeEarly | kModeVerify>));
        else if (quarter)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kQuarter | kModeVerify>));
        else if (halves)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kQuarter | kModeHalves | kModeVerify>));
        else if (small)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kSmall | kModeVerify>));
        else if (p.general == kGeneralItems)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeNoShift | kModeVerify>));
        else if (p.general == kGeneralShift)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeNoGItems | kModeVerify>));
        else if (p.general)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeGHoist | kModeVerify>));
        else
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kModeVerify>));
    } else {
        if (half_shift)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeGHoist | kModeHalfT>));
        else if (half)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeNoShift | kModeHalfT>));
        else if (early && !p.general)
            LAUNCH_B((hdfs_crc32c_plan_kernel<512, 2, kProd | kModeS4C | kModeQuarter | kModeEarly>), b8);
        else if (early)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kQuarter | kModeEarly>));
        else if (quarter)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kQuarter>));
        else if (halves)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kQuarter | kModeHalves>));
        else if (small)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kSmall>));
        else if (p.general == kGeneralItems)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeNoShift>));
        else if (p.general == kGeneralShift)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeNoGItems>));
        else if (p.general)
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd | kGen | kModeGHoist>));
        else
            LAUNCH((hdfs_crc32c_plan_kernel<768, 3, kProd>));
    }
#undef LAUNCH
#undef LAUNCH_B
    return hipGetLastError();
}

// Loads this file's code object (every build above) onto the current
// device: HIP loads it at its first use, which would otherwise land in the
// process's first checksum call (1.2-2.2 ms against 16 us,
// tools/first_call_probe.py).  crc32c_ctx_create calls it.
hipError_t preload_plan_kernels() {
    using namespace hdfs_crc_dev;
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&hdfs_crc32c_plan_kernel<768, 3, kModeS4 | kModeNt>));
}

}  // namespace hdfs_crc
