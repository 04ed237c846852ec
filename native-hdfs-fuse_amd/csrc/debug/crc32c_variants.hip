// crc32c_variants.hip -- A/B and DIAGNOSTIC instantiations of the CRC32C
// kernel (device code: ../crc32c_device.h).  Built only into
// libhdfs_crc32c_debug.so, which links against libhdfs_crc32c.so and adds
// crc32c_debug_plan_exec_variant; the product library launches nothing but
// the production kernel, whatever the environment says.
//
// Variant numbers are those of DESIGN.md (round 1 measured 37; the ones
// still built are listed below, the others were within noise of variant 0
// and were removed).
#include "../crc32c_device.h"
#include "../runtime_internal.h"
#include "hdfs_crc32c_debug.h"

namespace {

using namespace hdfs_crc_dev;
constexpr int kS4Nt = kModeS4 | kModeNt | kModeGeneral;  // A/B variants always carry the general-tile code

struct Variant {
    int id;
    const char *name;
    uint32_t threads, wg_per_cu;
    bool exact;  // computes the right checksums
    bool prod_grid = false;  // the production grid: min(items, CUs) workgroups
};

constexpr Variant kVariants[] = {
    {0, "s4_nt", 768, 1, true},                            // production (launched through the product library)
    {1, "nibble_wg1024x2_nt", 1024, 2, true},              // positional nibble tables, 32 waves per CU
    {2, "s4_wg1024x1_nt", 1024, 1, true},                  // 0 with 16 waves per CU
    {3, "s4_wg768x1_nt_memonly", 768, 1, false},           // memory ceiling of 0 (no lookups)
    {4, "s4_wg768x1_nt_compute_only", 768, 1, false},      // compute ceiling of 0 (no payload loads)
    {5, "s4_wg768x1_nt_stamps", 768, 1, true},             // 0 with per-wave timestamps
    {6, "s4_wg768x1_nt_memonly_stamps", 768, 1, false},    // 3 with per-wave timestamps
    {7, "s4_wg768x1_nt_memonly_nostage", 768, 1, false},   // 3 without the table staging
    {9, "s4_wg512x1_nt", 512, 1, true},                    // 0 with 8 waves per CU
    {40, "s4_nt_memonly_nostage_prodgrid", 768, 1, false, true},  // 7 on the production grid (launch floor)
    {41, "s4c_nt_prodgrid", 768, 1, true, true},           // compact image (28 KiB staged), production grid
    {42, "s4c_nt_stamps_prodgrid", 768, 1, true, true},    // 41 with per-wave timestamps
    {43, "s4_nt_stamps_prodgrid", 768, 1, true, true},     // 0 with per-wave timestamps, production grid
    // small batches: compact image, one tile per wave, smaller workgroups
    {44, "s4c_wg256_nt", 256, 4, true},                    // 4 waves per workgroup
    {45, "s4c_wg128_nt", 128, 8, true},                    // 2 waves per workgroup
    {46, "s4c_wg256_nt_early", 256, 4, true},              // 44, first tile's loads before the staging
    {47, "s4c_wg128_nt_early", 128, 8, true},              // 45, first tile's loads before the staging
    {48, "s4c_nt_early_prodgrid", 768, 1, true, true},     // 41, first tile's loads before the staging
    {49, "s4_nt_general_prodgrid", 768, 1, true, true},    // the full-image general build without the hoist (75), any batch
    {51, "s4c_nt_quarter_prodgrid", 768, 1, true, true},   // 41 with quarter units (4 per tile)
    {52, "s4c_nt_quarter_early_prodgrid", 768, 1, true, true},  // 51, first unit's loads before the staging
    {53, "s4_nt_quarter_prodgrid", 768, 1, true, true},    // 49 (full image) with quarter units
    {54, "s4c_nt_quarter_stamps_prodgrid", 768, 1, true, true},  // 51 with per-wave timestamps
    {55, "s4c_nt_quarter_early_stamps_prodgrid", 768, 1, true, true},  // 52 with per-wave timestamps
    {60, "s4c_nt_halves_prodgrid", 768, 1, true, true},    // 51 with 2 units of 8 blocks per tile
    {61, "s4_nt_halves_prodgrid", 768, 1, true, true},     // the same on the full image
    {62, "s4_nt_pow2only_prodgrid", 768, 1, true, true},   // the production power-of-two build (no general code)
    {63, "s4_nt_pow2only_xcdmap_prodgrid", 768, 1, true, true},  // 62, each XCD's ranges contiguous
    // general-item ablations (wrong results): what the per-subtile gather and
    // the chunk-start masks cost, with and without the payload loads
    {70, "s4_nt_compute_only_nogather", 768, 1, false},
    {71, "s4_nt_compute_only_nomask", 768, 1, false},
    {72, "s4_nt_compute_only_nogather_nomask", 768, 1, false},
    {73, "s4_nt_nogather", 768, 1, false},
    {74, "s4_nt_nomask", 768, 1, false},
    // (round 5, production since): the general build (49) with a general item's next
    // subtile facts computed right after the current subtile's loads
    {75, "s4_nt_general_hoist_prodgrid", 768, 1, true, true},
    // the general-tiles-only production build (what variant 0 runs for a
    // batch of general items and no shifted tiles) with the same hoist, with
    // a 2-subtile gather, and with both
    {76, "s4_nt_gitems_hoist_prodgrid", 768, 1, true, true},
    {77, "s4_nt_gitems_group2_prodgrid", 768, 1, true, true},
    {78, "s4_nt_gitems_group2_hoist_prodgrid", 768, 1, true, true},
    // the general-tiles-only production build itself (what a batch of padded
    // tiles and general items with no shifted tile runs), for any batch
    {79, "s4_nt_gitems_prodgrid", 768, 1, true, true},
    // the power-of-two production build (62) with the first tile's loads
    // issued right after the staging's, before the barrier; stamped twin
    {80, "s4_nt_pow2only_ovl_prodgrid", 768, 1, true, true},
    {81, "s4_nt_pow2only_ovl_stamps_prodgrid", 768, 1, true, true},
    // (round 6) the production quarter-unit build (no padded tiles), and the
    // same with the first unit's loads issued before the table staging
    {82, "s4c_nt_quarter_nopad_prodgrid", 768, 1, true, true},
    {83, "s4c_nt_quarter_nopad_early_prodgrid", 768, 1, true, true},
    // (round 6) the production small-batch build (compact image, whole
    // tiles, no padded tiles), and the same with the first tile's loads
    // before the table staging
    {84, "s4c_nt_nopad_prodgrid", 768, 1, true, true},
    {85, "s4c_nt_nopad_early_prodgrid", 768, 1, true, true},
    // (round 6) 82 with 2 units of 8 blocks per tile (halves)
    {86, "s4c_nt_halves_nopad_prodgrid", 768, 1, true, true},
    // (round 6) 86 and 84 with 16 waves per workgroup (one round of half
    // units / tiles at 4-8 tiles per CU)
    {87, "s4c_wg1024_nt_halves_nopad_prodgrid", 1024, 1, true, true},
    {88, "s4c_wg1024_nt_nopad_prodgrid", 1024, 1, true, true},
    // (round 6) the small-batch builds without the general-tile code (for
    // batches of aligned power-of-two tiles only): quarter units + early
    // loads, quarter units, half units
    {89, "s4c_nt_pow2only_quarter_early_prodgrid", 768, 1, true, true},
    {90, "s4c_nt_pow2only_quarter_prodgrid", 768, 1, true, true},
    {91, "s4c_nt_pow2only_halves_prodgrid", 768, 1, true, true},
    {92, "s4c_nt_pow2only_prodgrid", 768, 1, true, true},  // whole tiles, compact image
    // (round 6) 89 with 8 waves per workgroup (config 3: 8 units per CU, one per wave)
    {93, "s4c_wg512_nt_pow2only_quarter_early_prodgrid", 512, 1, true, true},
    // (round 6) 92 with 8 waves per workgroup (the 16 MiB shard: 8 tiles per CU)
    {94, "s4c_wg512_nt_pow2only_prodgrid", 512, 1, true, true},
    // (round 6) 83 (quarter units + early loads, general-tile code) with 8
    // waves per workgroup: one block off 16-byte alignment (an append)
    {95, "s4c_wg512_nt_quarter_nopad_early_prodgrid", 512, 1, true, true},
};

const Variant *find(int v) {
    for (const Variant &x : kVariants)
        if (x.id == v) return &x;
    return nullptr;
}

#define HDFS_LAUNCH(T, W, M) hipLaunchKernelGGL((hdfs_crc32c_plan_kernel<T, W, M>), g, b, 0, stream, p)

hipError_t launch_variant(const hdfs_crc::KParams &p, const Variant &v, uint32_t num_cu, hipStream_t stream) {
    const uint64_t items = uint64_t(p.ntiles) + (uint64_t(p.ngen) + 1) / 2 + (uint64_t(p.nseg) + 1) / 2 + p.nconst;
    const uint64_t waves = v.threads / 64;
    const uint32_t units = ((v.id >= 51 && v.id <= 55) || v.id == 82 || v.id == 83 || v.id == 89 || v.id == 90 ||
                            v.id == 93 || v.id == 95)
                               ? 4u
                           : (v.id == 60 || v.id == 61 || v.id == 86 || v.id == 87 || v.id == 91)             ? 2u
                                                                                                              : 1u;
    uint64_t grid = v.prod_grid ? hdfs_crc::production_grid(p, num_cu, units) : (items + waves - 1) / waves;
    const uint64_t cap = uint64_t(num_cu) * v.wg_per_cu;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    const dim3 g{uint32_t(grid), 1, 1}, b{v.threads, 1, 1};
    // (82-88 leave the padded- and half-tile code out, as the production
    // small-batch builds do: plans with such tiles are refused)
    if (((v.id >= 82 && v.id <= 88) || v.id == 95) && (p.general & (hdfs_crc::kGeneralPadded | hdfs_crc::kGeneralHalf)))
        return hipErrorInvalidValue;
    // (89-94 carry no general-tile code at all: aligned power-of-two plans only)
    if (v.id >= 89 && v.id <= 94 && p.general) return hipErrorInvalidValue;
    switch (v.id) {
    case 1: HDFS_LAUNCH(1024, 8, kModeNt | kModeGeneral); break;
    case 2: HDFS_LAUNCH(1024, 4, kS4Nt); break;
    case 3: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag); break;
    case 4: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompDiag); break;
    case 5: HDFS_LAUNCH(768, 3, kS4Nt | kModeStamps); break;
    case 6: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag | kModeStamps); break;
    case 7: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag | kModeNoStage); break;
    case 9: HDFS_LAUNCH(512, 2, kS4Nt); break;
    case 40: HDFS_LAUNCH(768, 3, kS4Nt | kModeMemDiag | kModeNoStage); break;
    case 41: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C); break;
    case 42: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeStamps); break;
    case 43: HDFS_LAUNCH(768, 3, kS4Nt | kModeStamps); break;
    case 44: HDFS_LAUNCH(256, 4, kS4Nt | kModeS4C); break;
    case 45: HDFS_LAUNCH(128, 4, kS4Nt | kModeS4C); break;
    case 46: HDFS_LAUNCH(256, 4, kS4Nt | kModeS4C | kModeEarly); break;
    case 47: HDFS_LAUNCH(128, 4, kS4Nt | kModeS4C | kModeEarly); break;
    case 48: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeEarly); break;
    case 49: HDFS_LAUNCH(768, 3, kS4Nt); break;
    case 51: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeQuarter); break;
    case 52: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeQuarter | kModeEarly); break;
    case 53: HDFS_LAUNCH(768, 3, kS4Nt | kModeQuarter); break;
    case 54: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeQuarter | kModeStamps); break;
    case 55: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeQuarter | kModeEarly | kModeStamps); break;
    case 60: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeQuarter | kModeHalves); break;
    case 61: HDFS_LAUNCH(768, 3, kS4Nt | kModeQuarter | kModeHalves); break;
    case 62: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt); break;
    case 63: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeXcdMap); break;
    case 70: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompDiag | kModeGDiagNoGather); break;
    case 71: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompDiag | kModeGDiagNoMask); break;
    case 72: HDFS_LAUNCH(768, 3, kS4Nt | kModeCompDiag | kModeGDiagNoGather | kModeGDiagNoMask); break;
    case 73: HDFS_LAUNCH(768, 3, kS4Nt | kModeGDiagNoGather); break;
    case 74: HDFS_LAUNCH(768, 3, kS4Nt | kModeGDiagNoMask); break;
    case 75: HDFS_LAUNCH(768, 3, kS4Nt | kModeGHoist); break;
    case 76: HDFS_LAUNCH(768, 3, kS4Nt | kModeNoShift | kModeGHoist); break;
    case 77: HDFS_LAUNCH(768, 3, kS4Nt | kModeNoShift | kModeGGroup2); break;
    case 78: HDFS_LAUNCH(768, 3, kS4Nt | kModeNoShift | kModeGGroup2 | kModeGHoist); break;
    case 79: HDFS_LAUNCH(768, 3, kS4Nt | kModeNoShift); break;
    case 80: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeOvl); break;
    case 81: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeOvl | kModeStamps); break;
    case 82: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeNoPadT | kModeQuarter); break;
    case 83: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeNoPadT | kModeQuarter | kModeEarly); break;
    case 84: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeNoPadT); break;
    case 85: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeNoPadT | kModeEarly); break;
    case 86: HDFS_LAUNCH(768, 3, kS4Nt | kModeS4C | kModeNoPadT | kModeQuarter | kModeHalves); break;
    case 87: HDFS_LAUNCH(1024, 4, kS4Nt | kModeS4C | kModeNoPadT | kModeQuarter | kModeHalves); break;
    case 88: HDFS_LAUNCH(1024, 4, kS4Nt | kModeS4C | kModeNoPadT); break;
    case 89: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeS4C | kModeQuarter | kModeEarly); break;
    case 90: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeS4C | kModeQuarter); break;
    case 91: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeS4C | kModeQuarter | kModeHalves); break;
    case 92: HDFS_LAUNCH(768, 3, kModeS4 | kModeNt | kModeS4C); break;
    case 93: HDFS_LAUNCH(512, 2, kModeS4 | kModeNt | kModeS4C | kModeQuarter | kModeEarly); break;
    case 94: HDFS_LAUNCH(512, 2, kModeS4 | kModeNt | kModeS4C); break;
    case 95: HDFS_LAUNCH(512, 2, kS4Nt | kModeS4C | kModeNoPadT | kModeQuarter | kModeEarly); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
#undef HDFS_LAUNCH

}  // namespace

extern "C" int crc32c_debug_plan_exec_variant(crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out,
                                              uint64_t *dev_stamps, int variant, void *stream) {
    using namespace hdfs_crc;
    if (!plan) return fail(-EINVAL, "plan == NULL");
    const Variant *v = find(variant);
    if (!v) return fail(-EINVAL, "kernel variant %d is not built", variant);
    if (plan->nchecksums == 0) return 0;
    if (plan->absolute) {
        if (dev_payload) return fail(-EINVAL, "a device-address plan takes dev_payload = NULL");
        dev_payload = reinterpret_cast<const void *>(uintptr_t(plan->abs_base));
    }
    DeviceGuard guard(plan->ctx->device);
    KParams p = plan_params(plan, dev_payload, dev_out);
    p.stamps = dev_stamps;
    p.done_ctr = nullptr;  // (not counted: the plan's block is never reused)
    const hipStream_t s = static_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lock(plan->mu);
    plan->unaccounted = true;
    if (int rc = prepare_launch(plan, s)) return rc;
    HIP_TRY(variant == 0 ? launch_plan_kernel(p, uint32_t(plan->ctx->num_cu), s)
                         : launch_variant(p, *v, uint32_t(plan->ctx->num_cu), s));
    return 0;
}

extern "C" const char *crc32c_debug_variant_name(int variant, int *exact) {
    const Variant *v = find(variant);
    if (exact) *exact = v ? int(v->exact) : 0;
    return v ? v->name : nullptr;
}
