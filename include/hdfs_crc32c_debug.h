/*
 * hdfs_crc32c_debug.h -- introspection hooks of libhdfs_crc32c.so used by the
 * CPU test-suite to check the GPU path's host-side inputs without a GPU:
 * the work decomposition and the LDS table image the kernel loads.
 * Not needed by a reference-side integration.
 */
#ifndef HDFS_CRC32C_DEBUG_H
#define HDFS_CRC32C_DEBUG_H

#include <stddef.h>
#include <stdint.h>

#include "hdfs_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Work items a plan would upload: 16-byte FastTile {u64 src, u32 out,
 * u32 meta = nblocks | lg << 8} and 16-byte GenItem {u64 src, u32 out,
 * u32 len}.  Copies at most *_cap items; counts go to *ntiles / *ngen. */
int crc32c_debug_plan(const crc32c_packet *pkts, size_t npkts, void *tiles, size_t tiles_cap, void *gen,
                      size_t gen_cap, uint64_t *ntiles, uint64_t *ngen);

/* The LDS image the kernel stages (returns its size; fills dst when cap is
 * large enough) and the affine constants crc32c(0, zeros(512 << lg)),
 * lg = 0..4, and crc32c(0, zeros(r)), r = 0..3. */
size_t crc32c_debug_lds_image(void *dst, size_t cap, uint32_t *c_lg5, uint32_t *c_small4);

#ifdef __cplusplus
}
#endif

#endif
