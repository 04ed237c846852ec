/*
 * hdfs_crc32c_debug.h -- introspection and diagnostic hooks.
 *
 * Section 1 is exported by libhdfs_crc32c.so (host-side only, no launch):
 * the CPU test-suite checks the GPU path's host-side inputs with it without a
 * GPU -- the work decomposition and the LDS table image the kernel loads.
 *
 * Section 2 is exported only by libhdfs_crc32c_debug.so (built beside the
 * product library, linked against it): A/B and diagnostic kernel variants
 * and a plain HBM read probe, for tools/ and the bench's read-rate
 * reference.  The product library never launches anything but the
 * production kernel.  Not needed by a reference-side integration.
 */
#ifndef HDFS_CRC32C_DEBUG_H
#define HDFS_CRC32C_DEBUG_H

#include <stddef.h>
#include <stdint.h>

#include "hdfs_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. libhdfs_crc32c.so ---- */

/* Work items a plan would upload: 16-byte FastTile {u64 src, u32 out,
 * u32 meta} (meta: nblocks | lg << 8, or bit 31 | nch * k | k << 8 |
 * nch << 13 | pad << 18 for a general tile) and 16-byte GenItem {u64 src,
 * u32 out, u32 len}.  Copies at most *_cap items; counts go to *ntiles /
 * *ngen. */
int crc32c_debug_plan(const crc32c_packet *pkts, size_t npkts, void *tiles, size_t tiles_cap, void *gen,
                      size_t gen_cap, uint64_t *ntiles, uint64_t *ngen);

/* Item counts of a crc32c_plan_create_buffers plan (CRC32C): counts[0..5] =
 * tiles, gen items, seg items, pieces, constant runs, checksums. */
int crc32c_debug_write_plan(const crc32c_buffer *buffers, uint32_t n_buffers, uint64_t bufferoffset, uint64_t len,
                            uint64_t blockoffset, uint32_t packetsize, uint32_t bpc, uint64_t counts[6]);

/* The LDS image the nibble variant stages (returns its size; fills dst when
 * cap is large enough) and the affine constants crc32c(0, zeros(512 << lg)),
 * lg = 0..4, and crc32c(0, zeros(r)), r = 0..3. */
size_t crc32c_debug_lds_image(void *dst, size_t cap, uint32_t *c_lg5, uint32_t *c_small4);

/* The slicing-by-4 kernel's LDS image for the checksum type in `flags`
 * (byte tables T0..T3 replicated over the 32 lane columns, the per-column
 * finishing operators N_q, the Z^(512 s) shifts); returns its size and
 * fills dst when cap is large enough. */
size_t crc32c_debug_lds_image_s4(void *dst, size_t cap, uint32_t flags);
/* The affine constants of the checksum type in `flags` (CRC32C_TYPE_CRC32 or not). */
void crc32c_debug_affine_constants(uint32_t flags, uint32_t *c_lg5, uint32_t *c_small4);

/* Fault injection for the block queue's error path (tests): the worker fails
 * the issue of the next `n` flushes of q as if their launch had failed
 * (-EIO, nothing launched); the waits of exactly those flushes' tickets
 * return the error. */
int crc32c_debug_blocks_fail_flushes(crc32c_blocks *q, uint32_t n);

/* Resident queues only: hold != 0 keeps the kernel from being launched
 * (submits queue up in the ring; 0 launches what is queued), and the next
 * fail_waits waits -- a submit's wait for a busy slot included -- return
 * -ETIMEDOUT at once. */
int crc32c_debug_blocks_resident_inject(crc32c_blocks *q, int hold, uint32_t fail_waits);

/* CPU time the queue's worker thread has used so far (its thread CPU clock),
 * in ns: what the queue itself costs beside the submitting threads. */
int crc32c_debug_blocks_worker_cpu_ns(crc32c_blocks *q, uint64_t *ns);

/* The device address of the pooled block holding a plan's descriptors (0:
 * none): tests see a destroyed plan's block come back from the pool. */
uint64_t crc32c_debug_plan_block(const crc32c_plan *plan);

/* ---- 2. libhdfs_crc32c_debug.so only ---- */

/* Launch of a plan with an explicit kernel variant (0 = production; see
 * debug/crc32c_variants.hip): 5, 6 and 36 write per-wave timestamps, 4 x
 * u64 per wave (s_memrealtime at start, after table staging, at exit;
 * XCC_ID << 32 | HW_ID) into dev_stamps, which must then hold 4 * (waves
 * launched) entries; 3, 4, 6 and 7 compute WRONG checksums on purpose
 * (memory-only / compute-only ceilings).  -EINVAL for a variant not built. */
int crc32c_debug_plan_exec_variant(crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out,
                                   uint64_t *dev_stamps, int variant, void *stream);
/* Name of a built variant (NULL if none); *exact = 1 when it computes the
 * right checksums. */
const char *crc32c_debug_variant_name(int variant, int *exact);

/* Plain streaming read of `bytes` device bytes; writes one dword per thread
 * to dev_out (at most 2^20 dwords).  Shapes 0-7: grid x 256 threads,
 * grid-stride, 16 B per lane, 4 / 8 / 4 nt / 16 / 2 nt / 8 nt / 16 nt / 1 nt
 * loads in flight per lane; shapes 8-15: tile reads like the CRC kernel's
 * (1024 or 512 threads, 8 or 4 KiB per wave, per-workgroup ranges or
 * grid-stride tiles), see debug/stream_probe.hip.  Prices the HBM read
 * roofline this device actually delivers (tools/probe_sweep.py). */
int crc32c_debug_stream_probe(const void *dev_src, uint64_t bytes, uint32_t *dev_out, uint32_t grid, int shape,
                              void *stream);

/* A/B experiment: a RESIDENT kernel for concurrent block writes (see
 * debug/resident.hip).  The kernel stays on the GPU (all CUs, tables staged
 * once) and takes blocks from a ring the submitting threads fill; it exits on
 * destroy, after idle_us (0: 2000) with nothing queued, or when stuck, and
 * submit / wait relaunch it on demand.  The plan must be aligned
 * power-of-two tiles only (one block's shape); payloads 16-byte aligned.
 * While it runs it holds every CU's LDS: other kernels wait. */
typedef struct crc32c_resident crc32c_resident;
int crc32c_debug_resident_create(crc32c_plan *plan, uint32_t idle_us, crc32c_resident **out);
int crc32c_debug_resident_submit(crc32c_resident *r, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket);
int crc32c_debug_resident_wait(crc32c_resident *r, uint64_t ticket);
int crc32c_debug_resident_stats(const crc32c_resident *r, uint64_t *launches);
/* Trace of a resident runner created with HDFS_CRC32C_RESIDENT_STAMPS=1:
 * ends the running launch (a later submit relaunches), then copies 4 x u64
 * s_memrealtime stamps (100 MHz) per ticket t at [4 (t % 4096)]: forwarded,
 * seen by workgroup 0's worker, that worker's tiles stored, completed by the
 * collector; and the sum / count of the forwarder's host-slot poll round
 * trips (ticks). -EINVAL without the trace. */
int crc32c_debug_resident_trace(crc32c_resident *r, uint64_t *stamps, uint64_t *rtt_ticks, uint64_t *rtt_polls);
int crc32c_debug_resident_destroy(crc32c_resident *r);

#ifdef __cplusplus
}
#endif

#endif
