/*
 * hdfs_crc32c.h -- C ABI of the MI355X-native CRC32C chunk-checksum path of
 * native-hdfs-fuse (libhdfs_crc32c.so).
 *
 * Every entry point is plain C: pointers, sizes and integers, no HIP or torch
 * types in the signatures (a HIP stream is passed as `void *`).  Batch entry
 * points return 0 on success or a negative errno, the reference's convention
 * (src/hadooprpc.c:440-486, 630-636).  They never fall back to a CPU
 * implementation: without a usable GPU they return -ENODEV.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   crc32c()             src/crc32c.c:333-343 (declared by hand at src/hadooprpc.c:31)
 *   crc32c_chunks*()     the per-chunk loop of hadoop_rpc_send_packet,
 *                        src/hadooprpc.c:639 + 727-748 (roundup, crc32c(0, ...), htonl)
 *   crc32c_packetize()   the packet cutting of hadoop_rpc_send_packets,
 *                        src/hadooprpc.c:827-857
 *   crc32c_multi_*()     no reference counterpart: blocks written in parallel
 *                        (src/fuse.c:580-647 writes them one at a time) sharded
 *                        over several GPUs of one node.
 */
#ifndef HDFS_CRC32C_H
#define HDFS_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDFS_CRC32C_ABI_VERSION 1

/* ---------------------------------------------------------------------------
 * 1. Drop-in scalar checksum (host CPU).
 *
 * Same signature and semantics as the reference export (src/crc32c.c:333):
 * `crc` is the finished CRC32C of the preceding bytes (0 to start), the result
 * is the CRC32C of the concatenation, in host byte order; any alignment;
 * len == 0 returns crc.  Cannot fail, reentrant, thread-safe.  This is the
 * per-call host path (a GPU round trip per 512-byte chunk would be absurd);
 * batches go through the GPU entry points below.
 * ------------------------------------------------------------------------- */
uint32_t crc32c(uint32_t crc, const void *buf, size_t len);

/* Hadoop's CHECKSUM_CRC32 on the host: zlib's crc32(crc, buf, len) (reflected
 * polynomial 0xEDB88320, same conditioning and incremental semantics as
 * crc32c above).  The reference has no implementation (hadooprpc.c:629-631). */
uint32_t hdfs_crc32(uint32_t crc, const void *buf, size_t len);

/* Checksum flags (batch entry points). */
#define CRC32C_BIG_ENDIAN 0x1u /* store htonl(crc), the wire order of hadooprpc.c:71-75 */
#define CRC32C_TYPE_CRC32 0x2u /* Hadoop CHECKSUM_CRC32 (IEEE 802.3 / zlib polynomial)
                                  instead of CHECKSUM_CRC32C; the reference returns
                                  -ENOSYS for it (hadooprpc.c:629-631) */
#define CRC32C_DEVICE_ADDRESSES 0x4u /* plan flag: every packet's payload_off is a device
                                        address, so one plan (one launch) covers packets in
                                        different device buffers, e.g. many HDFS blocks;
                                        exec / verify then take dev_payload = NULL.  Not
                                        valid for the host-resident calls. */

/* One packet of a batch: `len` payload bytes starting `payload_off` bytes into
 * the batch payload buffer, cut into chunks of `bpc` bytes
 * (bytesPerChecksum); its ceil(len / bpc) checksums go to out[out_idx ...].
 * Exactly hadooprpc.c:733-742 per packet: chunk i covers
 * [i*bpc, i*bpc + min(bpc, len - i*bpc)), checksummed from crc = 0. */
typedef struct crc32c_packet {
    uint64_t payload_off;
    uint64_t out_idx;
    uint32_t len;
    uint32_t bpc;
} crc32c_packet;

/* The reference's per-packet loop (hadooprpc.c:733-742) on the host CPU, in
 * one call: out[i] = crc32c(0, packet + i*bpc, min(bpc, len - i*bpc)) for the
 * ceil(len / bpc) chunks, htonl'd with CRC32C_BIG_ENDIAN (hadooprpc.c:71-75);
 * CRC32C_TYPE_CRC32 selects Hadoop's CHECKSUM_CRC32.  Whole chunks run as
 * three interleaved crc32q chains.  0, or -EINVAL (bpc == 0, unknown flags,
 * NULL buffers).  This is the per-packet replacement; batches of packets go
 * to the GPU (sections 3-4). */
int crc32c_chunks_cpu(const void *packet, size_t len, uint32_t bpc, uint32_t *out, uint32_t flags);

/* Number of checksums of one packet: roundup(len, bpc) (hadooprpc.c:639). */
uint64_t crc32c_nchunks(uint64_t len, uint32_t bpc);

/* Length of the checksum array a batch fills: max over packets with len > 0
 * of out_idx + crc32c_nchunks(len, bpc) (0 for none; bpc == 0 counts as 1). */
uint64_t crc32c_batch_nchecksums(const crc32c_packet *pkts, size_t npkts);

/* Packet lengths hadoop_rpc_send_packets produces for one block write of
 * `len` bytes starting at `blockoffset` (hadooprpc.c:827-857), including the
 * final empty packet.  Writes up to `max` lengths; returns the count. */
uint64_t crc32c_packetize(uint64_t len, uint64_t blockoffset, uint32_t packetsize, uint32_t bpc, uint64_t *lens,
                          uint64_t max);

/* ---------------------------------------------------------------------------
 * 2. GPU context (one HIP device).  Thread-safe: calls on one context are
 * serialised internally; use one context per thread for concurrency.
 * ------------------------------------------------------------------------- */
typedef struct crc32c_ctx crc32c_ctx;

int crc32c_ctx_create(int device, crc32c_ctx **out);
int crc32c_ctx_destroy(crc32c_ctx *ctx);
/* Number of visible HIP devices (0 when there is no GPU). */
int crc32c_device_count(void);

/* ---------------------------------------------------------------------------
 * 3. Device-resident batches.
 *
 * A plan is built once per batch SHAPE from host packet descriptors (work
 * decomposition into 8 KiB tiles, uploaded to the device) and executed on
 * any payload with that shape.  Payload and checksum buffers are device
 * pointers; execution is asynchronous on `stream` (a hipStream_t, NULL =
 * the default stream).  Exec launches of one plan are not ordered with each
 * other: independent batches may run on several streams at once, and two
 * streams let one launch start on the CUs the previous one has released
 * (config 2: 41.2 instead of 43.4 us per batch, tools/overlap_probe.py).
 * Fast path: every full chunk of a packet with bpc in {512, 1024, 2048,
 * 4096, 8192}, at any alignment (off 16-byte alignment the tile loads are
 * unaligned: config 2 five bytes off takes 55 instead of 42.5 us); short
 * tail chunks and other bpc values take the general path (exact, ~4x
 * slower).  The payload buffer must be readable up to the next 16-byte
 * boundary after each packet's last byte (device allocations always are).
 * ------------------------------------------------------------------------- */
typedef struct crc32c_plan crc32c_plan;

int crc32c_plan_create(crc32c_ctx *ctx, const crc32c_packet *pkts, size_t npkts, uint32_t flags,
                       crc32c_plan **out);
int crc32c_plan_exec(crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out, void *stream);
int crc32c_plan_destroy(crc32c_plan *plan);
/* Total checksums the plan writes (max over packets of out_idx + nchunks). */
uint64_t crc32c_plan_nchecksums(const crc32c_plan *plan);
/* Payload bytes the plan checksums (sum of packet lengths). */
uint64_t crc32c_plan_payload_bytes(const crc32c_plan *plan);

/* Verification, the read side ("next" row 1): a DataNode
 * sends each packet's checksums ahead of its data (received by
 * hadoop_rpc_receive_packets, src/hadooprpc.c:497-584; the reference asks for
 * none, src/fuse.c:1608-1609).  Computes every checksum of the plan's batch on
 * the GPU and compares it with dev_expected[same index] (in wire order when
 * the plan was created with CRC32C_BIG_ENDIAN) instead of storing it.
 * dev_result: 2 device u32s, set by this call (asynchronously on `stream`):
 * [0] = mismatching checksums, [1] = lowest mismatching index (0xffffffff
 * when none).  One launch: the last workgroup to finish publishes the result
 * (no separate reset of dev_result).  A plan's verify launches share its
 * device scratch, so the library keeps them in GPU order, also across
 * streams (a verify launch on another stream than the plan's previous one
 * waits for it).  Kernel variants other than 0 to 2
 * ($HDFS_CRC32C_KVARIANT, A/B only) return -EINVAL. */
int crc32c_plan_verify(crc32c_plan *plan, const void *dev_payload, const uint32_t *dev_expected,
                       uint32_t *dev_result, void *stream);

/* One-shot device batch: builds a plan, runs it on `stream` and waits for it. */
int crc32c_chunks_dev(crc32c_ctx *ctx, const crc32c_packet *pkts, size_t npkts, const void *dev_payload,
                      uint32_t *dev_out, uint32_t flags, void *stream);

/* ---------------------------------------------------------------------------
 * 4. Host-resident batches (file pages on their way to the DataNode socket).
 * The payload is copied to the GPU in 64 MiB slices on one copy stream
 * (straight from `payload` when it is pinned, else through pinned staging),
 * each slice is checksummed on one of two stage streams into mapped pinned
 * memory, and the checksums are scattered into `out` (host memory).
 * Blocking.
 * ------------------------------------------------------------------------- */
int crc32c_batch_host(crc32c_ctx *ctx, const void *payload, const crc32c_packet *pkts, size_t npkts,
                      uint32_t *out, uint32_t flags);

/* Host-resident verification (blocking): returns the number of checksums that
 * differ from expected[] (>= 0; only indices the packets cover are compared),
 * or -errno; *first_bad = the lowest such index (UINT64_MAX when none). */
int64_t crc32c_verify_host(crc32c_ctx *ctx, const void *payload, const crc32c_packet *pkts, size_t npkts,
                           const uint32_t *expected, uint32_t flags, uint64_t *first_bad);

/* The reference's per-packet loop (hadooprpc.c:733-742) on one host packet:
 * out receives ceil(len / bpc) checksums.  Uses the process-wide default
 * context (device 0, or $HDFS_CRC32C_DEVICE), created on first use. */
int crc32c_chunks(const void *packet, size_t len, uint32_t bpc, uint32_t *out, uint32_t flags);

/* ---------------------------------------------------------------------------
 * 5. Several GPUs of one node, one process.  Packets are sharded in groups of
 * `group_packets` consecutive packets (64 = one 4 MiB HDFS block of 64 KiB
 * packets) dealt round-robin over the devices; each device checksums its
 * shard and copies its checksums straight into the host `out` array.
 * ------------------------------------------------------------------------- */
typedef struct crc32c_multi crc32c_multi;

int crc32c_multi_create(const int *devices, int ndevices, crc32c_multi **out);
int crc32c_multi_destroy(crc32c_multi *m);
int crc32c_multi_batch_host(crc32c_multi *m, const void *payload, const crc32c_packet *pkts, size_t npkts,
                            uint32_t group_packets, uint32_t *out, uint32_t flags);

/* ---------------------------------------------------------------------------
 * 6. Host-side companions of the checksum path.
 * ------------------------------------------------------------------------- */

/* Batched packet framing ("next" row 2).  hadoop_rpc_send_packet sends every
 * packet as PLEN (u32 BE) | HLEN (u16 BE) | PacketHeaderProto | checksums
 * (u32 BE each) | data with 1 + 1 + 1 + n sendto calls (src/hadooprpc.c:
 * 596-664, 733-748).  This writes the prefixes (everything but the data) of
 * a whole batch back to back into `out`, so each packet can go out as one
 * sendmsg of two iovecs: out + prefix_off[i] .. prefix_off[i+1], then its
 * data.  Per packet i: offsetInBlock = block_offset + payload_off[i] -
 * payload_off[0], seqno = first_seqno + i (0 at a block start,
 * hadooprpc.c:825), lastPacketInBlock = (len == 0), dataLen = len;
 * PLEN = 4 + checksum_len * nchunks + len (hadooprpc.c:640).
 * `sums` holds each packet's checksums at out_idx (host order, or wire order
 * with CRC32C_BIG_ENDIAN in flags); checksum_len is 4 (CRC32C / CRC32) or 0
 * (CHECKSUM_NULL).  prefix_off (optional) receives npkts + 1 offsets.
 * Returns the bytes written, or the bytes needed when `out` is NULL or `cap`
 * is too small (nothing written then); 0 on invalid arguments. */
size_t crc32c_frame_packets(const crc32c_packet *pkts, size_t npkts, const uint32_t *sums, uint32_t flags,
                            uint64_t block_offset, int64_t first_seqno, uint32_t checksum_len, uint8_t *out,
                            size_t cap, uint64_t *prefix_off);

/* OpBlockChecksumResponseProto.md5 ("next" row 4, datatransfer.proto:262-267):
 * MD5 over a block's checksums as big-endian bytes (`sums` in host order, or
 * wire order with CRC32C_BIG_ENDIAN). */
void crc32c_block_md5(const uint32_t *sums, size_t n, uint32_t flags, uint8_t md5[16]);

/* Last error text of the calling thread (static storage, never NULL). */
const char *crc32c_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* HDFS_CRC32C_H */
