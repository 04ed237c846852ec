/*
 * hdfs_crc32c.h -- C ABI of the MI355X-native CRC32C chunk-checksum path of
 * native-hdfs-fuse (libhdfs_crc32c.so).
 *
 * Every entry point is plain C: pointers, sizes and integers, no HIP or torch
 * types in the signatures (a HIP stream is passed as `void *`).  Batch entry
 * points return 0 on success or a negative errno, the reference's convention
 * (src/hadooprpc.c:440-486, 630-636).  The GPU entry points never fall back
 * to a CPU implementation on their own: without a usable GPU they return
 * -ENODEV.  The two host-memory calls the per-packet loop uses
 * (crc32c_chunks, crc32c_batch_host) take CRC32C_CPU_FALLBACK to finish on
 * the host CPU instead (the reference's crc32c() cannot fail), and
 * crc32c_last_path() says which path ran.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   crc32c()             src/crc32c.c:333-343 (declared by hand at src/hadooprpc.c:31)
 *   crc32c_chunks*()     the per-chunk loop of hadoop_rpc_send_packet,
 *                        src/hadooprpc.c:639 + 727-748 (roundup, crc32c(0, ...), htonl)
 *   crc32c_packetize()   the packet cutting of hadoop_rpc_send_packets,
 *                        src/hadooprpc.c:827-857
 *   crc32c_plan_create_buffers()
 *                        hadoop_rpc_send_packets over a Hadoop_Fuse_Buffer_Pos
 *                        (src/hadooprpc.c:815-860 packet cutting, 666-725 packet
 *                        assembly, src/hadooprpc.h:33-45 the buffer types)
 *   crc32c_multi_*()     no reference counterpart: blocks written in parallel
 *                        (src/fuse.c:580-647 writes them one at a time) sharded
 *                        over several GPUs of one node, RCCL gather.
 *   crc32c_plan_verify*(), crc32c_verify_frames_host()
 *                        hadoop_rpc_receive_packets (src/hadooprpc.c:497-584)
 *                        with sendChecksums (the reference asks for none,
 *                        src/fuse.c:1608-1609)
 */
#ifndef HDFS_CRC32C_H
#define HDFS_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDFS_CRC32C_ABI_VERSION 2

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
#define CRC32C_CPU_FALLBACK 0x8u /* crc32c_chunks / crc32c_batch_host only: when the GPU
                                    is unavailable or a HIP call fails, compute on the host
                                    CPU (crc32c_chunks_cpu) and return 0; crc32c_last_path()
                                    then reports CRC32C_PATH_CPU */
#define CRC32C_COUNT_COMPLETION 0x20u /* plan flag: the plan's launches count their own
                                         completion on the GPU (every workgroup's last wave
                                         bumps a counter in the plan's block), so
                                         crc32c_plan_destroy touches none of the streams the
                                         plan ran on and the plan may be destroyed AFTER them
                                         (a FUSE worker that owns a short-lived stream).
                                         Costs ~0.65 us per launch (the counter's device-scope
                                         atomic ends each launch: one 4 MiB block 4.70 against
                                         4.0 us); off by default */

/* Which path the calling thread's last crc32c_chunks / crc32c_batch_host
 * call took. */
#define CRC32C_PATH_NONE 0 /* failed, or nothing to compute */
#define CRC32C_PATH_GPU 1
#define CRC32C_PATH_CPU 2  /* CRC32C_CPU_FALLBACK taken */
int crc32c_last_path(void);

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
 * of out_idx + crc32c_nchunks(len, bpc) (0 for none).  A packet with len == 0
 * (the block's final empty packet, hadooprpc.c:853-856) has no checksums
 * whatever its bpc, here and in every batch entry point; a packet with
 * len > 0 and bpc == 0 is invalid (the batch entry points return -EINVAL) and
 * counts nothing here. */
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
 * decomposition into 8 KiB tiles) and executed on any payload with that
 * shape.  Its descriptors go to the device asynchronously (the first launch
 * on a stream waits for that copy).  Destroying a plan whose launches are
 * still in flight is safe: for every stream a launch of the plan went on
 * that is still busy at destroy time an event is recorded there, and the
 * plan's device block is recycled only once those events (and its upload)
 * have completed.  So a plan is destroyed BEFORE the streams it was
 * launched on (an idle stream is only queried; HIP does not validate a
 * destroyed stream's handle) -- unless it was created with
 * CRC32C_COUNT_COMPLETION: its launches then count their own completion on
 * the GPU (+~0.65 us per launch), destroy touches none of its streams, and
 * the block is reused once the count is complete.  (An event record per
 * launch costs +2.6 us of GPU time per 4 MiB block; a stop event per launch
 * a cost that grows the longer a process runs)  A
 * context may be destroyed before its plans: it lives until its last plan
 * is destroyed, and is then torn down by the next crc32c_ctx_create /
 * crc32c_ctx_destroy call (crc32c_ctx_destroy(NULL) does only that), never
 * inside crc32c_plan_destroy.
 * No device-wide synchronisation on any plan create / destroy path, so work
 * of other streams and libraries is never waited on, and plans may be
 * created and destroyed while another thread captures a graph.  A plan must
 * outlive every HIP graph that captured its launches (the graph replays
 * read its descriptors); the block of a plan whose launches were captured
 * is not reused while the context lives.
 * Payload and checksum buffers are device
 * pointers; execution is asynchronous on `stream` (a hipStream_t, NULL =
 * the default stream).  Exec launches of one plan are not ordered with each
 * other: independent batches may run on several streams at once, and two
 * streams let one launch start on the CUs the previous one has released
 * (config 2: 41.2 instead of 43.4 us per batch, tools/overlap_probe.py).
 * Fast tiles: every full chunk of a packet with bpc in {512, 1024, 2048,
 * 4096, 8192}, at any alignment (off 16-byte alignment, loaded from the
 * aligned address below and shifted into place: config 2 five bytes off
 * 48.7-50.5 instead of 42.0-43.0 us); every full chunk of any other bpc in
 * [4, 8192] and every packet tail of at least 4 bytes (general items:
 * config 2 with bpc 1536 in 1.1x the time of bpc 512); the rest (shorter
 * tails, bpc outside [4, 8192]) takes the general path (exact, slower).
 * The payload buffer must be readable up to the next 16-byte boundary after
 * each packet's last byte (device allocations always are).
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
 * when none).  One launch: its first workgroup initialises dev_result and
 * tags the plan's device slot with the launch's key, and only workgroups
 * that found mismatches add to the result after they see that key (no
 * separate reset of dev_result, no grid-wide reduction; graph replays are
 * told apart by their dispatch).  A plan's verify launches share that slot,
 * so the library keeps them in GPU order, also across streams (a verify
 * launch on another stream than the plan's previous one waits for it).  It
 * cannot order a graph replay of captured verify launches against other
 * verify launches of the same plan: the caller must not let those overlap.
 * If they do, the kernels still finish (a mismatching workgroup waits for
 * its launch's key a bounded time) and bit 31 of dev_result[0]
 * (CRC32C_VERIFY_OVERLAP) marks the result indeterminate.  The same bit can
 * appear for a correct result when the launch's first workgroup starts late
 * -- e.g. while a resident block queue (section 3b) holds every CU -- and a
 * workgroup with more than 256 mismatches waits for it past its bound:
 * re-run such a verify once nothing else holds the device. */
#define CRC32C_VERIFY_OVERLAP 0x80000000u
int crc32c_plan_verify(crc32c_plan *plan, const void *dev_payload, const uint32_t *dev_expected,
                       uint32_t *dev_result, void *stream);

/* crc32c_plan_verify plus a mismatch bitmap (SURVEY.md section 8f row 1:
 * "compute + compare, emit a mismatch bitmap"): dev_bad_bits holds
 * ceil(crc32c_plan_nchecksums(plan) / 32) device u32s; bit i % 32 of word
 * i / 32 is set for every mismatching checksum i and cleared for every
 * other one (the launch itself zeroes the bitmap before any bit is set: no
 * separate memset on `stream`).
 * A reader that must report every corrupt chunk of a replica, not only the
 * first (the ChecksumException of hadooprpc.c:497-584's caller), takes it
 * from here; NULL = crc32c_plan_verify. */
int crc32c_plan_verify_bitmap(crc32c_plan *plan, const void *dev_payload, const uint32_t *dev_expected,
                              uint32_t *dev_result, uint32_t *dev_bad_bits, void *stream);

/* Packet assembly from scatter buffers (hadooprpc.h:33-45, hadooprpc.c:666-725).
 * The bytes a block write sends are `len` bytes starting `bufferoffset` into
 * the concatenation of buffers[0 .. n_buffers); a buffer with data == NULL is
 * `len` zero bytes (Hadoop_Fuse_Buffer).  FUSE writes use up to four:
 * TRUNCATE, NULLPADDING, THEDATA, TRAILINGDATA (fuse.c:1348-1354), and
 * ftruncate-extension one NULL buffer (fuse.c:1137-1142). */
typedef struct crc32c_buffer {
    const void *data; /* device address, or NULL = zero fill */
    uint64_t len;
} crc32c_buffer;

/* Plan of hadoop_rpc_send_packets(from = {buffers, n_buffers, bufferoffset},
 * len, blockoffset, packetsize, checksum{bpc}) (hadooprpc.c:815-860): the
 * packets crc32c_packetize(len, blockoffset, packetsize, bpc) lists, each
 * cut into chunks from its own start (hadooprpc.c:733-742), their checksums
 * at out indices 0, 1, ... in packet order.  Exec / verify take dev_payload
 * = NULL (the plan holds the buffer addresses, which must stay valid).
 * Chunks inside one data buffer are read in place (no assembly copy); a
 * chunk spanning buffers is read piece by piece; a chunk of zero fill only
 * is written from a plan-time constant without reading anything, so an
 * all-NULL write reads no payload at all.  flags: CRC32C_BIG_ENDIAN,
 * CRC32C_TYPE_CRC32.  -EINVAL when the range exceeds the buffers. */
int crc32c_plan_create_buffers(crc32c_ctx *ctx, const crc32c_buffer *buffers, uint32_t n_buffers,
                               uint64_t bufferoffset, uint64_t len, uint64_t blockoffset, uint32_t packetsize,
                               uint32_t bpc, uint32_t flags, crc32c_plan **out);

/* ---------------------------------------------------------------------------
 * 3b. Many blocks of one shape in one launch (concurrent block writes).
 *
 * libfuse runs hadoop_fuse_write_block (src/fuse.c:336-449) on many worker
 * threads at once (fuse.c:1771, no -s); each writes one block, cut into
 * packets by hadoop_rpc_send_packets (hadooprpc.c:815-860).  A launch per
 * 4 MiB block is bound by HIP's launch path (~3.5-4 us per block); one launch
 * over many blocks is not.  `plan` here describes ONE block's packets
 * (offsets from the block's start; not CRC32C_DEVICE_ADDRESSES).
 *
 * crc32c_plan_exec_blocks: the plan run once per block, block i's payload at
 * dev_payloads[i] and its checksums to dev_outs[i] (4-byte aligned), as ONE
 * launch per up to 32 blocks (the block table rides in the kernel arguments:
 * nothing is built or uploaded per call).  A plan with items other than
 * tiles (tails under 4 bytes, bpc outside [4, 8192]) runs one launch per
 * block instead.  Asynchronous on `stream`.
 *
 * crc32c_blocks: a coalescing queue for block writes arriving from several
 * threads without any batching by the caller.  crc32c_block_submit queues a
 * block (its bytes already in device memory) and returns a ticket (one
 * atomic add and a ring slot: no lock); the queue goes out as one
 * crc32c_plan_exec_blocks launch on the queue's own stream when it holds
 * max_blocks blocks, on crc32c_block_flush, or window_us after the queue's
 * worker saw the batch's first block (group commit).  The launches and
 * their completion are made by one worker thread the queue owns (every HIP
 * call of the queue is on it; crc32c_block_flush only asks it to launch
 * now); at most two launches are in flight, later blocks wait in the ring.
 * The GPU stays busy when about 2 x max_blocks blocks are in flight (e.g.
 * 16 writer threads keeping two blocks each in flight with submit / wait).  crc32c_block_wait returns when the ticket's checksums
 * are in device memory (and complete for any later stream or copy);
 * crc32c_block_checksums is submit + wait.  Thread-safe.  Destroy the queue
 * (it launches what is queued and waits) before its plan.
 * crc32c_blocks_stats: launches (flushes) made and blocks they carried.
 *
 * crc32c_blocks_create_resident: the same queue calls served by a RESIDENT
 * kernel (opt-in; replaces fuse.c:336's one-checksum-pass-per-call for many
 * concurrent writers, fuse.c:1771): one launch stays on the GPU and takes
 * each block as it is submitted from a ring in pinned host memory, so there
 * is no launch (nor launch boundary, table staging, tail) per block; a
 * waiter polls a completion word the kernel writes into host memory.
 * CU policy: while it runs the kernel holds one 16-wave workgroup with the
 * whole LDS on EVERY CU -- other kernels on the device (plan execs, other
 * queues) wait for CUs until it exits.  It exits idle_us after the last
 * block completes (0 = 2000 us), 50 ms after it stops making progress, or
 * at destroy; the next submit relaunches it.  Plans of power-of-two tiles
 * and general chunks (bpc 512 << k; packet tails and the trimmed first packet
 * of an append at an unaligned block offset, hadooprpc.c:832-840, included),
 * payload offsets from the block's start (not CRC32C_DEVICE_ADDRESSES, not
 * crc32c_plan_create_buffers): -EINVAL otherwise.  Payloads at any
 * alignment (a block off 16-byte alignment takes the kernel's shifted loads).
 * crc32c_block_flush does nothing (every block is taken at once);
 * crc32c_blocks_stats reports the kernel's launches and the blocks
 * submitted; destroy lets every submitted block complete, then stops the
 * kernel.  A wait gives up with -ETIMEDOUT after 5 s without its block; a
 * submit whose ring slot is still busy waits for it first and, if that wait
 * gives up, returns its error without taking a ticket (the queue goes on).
 *
 * crc32c_block_submit_plan: a block of ANOTHER shape through the same queue
 * -- e.g. the first block of an append at an unaligned offset
 * (hadoop_fuse_do_write, src/fuse.c:488-574, through write_block at
 * blockoffset > 0) beside the whole blocks of the queue's plan.  plan ==
 * NULL is the queue's plan (crc32c_block_submit).  The plan must be on the
 * queue's device and describe one block (offsets from its start); a
 * resident queue also needs the queue plan's checksum type and byte order
 * and the shapes above.  The group-commit queue sends consecutive blocks of
 * one plan out as one launch.  The plan must stay alive until its blocks'
 * waits have returned.
 * ------------------------------------------------------------------------- */
int crc32c_plan_exec_blocks(crc32c_plan *plan, const void *const *dev_payloads, uint32_t *const *dev_outs,
                            size_t nblocks, void *stream);

typedef struct crc32c_blocks crc32c_blocks;
int crc32c_blocks_create(crc32c_plan *plan, uint32_t max_blocks, uint32_t window_us, crc32c_blocks **out);
int crc32c_block_submit(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out, uint64_t *ticket);
int crc32c_block_submit_plan(crc32c_blocks *q, crc32c_plan *plan, const void *dev_payload, uint32_t *dev_out,
                             uint64_t *ticket);
int crc32c_block_flush(crc32c_blocks *q);
int crc32c_block_wait(crc32c_blocks *q, uint64_t ticket);
int crc32c_block_checksums(crc32c_blocks *q, const void *dev_payload, uint32_t *dev_out);
int crc32c_blocks_stats(const crc32c_blocks *q, uint64_t *flushes, uint64_t *blocks);
int crc32c_blocks_destroy(crc32c_blocks *q);
int crc32c_blocks_create_resident(crc32c_plan *plan, uint32_t idle_us, crc32c_blocks **out);

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
 * 5. Several GPUs of one node.  A file's packets are sharded in groups of
 * `group_packets` consecutive packets (64 = one 4 MiB HDFS block of 64 KiB
 * packets), group g on rank g % nranks.  Each rank checksums its shard on
 * its own GPU; RCCL point-to-point transfers over xGMI (one ncclGroupStart /
 * ncclGroupEnd) gather the u32 checksum arrays into block order on rank 0.
 * The communicator spans the devices of one process (crc32c_multi_create,
 * ranks = the devices in the order given) or one device per process
 * (crc32c_multi_create_rank: every rank calls it at the same time with the
 * id rank 0 got from crc32c_multi_unique_id and sent to the others).
 * ------------------------------------------------------------------------- */
typedef struct crc32c_multi crc32c_multi;

int crc32c_multi_create(const int *devices, int ndevices, crc32c_multi **out);
int crc32c_multi_unique_id(uint8_t id[128]);
int crc32c_multi_create_rank(int device, int rank, int nranks, const uint8_t id[128], crc32c_multi **out);
int crc32c_multi_destroy(crc32c_multi *m);
/* Waits for the library's own per-device streams (used when exec gets none). */
int crc32c_multi_sync(crc32c_multi *m);

/* Shard layout (host only, no GPU): returns the number of groups G and, per
 * group g, layout[4g .. 4g+3] = {rank, offset of the group's first byte in
 * that rank's shard buffer, offset of that byte in the caller's payload,
 * bytes}; a group's bytes move as one range (its 16-byte phase is kept).
 * shard_bytes[r] (optional) = bytes of rank r's shard.  A group's checksums
 * must form one contiguous range of out indices. */
int64_t crc32c_multi_layout(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                            uint64_t *layout, uint64_t *shard_bytes);
/* Rank `rank`'s packets with payload offsets into its shard buffer (out
 * indices unchanged); returns their count (copies at most cap). */
int64_t crc32c_multi_shard_packets(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                                   int rank, crc32c_packet *local, size_t cap);

/* The two halves of crc32c_multi_plan_exec's gather, host only (no GPU), so
 * that the N-rank exchange can be checked without N GPUs.
 *
 * crc32c_multi_rank_packets: the packets rank `rank`'s plan computes --
 * payload offsets into its shard, out indices into the u32 array it sends to
 * rank 0 (its groups' checksum ranges back to back, in group order); rank 0's
 * out indices are the global ones (it writes its groups in place) unless
 * flags has CRC32C_MULTI_SELF_SEND.  Returns their count (copies at most cap).
 *
 * crc32c_multi_transfers: local_nout[r] = length of rank r's local array (0
 * for rank 0 in place; nranks entries, optional), and per transfer t, in the
 * order exec posts them, xfers[4t .. 4t+3] = {sending rank, index in its
 * local array, index in the file-order output on rank 0, count} -- one per
 * received group, merged with the previous one when both come from the same
 * rank and stay contiguous on both sides.  Returns the number of transfers
 * (fills at most cap).  These are the gather's placements.  When no sender
 * has more than one (each rank's groups are one file-order range),
 * crc32c_multi_plan_exec posts exactly these: each sender one ncclSend, rank
 * 0 one ncclRecv straight into root_out.  Otherwise (round-robin blocks over
 * N > 1 ranks) the exec is packed: each sender posts ONE ncclSend of its
 * whole local array, rank 0 one ncclRecv per sender into a staging array of
 * the plan's, and one scatter kernel on rank 0's stream copies every
 * placement into root_out -- unless the plan has CRC32C_MULTI_PER_GROUP_RECV,
 * which posts one ncclSend / ncclRecv pair per placement. */
int64_t crc32c_multi_rank_packets(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                                  int rank, uint32_t flags, crc32c_packet *local, size_t cap);
int64_t crc32c_multi_transfers(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                               uint32_t flags, uint64_t *local_nout, uint64_t *xfers, size_t cap);
/* crc32c_multi_scatter: the packed gather's layout (host only).  Returns the
 * number of scatter tiles, 0 when the gather is not packed (no sender has
 * more than one placement, or CRC32C_MULTI_PER_GROUP_RECV); stage_off[r]
 * (nranks entries, optional) = index in rank 0's staging array where rank
 * r's whole local array is received (senders in rank order); per tile t
 * (fills at most cap), tiles[3t .. 3t+2] = {staging index, file index,
 * count <= 1024}: what the scatter kernel copies into root_out. */
int64_t crc32c_multi_scatter(const crc32c_packet *pkts, size_t npkts, uint32_t group_packets, int nranks,
                             uint32_t flags, uint64_t *stage_off, uint64_t *tiles, size_t cap);

/* Device-resident multi-GPU plan of a file's packets (offsets in the caller's
 * file layout; every process passes the same list).  Exec: dev_shards[i] =
 * the shard of the i-th local device (laid out as crc32c_multi_layout says),
 * root_out = nchecksums device u32s on rank 0's device (rank 0's process
 * only), streams[i] = the local device i's stream (NULL entry = its default
 * stream; streams == NULL = the library's own streams, see
 * crc32c_multi_sync).  Asynchronous: the
 * checksum launches, then the RCCL gather (crc32c_multi_transfers: every
 * other rank's group ranges sent straight into their file-order places in
 * root_out; rank 0 computes its own groups in place), on the local devices'
 * streams; root_out is complete when rank 0's stream is.  An exec may be
 * captured into a HIP graph (kernels and the RCCL group; the communicator is
 * created by the first exec, so run one exec before capturing).  Successive
 * execs on the same stream cost no extra HIP call; an exec on another stream
 * than the plan's previous one records an event on that previous stream, so
 * that stream must still exist then.  flags: CRC32C_BIG_ENDIAN,
 * CRC32C_TYPE_CRC32, CRC32C_MULTI_SELF_SEND, CRC32C_MULTI_PIPELINE,
 * CRC32C_MULTI_PER_GROUP_RECV, CRC32C_COUNT_COMPLETION.  A plan with
 * CRC32C_MULTI_PER_GROUP_RECV whose gather would post more than 4096
 * transfers (a tiny group_packets over a large file) is refused with -E2BIG.
 * crc32c_multi_plan_gather_ops: the point-to-point operations (sends +
 * receives, whole communicator) one exec's RCCL group posts; *packed
 * (optional) = 1 when the exec is packed (staging array + scatter kernel). */
#define CRC32C_MULTI_SELF_SEND 0x10u /* crc32c_multi_plan_create: rank 0's own checksums also travel
                                       through RCCL (a send to itself) instead of being written in
                                       place -- exercises the transport on a one-GPU communicator */
/* CRC32C_MULTI_PIPELINE (plan flag): consecutive execs overlap -- exec k + 1's
 * shard launch runs beside exec k's tail and RCCL gather (the files of a
 * stream of block writes, src/fuse.c:580-647, are independent).  An exec
 * forks from the caller's stream (it starts after the caller's work so far)
 * onto one of the plan's two exec streams (alternating), into one of two
 * local arrays (alternating), and issues the PREVIOUS exec's gather on the
 * caller's stream (after that exec's launch); the last exec's gather is
 * issued by crc32c_multi_plan_join(mp, streams), which then makes every
 * local stream wait for every launch.  So root_out and the shards belong to
 * the plan until the join; call it before reading root_out, before a graph
 * capture of execs begins and before it ends (on the capturing stream).
 * Execs writing the same root_out keep their in-place launches on rank 0 in
 * order (an exec waits for the previous one's launch); execs into different
 * root_out arrays overlap fully.  crc32c_multi_plan_join on a plan without
 * the flag does nothing. */
#define CRC32C_MULTI_PIPELINE 0x40u
/* CRC32C_MULTI_PER_GROUP_RECV (plan flag, A/B): one ncclSend / ncclRecv pair
 * per placement (crc32c_multi_transfers), received straight into root_out,
 * even when a sender has several -- instead of the packed gather. */
#define CRC32C_MULTI_PER_GROUP_RECV 0x80u
typedef struct crc32c_multi_plan crc32c_multi_plan;
int crc32c_multi_plan_create(crc32c_multi *m, const crc32c_packet *pkts, size_t npkts, uint32_t group_packets,
                             uint32_t flags, crc32c_multi_plan **out);
int crc32c_multi_plan_exec(crc32c_multi_plan *mp, const void *const *dev_shards, uint32_t *root_out,
                           void *const *streams);
int crc32c_multi_plan_join(crc32c_multi_plan *mp, void *const *streams);
int crc32c_multi_plan_destroy(crc32c_multi_plan *mp);
uint64_t crc32c_multi_plan_nchecksums(const crc32c_multi_plan *mp);
uint64_t crc32c_multi_plan_shard_bytes(const crc32c_multi_plan *mp, int rank);
uint64_t crc32c_multi_plan_gather_ops(const crc32c_multi_plan *mp, int *packed);

/* Host-resident: each local device checksums its groups (dealt round-robin
 * over the local devices) from host memory over its own PCIe link and
 * copies its checksums straight into the host `out` array. */
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

/* The read side ("next" row 1): the packet stream a DataNode sends for
 * OP_READ_BLOCK with sendChecksums, per packet PLEN (u32 BE) | HLEN (u16 BE)
 * | PacketHeaderProto | checksums (u32 BE) | data (hadoop_rpc_receive_packets,
 * src/hadooprpc.c:497-584; datatransfer.proto:184-191). */
typedef struct crc32c_frame_info {
    uint64_t frame_off;      /* offset of the frame's PLEN in the buffer */
    uint64_t sums_off;       /* offset of its checksums */
    uint64_t data_off;       /* offset of its data */
    int64_t offset_in_block; /* PacketHeaderProto.offsetInBlock */
    int64_t seqno;           /* PacketHeaderProto.seqno */
    uint32_t data_len;       /* PacketHeaderProto.dataLen */
    uint32_t nsums;          /* checksums in the frame ((PLEN - 4 - dataLen) / 4) */
    uint32_t last;           /* PacketHeaderProto.lastPacketInBlock */
    uint32_t reserved;
} crc32c_frame_info;

/* Whole frames at the start of `frames` (stops before a partial frame and
 * after a lastPacketInBlock frame): returns their count (fills at most cap
 * entries of info), *consumed = their bytes; -EBADMSG for a malformed frame. */
int64_t crc32c_parse_frames(const void *frames, size_t bytes, crc32c_frame_info *info, size_t cap,
                            uint64_t *consumed);

typedef struct crc32c_frames_result {
    uint64_t packets;          /* frames parsed (whole frames) */
    uint64_t data_bytes;
    uint64_t checksums;        /* checksums compared */
    uint64_t mismatches;
    uint64_t first_bad;        /* index of the first bad checksum in the run, UINT64_MAX if none */
    int64_t first_bad_offset;  /* offsetInBlock of its chunk, -1 if none */
    uint64_t consumed;         /* bytes of the whole frames parsed */
    uint32_t last_packet;      /* a lastPacketInBlock frame was seen */
    uint32_t reserved;
} crc32c_frames_result;

/* Verifies a run of received frames on the GPU (host-resident: the frame
 * buffer is copied once and every chunk is checked against the checksums in
 * front of it; nothing is de-interleaved by the caller).  chunk_offset =
 * ReadOpChecksumInfoProto.chunkOffset (datatransfer.proto:218-227): the
 * first data packet must start there, every packet on a chunk boundary
 * right after the previous one; the caller skips requested offset -
 * chunkOffset bytes of the first packet's data, as hadooprpc.c:548-560
 * does.  flags: CRC32C_TYPE_CRC32 for CHECKSUM_CRC32, CRC32C_CPU_FALLBACK.
 * 0 (result in *res), -EBADMSG for a malformed or misplaced frame, or -errno. */
int crc32c_verify_frames_host(crc32c_ctx *ctx, const void *frames, size_t bytes, uint32_t bpc,
                              uint64_t chunk_offset, uint32_t flags, crc32c_frames_result *res);

/* Last error text of the calling thread (static storage, never NULL). */
const char *crc32c_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* HDFS_CRC32C_H */
