/* fuse_write.c -- hadoop_fuse_write's checksum path called from C through
 * libhdfs_crc32c.so, with the write's bytes in device memory (INTEGRATION.md
 * section 3, "Assembling packets from the FUSE write buffers").
 *
 * hadoop_fuse_write (src/fuse.c:1348-1354) sends a block write as up to four
 * Hadoop_Fuse_Buffers: TRUNCATE (the block's old bytes before the write),
 * NULLPADDING (zeros, data == NULL), THEDATA (the write) and TRAILINGDATA (old
 * bytes after it); hadoop_rpc_send_packet memcpy/memsets every packet that
 * spans two of them into one buffer (src/hadooprpc.c:666-725) before the
 * per-chunk loop (hadooprpc.c:733-742).  Here:
 *   1. the non-NULL buffers are copied to the GPU (hipMalloc / hipMemcpy);
 *   2. crc32c_plan_create_buffers plans the whole block write over them
 *      (packets as hadoop_rpc_send_packets cuts them, hadooprpc.c:815-860);
 *   3. crc32c_plan_exec checksums every packet, reading each byte in place
 *      and no NULL byte at all;
 *   4. crc32c_plan_verify_bitmap verifies the block, then with three flipped
 *      checksums, which the bitmap must name exactly;
 *   5. an ftruncate extension (fuse.c:1137-1142: one NULL buffer) gives the
 *      zero-chunk constant for every checksum.
 * Every result is checked against the reference's loop done with the drop-in
 * scalar crc32c() over the stream assembled on the host.  Exit 0 = exact.
 *
 *   fuse_write [truncate_len null_len data_len trailing_len [blockoffset [bpc]]]
 */
#include <arpa/inet.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "hdfs_crc32c.h"

static int fails = 0;
#define CHECK(cond, ...)                                         \
    do {                                                         \
        if (!(cond)) {                                           \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                        \
            fputc('\n', stderr);                                 \
            ++fails;                                             \
        }                                                        \
    } while (0)
#define HIP_OK(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d: %s: %s\n", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

static uint64_t xs = 0x243F6A8885A308D3ull;
static uint8_t next_byte(void) {
    xs ^= xs << 13;
    xs ^= xs >> 7;
    xs ^= xs << 17;
    return (uint8_t)(xs >> 56);
}

/* The reference's checksums of a block write: hadoop_rpc_send_packets' packets
 * (crc32c_packetize) over the assembled stream, crc32c(0, chunk) per chunk,
 * htonl on the wire.  Returns the count written to want. */
static uint64_t reference_sums(const uint8_t *stream, uint64_t len, uint64_t blockoffset, uint32_t bpc,
                               uint32_t *want) {
    const uint64_t np = crc32c_packetize(len, blockoffset, 65536, bpc, NULL, 0);
    uint64_t *lens = malloc(np * sizeof *lens);
    crc32c_packetize(len, blockoffset, 65536, bpc, lens, np);
    uint64_t pos = 0, n = 0;
    for (uint64_t p = 0; p < np; ++p) {
        for (uint64_t o = 0; o < lens[p]; o += bpc) {
            const uint64_t c = lens[p] - o < bpc ? lens[p] - o : bpc;
            want[n++] = htonl(crc32c(0, stream + pos + o, c));
        }
        pos += lens[p];
    }
    free(lens);
    return n;
}

static int verify_bits(crc32c_plan *plan, const uint32_t *expect, uint64_t n, uint32_t *result,
                       uint64_t *count, uint64_t *first, uint32_t **bits_out) {
    uint32_t *d_exp, *d_res, *d_bits;
    const uint64_t words = (n + 31) / 32;
    HIP_OK(hipMalloc((void **)&d_exp, n * 4 + 4));
    HIP_OK(hipMalloc((void **)&d_res, 8));
    HIP_OK(hipMalloc((void **)&d_bits, words * 4 + 4));
    HIP_OK(hipMemcpy(d_exp, expect, n * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(d_bits, 0xff, words * 4 + 4)); /* stale bits: the call clears them */
    int rc = crc32c_plan_verify_bitmap(plan, NULL, d_exp, d_res, d_bits, NULL);
    CHECK(rc == 0, "plan_verify_bitmap: %d (%s)", rc, crc32c_last_error());
    HIP_OK(hipDeviceSynchronize());
    uint32_t *bits = malloc(words * 4 + 4);
    HIP_OK(hipMemcpy(result, d_res, 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(bits, d_bits, words * 4, hipMemcpyDeviceToHost));
    *count = result[0];
    *first = result[1];
    *bits_out = bits;
    HIP_OK(hipFree(d_exp));
    HIP_OK(hipFree(d_res));
    HIP_OK(hipFree(d_bits));
    return 0;
}

int main(int argc, char **argv) {
    uint64_t lens[4] = {10000, 300000, 1u << 20, 77777}; /* TRUNCATE, NULLPADDING, THEDATA, TRAILINGDATA */
    for (int i = 0; i < 4 && i + 1 < argc; ++i) lens[i] = strtoull(argv[i + 1], NULL, 0);
    const uint64_t blockoffset = argc > 5 ? strtoull(argv[5], NULL, 0) : 0;
    const uint32_t bpc = argc > 6 ? (uint32_t)strtoul(argv[6], NULL, 0) : 512;
    const uint64_t len = lens[0] + lens[1] + lens[2] + lens[3];

    /* the host-assembled stream (what hadooprpc.c:666-725 would memcpy) and
     * the device copies of the data buffers (NULLPADDING stays NULL) */
    uint8_t *stream = calloc(len + 1, 1);
    crc32c_buffer bufs[4];
    void *dev[4] = {NULL, NULL, NULL, NULL};
    uint64_t pos = 0;
    for (int i = 0; i < 4; ++i) {
        if (i != 1)
            for (uint64_t k = 0; k < lens[i]; ++k) stream[pos + k] = next_byte();
        if (i != 1 && lens[i]) {
            HIP_OK(hipMalloc(&dev[i], lens[i]));
            HIP_OK(hipMemcpy(dev[i], stream + pos, lens[i], hipMemcpyHostToDevice));
        }
        bufs[i].data = dev[i];
        bufs[i].len = lens[i];
        pos += lens[i];
    }
    const uint64_t maxsums = len / (bpc ? bpc : 1) + 2 * (len / 65536 + 2);
    uint32_t *want = malloc(maxsums * 4);
    const uint64_t n = reference_sums(stream, len, blockoffset, bpc, want);

    crc32c_ctx *ctx = NULL;
    int rc = crc32c_ctx_create(0, &ctx);
    CHECK(rc == 0, "ctx_create: %d (%s)", rc, crc32c_last_error());
    if (rc) return 1;

    /* 2-3. the block write's plan over the four buffers, and its checksums */
    crc32c_plan *plan = NULL;
    rc = crc32c_plan_create_buffers(ctx, bufs, 4, 0, len, blockoffset, 65536, bpc, CRC32C_BIG_ENDIAN, &plan);
    CHECK(rc == 0, "plan_create_buffers: %d (%s)", rc, crc32c_last_error());
    if (rc) return 1;
    CHECK(crc32c_plan_nchecksums(plan) == n, "nchecksums %" PRIu64 " vs %" PRIu64, crc32c_plan_nchecksums(plan), n);
    uint32_t *d_sums;
    HIP_OK(hipMalloc((void **)&d_sums, n * 4 + 4));
    rc = crc32c_plan_exec(plan, NULL, d_sums, NULL);
    CHECK(rc == 0, "plan_exec: %d (%s)", rc, crc32c_last_error());
    HIP_OK(hipDeviceSynchronize());
    uint32_t *got = malloc(n * 4 + 4);
    HIP_OK(hipMemcpy(got, d_sums, n * 4, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t k = 0; k < n; ++k) bad += got[k] != want[k];
    CHECK(bad == 0, "%" PRIu64 " of %" PRIu64 " checksums differ from crc32c() over the assembled stream", bad, n);

    /* 4. read side: clean, then three flipped checksums named by the bitmap */
    uint32_t result[2];
    uint64_t count, first;
    uint32_t *bits;
    if (verify_bits(plan, want, n, result, &count, &first, &bits)) return 1;
    uint64_t set = 0;
    for (uint64_t w = 0; w < (n + 31) / 32; ++w) set += (uint64_t)__builtin_popcount(bits[w]);
    CHECK(count == 0 && first == 0xffffffffu && set == 0, "verify clean: %" PRIu64 " / %" PRIu64 " bits", count, set);
    free(bits);
    if (n >= 3) {
        const uint64_t flip[3] = {0, n / 2, n - 1};
        for (int i = 0; i < 3; ++i) want[flip[i]] ^= htonl(0x10000u);
        if (verify_bits(plan, want, n, result, &count, &first, &bits)) return 1;
        set = 0;
        for (uint64_t w = 0; w < (n + 31) / 32; ++w) set += (uint64_t)__builtin_popcount(bits[w]);
        const uint64_t distinct = (n / 2 == 0 || n / 2 == n - 1) ? 2 : 3;
        CHECK(count == distinct && first == 0 && set == distinct, "verify flipped: %" PRIu64 " / %" PRIu64, count,
              set);
        for (int i = 0; i < 3; ++i)
            CHECK((bits[flip[i] / 32] >> (flip[i] % 32)) & 1u, "bit %" PRIu64 " not set", flip[i]);
        free(bits);
    }
    crc32c_plan_destroy(plan);

    /* 5. ftruncate extension of a whole 4 MiB block: one NULL buffer */
    const crc32c_buffer zeros = {NULL, 4u << 20};
    rc = crc32c_plan_create_buffers(ctx, &zeros, 1, 0, zeros.len, 0, 65536, 512, CRC32C_BIG_ENDIAN, &plan);
    CHECK(rc == 0, "plan_create_buffers (NULL): %d", rc);
    if (rc == 0) {
        const uint64_t nz = crc32c_plan_nchecksums(plan);
        CHECK(nz == 8192, "ftruncate: %" PRIu64 " checksums", nz);
        uint32_t *d_z;
        HIP_OK(hipMalloc((void **)&d_z, nz * 4));
        CHECK(crc32c_plan_exec(plan, NULL, d_z, NULL) == 0, "plan_exec (NULL)");
        HIP_OK(hipDeviceSynchronize());
        uint32_t *z = malloc(nz * 4);
        HIP_OK(hipMemcpy(z, d_z, nz * 4, hipMemcpyDeviceToHost));
        const uint8_t zero512[512] = {0};
        const uint32_t c = htonl(crc32c(0, zero512, 512)); /* 30fcedc0 */
        uint64_t zb = 0;
        for (uint64_t k = 0; k < nz; ++k) zb += z[k] != c;
        CHECK(zb == 0, "ftruncate: %" PRIu64 " checksums differ from crc32c(512 zeros)", zb);
        free(z);
        HIP_OK(hipFree(d_z));
        crc32c_plan_destroy(plan);
    }

    printf("%s: %" PRIu64 " + %" PRIu64 " (NULL) + %" PRIu64 " + %" PRIu64 " bytes at block offset %" PRIu64
           ", bpc %u, %" PRIu64 " checksums\n",
           fails ? "FAILED" : "ok", lens[0], lens[1], lens[2], lens[3], blockoffset, bpc, n);
    crc32c_ctx_destroy(ctx);
    for (int i = 0; i < 4; ++i)
        if (dev[i]) HIP_OK(hipFree(dev[i]));
    HIP_OK(hipFree(d_sums));
    free(got);
    free(want);
    free(stream);
    return fails ? 1 : 0;
}
