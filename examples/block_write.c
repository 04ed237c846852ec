/* block_write.c -- the reference's block-write checksum path, written the way
 * INTEGRATION.md tells a maintainer to call libhdfs_crc32c.so from C.
 *
 * For one block write of `len` bytes at `blockoffset` (defaults: a 4 MiB
 * block at 0, 64 KiB packets, 512-byte chunks):
 *   1. cut it into packets like hadoop_rpc_send_packets (hadooprpc.c:815-860)
 *      with crc32c_packetize;
 *   2. checksum every packet at once with crc32c_batch_host, in wire order;
 *   3. frame every packet's PLEN | HLEN | header | checksums prefix with
 *      crc32c_frame_packets (hadooprpc.c:596-664, 733-748);
 *   4. verify the block with crc32c_verify_host, then again with one flipped
 *      checksum;
 * and checks each step against the per-chunk loop of hadooprpc.c:733-742
 * done with the drop-in scalar crc32c().  Exit status 0 = all exact.
 *
 *   block_write [len [blockoffset [bpc]]]
 *   block_write --cpu      (no GPU: scalar, packetize and framing only; the GPU
 *                           entry points must fail with -ENODEV)
 */
#include <arpa/inet.h>
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hdfs_crc32c.h"

static int fails = 0;
#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fputc('\n', stderr);                          \
            ++fails;                                      \
        }                                                 \
    } while (0)

static uint64_t xs = 0x9E3779B97F4A7C15ull;
static uint8_t next_byte(void) {
    xs ^= xs << 13;
    xs ^= xs >> 7;
    xs ^= xs << 17;
    return (uint8_t)(xs >> 56);
}

int main(int argc, char **argv) {
    int cpu_only = argc > 1 && strcmp(argv[1], "--cpu") == 0;
    int a = cpu_only ? 2 : 1;
    const uint64_t len = argc > a ? strtoull(argv[a], NULL, 0) : (4u << 20);
    const uint64_t blockoffset = argc > a + 1 ? strtoull(argv[a + 1], NULL, 0) : 0;
    const uint32_t bpc = argc > a + 2 ? (uint32_t)strtoul(argv[a + 2], NULL, 0) : 512;
    const uint32_t packetsize = 65536;

    uint8_t *data = malloc(len + 16);
    for (uint64_t i = 0; i < len; ++i) data[i] = next_byte();

    /* 1. packets of the block write */
    const uint64_t np = crc32c_packetize(len, blockoffset, packetsize, bpc, NULL, 0);
    uint64_t *lens = malloc(np * sizeof *lens);
    crc32c_packetize(len, blockoffset, packetsize, bpc, lens, np);
    crc32c_packet *pk = malloc(np * sizeof *pk);
    uint64_t off = 0, nsum = 0;
    for (uint64_t i = 0; i < np; ++i) {
        pk[i].payload_off = off;
        pk[i].out_idx = nsum;
        pk[i].len = (uint32_t)lens[i];
        pk[i].bpc = bpc;
        off += lens[i];
        nsum += crc32c_nchunks(lens[i], bpc);
    }
    CHECK(off == len, "packets cover %" PRIu64 " of %" PRIu64 " bytes", off, len);
    CHECK(lens[np - 1] == 0, "no final empty packet");
    CHECK(crc32c_batch_nchecksums(pk, np) == nsum, "batch_nchecksums");

    /* the reference's loop: crc32c(0, packet + i*bpc, min(bpc, len - i*bpc)), htonl */
    uint32_t *want = malloc((nsum + 1) * sizeof *want);
    for (uint64_t p = 0; p < np; ++p)
        for (uint64_t i = 0; i < crc32c_nchunks(pk[p].len, bpc); ++i) {
            const uint64_t o = (uint64_t)i * bpc;
            const uint64_t n = pk[p].len - o < bpc ? pk[p].len - o : bpc;
            want[pk[p].out_idx + i] = htonl(crc32c(0, data + pk[p].payload_off + o, n));
        }

    /* 2. all checksums of the block in one call */
    uint32_t *sums = calloc(nsum + 1, sizeof *sums);
    crc32c_ctx *ctx = NULL;
    int rc = crc32c_ctx_create(0, &ctx);
    if (cpu_only) {
        CHECK(rc == -ENODEV, "ctx_create without a GPU: %d", rc);
        CHECK(crc32c_chunks(data, 1000, 512, sums, 0) == -ENODEV, "crc32c_chunks without a GPU");
        memcpy(sums, want, nsum * sizeof *sums);
    } else {
        CHECK(rc == 0, "ctx_create: %d (%s)", rc, crc32c_last_error());
        if (rc) return 1;
        rc = crc32c_batch_host(ctx, data, pk, np, sums, CRC32C_BIG_ENDIAN);
        CHECK(rc == 0, "batch_host: %d (%s)", rc, crc32c_last_error());
        uint64_t bad = 0;
        for (uint64_t k = 0; k < nsum; ++k) bad += sums[k] != want[k];
        CHECK(bad == 0, "%" PRIu64 " of %" PRIu64 " checksums differ from crc32c()", bad, nsum);
    }

    /* 3. one prefix per packet: PLEN | HLEN | PacketHeaderProto | checksums */
    const size_t need = crc32c_frame_packets(pk, np, sums, CRC32C_BIG_ENDIAN, blockoffset, 0, 4, NULL, 0, NULL);
    uint8_t *prefix = malloc(need);
    uint64_t *poff = malloc((np + 1) * sizeof *poff);
    CHECK(crc32c_frame_packets(pk, np, sums, CRC32C_BIG_ENDIAN, blockoffset, 0, 4, prefix, need, poff) == need,
          "frame_packets size");
    for (uint64_t p = 0; p < np; ++p) {
        const uint8_t *q = prefix + poff[p];
        const uint64_t n = crc32c_nchunks(pk[p].len, bpc);
        uint32_t plen;
        uint16_t hlen;
        memcpy(&plen, q, 4);
        memcpy(&hlen, q + 4, 2);
        CHECK(ntohl(plen) == 4 + 4 * n + pk[p].len, "packet %" PRIu64 ": PLEN", p);  /* hadooprpc.c:640 */
        CHECK(poff[p + 1] - poff[p] == 6 + ntohs(hlen) + 4 * n, "packet %" PRIu64 ": prefix size", p);
        CHECK(memcmp(q + 6 + ntohs(hlen), want + pk[p].out_idx, 4 * n) == 0, "packet %" PRIu64 ": checksums", p);
    }

    /* 4. read side: verify the block, then with one flipped checksum */
    if (!cpu_only) {
        uint64_t first = 0;
        int64_t nbad = crc32c_verify_host(ctx, data, pk, np, want, CRC32C_BIG_ENDIAN, &first);
        CHECK(nbad == 0 && first == UINT64_MAX, "verify clean: %" PRId64, nbad);
        if (nsum > 3) {
            want[nsum / 3] ^= htonl(1);
            nbad = crc32c_verify_host(ctx, data, pk, np, want, CRC32C_BIG_ENDIAN, &first);
            CHECK(nbad == 1 && first == nsum / 3, "verify flipped: %" PRId64 " first %" PRIu64, nbad, first);
        }
        crc32c_ctx_destroy(ctx);
    }

    printf("%s: %" PRIu64 " bytes at %" PRIu64 ", %" PRIu64 " packets, %" PRIu64 " checksums, bpc %u%s\n",
           fails ? "FAILED" : "ok", len, blockoffset, np, nsum, bpc, cpu_only ? " (CPU only)" : "");
    free(poff);
    free(prefix);
    free(sums);
    free(want);
    free(pk);
    free(lens);
    free(data);
    return fails ? 1 : 0;
}
