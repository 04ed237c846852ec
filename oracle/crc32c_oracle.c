/*
 * crc32c_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A clean-room CPU restatement of the reference's per-chunk CRC32C path, used
 * as the parity checker for the HIP implementation. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code.
 * The product library (native-hdfs-fuse_amd/csrc) never links it.
 *
 * Parity pin: this restatement is checked against
 *   - the RFC 3720 B.4 / "123456789" known answers (tests/golden/known_answers.json),
 *   - outputs of the reference itself (/root/reference/src/crc32c.c compiled by
 *     oracle/Makefile into oracle/_ref/, see tests/golden/make_golden.py).
 *
 * Reference algorithm being restated (file:line under /root/reference):
 *   src/crc32c.c:43        reflected Castagnoli polynomial 0x82f63b78
 *   src/crc32c.c:50-73     byte table and slicing-by-8 tables
 *   src/crc32c.c:78-107    pre-inversion, byte/word update, post-inversion
 *   src/crc32c.c:333-343   public entry point crc32c(crc, buf, len)
 *   src/hadooprpc.c:639    n_checksums = roundup(len, bytesperchecksum)
 *   src/hadooprpc.c:733-742 per-chunk loop crc32c(0, packet + i*bpc, min(bpc, len - i*bpc))
 *   src/hadooprpc.c:71-75  htonl() of every checksum on the wire
 *   src/hadooprpc.c:827-857 packetisation (packet = min(remaining, packetsize),
 *                           first packet trimmed to a chunk boundary, final empty packet)
 *   src/roundup.h:7-11, src/minmax.h:9-19 ceil-div and min
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#define ORACLE_POLY 0x82f63b78u /* crc32c.c:43 */

static uint32_t g_tab[8][256];
static pthread_once_t g_tab_once = PTHREAD_ONCE_INIT;

/* crc32c.c:50-73: T0[b] is eight reflected shift/xor steps on b; Tk[b] is
 * T0 applied to T(k-1)[b] shifted by one more byte. */
static void oracle_build_tables(void)
{
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t r = b;
        for (int bit = 0; bit < 8; bit++)
            r = (r >> 1) ^ (ORACLE_POLY & (0u - (r & 1u)));
        g_tab[0][b] = r;
    }
    for (uint32_t b = 0; b < 256; b++)
        for (int k = 1; k < 8; k++)
            g_tab[k][b] = (g_tab[k - 1][b] >> 8) ^ g_tab[0][g_tab[k - 1][b] & 0xffu];
}

/* Byte-at-a-time restatement of crc32c_sw's scalar loops (crc32c.c:84-87,
 * 102-106). */
uint32_t oracle_crc32c_bytewise(uint32_t crc, const void *buf, size_t len)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t r = ~crc;
    pthread_once(&g_tab_once, oracle_build_tables);
    for (size_t i = 0; i < len; i++)
        r = (r >> 8) ^ g_tab[0][(r ^ p[i]) & 0xffu];
    return ~r;
}

/* Slicing-by-8 restatement of crc32c_sw (crc32c.c:78-107); little-endian
 * load of each 8-byte word, as the reference assumes (crc32c.c:75-77). The
 * result must not depend on the alignment of buf. */
uint32_t oracle_crc32c_slice8(uint32_t crc, const void *buf, size_t len)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint64_t r = (uint64_t)(~crc);
    pthread_once(&g_tab_once, oracle_build_tables);
    while (len && ((uintptr_t)p & 7u)) {
        r = (r >> 8) ^ g_tab[0][(r ^ *p++) & 0xffu];
        len--;
    }
    for (; len >= 8; len -= 8, p += 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        w ^= r;
        r = g_tab[7][w & 0xff] ^ g_tab[6][(w >> 8) & 0xff] ^ g_tab[5][(w >> 16) & 0xff] ^
            g_tab[4][(w >> 24) & 0xff] ^ g_tab[3][(w >> 32) & 0xff] ^ g_tab[2][(w >> 40) & 0xff] ^
            g_tab[1][(w >> 48) & 0xff] ^ g_tab[0][w >> 56];
    }
    while (len--)
        r = (r >> 8) ^ g_tab[0][(r ^ *p++) & 0xffu];
    return ~(uint32_t)r;
}

static inline uint32_t oracle_bswap32(uint32_t v)
{
    return (v >> 24) | ((v >> 8) & 0xff00u) | ((v << 8) & 0xff0000u) | (v << 24);
}

/* Number of checksums of one packet: roundup(len, bpc), hadooprpc.c:639 and
 * roundup.h:7-11. */
uint64_t oracle_nchunks(uint64_t len, uint32_t bpc)
{
    return bpc ? (len + bpc - 1) / bpc : 0;
}

/* One packet, exactly hadooprpc.c:733-742: chunk i covers
 * [i*bpc, i*bpc + min(bpc, len - i*bpc)) and is checksummed from crc = 0.
 * big_endian != 0 stores htonl() of each value (hadooprpc.c:71-75). */
uint64_t oracle_chunks(const void *packet, uint64_t len, uint32_t bpc, uint32_t *out, int big_endian)
{
    const uint8_t *p = (const uint8_t *)packet;
    uint64_t n = oracle_nchunks(len, bpc);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t at = i * (uint64_t)bpc;
        uint64_t m = len - at < bpc ? len - at : bpc;
        uint32_t c = oracle_crc32c_slice8(0, p + at, (size_t)m);
        out[i] = big_endian ? oracle_bswap32(c) : c;
    }
    return n;
}

/* A batch descriptor mirrors the product ABI's crc32c_packet. */
typedef struct {
    uint64_t payload_off;
    uint64_t out_idx;
    uint32_t len;
    uint32_t bpc;
} oracle_packet;

void oracle_batch(const void *payload, const oracle_packet *pkts, uint64_t npkts, uint32_t *out, int big_endian)
{
    const uint8_t *base = (const uint8_t *)payload;
    for (uint64_t i = 0; i < npkts; i++)
        oracle_chunks(base + pkts[i].payload_off, pkts[i].len, pkts[i].bpc, out + pkts[i].out_idx, big_endian);
}

/* Packetisation of one block write, hadooprpc.c:827-857: packet length is
 * min(len - sent, packetsize); if the packet would start off a chunk
 * boundary it is trimmed to finish the partial chunk (hadooprpc.c:832-840);
 * a zero-length packet terminates the block (hadooprpc.c:644, 853-856).
 * Writes up to max lengths and returns the number of packets produced. */
uint64_t oracle_packetize(uint64_t len, uint64_t blockoffset, uint32_t packetsize, uint32_t bpc,
                          uint64_t *lens, uint64_t max)
{
    uint64_t sent = 0, n = 0;
    for (;;) {
        uint64_t plen = len - sent < packetsize ? len - sent : packetsize;
        uint64_t past = (blockoffset + sent) % bpc;
        if (plen > 0 && past != 0) {
            plen = bpc - past;
            /* hadooprpc.c:622 only asserts the trimmed packet fits; a trim past
             * the remaining bytes is undefined there, so it is clamped here. */
            if (plen > len - sent)
                plen = len - sent;
        }
        if (n < max)
            lens[n] = plen;
        n++;
        if (plen == 0)
            break;
        sent += plen;
    }
    return n;
}

/* Synthetic payload generator used by the fixtures and the bench (SURVEY.md
 * §8d): xorshift64 (13, 7, 17), each state emitted as 8 little-endian bytes. */
void oracle_xorshift64_fill(uint64_t seed, void *buf, uint64_t len)
{
    uint8_t *p = (uint8_t *)buf;
    uint64_t s = seed ? seed : 0x9E3779B97F4A7C15ull;
    uint64_t i = 0;
    while (i < len) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        for (int b = 0; b < 8 && i < len; b++, i++)
            p[i] = (uint8_t)(s >> (8 * b));
    }
}

/* ---- multi-threaded timing harness for the "port" CPU baseline ---- */
typedef struct {
    const uint8_t *payload;
    const oracle_packet *pkts;
    uint64_t lo, hi;
    uint32_t *out;
} oracle_job;

static void *oracle_worker(void *arg)
{
    oracle_job *j = (oracle_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++)
        oracle_chunks(j->payload + j->pkts[i].payload_off, j->pkts[i].len, j->pkts[i].bpc,
                      j->out + j->pkts[i].out_idx, 0);
    return NULL;
}

/* Runs the batch on nthreads threads (contiguous packet slices) `reps`
 * times; returns elapsed seconds. */
double oracle_batch_mt(const void *payload, const oracle_packet *pkts, uint64_t npkts, uint32_t *out,
                       int nthreads, int reps)
{
    enum { MAXT = 256 };
    pthread_t th[MAXT];
    oracle_job jobs[MAXT];
    struct timespec t0, t1;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > MAXT)
        nthreads = MAXT;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        for (int t = 0; t < nthreads; t++) {
            jobs[t].payload = (const uint8_t *)payload;
            jobs[t].pkts = pkts;
            jobs[t].lo = npkts * (uint64_t)t / (uint64_t)nthreads;
            jobs[t].hi = npkts * (uint64_t)(t + 1) / (uint64_t)nthreads;
            jobs[t].out = out;
            pthread_create(&th[t], NULL, oracle_worker, &jobs[t]);
        }
        for (int t = 0; t < nthreads; t++)
            pthread_join(th[t], NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
