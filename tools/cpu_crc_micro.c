/* cpu_crc_micro.c -- DIAGNOSTIC: single-thread host CRC32C per 512-byte chunk on
 * this machine's CPU, L2-resident (256 KiB) and streaming (256 MiB):
 *   serial   one dependent crc32q chain per chunk (the reference's path for
 *            512 B, crc32c.c:293-299; restated here, not copied)
 *   scalar   libhdfs_crc32c.so crc32c() per chunk (three 168-byte stripes)
 *   chunks   crc32c_chunks_cpu() (three chunks as interleaved chains)
 *   cc -O2 -msse4.2 -Iinclude tools/cpu_crc_micro.c -Lnative-hdfs-fuse_amd -lhdfs_crc32c */
#include <nmmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hdfs_crc32c.h"

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint32_t serial512(const uint8_t *p) {
    uint64_t r = 0xffffffffu;
    for (int i = 0; i < 512; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        r = _mm_crc32_u64(r, w);
    }
    return ~(uint32_t)r;
}

int main(void) {
    const size_t sizes[2] = {256u << 10, 256u << 20};
    uint8_t *b = malloc(sizes[1]);
    uint32_t *o = malloc(sizes[1] / 512 * 4);
    for (size_t i = 0; i < sizes[1]; ++i) b[i] = (uint8_t)((i * 2654435761u) >> 13);
    for (int s = 0; s < 2; ++s) {
        const size_t n = sizes[s], reps = (size_t)(2u << 30) / n;
        for (int round = 0; round < 2; ++round) {
            double t0 = now();
            for (size_t r = 0; r < reps; ++r)
                for (size_t i = 0; i < n / 512; ++i) o[i] = serial512(b + i * 512);
            double t1 = now();
            uint32_t chk = o[n / 512 - 1];
            for (size_t r = 0; r < reps; ++r)
                for (size_t i = 0; i < n / 512; ++i) o[i] = crc32c(0, b + i * 512, 512);
            double t2 = now();
            if (o[n / 512 - 1] != chk) return 2;
            for (size_t r = 0; r < reps; ++r) crc32c_chunks_cpu(b, n, 512, o, 0);
            double t3 = now();
            if (o[n / 512 - 1] != chk) return 3;
            const double g = (double)n * reps / 1073741824.0;
            printf("%s: serial %.2f  scalar %.2f  chunks %.2f GiB/s\n", s ? "256 MiB" : "256 KiB", g / (t1 - t0),
                   g / (t2 - t1), g / (t3 - t2));
        }
    }
    return 0;
}
