/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives the UNMODIFIED reference implementation (/root/reference/src/crc32c.c,
 * compiled where it lies by oracle/Makefile into oracle/_ref/) the way the
 * reference's packet writer does: one crc32c(0, chunk, min(bpc, len - i*bpc))
 * call per chunk (src/hadooprpc.c:733-742). Used to generate golden fixtures
 * (tests/golden/make_golden.py) and as bench.py's cpu_baseline
 * ("kind": "reference"). No reference source is copied into this repository.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

/* The reference exports exactly this symbol (src/crc32c.c:333) and its only
 * caller declares it by hand (src/hadooprpc.c:31). */
uint32_t crc32c(uint32_t crc, const void *buf, size_t len);

uint32_t ref_crc32c(uint32_t crc, const void *buf, size_t len)
{
    return crc32c(crc, buf, len);
}

typedef struct {
    uint64_t payload_off;
    uint64_t out_idx;
    uint32_t len;
    uint32_t bpc;
} ref_packet;

/* hadooprpc.c:639 + 733-742 for one packet. */
static void ref_packet_chunks(const uint8_t *packet, uint64_t len, uint32_t bpc, uint32_t *out)
{
    uint64_t n = (len + bpc - 1) / bpc;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t idx = i * (uint64_t)bpc;
        uint64_t m = len - idx < bpc ? len - idx : bpc;
        out[i] = crc32c(0, packet + idx, (size_t)m);
    }
}

void ref_batch(const void *payload, const ref_packet *pkts, uint64_t npkts, uint32_t *out)
{
    for (uint64_t i = 0; i < npkts; i++)
        ref_packet_chunks((const uint8_t *)payload + pkts[i].payload_off, pkts[i].len, pkts[i].bpc,
                          out + pkts[i].out_idx);
}

typedef struct {
    const uint8_t *payload;
    const ref_packet *pkts;
    uint64_t lo, hi;
    uint32_t *out;
} ref_job;

static void *ref_worker(void *arg)
{
    ref_job *j = (ref_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++)
        ref_packet_chunks(j->payload + j->pkts[i].payload_off, j->pkts[i].len, j->pkts[i].bpc,
                          j->out + j->pkts[i].out_idx);
    return NULL;
}

/* The batch on nthreads threads (contiguous packet slices), `reps` times.
 * Returns elapsed wall seconds. */
double ref_batch_mt(const void *payload, const ref_packet *pkts, uint64_t npkts, uint32_t *out, int nthreads,
                    int reps)
{
    enum { MAXT = 256 };
    pthread_t th[MAXT];
    ref_job jobs[MAXT];
    struct timespec t0, t1;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > MAXT)
        nthreads = MAXT;
    /* First call resolves the reference's lazy SSE4.2 dispatch (crc32c.c:335-341)
     * outside the timed region so threads do not race on it. */
    (void)crc32c(0, "", 0);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        for (int t = 0; t < nthreads; t++) {
            jobs[t].payload = (const uint8_t *)payload;
            jobs[t].pkts = pkts;
            jobs[t].lo = npkts * (uint64_t)t / (uint64_t)nthreads;
            jobs[t].hi = npkts * (uint64_t)(t + 1) / (uint64_t)nthreads;
            jobs[t].out = out;
            pthread_create(&th[t], NULL, ref_worker, &jobs[t]);
        }
        for (int t = 0; t < nthreads; t++)
            pthread_join(th[t], NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- cpu_baseline at full host width, streaming from DRAM ----------------
 * nbuf distinct copies of the batch (first-touched by the threads that read
 * them, so each NUMA node streams its own memory), nthreads persistent
 * threads each owning a contiguous packet slice, rep r reading copy r % nbuf:
 * consecutive reps cannot be served from the L3.  Timed from the moment
 * every thread is ready to the last thread's finish.  Returns wall seconds,
 * or a negative value when memory could not be allocated. */
typedef struct {
    const uint8_t *src;
    uint8_t **bufs;
    int nbuf, reps;
    const ref_packet *pkts;
    uint64_t lo, hi;
    uint32_t *out;
    pthread_barrier_t *ready, *go;
} ref_rot_job;

static void *ref_rot_worker(void *arg)
{
    ref_rot_job *j = (ref_rot_job *)arg;
    if (j->hi > j->lo) {
        uint64_t b0 = j->pkts[j->lo].payload_off, b1 = b0;
        for (uint64_t i = j->lo; i < j->hi; i++) {
            if (j->pkts[i].payload_off < b0)
                b0 = j->pkts[i].payload_off;
            if (j->pkts[i].payload_off + j->pkts[i].len > b1)
                b1 = j->pkts[i].payload_off + j->pkts[i].len;
        }
        for (int b = 0; b < j->nbuf; b++)
            for (uint64_t o = b0; o < b1; o++)
                j->bufs[b][o] = j->src[o];
    }
    pthread_barrier_wait(j->ready);
    pthread_barrier_wait(j->go);
    for (int r = 0; r < j->reps; r++) {
        const uint8_t *p = j->bufs[r % j->nbuf];
        for (uint64_t i = j->lo; i < j->hi; i++)
            ref_packet_chunks(p + j->pkts[i].payload_off, j->pkts[i].len, j->pkts[i].bpc, j->out + j->pkts[i].out_idx);
    }
    return NULL;
}

double ref_batch_mt_rot(const void *payload, uint64_t bytes, const ref_packet *pkts, uint64_t npkts, uint32_t *out,
                        int nthreads, int nbuf, int reps)
{
    enum { MAXT = 1024, MAXB = 16 };
    static pthread_t th[MAXT];
    static ref_rot_job jobs[MAXT];
    uint8_t *bufs[MAXB];
    pthread_barrier_t ready, go;
    struct timespec t0, t1;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > MAXT)
        nthreads = MAXT;
    if (nbuf < 1)
        nbuf = 1;
    if (nbuf > MAXB)
        nbuf = MAXB;
    for (int b = 0; b < nbuf; b++) {
        bufs[b] = (uint8_t *)malloc(bytes ? bytes : 1);
        if (!bufs[b]) {
            for (int k = 0; k < b; k++)
                free(bufs[k]);
            return -1.0;
        }
    }
    (void)crc32c(0, "", 0);
    pthread_barrier_init(&ready, NULL, (unsigned)nthreads + 1);
    pthread_barrier_init(&go, NULL, (unsigned)nthreads + 1);
    for (int t = 0; t < nthreads; t++) {
        jobs[t].src = (const uint8_t *)payload;
        jobs[t].bufs = bufs;
        jobs[t].nbuf = nbuf;
        jobs[t].reps = reps;
        jobs[t].pkts = pkts;
        jobs[t].lo = npkts * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].hi = npkts * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].out = out;
        jobs[t].ready = &ready;
        jobs[t].go = &go;
        pthread_create(&th[t], NULL, ref_rot_worker, &jobs[t]);
    }
    pthread_barrier_wait(&ready);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_barrier_wait(&go);
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    pthread_barrier_destroy(&ready);
    pthread_barrier_destroy(&go);
    for (int b = 0; b < nbuf; b++)
        free(bufs[b]);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- per-block latency: one batch split over nthreads, reps times ---------
 * The reference's unit of work is one block written by one libfuse worker
 * (src/fuse.c:336-449); this times one call over the batch (e.g. one 4 MiB
 * block) as a caller would issue it: the batch split into nthreads
 * contiguous packet slices computed at once by persistent threads (the
 * calling thread is slice 0), each rep between two barriers.  Returns the
 * mean wall seconds per rep (in-cache: the same buffer every rep, as a block
 * just written by the application). */
typedef struct {
    const uint8_t *payload;
    const ref_packet *pkts;
    uint64_t lo, hi;
    uint32_t *out;
    int reps;
    pthread_barrier_t *bar;
} ref_lat_job;

static void ref_lat_slice(const ref_lat_job *j)
{
    for (uint64_t i = j->lo; i < j->hi; i++)
        ref_packet_chunks(j->payload + j->pkts[i].payload_off, j->pkts[i].len, j->pkts[i].bpc,
                          j->out + j->pkts[i].out_idx);
}

static void *ref_lat_worker(void *arg)
{
    ref_lat_job *j = (ref_lat_job *)arg;
    for (int r = 0; r < j->reps; r++) {
        pthread_barrier_wait(j->bar);
        ref_lat_slice(j);
        pthread_barrier_wait(j->bar);
    }
    return NULL;
}

double ref_block_latency(const void *payload, const ref_packet *pkts, uint64_t npkts, uint32_t *out, int nthreads,
                         int reps)
{
    enum { MAXT = 256 };
    pthread_t th[MAXT];
    ref_lat_job jobs[MAXT];
    pthread_barrier_t bar;
    struct timespec t0, t1;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > MAXT)
        nthreads = MAXT;
    if (reps < 1)
        reps = 1;
    (void)crc32c(0, "", 0);
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (int t = 0; t < nthreads; t++) {
        jobs[t].payload = (const uint8_t *)payload;
        jobs[t].pkts = pkts;
        jobs[t].lo = npkts * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].hi = npkts * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].out = out;
        jobs[t].reps = reps;
        jobs[t].bar = &bar;
        if (t)
            pthread_create(&th[t], NULL, ref_lat_worker, &jobs[t]);
    }
    ref_lat_slice(&jobs[0]); /* (warm: caches, page mappings) */
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        pthread_barrier_wait(&bar);
        ref_lat_slice(&jobs[0]);
        pthread_barrier_wait(&bar);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (int t = 1; t < nthreads; t++)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&bar);
    return ((double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec)) / reps;
}
