/*
 * zk_kv_port.c — TEST/BENCH INFRASTRUCTURE ONLY: a multithreaded C restatement of the key-value
 * popularity sketch behind Aggregates.getTopKeyValueAnnotations
 * (zipkin-common/src/main/scala/com/twitter/zipkin/storage/Aggregates.scala:34; the top lists the
 * reference stores, CassandraAggregates.scala:86-88,100-108), for one batch from a reset sketch.
 * It is the C4 line's parity checker on large prefixes and its CPU baseline (kind "port"); it
 * restates oracle/kv.py (the numpy definition, pinned against it by tests/test_kv.py) for speed:
 *
 *   per service a count-min sketch of `depth` rows x `width` counters: h = mix64(key ^ seed0),
 *   seed0 = mix64(seed + GOLDEN), row r of key k = the top log2(width) bits of the 32-bit
 *   (lo32(h) + r * (hi32(h) | 1)); per service the best `cand` distinct keys of the batch by
 *   (estimate desc, key asc), estimates read from the counters after the whole batch.
 *
 * Pass 1 (threads over item ranges): counters by relaxed atomic adds, per-service totals, and a
 * service histogram per thread. Pass 2: items scattered into service order. Pass 3 (threads over
 * services): sort the service's keys, estimate every distinct key, keep the best `cand`.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define GOLDEN 0x9E3779B97F4A7C15ull

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct {
    const uint32_t* svc;
    const uint64_t* keys;
    uint64_t n, lo, hi;
    uint32_t S, width, depth, cand, wbits;
    uint64_t seed0;
    uint32_t* cm;        /* [S][depth][width] */
    uint64_t* totals;    /* [S] */
    uint64_t* hist;      /* [threads][S + 1] */
    uint64_t* sorted;    /* keys in service order */
    uint64_t* base;      /* [S + 1] service starts in `sorted` */
    uint64_t* out_keys;  /* [S][cand] */
    uint32_t* out_est;   /* [S][cand] */
    uint32_t* out_cnt;   /* [S] */
    int tid, nthreads;
    uint64_t dropped;
} kv_job;

static inline uint32_t row_idx(uint64_t h, uint32_t r, uint32_t wbits) {
    const uint32_t h1 = (uint32_t)h, h2 = (uint32_t)(h >> 32) | 1u;
    return (uint32_t)(h1 + r * h2) >> (32 - wbits);
}

static void* pass1(void* p) {
    kv_job* j = (kv_job*)p;
    uint64_t* h = j->hist + (uint64_t)j->tid * (j->S + 1);
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint32_t s = j->svc[i];
        if (s >= j->S) {
            ++j->dropped;
            continue;
        }
        const uint64_t hh = mix64(j->keys[i] ^ j->seed0);
        uint32_t* row = j->cm + (uint64_t)s * j->depth * j->width;
        for (uint32_t r = 0; r < j->depth; ++r)
            __atomic_fetch_add(&row[(uint64_t)r * j->width + row_idx(hh, r, j->wbits)], 1u, __ATOMIC_RELAXED);
        ++h[s];
    }
    return NULL;
}

static void* pass2(void* p) {
    kv_job* j = (kv_job*)p;
    uint64_t* cur = j->hist + (uint64_t)j->tid * (j->S + 1);  /* this thread's start per service */
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint32_t s = j->svc[i];
        if (s < j->S) j->sorted[cur[s]++] = j->keys[i];
    }
    return NULL;
}

static int cmp_u64(const void* a, const void* b) {
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* (estimate desc, key asc): does (e1, k1) rank before (e2, k2)? */
static inline int better(uint32_t e1, uint64_t k1, uint32_t e2, uint64_t k2) {
    return e1 > e2 || (e1 == e2 && k1 < k2);
}

static void* pass3(void* p) {
    kv_job* j = (kv_job*)p;
    for (uint32_t s = (uint32_t)j->tid; s < j->S; s += (uint32_t)j->nthreads) {
        uint64_t* k = j->sorted + j->base[s];
        const uint64_t m = j->base[s + 1] - j->base[s];
        qsort(k, m, 8, cmp_u64);
        uint64_t* ok = j->out_keys + (uint64_t)s * j->cand;
        uint32_t* oe = j->out_est + (uint64_t)s * j->cand;
        uint32_t cnt = 0;  /* ok/oe kept sorted best first; insertion into a list of <= cand */
        const uint32_t* cm = j->cm + (uint64_t)s * j->depth * j->width;
        for (uint64_t i = 0; i < m; ++i) {
            if (i > 0 && k[i] == k[i - 1]) continue;
            const uint64_t hh = mix64(k[i] ^ j->seed0);
            uint32_t e = 0xFFFFFFFFu;
            for (uint32_t r = 0; r < j->depth; ++r) {
                const uint32_t c = cm[(uint64_t)r * j->width + row_idx(hh, r, j->wbits)];
                if (c < e) e = c;
            }
            if (cnt == j->cand && !better(e, k[i], oe[cnt - 1], ok[cnt - 1])) continue;
            uint32_t at = cnt < j->cand ? cnt : j->cand - 1;
            while (at > 0 && better(e, k[i], oe[at - 1], ok[at - 1])) {
                oe[at] = oe[at - 1];
                ok[at] = ok[at - 1];
                --at;
            }
            oe[at] = e;
            ok[at] = k[i];
            if (cnt < j->cand) ++cnt;
        }
        j->out_cnt[s] = cnt;
    }
    return NULL;
}

static void run(kv_job* jobs, int T, void* (*fn)(void*)) {
    pthread_t th[256];
    for (int t = 1; t < T; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    fn(&jobs[0]);
    for (int t = 1; t < T; ++t) pthread_join(th[t], NULL);
}

/* One batch into a fresh sketch. Outputs: cm [S][depth][width] (u32), totals [S], the top lists
 * out_keys / out_est [S][cand] best first (zero past out_cnt[s]), *dropped = items with svc >= S.
 * Returns 0, or -1 on bad arguments / no memory. *seconds = wall time of the three passes. */
int zkv_port(const uint32_t* svc, const uint64_t* keys, uint64_t n, uint32_t S, uint32_t width, uint32_t depth,
             uint32_t cand, uint64_t seed, int threads, uint32_t* cm, uint64_t* totals, uint64_t* out_keys,
             uint32_t* out_est, uint32_t* out_cnt, uint64_t* dropped, double* seconds) {
    if (S == 0 || width < 2 || (width & (width - 1)) || depth == 0 || cand == 0) return -1;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint32_t wbits = 0;
    while ((1u << wbits) < width) ++wbits;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    memset(cm, 0, (size_t)S * depth * width * 4);
    memset(out_keys, 0, (size_t)S * cand * 8);
    memset(out_est, 0, (size_t)S * cand * 4);
    uint64_t* hist = calloc((size_t)threads * (S + 1), 8);
    uint64_t* sorted = malloc((n ? n : 1) * 8);
    uint64_t* base = calloc(S + 1, 8);
    kv_job* jobs = calloc(threads, sizeof(kv_job));
    if (!hist || !sorted || !base || !jobs) {
        free(hist), free(sorted), free(base), free(jobs);
        return -1;
    }
    for (int t = 0; t < threads; ++t) {
        kv_job* j = &jobs[t];
        j->svc = svc, j->keys = keys, j->n = n, j->S = S, j->width = width, j->depth = depth, j->cand = cand;
        j->wbits = wbits, j->seed0 = mix64(seed + GOLDEN), j->cm = cm, j->totals = totals, j->hist = hist;
        j->sorted = sorted, j->base = base, j->out_keys = out_keys, j->out_est = out_est, j->out_cnt = out_cnt;
        j->tid = t, j->nthreads = threads;
        j->lo = n * (uint64_t)t / threads, j->hi = n * (uint64_t)(t + 1) / threads;
    }
    run(jobs, threads, pass1);
    /* service starts, and each thread's start inside its service's run (thread order = item order) */
    uint64_t pos = 0;
    *dropped = 0;
    for (uint32_t s = 0; s < S; ++s) {
        base[s] = pos;
        totals[s] = 0;
        for (int t = 0; t < threads; ++t) {
            const uint64_t c = hist[(uint64_t)t * (S + 1) + s];
            hist[(uint64_t)t * (S + 1) + s] = pos;
            pos += c;
            totals[s] += c;
        }
    }
    base[S] = pos;
    for (int t = 0; t < threads; ++t) *dropped += jobs[t].dropped;
    run(jobs, threads, pass2);
    run(jobs, threads, pass3);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    free(hist), free(sorted), free(base), free(jobs);
    return 0;
}
