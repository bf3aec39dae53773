/*
 * zk_rt_port.c — TEST/BENCH INFRASTRUCTURE ONLY: a multithreaded C restatement of the realtime span
 * sketches (include/zksketch.h zk_rt_*, BASELINE configs[4]: per-service distinct traceIds and
 * duration quantiles; RealtimeAggregates.scala:26-38 declares them, the reference implements none)
 * for one batch of TRACE-CLUSTERED span fragments into fresh sketches. It is the C5 line's parity
 * checker on large prefixes and its CPU baseline (kind "port"); it restates oracle/realtime.py (the
 * numpy definition, pinned against it by tests/test_realtime.py) for speed:
 *
 *   items: fragments grouped by (traceId, spanId) -- Span.mergeSpan (Span.scala:148-169) -- kept
 *   when every core annotation occurs at most once over the fragments (isValid, :236-240), some
 *   fragment names a service (serviceName, :125-131: server side first, then the lowest id) and
 *   some fragment has annotations; duration = max last - min first over those fragments (:228-230),
 *   dropped (counted) outside [0, 2^40) us;
 *   HyperLogLog: h = mix64(traceId ^ seed ^ SALT), register = top p bits, value = leading zeros of
 *   h << p plus one; log-linear histogram with m mantissa bits.
 *
 * Threads take contiguous record ranges cut at trace boundaries, each with private registers and
 * bins, merged by MAX / SUM at the end. Inside a trace the fragments are grouped by sorting their
 * spanIds.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define SALT 0xD6E8FEB86659FD93ull
#define F_HAS_ANNOTATIONS (1u << 1)
#define F_SVC_CLIENT (1u << 2)
#define F_SVC_SERVER (1u << 3)
#define MAX_DURATION (1ull << 40)
#define NO_KEY (1ull << 62)

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct {
    const uint64_t *tid, *sid;
    const int64_t *first, *last;
    const uint32_t *svc, *flags;
    uint64_t lo, hi;
    uint32_t S, p, m, nbins;
    uint64_t seed;
    uint8_t* regs;   /* [S][2^p] */
    uint64_t* hist;  /* [S][nbins] */
    uint64_t dropped_duration;
    int failed;
} rt_job;

static uint32_t bin_of(uint64_t d, uint32_t m) {
    if (d < (1ull << m)) return (uint32_t)d;
    const uint32_t e = 63u - (uint32_t)__builtin_clzll(d);
    return ((e - m + 1u) << m) | (uint32_t)((d >> (e - m)) & ((1ull << m) - 1ull));
}

typedef struct {
    uint64_t sid;
    uint64_t i;
} ent;

static int ent_cmp(const void* a, const void* b) {
    const ent *x = (const ent*)a, *y = (const ent*)b;
    if (x->sid != y->sid) return x->sid < y->sid ? -1 : 1;
    return x->i < y->i ? -1 : x->i > y->i;
}

static void item(rt_job* j, uint64_t key, uint64_t tid, uint64_t d) {
    const uint32_t s = (uint32_t)(key & ((1u << 30) - 1u));
    const uint64_t h = mix64(tid ^ j->seed ^ SALT);
    const uint64_t idx = h >> (64u - j->p);
    const uint64_t w = h << j->p;
    const uint8_t rho = (uint8_t)(w ? (uint64_t)__builtin_clzll(w) + 1u : 64u - j->p + 1u);
    uint8_t* r = j->regs + ((uint64_t)s << j->p) + idx;
    if (*r < rho) *r = rho;
    j->hist[(uint64_t)s * j->nbins + bin_of(d, j->m)] += 1;
}

static void* run(void* arg) {
    rt_job* j = (rt_job*)arg;
    uint64_t cap = 1024;
    ent* e = (ent*)malloc(cap * sizeof(ent));
    if (!e) {
        j->failed = 1;
        return NULL;
    }
    uint64_t a = j->lo;
    while (a < j->hi) {
        uint64_t b = a + 1;
        while (b < j->hi && j->tid[b] == j->tid[a]) ++b;
        const uint64_t L = b - a;
        if (L > cap) {
            while (cap < L) cap *= 2;
            ent* ne = (ent*)realloc(e, cap * sizeof(ent));
            if (!ne) {
                j->failed = 1;
                free(e);
                return NULL;
            }
            e = ne;
        }
        for (uint64_t k = 0; k < L; ++k) {
            e[k].sid = j->sid[a + k];
            e[k].i = a + k;
        }
        qsort(e, L, sizeof(ent), ent_cmp);
        for (uint64_t g = 0; g < L;) {  /* one span: the run of equal spanIds */
            uint64_t h = g;
            int64_t fmin = INT64_MAX, lmax = INT64_MIN;
            uint64_t key = NO_KEY;
            uint32_t cnt[4] = {0, 0, 0, 0};
            while (h < L && e[h].sid == e[g].sid) {
                const uint64_t i = e[h].i;
                const uint32_t f = j->flags[i];
                if (f & F_HAS_ANNOTATIONS) {
                    if (j->first[i] < fmin) fmin = j->first[i];
                    if (j->last[i] > lmax) lmax = j->last[i];
                }
                const uint64_t kind = (f & F_SVC_SERVER) ? 0 : (f & F_SVC_CLIENT) ? 1 : 2;
                if (kind < 2 && j->svc[i] < j->S) {
                    const uint64_t k = (kind << 30) | j->svc[i];
                    if (k < key) key = k;
                }
                for (int c = 0; c < 4; ++c) cnt[c] += (f >> (8 + 2 * c)) & 3u;
                ++h;
            }
            const int valid = cnt[0] <= 1 && cnt[1] <= 1 && cnt[2] <= 1 && cnt[3] <= 1;
            if (valid && key != NO_KEY && fmin != INT64_MAX) {
                const int64_t d = lmax - fmin;
                if (d < 0 || (uint64_t)d >= MAX_DURATION)
                    j->dropped_duration += 1;
                else
                    item(j, key, j->tid[a], (uint64_t)d);
            }
            g = h;
        }
        a = b;
    }
    free(e);
    return NULL;
}

/* regs u8[S][2^p] and hist u64[S][(41-m) << m] are zeroed and filled here; dropped[0] = service
   (always 0: keys are < S), dropped[1] = duration. Returns 0, or -1 on bad arguments / memory. */
int zkr_port(const uint64_t* tid, const uint64_t* sid, const int64_t* first, const int64_t* last,
             const uint32_t* svc, const uint32_t* flags, uint64_t n, uint32_t S, uint32_t p, uint32_t m, uint64_t seed,
             int threads, uint8_t* regs, uint64_t* hist, uint64_t* dropped, double* seconds) {
    if (S == 0 || p < 4 || p > 16 || m < 2 || m > 8 || threads < 1 || threads > 256) return -1;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const uint32_t nbins = (41u - m) << m;
    const uint64_t rbytes = (uint64_t)S << p, hwords = (uint64_t)S * nbins;
    rt_job* jobs = (rt_job*)calloc((size_t)threads, sizeof(rt_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    int rc = 0;
    uint64_t prev = 0;
    for (int t = 0; t < threads; ++t) {
        rt_job* j = &jobs[t];
        uint64_t cut = t + 1 == threads ? n : n / (uint64_t)threads * (uint64_t)(t + 1);
        if (cut < prev) cut = prev;
        while (cut < n && cut > 0 && tid[cut] == tid[cut - 1]) ++cut;  /* a trace belongs to one thread */
        j->tid = tid;
        j->sid = sid;
        j->first = first;
        j->last = last;
        j->svc = svc;
        j->flags = flags;
        j->lo = prev;
        j->hi = cut;
        prev = cut;
        j->S = S;
        j->p = p;
        j->m = m;
        j->nbins = nbins;
        j->seed = seed;
        j->regs = t == 0 ? regs : (uint8_t*)calloc(rbytes, 1);
        j->hist = t == 0 ? hist : (uint64_t*)calloc(hwords, 8);
        if (!j->regs || !j->hist) rc = -1;
    }
    if (rc == 0) {
        memset(regs, 0, rbytes);
        memset(hist, 0, hwords * 8);
        for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, run, &jobs[t]);
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
        dropped[0] = 0;
        dropped[1] = 0;
        for (int t = 0; t < threads; ++t) {
            if (jobs[t].failed) rc = -1;
            dropped[1] += jobs[t].dropped_duration;
            if (t == 0) continue;
            for (uint64_t k = 0; k < rbytes; ++k)
                if (jobs[t].regs[k] > regs[k]) regs[k] = jobs[t].regs[k];
            for (uint64_t k = 0; k < hwords; ++k) hist[k] += jobs[t].hist[k];
        }
    }
    for (int t = 1; t < threads; ++t) {
        free(jobs[t].regs);
        free(jobs[t].hist);
    }
    free(jobs);
    free(th);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return rc;
}
