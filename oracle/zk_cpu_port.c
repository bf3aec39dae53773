/*
 * zk_cpu_port.c — TEST/BENCH INFRASTRUCTURE ONLY: the CPU baseline of bench.py (cpu_baseline,
 * kind "port"), never the product. A reasonable multithreaded CPU implementation of the same job
 * the oracle restates (zk_oracle.c, whose header cites ZipkinAggregateJob.scala:20-43 line by
 * line), written for speed instead of literalness, with the same deterministic build rules and
 * counters, so its output equals the oracle's bit for bit (tests/test_cpu_port.py).
 *
 * Two modes, each one pass over the input:
 *  - clustered: the promise the GPU fast path runs under (all fragments of a trace adjacent, as
 *    Cassandra's row-per-trace reads deliver them). Threads take contiguous ranges cut at trace
 *    boundaries and merge / validate / join one trace at a time in a small cache-resident hash map.
 *  - general: any record order, like the reference's shuffles. One histogram pass and one scatter
 *    pass partition the records by hash(traceId) (every merge and join key contains traceId), then
 *    each thread merges and joins its partition in one hash map.
 * Each thread sums exact power sums into a private S x S table; the tables are added at the end.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define F_HAS_PARENT 1u
#define F_HAS_ANN 2u
#define F_SVC_CLIENT 4u
#define F_SVC_SERVER 8u
#define SVC_NONE 0xFFFFFFFFu
#define MAX_DURATION (1ull << 40)
#define CELL_WORDS 17

enum {
    ST_RECORDS = 0, ST_MERGED, ST_VALID, ST_INVALID, ST_CHILD, ST_JOINED, ST_MISSING_PARENT,
    ST_NO_SERVICE, ST_AMBIGUOUS, ST_SPILLED, ST_DUR_RANGE, ST_SVC_RANGE, ST_TOO_LARGE, ST_N = 16
};

typedef struct {
    uint64_t tid, sid, pid;
    int64_t first, last;
    uint32_t svc, flags;
} rec_t;

typedef struct {
    uint64_t tid, sid, pid;
    int64_t first, last;
    uint32_t cnt;   /* cs | cr << 8 | sr << 16 | ss << 24, saturating at 2 */
    uint32_t npar;
    uint32_t svck;
    uint32_t used;
} ent_t;

typedef struct {
    const uint64_t *tid, *sid, *pid;
    const int64_t *first, *last;
    const uint32_t *svc, *flags;
    uint64_t n;
    uint32_t S;
    int T, t, clustered;
    uint64_t lo, hi;     /* clustered: record range; general: partition bounds in `part` */
    rec_t *part;
    uint64_t *counts;    /* general: [T][T] histogram */
    uint64_t *cells;
    uint64_t stats[ST_N];
    ent_t *map;
    uint64_t cap;
    uint32_t *used_list;
    int oom;
} job_t;

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint32_t svc_key(uint32_t f, uint32_t svc, uint32_t S, int *range_err) {
    const uint32_t kind = (f & F_SVC_SERVER) ? 0u : (f & F_SVC_CLIENT) ? 1u : 2u;
    if (kind == 2u) return SVC_NONE;
    if (svc >= S) { *range_err = 1; return SVC_NONE; }
    return (kind << 30) | svc;
}

/* merged cs|cr|sr|ss occurrence counts, 8 bits each, saturating at 2 (isValid needs only "<= 1") */
static inline uint32_t counts_add(uint32_t c, uint32_t f) {
    uint32_t out = 0;
    for (int k = 0; k < 4; ++k) {
        uint32_t v = ((c >> (8 * k)) & 0xFFu) + ((f >> (8 + 2 * k)) & 3u);
        out |= (v > 2 ? 2u : v) << (8 * k);
    }
    return out;
}
static inline int counts_valid(uint32_t c) {
    return (c & 0xFF) <= 1 && ((c >> 8) & 0xFF) <= 1 && ((c >> 16) & 0xFF) <= 1 && (c >> 24) <= 1;
}

static inline void add256(uint64_t *acc, const uint64_t *v, int nw) {
    unsigned __int128 carry = 0;
    for (int i = 0; i < 4; ++i) {
        const unsigned __int128 s = (unsigned __int128)acc[i] + (i < nw ? v[i] : 0) + carry;
        acc[i] = (uint64_t)s;
        carry = s >> 64;
        if (i >= nw && !carry) break;
    }
}

static void add_link(uint64_t *cell, uint64_t d) {
    cell[0] += 1;
    uint64_t w[4] = {d, 0, 0, 0};
    add256(cell + 1, w, 1);
    const unsigned __int128 d2 = (unsigned __int128)d * d;
    w[0] = (uint64_t)d2;
    w[1] = (uint64_t)(d2 >> 64);
    add256(cell + 5, w, 2);
    const unsigned __int128 lo = (unsigned __int128)w[0] * d, hi = (unsigned __int128)w[1] * d + (uint64_t)(lo >> 64);
    const uint64_t d3[3] = {(uint64_t)lo, (uint64_t)hi, (uint64_t)(hi >> 64)};
    add256(cell + 9, d3, 3);
    const unsigned __int128 a = (unsigned __int128)d3[0] * d;
    const unsigned __int128 b = (unsigned __int128)d3[1] * d + (uint64_t)(a >> 64);
    const unsigned __int128 c = (unsigned __int128)d3[2] * d + (uint64_t)(b >> 64);
    const uint64_t d4[4] = {(uint64_t)a, (uint64_t)b, (uint64_t)c, (uint64_t)(c >> 64)};
    add256(cell + 13, d4, 4);
}

static int ensure_map(job_t *J, uint64_t records) {
    uint64_t cap = 16;
    while (cap < 2 * records + 16) cap <<= 1;
    if (cap <= J->cap) return 0;
    free(J->map);
    free(J->used_list);
    J->map = (ent_t *)calloc(cap, sizeof(ent_t));
    J->used_list = (uint32_t *)malloc(cap * sizeof(uint32_t));
    J->cap = cap;
    return J->map && J->used_list ? 0 : -1;
}

/* merge -> ambiguity -> validate / join / emit over records r[0..m) of whole traces */
static void aggregate_records(job_t *J, const rec_t *r, uint64_t m, int by_trace_hash) {
    const uint64_t mask = J->cap - 1;
    ent_t *map = J->map;
    uint64_t nused = 0;
    for (uint64_t i = 0; i < m; ++i) {
        const rec_t *x = &r[i];
        int rerr = 0;
        const uint32_t sk = svc_key(x->flags, x->svc, J->S, &rerr);
        J->stats[ST_RECORDS]++;
        if (rerr) J->stats[ST_SVC_RANGE]++;
        uint64_t h = (by_trace_hash ? mix64(x->tid ^ mix64(x->sid)) : mix64(x->sid)) & mask;
        ent_t *e;
        for (;;) {
            e = &map[h];
            if (!e->used) {
                e->used = 1;
                e->tid = x->tid;
                e->sid = x->sid;
                e->first = INT64_MAX;
                e->last = INT64_MIN;
                e->pid = UINT64_MAX;
                e->svck = SVC_NONE;
                e->cnt = 0;
                e->npar = 0;
                J->used_list[nused++] = (uint32_t)h;
                break;
            }
            if (e->sid == x->sid && e->tid == x->tid) break;
            h = (h + 1) & mask;
        }
        if (x->flags & F_HAS_ANN) {
            if (x->first < e->first) e->first = x->first;
            if (x->last > e->last) e->last = x->last;
        }
        e->cnt = counts_add(e->cnt, x->flags);
        if (x->flags & F_HAS_PARENT) {
            e->npar++;
            if (x->pid < e->pid) e->pid = x->pid;
        }
        if (sk < e->svck) e->svck = sk;
    }
    for (uint64_t i = 0; i < m; ++i) {  /* fragments disagreeing with their merged span */
        const rec_t *x = &r[i];
        uint64_t h = (by_trace_hash ? mix64(x->tid ^ mix64(x->sid)) : mix64(x->sid)) & mask;
        while (!(map[h].used && map[h].sid == x->sid && map[h].tid == x->tid)) h = (h + 1) & mask;
        const ent_t *e = &map[h];
        int rerr = 0;
        const uint32_t sk = svc_key(x->flags, x->svc, J->S, &rerr);
        int amb = (x->flags & F_HAS_PARENT) ? (x->pid != e->pid) : (e->npar > 0);
        if (sk != SVC_NONE && (sk >> 30) == (e->svck >> 30) && sk != e->svck) amb = 1;
        if (amb) J->stats[ST_AMBIGUOUS]++;
    }
    for (uint64_t u = 0; u < nused; ++u) {
        const ent_t *e = &map[J->used_list[u]];
        J->stats[ST_MERGED]++;
        const int valid = counts_valid(e->cnt);
        J->stats[valid ? ST_VALID : ST_INVALID]++;
        if (!valid || e->npar == 0) continue;
        J->stats[ST_CHILD]++;
        uint64_t h = (by_trace_hash ? mix64(e->tid ^ mix64(e->pid)) : mix64(e->pid)) & mask;
        const ent_t *p = NULL;
        while (map[h].used) {
            if (map[h].sid == e->pid && map[h].tid == e->tid) { p = &map[h]; break; }
            h = (h + 1) & mask;
        }
        if (!p || !counts_valid(p->cnt)) { J->stats[ST_MISSING_PARENT]++; continue; }
        J->stats[ST_JOINED]++;
        if (p->svck == SVC_NONE || e->svck == SVC_NONE) { J->stats[ST_NO_SERVICE]++; continue; }
        const uint64_t d = (uint64_t)(e->last - e->first);
        if (d >= MAX_DURATION) { J->stats[ST_DUR_RANGE]++; continue; }
        add_link(J->cells + ((uint64_t)(p->svck & 0x3FFFFFFFu) * J->S + (e->svck & 0x3FFFFFFFu)) * CELL_WORDS, d);
    }
    for (uint64_t u = 0; u < nused; ++u) map[J->used_list[u]].used = 0;
}

static void *run_clustered(void *arg) {
    job_t *J = (job_t *)arg;
    rec_t *buf = NULL;
    uint64_t bcap = 0;
    uint64_t i = J->lo;
    while (i < J->hi) {
        uint64_t e = i + 1;
        while (e < J->n && J->tid[e] == J->tid[i]) ++e;
        const uint64_t m = e - i;
        if (m > bcap) {
            free(buf);
            bcap = m < 4096 ? 4096 : m;
            buf = (rec_t *)malloc(bcap * sizeof(rec_t));
            if (!buf) { J->oom = 1; return NULL; }
        }
        for (uint64_t k = 0; k < m; ++k) {
            rec_t *x = &buf[k];
            x->tid = J->tid[i + k];
            x->sid = J->sid[i + k];
            x->pid = J->pid[i + k];
            x->first = J->first[i + k];
            x->last = J->last[i + k];
            x->svc = J->svc[i + k];
            x->flags = J->flags[i + k];
        }
        if (ensure_map(J, m) != 0) { J->oom = 1; free(buf); return NULL; }
        aggregate_records(J, buf, m, 0);
        i = e;
    }
    free(buf);
    return NULL;
}

static inline int part_of(uint64_t tid, int T) { return (int)(mix64(tid) % (uint64_t)T); }

static void *run_hist(void *arg) {
    job_t *J = (job_t *)arg;
    uint64_t *c = J->counts + (uint64_t)J->t * J->T;
    for (uint64_t i = J->lo; i < J->hi; ++i) c[part_of(J->tid[i], J->T)]++;
    return NULL;
}

static void *run_scatter(void *arg) {  /* counts[t][p] now holds this thread's write offsets */
    job_t *J = (job_t *)arg;
    uint64_t *pos = J->counts + (uint64_t)J->t * J->T;
    for (uint64_t i = J->lo; i < J->hi; ++i) {
        rec_t *x = &J->part[pos[part_of(J->tid[i], J->T)]++];
        x->tid = J->tid[i];
        x->sid = J->sid[i];
        x->pid = J->pid[i];
        x->first = J->first[i];
        x->last = J->last[i];
        x->svc = J->svc[i];
        x->flags = J->flags[i];
    }
    return NULL;
}

static void *run_partition(void *arg) {
    job_t *J = (job_t *)arg;
    if (ensure_map(J, J->hi - J->lo) != 0) { J->oom = 1; return NULL; }
    aggregate_records(J, J->part + J->lo, J->hi - J->lo, 1);
    return NULL;
}

typedef struct {
    job_t *jobs;
    int T;
    uint64_t c0, c1;
} merge_t;

/* table 0 += tables 1..T-1 over cells [c0, c1) */
static void *run_merge(void *arg) {
    merge_t *M = (merge_t *)arg;
    uint64_t *dst0 = M->jobs[0].cells;
    for (int t = 1; t < M->T; ++t) {
        const uint64_t *srcT = M->jobs[t].cells;
        for (uint64_t c = M->c0; c < M->c1; ++c) {
            const uint64_t *src = srcT + c * CELL_WORDS;
            if (!src[0]) continue;
            uint64_t *dst = dst0 + c * CELL_WORDS;
            dst[0] += src[0];
            for (int k = 0; k < 4; ++k) add256(dst + 1 + 4 * k, src + 1 + 4 * k, 4);
        }
    }
    return NULL;
}

static void run_all(job_t *jobs, int T, void *(*fn)(void *)) {
    pthread_t th[256];
    for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
}

/* Same output layout and counters as zko_aggregate. Returns 0, or -1 on allocation failure. */
int zkp_aggregate(const uint64_t *tid, const uint64_t *sid, const uint64_t *pid, const int64_t *first,
                  const int64_t *last, const uint32_t *svc, const uint32_t *flags, uint64_t n, uint32_t S,
                  int threads, int clustered, uint64_t *out_cells, uint64_t *out_stats) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    const uint64_t cells = (uint64_t)S * S;
    memset(out_cells, 0, cells * CELL_WORDS * 8);
    memset(out_stats, 0, ST_N * 8);
    job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
    if (!jobs) return -1;
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        job_t *J = &jobs[t];
        J->tid = tid; J->sid = sid; J->pid = pid; J->first = first; J->last = last;
        J->svc = svc; J->flags = flags; J->n = n; J->S = S; J->T = threads; J->t = t; J->clustered = clustered;
        J->cells = t == 0 ? out_cells : (uint64_t *)calloc(cells * CELL_WORDS, 8);
        if (!J->cells) { rc = -1; threads = t; break; }
        uint64_t lo = n * (uint64_t)t / (uint64_t)J->T, hi = n * (uint64_t)(t + 1) / (uint64_t)J->T;
        if (clustered) {  /* cut at trace starts */
            while (lo > 0 && lo < n && tid[lo] == tid[lo - 1]) ++lo;
            while (hi > 0 && hi < n && tid[hi] == tid[hi - 1]) ++hi;
        }
        J->lo = lo;
        J->hi = hi;
    }
    if (rc == 0 && clustered) {
        run_all(jobs, threads, run_clustered);
    } else if (rc == 0) {
        uint64_t *counts = (uint64_t *)calloc((size_t)threads * threads, 8);
        rec_t *part = (rec_t *)malloc((n ? n : 1) * sizeof(rec_t));
        if (!counts || !part) {
            rc = -1;
        } else {
            for (int t = 0; t < threads; ++t) { jobs[t].counts = counts; jobs[t].part = part; }
            run_all(jobs, threads, run_hist);
            uint64_t off = 0;  /* partition-major offsets: part p = all threads' records of p */
            uint64_t *bounds = (uint64_t *)calloc((size_t)threads + 1, 8);
            for (int p = 0; p < threads; ++p) {
                bounds[p] = off;
                for (int t = 0; t < threads; ++t) {
                    const uint64_t c = counts[(uint64_t)t * threads + p];
                    counts[(uint64_t)t * threads + p] = off;
                    off += c;
                }
            }
            bounds[threads] = off;
            run_all(jobs, threads, run_scatter);
            for (int t = 0; t < threads; ++t) { jobs[t].lo = bounds[t]; jobs[t].hi = bounds[t + 1]; }
            run_all(jobs, threads, run_partition);
            free(bounds);
        }
        free(counts);
        free(part);
    }
    if (threads > 1) {  /* the private tables are added in parallel, by cell range */
        merge_t ms[256];
        pthread_t th[256];
        for (int t = 0; t < threads; ++t) {
            ms[t].jobs = jobs;
            ms[t].T = threads;
            ms[t].c0 = cells * (uint64_t)t / (uint64_t)threads;
            ms[t].c1 = cells * (uint64_t)(t + 1) / (uint64_t)threads;
            pthread_create(&th[t], NULL, run_merge, &ms[t]);
        }
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    }
    for (int t = 0; t < threads; ++t) {
        if (jobs[t].oom) rc = -1;
        for (int s = 0; s < ST_N; ++s) out_stats[s] += jobs[t].stats[s];
        free(jobs[t].map);
        free(jobs[t].used_list);
        if (t) free(jobs[t].cells);
    }
    free(jobs);
    return rc;
}
