/*
 * zk_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of the zipkin-aggregate dependency job over columnar span fragments,
 * used by tests/ and by bench.py's cpu_baseline leg. It follows the reference's relational
 * formulation literally and assumes NOTHING about record order (no trace clustering):
 *
 *   ZipkinAggregateJob.scala:21-22  groupBy((span.id, span.traceId)).reduce(mergeSpan)
 *        -> open-addressing hash map keyed by (traceId, spanId); Span.mergeSpan (Span.scala:148-169)
 *           concatenates annotations, so first = min, last = max, core counts add
 *   ZipkinAggregateJob.scala:23     filter(isValid) -> Span.isValid (Span.scala:236-240)
 *   ZipkinAggregateJob.scala:25-33  join on (parentId, traceId) -> hash lookup of (traceId, parentId)
 *   ZipkinAggregateJob.scala:34-37  Moments(child.duration) keyed by (parent.serviceName, child.serviceName);
 *                                   duration = last - first (Span.scala:228-230);
 *                                   serviceName prefers sr/ss hosts over cs/cr (Span.scala:125-131)
 *   ZipkinAggregateJob.scala:39-40  group.sum -> exact integer power sums n, S1..S4 per cell
 *
 * Build rules where the reference depends on reduce order (fragments of one span disagreeing on
 * parentId or service): parentId = min over fragments that carry one, service = min over
 * (side, id) with server side first; such fragments are counted as "ambiguous" exactly as the
 * product counts them, and parity tests on reference semantics exclude them.
 *
 * Parallelism: T threads partition traces by a hash of traceId (every merge and join key contains
 * traceId, so the partitions are independent), each with private maps and cell tables.
 *
 * Output per cell (S*S cells, 17 u64): n, then S1, S2, S3, S4 as 256-bit little-endian integers.
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
    uint64_t tid, sid;
    int64_t first, last;
    uint64_t pid;       /* min parentId over fragments carrying one */
    uint32_t cnt[4];    /* cs, cr, sr, ss occurrence counts (each fragment adds 0..2) */
    uint32_t npar;      /* fragments carrying a parentId */
    uint32_t svck;      /* (side << 30) | id, side 0 = server, 1 = client; SVC_NONE if none */
    uint32_t used;
} entry_t;

typedef struct {
    const uint64_t *tid, *sid, *pid;
    const int64_t *first, *last;
    const uint32_t *svc, *flags;
    uint64_t n;
    uint32_t S;
    int T, t;
    uint64_t *cells; /* private S*S*CELL_WORDS */
    uint64_t stats[ST_N];
    int oom;
} job_t;

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t key_hash(uint64_t tid, uint64_t sid) { return mix64(tid ^ mix64(sid + 0x632BE59BD9B4E019ull)); }

static inline uint32_t svc_key(uint32_t f, uint32_t svc, uint32_t S, int *range_err) {
    uint32_t kind = (f & F_SVC_SERVER) ? 0u : (f & F_SVC_CLIENT) ? 1u : 2u;
    if (kind == 2u) return SVC_NONE;
    if (svc >= S) { *range_err = 1; return SVC_NONE; }
    return (kind << 30) | svc;
}

static entry_t *lookup(entry_t *map, uint64_t mask, uint64_t tid, uint64_t sid) {
    uint64_t h = key_hash(tid, sid) & mask;
    for (;;) {
        entry_t *e = &map[h];
        if (!e->used) return NULL;
        if (e->tid == tid && e->sid == sid) return e;
        h = (h + 1) & mask;
    }
}

/* add v (up to 4 words) into 4-word accumulator */
static inline void add256(uint64_t *acc, const uint64_t *v, int nw) {
    unsigned __int128 carry = 0;
    for (int i = 0; i < 4; ++i) {
        unsigned __int128 s = (unsigned __int128)acc[i] + (i < nw ? v[i] : 0) + carry;
        acc[i] = (uint64_t)s;
        carry = s >> 64;
    }
}

static void add_link(uint64_t *cell, uint64_t d) {
    cell[0] += 1;
    uint64_t w[4];
    w[0] = d; w[1] = 0;
    add256(cell + 1, w, 1);
    unsigned __int128 d2 = (unsigned __int128)d * d;
    w[0] = (uint64_t)d2; w[1] = (uint64_t)(d2 >> 64);
    add256(cell + 5, w, 2);
    unsigned __int128 lo = (unsigned __int128)w[0] * d, hi = (unsigned __int128)w[1] * d + (uint64_t)(lo >> 64);
    uint64_t d3[3] = {(uint64_t)lo, (uint64_t)hi, (uint64_t)(hi >> 64)};
    add256(cell + 9, d3, 3);
    unsigned __int128 a = (unsigned __int128)d3[0] * d;
    unsigned __int128 b = (unsigned __int128)d3[1] * d + (uint64_t)(a >> 64);
    unsigned __int128 c = (unsigned __int128)d3[2] * d + (uint64_t)(b >> 64);
    uint64_t d4[4] = {(uint64_t)a, (uint64_t)b, (uint64_t)c, (uint64_t)(c >> 64)};
    add256(cell + 13, d4, 4);
}

static void *run_job(void *arg) {
    job_t *J = (job_t *)arg;
    const uint64_t n = J->n;
    uint64_t mine = 0;
    for (uint64_t i = 0; i < n; ++i)
        if ((int)(mix64(J->tid[i]) % (uint64_t)J->T) == J->t) ++mine;
    uint64_t cap = 16;
    while (cap < 2 * mine + 16) cap <<= 1;
    entry_t *map = (entry_t *)calloc(cap, sizeof(entry_t));
    if (!map) { J->oom = 1; return NULL; }
    const uint64_t mask = cap - 1;
    /* groupBy((id, traceId)).reduce(mergeSpan), fragments in input order */
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t tid = J->tid[i];
        if ((int)(mix64(tid) % (uint64_t)J->T) != J->t) continue;
        const uint64_t sid = J->sid[i];
        const uint32_t f = J->flags[i];
        int rerr = 0;
        const uint32_t sk = svc_key(f, J->svc[i], J->S, &rerr);
        J->stats[ST_RECORDS]++;
        if (rerr) J->stats[ST_SVC_RANGE]++;
        uint64_t h = key_hash(tid, sid) & mask;
        entry_t *e;
        for (;;) {
            e = &map[h];
            if (!e->used) {
                e->used = 1;
                e->tid = tid;
                e->sid = sid;
                e->first = INT64_MAX;
                e->last = INT64_MIN;
                e->pid = UINT64_MAX;
                e->svck = SVC_NONE;
                break;
            }
            if (e->tid == tid && e->sid == sid) break;
            h = (h + 1) & mask;
        }
        if (f & F_HAS_ANN) {
            if (J->first[i] < e->first) e->first = J->first[i];
            if (J->last[i] > e->last) e->last = J->last[i];
        }
        e->cnt[0] += (f >> 8) & 3u;
        e->cnt[1] += (f >> 10) & 3u;
        e->cnt[2] += (f >> 12) & 3u;
        e->cnt[3] += (f >> 14) & 3u;
        if (f & F_HAS_PARENT) {
            e->npar++;
            if (J->pid[i] < e->pid) e->pid = J->pid[i];
        }
        if (sk < e->svck) e->svck = sk;
    }
    /* fragments whose own parentId / service disagree with the merged span (order-dependent) */
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t tid = J->tid[i];
        if ((int)(mix64(tid) % (uint64_t)J->T) != J->t) continue;
        const entry_t *e = lookup(map, mask, tid, J->sid[i]);
        const uint32_t f = J->flags[i];
        int rerr = 0;
        const uint32_t sk = svc_key(f, J->svc[i], J->S, &rerr);
        int amb = (f & F_HAS_PARENT) ? (J->pid[i] != e->pid) : (e->npar > 0);
        if (sk != SVC_NONE && (sk >> 30) == (e->svck >> 30) && sk != e->svck) amb = 1;
        if (amb) J->stats[ST_AMBIGUOUS]++;
    }
    /* filter(isValid), join child -> parent on (parentId, traceId), Moments, sum */
    for (uint64_t h = 0; h < cap; ++h) {
        const entry_t *e = &map[h];
        if (!e->used) continue;
        J->stats[ST_MERGED]++;
        const int valid = e->cnt[0] <= 1 && e->cnt[1] <= 1 && e->cnt[2] <= 1 && e->cnt[3] <= 1;
        J->stats[valid ? ST_VALID : ST_INVALID]++;
        if (!valid || e->npar == 0) continue;
        J->stats[ST_CHILD]++;
        const entry_t *p = lookup(map, mask, e->tid, e->pid);
        const int pvalid = p && p->cnt[0] <= 1 && p->cnt[1] <= 1 && p->cnt[2] <= 1 && p->cnt[3] <= 1;
        if (!pvalid) { J->stats[ST_MISSING_PARENT]++; continue; }
        J->stats[ST_JOINED]++;
        if (p->svck == SVC_NONE || e->svck == SVC_NONE) { J->stats[ST_NO_SERVICE]++; continue; }
        const uint64_t d = (uint64_t)(e->last - e->first);
        if (d >= MAX_DURATION) { J->stats[ST_DUR_RANGE]++; continue; }
        const uint64_t cell = (uint64_t)(p->svck & 0x3FFFFFFFu) * J->S + (e->svck & 0x3FFFFFFFu);
        add_link(J->cells + cell * CELL_WORDS, d);
    }
    free(map);
    return NULL;
}

/* returns 0 on success, -1 on allocation failure */
int zko_aggregate(const uint64_t *tid, const uint64_t *sid, const uint64_t *pid, const int64_t *first,
                  const int64_t *last, const uint32_t *svc, const uint32_t *flags, uint64_t n, uint32_t S,
                  int threads, uint64_t *out_cells, uint64_t *out_stats) {
    if (threads < 1) threads = 1;
    const uint64_t cells = (uint64_t)S * S;
    memset(out_cells, 0, cells * CELL_WORDS * 8);
    memset(out_stats, 0, ST_N * 8);
    job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) return -1;
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        job_t *J = &jobs[t];
        J->tid = tid; J->sid = sid; J->pid = pid; J->first = first; J->last = last;
        J->svc = svc; J->flags = flags; J->n = n; J->S = S; J->T = threads; J->t = t;
        J->cells = t == 0 ? out_cells : (uint64_t *)calloc(cells * CELL_WORDS, 8);
        if (!J->cells) { rc = -1; threads = t; break; }
    }
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, run_job, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    for (int t = 0; t < threads; ++t) {
        if (jobs[t].oom) rc = -1;
        for (int s = 0; s < ST_N; ++s) out_stats[s] += jobs[t].stats[s];
        if (t == 0) continue;
        for (uint64_t c = 0; c < cells; ++c) {
            uint64_t *dst = out_cells + c * CELL_WORDS;
            const uint64_t *src = jobs[t].cells + c * CELL_WORDS;
            if (!src[0]) continue;
            dst[0] += src[0];
            for (int k = 0; k < 4; ++k) add256(dst + 1 + 4 * k, src + 1 + 4 * k, 4);
        }
        free(jobs[t].cells);
    }
    free(jobs);
    free(th);
    return rc;
}
