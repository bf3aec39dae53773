/*
 * zksketch.h — C ABI of the per-service sketches of libzkagg (MI355X, gfx950).
 *
 * Key-value annotation popularity, behind
 *   Aggregates.getTopKeyValueAnnotations(serviceName): Future[Seq[String]]
 *   (zipkin-common/src/main/scala/com/twitter/zipkin/storage/Aggregates.scala:34; stored per
 *   service by CassandraAggregates.scala:86-88,104-108,141-142 and HBaseAggregates.scala:66-68).
 * The reference keeps a precomputed list per service; its producer was removed (CHANGELOG:7-8).
 * Items follow the span indexer's key definition: one item per binary annotation whose host has
 * a service name, (service id, 64-bit hash of the annotation key) (CassieSpanStore.scala:235-241).
 * The host owns both dictionaries (service name <-> id, key string <-> hash), exactly like the
 * dependency path (zkagg.h).
 *
 * Sketch: per service a count-min sketch of `depth` rows x `width` u32 counters and the
 * `candidates` best keys by estimate. Estimates never undercount; with N_s keys counted for the
 * service, est - true <= e / width * N_s for any key with probability >= 1 - e^-depth
 * (Cormode & Muthukrishnan 2005). Defaults: depth 4, width = 2^20 / S rounded to a power of two
 * (the BASELINE C4 budget of 4 x 2^20 counters shared by all services), 64 candidates.
 *
 * Conventions: as zkagg.h (zk_status codes, borrowed inputs, caller-owned outputs, one HIP
 * stream per handle, not thread-safe, no host compute fallback).
 */
#ifndef ZKSKETCH_H
#define ZKSKETCH_H

#include <stddef.h>
#include <stdint.h>

#include "zkagg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct zk_kv_config {
    uint32_t num_services;  /* S <= 4096 */
    int32_t  device;
    void*    stream;        /* hipStream_t or NULL for a private stream */
    uint32_t width;         /* counters per row per service: power of two in [64, 4096]; 0 = auto */
    uint32_t depth;         /* rows, 1..8; 0 = 4 */
    uint32_t candidates;    /* keys kept per service (>= any k queried), <= 256; 0 = 64 */
    uint64_t seed;          /* hash seed of the rows */
    uint32_t reserved[8];
} zk_kv_config;

typedef struct zk_kv zk_kv;

zk_status   zk_kv_create(const zk_kv_config* cfg, zk_kv** out);
zk_status   zk_kv_destroy(zk_kv* kv);
const char* zk_kv_last_error(const zk_kv* kv);
/* effective geometry after defaults */
zk_status   zk_kv_geometry(const zk_kv* kv, uint32_t* width, uint32_t* depth, uint32_t* candidates);
zk_status   zk_kv_reset(zk_kv* kv);
/* One batch of n < 2^32 items (service_id u32[n], key_hash u64[n]); host or device pointers
 * (ZK_BATCH_DEVICE_PTRS). Items with service_id >= S are dropped and reported by the queries as
 * ZK_ERR_SERVICE_RANGE (like zk_deps_finalize). */
zk_status   zk_kv_accumulate(zk_kv* kv, const uint32_t* service_id, const uint64_t* key_hash, uint64_t n,
                             uint32_t batch_flags);
/* Top-k keys of every service, best first (estimate desc, key hash asc): keys/est are S*k host
 * arrays (row s = service s, unused slots have est 0), count[s] = valid entries (may be NULL).
 * k <= candidates. ZK_ERR_CAPACITY when a service counted >= 2^32 keys since reset. */
zk_status   zk_kv_topk_all(zk_kv* kv, uint32_t k, uint64_t* keys, uint32_t* est, uint32_t* count);
/* Top-k of one service (getTopKeyValueAnnotations(service)) into host arrays of k entries. */
zk_status   zk_kv_topk(zk_kv* kv, uint32_t service, uint32_t k, uint64_t* keys, uint32_t* est, uint32_t* count);
/* Count-min point estimates of host keys for one service. */
zk_status   zk_kv_estimate(zk_kv* kv, uint32_t service, const uint64_t* key_hash, uint64_t n, uint32_t* est);
/* Keys counted per service since reset (N_s of the error bound), host u64[S]. */
zk_status   zk_kv_totals(zk_kv* kv, uint64_t* totals);
/* Multi-GPU (traceId or item sharding, one process per GPU):
 *   zk_kv_partial     device pointers of the counters (u32, SUM all-reduce) and totals (u64, SUM)
 *   zk_kv_candidates  device pointers of the candidate lists [S][candidates] keys u64 / est u32
 *                     (all-gather them)
 *   zk_kv_merge_candidates  after the SUM all-reduce: re-estimate this handle's candidates plus
 *                     `lists` gathered lists (device, layout [lists][S][candidates]) against the
 *                     merged counters and keep the best. Every rank then holds the same top-K. */
zk_status   zk_kv_partial(zk_kv* kv, void** counters, uint64_t* counter_bytes, void** totals,
                          uint64_t* totals_bytes);
zk_status   zk_kv_candidates(zk_kv* kv, void** keys, void** est, uint64_t* bytes_keys, uint64_t* bytes_est);
zk_status   zk_kv_merge_candidates(zk_kv* kv, const uint64_t* keys, const uint32_t* est, uint32_t lists);
/* Device time (ms, HIP events on the handle's stream) of the last zk_kv_accumulate's phases:
 * [0] service partition (histogram + scan + line scatter), [1] count-min sketch, [2] candidate
 * pass, [3] merge. Recorded only when zk_kv_config.reserved[0] has bit 0 set (ZK_KV_TIMING);
 * syncs the stream. */
#define ZK_KV_TIMING 1u
zk_status   zk_kv_phase_ms(zk_kv* kv, double out[4]);

/* ------------------------------------------------------------------------------------------
 * Realtime span sketches per service: distinct traces (HyperLogLog) and duration quantiles.
 *
 * The reference declares these aggregates (RealtimeAggregates.getSpanDurations /
 * getServiceNamesToTraceIds, zipkin-common/.../storage/RealtimeAggregates.scala:26-38;
 * zipkinQuery.thrift:242,251) but implements none (QueryService.scala:416-430 returns "Not
 * Implemented"); BASELINE.json asks for per-service distinct traceIds and duration p50/p99.
 * One item per MERGED span (after mergeSpan, Span.scala:148-169) that passes isValid
 * (Span.scala:236-240) and has a service name (Span.serviceName, :125-131): (service, traceId,
 * duration = last - first annotation, Span.scala:228-230).
 *
 * HyperLogLog (Flajolet et al. 2007): 2^p one-byte registers per service; register index = top p
 * bits of h = mix64(traceId ^ seed ^ 0xD6E8FEB86659FD93) (splitmix64 finalizer, salted apart from
 * the traceId shard hash), value = leading zeros of the remaining bits + 1. Standard
 * estimator with linear counting below 2.5 * 2^p; relative standard error ~1.04 / sqrt(2^p)
 * (0.81 % at p = 14). Mergeable by register-wise MAX (RCCL all-reduce MAX, u8).
 * Durations: a log-linear histogram (the HDR-histogram layout) instead of a t-digest: bin = the
 * value itself below 2^m, else (exponent, top m mantissa bits). Every bin spans at most
 * 2^-m of its lower bound, so the reported quantile bin [lo, hi] contains the exact
 * nearest-rank quantile and its midpoint is within 2^-(m+1) relative of it. Counts are integers,
 * so it is order-independent and mergeable by SUM (RCCL all-reduce SUM, u32) -- which a
 * t-digest is not.
 * ------------------------------------------------------------------------------------------ */
typedef struct zk_rt_config {
    uint32_t num_services;  /* S <= 4096 */
    int32_t  device;
    void*    stream;        /* hipStream_t or NULL for a private stream */
    uint32_t hll_p;         /* register index bits, 4..16; 0 = 14 */
    uint32_t sub_bits;      /* histogram mantissa bits m, 2..8; 0 = 7 (<= 0.39 % from the midpoint) */
    uint64_t seed;          /* traceId hash seed */
    uint32_t reserved[8];
} zk_rt_config;

typedef struct zk_rt zk_rt;

zk_status   zk_rt_create(const zk_rt_config* cfg, zk_rt** out);
zk_status   zk_rt_destroy(zk_rt* rt);
const char* zk_rt_last_error(const zk_rt* rt);
/* geometry: registers per service (2^p) and histogram bins per service */
zk_status   zk_rt_geometry(const zk_rt* rt, uint32_t* registers, uint32_t* bins);
zk_status   zk_rt_reset(zk_rt* rt);
/* Bind a sketch to a dependency ctx (same device): every later zk_deps_accumulate of the ctx
 * also feeds the sketch, in the same pass over the span records (K1 emits one item per merged
 * span). mode ZK_RT_WITH_DEPS keeps the dependency path; ZK_RT_ONLY skips it (no parent join,
 * no links, parent_id is not read). rt = NULL unbinds. */
#define ZK_RT_WITH_DEPS 0u
#define ZK_RT_ONLY      1u
zk_status   zk_rt_bind(zk_ctx* ctx, zk_rt* rt, uint32_t mode);
/* Already-merged spans: service_id u32[n], trace_id u64[n], duration i64[n] (us, >= 0);
 * host or device pointers (ZK_BATCH_DEVICE_PTRS). */
zk_status   zk_rt_accumulate_merged(zk_rt* rt, const uint32_t* service_id, const uint64_t* trace_id,
                                    const int64_t* duration, uint64_t n, uint32_t batch_flags);
/* Distinct-trace estimates of every service (host double[S]). */
zk_status   zk_rt_distinct_traces(zk_rt* rt, double* estimate);
/* Duration quantiles of one service: for each q[i] in [0, 1], the histogram bin holding the
 * nearest-rank quantile (rank = max(1, ceil(q * N))): lo[i] <= exact <= hi[i] (us); count =
 * N. With N = 0 all outputs are 0. */
zk_status   zk_rt_quantiles(zk_rt* rt, uint32_t service, const double* q, uint32_t nq, int64_t* lo, int64_t* hi,
                            uint64_t* count);
/* The same for every service at once (the query path of a dashboard over all services): lo/hi are
 * host int64[S][nq], count host u64[S] (may be NULL). One device pass over the histograms and one
 * copy of S x (4 + nq) words, instead of a copy and a synchronisation per service. */
zk_status   zk_rt_quantiles_all(zk_rt* rt, const double* q, uint32_t nq, int64_t* lo, int64_t* hi, uint64_t* count);
/* Duration t-digest of one service (BASELINE configs[4]: "duration t-digest p50/p99"): a merging
 * t-digest with the k1 scale function at the given compression (delta, e.g. 200), built from the
 * service's exact histogram -- bins in ascending order, each its midpoint weighted by its count,
 * merged while a centroid's quantile span stays within one unit of k(q) = delta/(2 pi) asin(2q-1).
 * Because the histogram is merged exactly across shards (SUM), the digest is the same on every
 * rank and for every world size and batch order (a digest merged centroid-by-centroid is not).
 * Outputs: the centroids (mean, weight: host double[cap], NULL to size with *n), the t-digest
 * estimate of each quantile q[i] (host double[nq]; interpolation between centroid centres), and
 * the item count. */
zk_status   zk_rt_tdigest(zk_rt* rt, uint32_t service, double compression, double* mean, double* weight,
                          uint32_t cap, uint32_t* n, const double* q, uint32_t nq, double* value, uint64_t* count);
/* Raw state for tests and multi-GPU merging: registers u8[S][2^p] (MAX all-reduce) and histogram
 * u32[S][bins] (SUM all-reduce), device pointers; and host copies. */
zk_status   zk_rt_partial(zk_rt* rt, void** registers, uint64_t* register_bytes, void** histogram,
                          uint64_t* histogram_bytes);
zk_status   zk_rt_read(zk_rt* rt, uint8_t* registers, uint32_t* histogram);
/* items dropped since reset: service_id >= S, or duration outside [0, 2^40) us */
zk_status   zk_rt_dropped(zk_rt* rt, uint64_t* service_range, uint64_t* duration_range);

/* ------------------------------------------------------------------------------------------
 * Realtime link store: the state behind RealtimeAggregates (zipkin-common/.../storage/
 * RealtimeAggregates.scala:26-38; zipkinQuery.thrift:234-251 -- "given a time stamp, server
 * service name and rpc name, fetch all of the client services calling in paired with the lists of
 * every span duration / every trace id from the server to client"). The reference declares the
 * trait but only implements NullRealtimeAggregates.
 *
 * Those lists are the dependency job's join rows before its group.sum: one (parent = client
 * service, child = server service, child duration, traceId) row per joined child span
 * (ZipkinAggregateJob.scala:25-37). Bound to a dependency ctx, every later zk_deps_accumulate writes
 * one item per link it emits (K1 and the spill kernel, beside the link, in the same pass) and
 * appends them to the store's window in HBM (16 B per link; grown as it fills: one link per record at
 * most). zk_rl_server_links answers one server service: every row whose child is `server`, as
 * parent ids, durations (us) and traceIds, ordered by (parent, duration, traceId) -- one filter pass
 * over the window, then a host sort of that server's rows. zk_rl_reset starts a new window (the
 * host keeps one store per time window). The ctx and the store must agree on num_services; a store
 * cannot share a ctx with a ZK_RT_WITH_DEPS sketch (ZK_ERR_UNSUPPORTED), and unclustered batches take
 * the streaming join (not the group join) while a store is bound. The record has no span name, so the
 * trait's rpcName is not a key here (GpuRealtimeAggregates).
 * ------------------------------------------------------------------------------------------ */
typedef struct zk_rl_config {
    uint32_t num_services;  /* S <= 4096, the ctx's */
    int32_t  device;
    void*    stream;        /* hipStream_t or NULL for a private stream (the bound ctx's while bound) */
    uint32_t reserved[8];
} zk_rl_config;

typedef struct zk_rl zk_rl;

zk_status   zk_rl_create(const zk_rl_config* cfg, zk_rl** out);
zk_status   zk_rl_destroy(zk_rl* rl);
const char* zk_rl_last_error(const zk_rl* rl);
zk_status   zk_rl_reset(zk_rl* rl);
zk_status   zk_rl_bind(zk_ctx* ctx, zk_rl* rl);   /* rl = NULL unbinds */
/* links in the window since reset (syncs); dropped: items past the window's capacity (0) */
zk_status   zk_rl_count(zk_rl* rl, uint64_t* items, uint64_t* dropped);
/* every link whose child service is `server` (host arrays of cap entries; all NULL: *n = the count) */
zk_status   zk_rl_server_links(zk_rl* rl, uint32_t server, uint32_t* parent, int64_t* duration,
                               uint64_t* trace_id, uint64_t cap, uint64_t* n);

#ifdef __cplusplus
}
#endif

#endif /* ZKSKETCH_H */
