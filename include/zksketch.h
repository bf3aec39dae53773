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

#ifdef __cplusplus
}
#endif

#endif /* ZKSKETCH_H */
