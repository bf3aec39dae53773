/*
 * zkagg.h — C ABI of the MI355X-native zipkin-aggregate dependency path.
 *
 * This library replaces the compute of ONE reference path: the Scalding job
 *   zipkin-aggregate/src/main/scala/com/twitter/zipkin/aggregate/ZipkinAggregateJob.scala:20-43
 * (TypedPipe[Span] -> groupBy(id,traceId).reduce(mergeSpan) -> filter(isValid)
 *  -> join child on (parentId,traceId) -> Moments(duration) -> group.sum -> Dependencies)
 * and provides the device-side state behind the store surface
 *   zipkin-common/src/main/scala/com/twitter/zipkin/storage/Aggregates.scala:26-37
 * (getDependencies / storeDependencies / getTopKeyValueAnnotations).
 *
 * Conventions (mirroring the reference's error behaviour without exceptions):
 *  - every entry point returns zk_status (0 = OK) and never throws or aborts;
 *  - zk_last_error(ctx) gives a human-readable message for the last failure;
 *  - inputs are caller-owned. HOST pointers are borrowed for the duration of the
 *    call only: an entry point that stages host inputs waits until its copies have
 *    read them (page-locked memory included), so the caller may reuse the buffers as
 *    soon as it returns. DEVICE pointers (ZK_BATCH_DEVICE_PTRS) are read by kernels
 *    queued on the ctx stream and must stay valid and unmodified until that stream has
 *    drained them (zk_ctx_sync, or an event recorded after the call);
 *  - outputs go to caller buffers; sizes are queried by passing NULL;
 *  - a ctx is NOT thread-safe (one ctx per host thread, or an external lock:
 *    the reference serialises store writes with `synchronized`,
 *    zipkin-cassandra/.../storage/cassandra/CassandraAggregates.scala:122);
 *  - all device work of a ctx is ordered on ONE HIP stream (its own, or the
 *    caller's when zk_config.stream is set).
 *
 * The library has no host compute fallback: without a usable gfx950 device
 * zk_ctx_create returns ZK_ERR_NO_DEVICE.
 */
#ifndef ZKAGG_H
#define ZKAGG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZK_ABI_VERSION 3

typedef enum zk_status {
    ZK_OK = 0,
    ZK_ERR_INVALID_ARG = 1,
    ZK_ERR_HIP = 2,              /* HIP runtime failure; see zk_last_error */
    ZK_ERR_NO_SERVICE = 3,       /* a joined parent/child span has no service name: the
                                    reference throws None.get (ZipkinAggregateJob.scala:36-37).
                                    Returned by finalize in strict mode only. */
    ZK_ERR_DURATION_RANGE = 4,   /* a joined child duration >= 2^40 us (12.7 days, longer than the
                                    7-day span TTL, CassieSpanStore.scala:47); link not counted */
    ZK_ERR_TRACE_TOO_LARGE = 5,  /* a trace longer than zk_config.max_trace_records */
    ZK_ERR_CAPACITY = 6,         /* exact-accumulator headroom exhausted (> 2^32-1 records since reset),
                                    or a caller buffer too small */
    ZK_ERR_NOT_CLUSTERED = 7,    /* ZK_BATCH_VERIFY_TRACES found a trace split into non-adjacent
                                    runs, or over two accumulate calls since the last reset */
    ZK_ERR_NO_DEVICE = 8,        /* no HIP device / not gfx950 */
    ZK_ERR_SERVICE_RANGE = 9,    /* a record carries service_id >= num_services */
    ZK_ERR_UNSUPPORTED = 10,
    ZK_ERR_INVALID_SPAN = 11,    /* ingest: a span the reference's thrift conversion rejects (null
                                    name, annotation timestamp <= 0 or empty value,
                                    thrift.scala:64-121), or bytes that do not decode */
    ZK_ERR_RANK_FAILED = 12,     /* multi-GPU: another rank of the job failed before the exchange
                                    (zk_deps_abort); the merged table is incomplete */
} zk_status;

/* ------------------------------------------------------------------------------------------
 * Columnar span records (the algorithmic input: 48 B per stored span fragment).
 *
 * One record = one stored Thrift Span fragment (one Cassandra column,
 * CassieSpanStore.scala:76-77,295) after host ingest (thrift.scala:36-121):
 *   trace_id, span_id, parent_id   Span.traceId/id/parentId (zipkinCore.thrift:50-58)
 *   first_ts, last_ts              min/max annotation timestamp, us (Span.scala:174-191,72-74)
 *   service_id                     dictionary id of the fragment's service name (Span.scala:125-131):
 *                                  the host of its first sr/ss annotation, else of its first cs/cr
 *   flags                          ZK_F_* below
 * ------------------------------------------------------------------------------------------ */
#define ZK_F_HAS_PARENT      (1u << 0)   /* parentId.isDefined */
#define ZK_F_HAS_ANNOTATIONS (1u << 1)   /* first_ts/last_ts are meaningful */
#define ZK_F_SVC_CLIENT      (1u << 2)   /* service_id came from a cs/cr host (Constants.CoreClient) */
#define ZK_F_SVC_SERVER      (1u << 3)   /* service_id came from a sr/ss host (Constants.CoreServer) */
/* 2-bit saturating (0,1,2=">=2") occurrence counts of each core annotation
   (Constants.scala:20-32), used by Span.isValid (Span.scala:236-240). */
#define ZK_F_CS_SHIFT 8
#define ZK_F_CR_SHIFT 10
#define ZK_F_SR_SHIFT 12
#define ZK_F_SS_SHIFT 14
#define ZK_F_COUNT_MASK 3u

typedef struct zk_span_cols {
    const uint64_t* trace_id;
    const uint64_t* span_id;
    const uint64_t* parent_id;
    const int64_t*  first_ts;
    const int64_t*  last_ts;
    const uint32_t* service_id;
    const uint32_t* flags;
    uint64_t        n;
} zk_span_cols;

/* batch flags for zk_deps_accumulate
 *
 * Fragments may come in ANY order, as the reference's shuffles allow (ZipkinAggregateJob.scala:21,
 * 28-33): without ZK_BATCH_TRACE_CLUSTERED the batch first goes through a device partition: a
 * two-level MSD radix partition of the records on a hash of the traceId (a histogram pass, two
 * scatter passes that move all seven columns), after which every trace lies inside one sub-bucket.
 * Batches of more than 2^18 records without ZK_BATCH_VERIFY_TRACES are then joined per run of whole
 * sub-buckets in LDS with the traceId in the keys (the group join; sub-buckets longer than its LDS
 * tile are clustered and go through the streaming join); otherwise one more pass groups each
 * sub-bucket's records into whole traces for the streaming join. Measured on MI355X: a shuffled
 * 1e8-record batch takes 6.6-7.0 ms per accumulate with the group join (8.6 ms with the trace pass)
 * against 1.3-1.5 ms clustered, about 208 B of HBM traffic per 48-B record; the partition needs two
 * extra 48-B/record column buffers. ZK_BATCH_TRACE_CLUSTERED is the caller's promise that it is
 * unnecessary (Cassandra row-per-trace reads deliver clustered batches).
 * ZK_BATCH_VERIFY_TRACES checks that promise, and the trace-complete-batch contract, exactly: every
 * trace run's traceId is inserted into a device set of all traceIds accumulated since the last
 * reset, and a traceId seen again (a trace split into non-adjacent runs, or spread over two
 * accumulate calls -- either would be mis-joined) is counted in zk_stats.not_clustered and makes
 * finalize return ZK_ERR_NOT_CLUSTERED. The set costs 16 B of HBM per record since reset (about
 * 24 B per record while it is rehashed into a larger set: both are live) and one extra read of the
 * traceId column; when that memory cannot be allocated accumulate returns ZK_ERR_CAPACITY. */
#define ZK_BATCH_DEVICE_PTRS     (1u << 0) /* column pointers are device (HBM) pointers; else host */
#define ZK_BATCH_TRACE_CLUSTERED (1u << 1) /* all fragments of a trace are adjacent (Cassandra
                                              row-per-trace reads, StorageRecordReader.scala:49-54) */
#define ZK_BATCH_VERIFY_TRACES   (1u << 2) /* check clustering and trace-completeness (see above) */
/* ZK_BATCH_CONTINUES (with ZK_BATCH_TRACE_CLUSTERED): the batch's last trace may continue in the next
 * accumulate -- a trace cut at a batch edge, as a streaming reader of row-per-trace storage cuts
 * them. Its fragments are held back in HBM (up to max_trace_records) and joined with the next
 * batch's leading fragments of the same traceId; a held trace may continue over any number of
 * batches. The held trace is aggregated when a batch moves on to another traceId, when a batch
 * arrives without the flag, at finalize and at zk_deps_partial; zk_ctx_stats does not count it
 * before then. Decided on the device (no host round trip): one small kernel finds the batch's
 * edge runs (scanning from both ends until a trace boundary) and applies these rules. */
#define ZK_BATCH_CONTINUES       (1u << 3)

typedef struct zk_config {
    uint32_t num_services;       /* S <= 4096: service ids are 0..S-1, link table is S x S */
    int32_t  device;             /* HIP device ordinal */
    void*    stream;             /* hipStream_t to run on, or NULL for a private stream */
    uint32_t strict;             /* 1: finalize returns ZK_ERR_NO_SERVICE like the reference's
                                    None.get; 0: such pairs are skipped and counted */
    uint32_t max_trace_records;  /* largest trace handled (default 131072 > MaxTraceCols=100000,
                                    CassieSpanStore.scala:50) */
    uint32_t timing;             /* 1: record per-kernel HIP events (zk_ctx_timing) */
    void*    table;              /* optional caller-owned device buffer for the exact accumulator
                                    (table_bytes >= ZK_TABLE_BYTES(S)), e.g. to place it in a pool the
                                    caller manages. It is NOT the exchange buffer: only the buffer
                                    zk_deps_partial returns may be all-reduced, and
                                    zk_deps_note_merged overwrites this table from that buffer (an
                                    all-reduce of the table itself would be lost) */
    uint64_t table_bytes;
    uint32_t trace_pass;         /* 1: unclustered batches always take the trace pass + streaming join
                                    (P3 + K1) instead of the group join (the A/B of DESIGN.md §7b);
                                    0: the library picks (group join for > 2^18 records without
                                    ZK_BATCH_VERIFY_TRACES, when max_trace_records >= its LDS tile) */
    uint32_t reserved[7];
} zk_config;

typedef struct zk_ctx zk_ctx;

/* Per-ctx counters since the last zk_deps_reset (all device-counted, exact). */
typedef struct zk_stats {
    uint64_t records;          /* span fragments accumulated */
    uint64_t merged_spans;     /* distinct (traceId, spanId) after mergeSpan */
    uint64_t valid_spans;      /* merged spans passing isValid */
    uint64_t invalid_spans;    /* dropped by isValid (a core annotation > once) */
    uint64_t child_spans;      /* valid merged spans with parentId defined */
    uint64_t joined_links;     /* child x parent join rows turned into Moments */
    uint64_t missing_parent;   /* valid child whose parent is absent or invalid */
    uint64_t no_service;       /* joined pair with a side lacking a service (reference: throws) */
    uint64_t ambiguous;        /* fragments of one span disagreeing on parentId/service: the
                                  reference result depends on reduce order (Span.scala:160-168) */
    uint64_t spilled_traces;   /* traces too long for one LDS tile, handled by the spill kernel */
    uint64_t duration_range;   /* links dropped for duration >= 2^40 us */
    uint64_t service_range;    /* records with service_id >= num_services */
    uint64_t trace_too_large;  /* traces longer than max_trace_records (not aggregated) */
    uint64_t not_clustered;    /* trace runs whose traceId was already accumulated (VERIFY_TRACES) */
    uint64_t reserved[2];
} zk_stats;

/* Device time of the last accumulate/finalize, from HIP events (config.timing = 1). */
typedef struct zk_timing {
    double join_ms;        /* K1 span_join (merge + validate + parent join + link emit) */
    double reduce_ms;      /* link reduction into the exact limb table */
    double spill_ms;       /* giant-trace spill kernel */
    double finalize_ms;    /* exact power sums -> Algebird Moments */
    uint64_t join_calls;   /* cumulative number of timed K1 launches */
    double join_ms_total;  /* cumulative K1 time */
    double reduce_ms_total;
    double cluster_ms;        /* clustering pass of the last unclustered batch (0 when none) */
    double cluster_ms_total;  /* cumulative clustering-pass time */
    double reserved[2];
} zk_timing;

/* Dense S x S output table of DependencyLink(parent=i, child=j, Moments) for cell i*S+j
   (Dependencies.scala:34, zipkinDependencies.thrift:24-37). m1..m4 are the Algebird central
   moments (mean, sum (x-mean)^2, sum (x-mean)^3, sum (x-mean)^4), computed exactly and rounded
   once to fp64. present[c] = (m0[c] > 0). */
typedef struct zk_link_table {
    uint64_t* m0;
    double*   m1;
    double*   m2;
    double*   m3;
    double*   m4;
    uint8_t*  present;
    uint32_t  device_ptrs;   /* 1: the arrays above are device pointers */
} zk_link_table;

/* ---- lifecycle ------------------------------------------------------------------------- */
uint32_t    zk_abi_version(void);
zk_status   zk_ctx_create(const zk_config* cfg, zk_ctx** out);
zk_status   zk_ctx_destroy(zk_ctx* ctx);
const char* zk_last_error(const zk_ctx* ctx);
const char* zk_status_str(zk_status s);
zk_status   zk_ctx_sync(zk_ctx* ctx);                       /* wait for the ctx stream */
zk_status   zk_ctx_stats(zk_ctx* ctx, zk_stats* out);       /* syncs */
zk_status   zk_ctx_timing(zk_ctx* ctx, zk_timing* out);     /* syncs */

/* ---- dependency path (ZipkinAggregateJob.scala:20-43) -------------------------------------
 * reset       : zero the exact accumulators (Monoid.zero[Dependencies], Dependencies.scala:81)
 * accumulate  : one trace-complete batch of fragments; may be called many times (the link table
 *               is a monoid, so incremental runs are exact and order-independent)
 * finalize    : power sums -> m0..m4 into the caller's table; links with m0 = 0 are absent
 *               (the reference emits nothing for them, ZipkinAggregateJob.scala:43-45) */
zk_status zk_deps_reset(zk_ctx* ctx);
zk_status zk_deps_accumulate(zk_ctx* ctx, const zk_span_cols* cols, uint32_t batch_flags);
zk_status zk_deps_finalize(zk_ctx* ctx, const zk_link_table* out);

/* Exact accumulator exchange for an external SUM all-reduce (RCCL over xGMI) across traceId-hash
   shards, replacing the cross-reducer .group.sum / .sum of ZipkinAggregateJob.scala:39-43.
   The accumulator (zk_config.table, ZK_TABLE_BYTES(S) bytes) is S*S cells x 16 u64 limbs of
   32-bit chunks, carry-free, then a tail of 16 u64 = this ctx's zk_stats counters.
   zk_deps_partial enqueues on the ctx stream the fold of the counters into the tail and the
   carry-normalisation of every cell into the ctx-owned EXCHANGE buffer it returns
   (ZK_XCHG_BYTES(S): S*S cells x 12 u64 limbs of 56 bits -- m0 one, S1 two, S2 two, S3 three, S4
   four, a sum's top limb holding its remaining bits -- then the counter tail): 25 % fewer bytes to
   move than the accumulator, and every field is a plain sum that cannot carry out of its u64
   for up to 256 ranks, so ONE int64/uint64 SUM all-reduce of the returned buffer merges the exact
   power sums and the job-wide counters. zk_deps_note_merged (after the all-reduce, on the same
   stream) rebuilds the merged exact sums into the accumulator and tells the ctx that it holds the
   merged job: total_records bounds the ZK_ERR_CAPACITY headroom (0: read it from the merged tail,
   which costs one stream synchronisation), and finalize / zk_ctx_stats read the merged counters,
   so every rank reaches the same status (a strict-mode ZK_ERR_NO_SERVICE on one shard fails all
   ranks alike instead of one rank leaving the others blocked in the next collective).
   note_merged without a partial since the last reset/accumulate returns ZK_ERR_INVALID_ARG. The
   next reset leaves the merged state. An accumulate into a merged table continues the job on THIS
   rank (finalize then reports the merged job plus the batch), but such a ctx holds the whole job, so
   zk_deps_partial refuses it (ZK_ERR_INVALID_ARG) until the next reset: exchanging it again would
   add the job once per rank. */
#define ZK_TABLE_BYTES(S) ((uint64_t)(S) * (uint64_t)(S) * 128u + 128u)
#define ZK_XCHG_BYTES(S) ((uint64_t)(S) * (uint64_t)(S) * 96u + 128u)
zk_status zk_deps_partial(zk_ctx* ctx, void** dev_ptr, uint64_t* bytes);
zk_status zk_deps_note_merged(zk_ctx* ctx, uint64_t total_records);
/* A rank that fails on the host before the exchange (an undecodable span, a batch the library
   refused, a service outside the job's list) must still make the job's collective call, or every
   other rank waits in it forever. zk_deps_abort marks this ctx's part of the job as failed: its next
   zk_deps_partial returns a zero table whose counter tail carries one abort mark (2^48 added to the
   records word; records per job stay < 2^40, so up to 256 marks never reach the count), the
   all-reduce adds it into every rank's tail, and after zk_deps_note_merged finalize returns
   ZK_ERR_RANK_FAILED on EVERY rank. The records count the merged tail reports excludes the marks.
   zk_deps_reset clears the mark. */
zk_status zk_deps_abort(zk_ctx* ctx);

/* ---- synthetic zipkin-tracegen workload (TraceGen.scala:50-143) ------------------------------
 * Counter-based, so host and device produce bit-identical records for the same parameters.
 * Traces are emitted trace-clustered, in TraceGen's own post-order. Sharding: trace k of shard
 * (rank, world) gets a unique traceId whose zk_trace_shard(traceId, world) == rank (each shard its
 * own traces), or with global_ids the shards split ONE set of traces by that hash. */
typedef struct zk_tracegen_params {
    uint64_t seed;
    uint64_t num_traces;      /* traces to generate (upper bound when target_records > 0) */
    uint64_t target_records;  /* 0: all num_traces; else stop at the last whole trace <= target */
    uint32_t max_depth;       /* TraceGen maxDepth (tracegen Main.scala:31-32 default 7) */
    uint32_t num_services;    /* service ids 0..S-1 */
    int64_t  base_ts;         /* "now" in us; traces start 1..8 hours before it */
    uint32_t rank;
    uint32_t world;
    uint32_t global_ids;      /* 1: ONE trace set for every world size (configs[2]): trace k has a
                                 traceId independent of world, and shard (rank, world) generates only
                                 the traces of that set with zk_trace_shard(traceId, world) == rank;
                                 num_traces / target_records then describe the WHOLE set (the cut is
                                 the same on every rank) and n_records / n_traces the shard's part */
    uint32_t reserved[3];
} zk_tracegen_params;

uint32_t  zk_trace_shard(uint64_t trace_id, uint32_t world);
/* host generator: cols point at host arrays of capacity `cap` (NULL arrays: count only) */
zk_status zk_tracegen_host(const zk_tracegen_params* p, const zk_span_cols* out, uint64_t cap,
                           uint64_t* n_records, uint64_t* n_traces);
/* device generator on the ctx stream: cols point at device arrays of capacity `cap` */
zk_status zk_tracegen_device(zk_ctx* ctx, const zk_tracegen_params* p, const zk_span_cols* out,
                             uint64_t cap, uint64_t* n_records, uint64_t* n_traces);

#ifdef __cplusplus
}
#endif
#endif /* ZKAGG_H */
