/*
 * zkingest.h — C ABI of the span ingest decoders of libzkagg (host, and device: zk_ingest_dev).
 *
 * Turns stored span fragments into the 48-B columnar records of zkagg.h, replacing the job's
 * input decode: the Cassandra column value of one span fragment is
 *   Snappy(TBinaryProtocol(thrift Span))      CassieSpanStoreDefaults.SpanCodec
 *                                             (zipkin-cassandra/.../storage/cassandra/CassieSpanStore.scala:52;
 *                                             SnappyCodec.scala:32-51, ScroogeThriftCodec.scala:23-40)
 * with the Span / Annotation / BinaryAnnotation / Endpoint structs of
 *   zipkin-thrift/src/main/thrift/com/twitter/zipkin/zipkinCore.thrift:27-58.
 * The reference decodes each fragment twice (StorageRecordReader.scala:58 for the key, then
 * SpanSource.scala:20-22); this decodes once, straight into columns.
 *
 * Validation is the reference's thrift -> Span conversion (zipkin-scrooge/.../conversions/
 * thrift.scala): a null span name throws IncompleteTraceDataException (:101-104); an annotation
 * with timestamp <= 0 or an empty value throws IllegalArgumentException (:66-71); a null or empty
 * endpoint service name becomes "Unknown service name" (:36-43). ZK_INGEST_STRICT mirrors the
 * throw (the batch fails with ZK_ERR_INVALID_SPAN at the first bad span); otherwise bad spans are
 * skipped and counted. Bytes that do not decode are always ZK_ERR_INVALID_SPAN in strict mode.
 *
 * Record derivation (Span.scala:72-74,125-131,174-191,216-240): first/last
 * = min/max annotation timestamp; service = host of the first sr/ss annotation with a host, else
 * of the first cs/cr; 2-bit saturating counts of cs/cr/sr/ss; parentId presence.
 *
 * Side outputs for the sketches (zksketch.h), following the span indexer
 * (CassieSpanStore.scala:214-242; only spans with >= 1 annotation are indexed):
 *   key-value items   one per binary annotation with a host: (host service id, key hash)
 *   annotation items  one per distinct non-core annotation value with a host: (service id, value hash)
 * Hashes are zk_hash_string (64-bit FNV-1a, then the splitmix64 finalizer); the decoder keeps the
 * strings so hashes map back to names (zk_ingest_string).
 *
 * A zk_ingest owns the service-name dictionary (ids in order of first appearance, names
 * case-sensitive as Service(name) compares them, Dependencies.scala:25). It is not thread-safe.
 */
#ifndef ZKINGEST_H
#define ZKINGEST_H

#include <stddef.h>
#include <stdint.h>

#include "zkagg.h"
#include "zkstore.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ZK_CODEC_THRIFT        0u  /* TBinaryProtocol-encoded Span */
#define ZK_CODEC_SNAPPY_THRIFT 1u  /* raw Snappy block of the above (the stored Cassandra value) */

#define ZK_INGEST_STRICT 1u        /* fail the batch on the first span the reference rejects */
#define ZK_INGEST_ONE_THREAD 2u    /* host decoder: decode on the calling thread only (by default up to
                                      16 threads decode contiguous ranges; records, items, service ids
                                      and errors are the same either way) */
/* Both decoders (host zk_ingest_spans, device zk_ingest_dev_spans) reject a Snappy fragment whose
 * header announces more than ZK_INGEST_MAX_FRAGMENT bytes, or more than the format can expand its
 * payload to (a 3-byte copy emits at most 64 bytes: < ZK_SNAPPY_MAX_EXPANSION x), before any
 * allocation -- a 5-byte hostile header cannot make either decoder allocate gigabytes. */
#define ZK_INGEST_MAX_FRAGMENT   (1u << 24)
#define ZK_SNAPPY_MAX_EXPANSION  22u

typedef struct zk_ingest zk_ingest;

/* caller buffers for the sketch items (any may be NULL / cap 0: not produced) */
typedef struct zk_ingest_items {
    uint32_t* kv_service;     /* binary annotations: host service id */
    uint64_t* kv_key;         /* zk_hash_string(key) */
    uint64_t  kv_cap;
    uint64_t  kv_n;           /* out: items written */
    uint32_t* ann_service;    /* non-core annotation values */
    uint64_t* ann_value;      /* zk_hash_string(value) */
    uint64_t  ann_cap;
    uint64_t  ann_n;          /* out */
} zk_ingest_items;

zk_status   zk_ingest_create(zk_ingest** out);
zk_status   zk_ingest_destroy(zk_ingest* ing);
const char* zk_ingest_last_error(const zk_ingest* ing);

/* Decode n stored fragments: fragment i is buf[offsets[i] .. offsets[i+1]) (offsets has n+1
 * entries). Records go to the host columns of `out` (capacity >= n); *n_out = records written
 * (in input order), *n_rejected = spans skipped (lenient mode). items may be NULL.
 * ZK_ERR_CAPACITY when an item buffer is too small (the records are still written). */
zk_status zk_ingest_spans(zk_ingest* ing, const uint8_t* buf, const uint64_t* offsets, uint64_t n, uint32_t codec,
                          uint32_t flags, const zk_span_cols* out, uint64_t* n_out, uint64_t* n_rejected,
                          zk_ingest_items* items);

/* the service dictionary */
zk_status zk_ingest_num_services(const zk_ingest* ing, uint32_t* n);
zk_status zk_ingest_service_id(zk_ingest* ing, const char* name, uint64_t len, uint32_t* id);  /* adds if new */
zk_status zk_ingest_service_name(const zk_ingest* ing, uint32_t id, char* buf, uint64_t cap, uint64_t* len);
/* the string behind a key / value hash seen by this decoder (two-phase: buf NULL -> *len) */
zk_status zk_ingest_string(const zk_ingest* ing, uint64_t hash, char* buf, uint64_t cap, uint64_t* len);

/* ---- the same decoder on the device -------------------------------------------------------
 * zk_ingest_dev decodes fragments that are already in HBM (buf and offsets are device pointers)
 * into device columns, one lane per fragment (Snappy block, thrift walk, validation and record as
 * above; the indexer items through zk_ingest_dev_spans_items). Its service dictionary lives on the device: a batch's new names get ids
 * in the order of their hash-table slots (not in order of first appearance; names whose hashes
 * collide in the table may swap ids between runs), names are compared byte for byte. At most `max_services` distinct names
 * (ZK_ERR_SERVICE_RANGE past that). Thrift nesting deeper than 16 levels inside skipped fields is
 * treated as undecodable. Results are synchronous with respect to the host (the call waits). */
typedef struct zk_ingest_dev zk_ingest_dev;
zk_status   zk_ingest_dev_create(int32_t device, void* stream, uint32_t max_services, zk_ingest_dev** out);
zk_status   zk_ingest_dev_destroy(zk_ingest_dev* ing);
const char* zk_ingest_dev_last_error(const zk_ingest_dev* ing);
zk_status   zk_ingest_dev_spans(zk_ingest_dev* ing, const uint8_t* buf, const uint64_t* offsets, uint64_t n,
                                uint32_t codec, uint32_t flags, const zk_span_cols* out, uint64_t* n_out,
                                uint64_t* n_rejected);
/* The same decode with the span indexer's items (as zk_ingest_spans: CassieSpanStore.scala:214-242),
 * written to DEVICE buffers: kv_service / kv_key and ann_service / ann_value are device pointers
 * (either pair NULL or cap 0: not produced). Service ids are this decoder's; within a batch the items
 * come in no particular order (the sketches take a batch as a set), the multiset per batch equals the
 * host decoder's. ZK_ERR_CAPACITY when a buffer is too small (records and the first cap items are
 * still written; kv_n / ann_n are the items written). n < 2^30. The strings behind key / value hashes
 * are kept on the host side of the decoder: zk_ingest_dev_string. Slower than zk_ingest_dev_spans
 * (a second build of the decoder: a captured-string set probe per item, no copy-in prefetch). */
zk_status   zk_ingest_dev_spans_items(zk_ingest_dev* ing, const uint8_t* buf, const uint64_t* offsets, uint64_t n,
                                      uint32_t codec, uint32_t flags, const zk_span_cols* out, uint64_t* n_out,
                                      uint64_t* n_rejected, zk_ingest_items* items);
/* Several stored batches in one decode: batch b is bufs[b] + offsets[b][0..ns[b]] (device pointers;
 * host arrays of nb entries; ns[b] == 0 allowed). Records, rejected count and items (items may be
 * NULL: none) are those of zk_ingest_dev_spans(_items) over the batches joined in order; fragment
 * numbers in errors count across the batches. One set of launches and one host round trip for all
 * of them: a job reading many small stored batches (StorageRecordReader.scala:49-54, one row batch
 * per read) decodes them at the large-batch rate. */
zk_status   zk_ingest_dev_spans_multi(zk_ingest_dev* ing, uint32_t nb, const uint8_t* const* bufs,
                                      const uint64_t* const* offsets, const uint64_t* ns, uint32_t codec,
                                      uint32_t flags, const zk_span_cols* out, uint64_t* n_out,
                                      uint64_t* n_rejected, zk_ingest_items* items);
/* the string behind a key / value hash an items batch of this decoder has seen (two-phase) */
zk_status   zk_ingest_dev_string(const zk_ingest_dev* ing, uint64_t hash, char* buf, uint64_t cap, uint64_t* len);
zk_status   zk_ingest_dev_num_services(const zk_ingest_dev* ing, uint32_t* n);
/* Snappy scratch (deferred fragments' Spans, names not yet in the dictionary): bump-allocated per
 * batch and grown when a batch runs out (the fragments that missed out are decoded again). `bytes`
 * sets its size from the next batch on; 0 = automatic (max(64 MiB, 24 B per fragment)). */
zk_status   zk_ingest_dev_set_scratch(zk_ingest_dev* ing, uint64_t bytes);
zk_status   zk_ingest_dev_service_name(const zk_ingest_dev* ing, uint32_t id, char* buf, uint64_t cap,
                                       uint64_t* len);

/* ---- the Dependencies record on the wire ----------------------------------------------------
 * TBinaryProtocol thriftscala.Dependencies (zipkinDependencies.thrift:24-43) as the Cassandra
 * store writes it: WrappedDependencies.toThrift (zipkin-scrooge/.../conversions/thrift.scala:
 * 330-333) through ScroogeThriftCodec (zipkin-cassandra/.../cassandra/AggregatesBuilder.scala:31),
 * one column per record (CassandraAggregates.scala:111-116). Fields in id order, all written.
 * encode: service ids resolve through names[id] (name_lens[id] bytes, case-sensitive);
 * two-phase (out == NULL -> *len). decode: names map to ids through the dictionary of `dict`
 * exactly as stored ("" stays ""; new names are added); two-phase on the link count; bytes that
 * do not decode -> ZK_ERR_INVALID_SPAN. */
zk_status zk_dependencies_encode(int64_t start_us, int64_t end_us, const zk_dep_link* links, uint64_t n_links,
                                 const char* const* names, const uint32_t* name_lens, uint32_t num_names,
                                 uint8_t* out, uint64_t cap, uint64_t* len);
zk_status zk_dependencies_decode(zk_ingest* dict, const uint8_t* buf, uint64_t len, int64_t* start_us,
                                 int64_t* end_us, zk_dep_link* out, uint64_t cap, uint64_t* n_links);
/* the record's Cassandra row key: deps.startTime.floor(1.day).inMicroseconds
 * (CassandraAggregates.scala:111-113), integer division toward zero */
int64_t   zk_dependencies_row_key(int64_t start_us);

uint64_t  zk_hash_string(const char* s, uint64_t len);
/* raw Snappy block decompression (exposed for tools/tests): *out_len = uncompressed size; with
 * out == NULL only the size is read from the header */
zk_status zk_snappy_uncompress(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t cap, uint64_t* out_len);

#ifdef __cplusplus
}
#endif

#endif /* ZKINGEST_H */
