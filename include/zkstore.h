/*
 * zkstore.h — C ABI of the Aggregates store surface of libzkagg (host side, no device work).
 *
 * Replaces the storage half of
 *   trait Aggregates  (zipkin-common/src/main/scala/com/twitter/zipkin/storage/Aggregates.scala:26-37)
 *     getDependencies(startDate: Option[Time], endDate: Option[Time] = None): Future[Dependencies]   :30
 *     storeDependencies(dependencies: Dependencies): Future[Unit]                                  :31
 *     getTopAnnotations(serviceName) / getTopKeyValueAnnotations(serviceName): Future[Seq[String]]  :33-34
 *     storeTopAnnotations(serviceName, a) / storeTopKeyValueAnnotations(serviceName, a)            :35-36
 * and the value types it moves:
 *   Moments(m0: Long, m1..m4: Double)           algebird-core 0.8.1 (project/Project.scala:42,50)
 *   DependencyLink(parent, child, Moments)      zipkin-common/.../common/Dependencies.scala:34
 *   Dependencies(startTime, endTime, links)     Dependencies.scala:59-63; wire form
 *                                               zipkin-thrift/.../zipkinDependencies.thrift:24-43 (us)
 *
 * The producer side of the store is the device path: zk_deps_finalize (zkagg.h) gives the dense
 * link table, zk_link_table_compact turns it into the job's single Dependencies record
 * (ZipkinAggregateJob.scala:41-45), and zk_kv_topk (zksketch.h) produces the per-service
 * top key-value annotation list that storeTopKeyValueAnnotations persists.
 *
 * Services and annotation strings are dictionary ids owned by the host (like zkagg.h); the store
 * never sees strings. Unlike a zk_ctx, a zk_store IS thread-safe: every call takes the store's
 * lock, mirroring the reference's `synchronized` writes (CassandraAggregates.scala:110,122) and
 * the transaction of AnormAggregates.storeDependencies (AnormAggregates.scala:83-109).
 */
#ifndef ZKSTORE_H
#define ZKSTORE_H

#include <stddef.h>
#include <stdint.h>

#include "zkagg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* algebird Moments: count, mean, sum (x-mean)^2, sum (x-mean)^3, sum (x-mean)^4 */
typedef struct zk_moments {
    int64_t m0;
    double  m1, m2, m3, m4;
} zk_moments;

/* DependencyLink(parent = Service(parent name), child = Service(child name), durationMoments) */
typedef struct zk_dep_link {
    uint32_t   parent;   /* host dictionary id of the parent service name (case-sensitive) */
    uint32_t   child;
    zk_moments moments;
} zk_dep_link;

/* Time.Top / Time.Bottom of the Dependencies monoid zero (Dependencies.scala:81), in us */
#define ZK_TIME_TOP    INT64_MAX
#define ZK_TIME_BOTTOM INT64_MIN

/* Storage semantics of the reference backends (each mode reproduces one, quirks included):
 *   ZK_STORE_ANORM      one row per stored record; getDependencies returns the links of the rows
 *                       with start_ts >= start AND end_ts <= end, newest record first, times = the
 *                       query window; absent bounds: start = now - 1 day, end = now
 *                       (AnormAggregates.scala:52-76; `now_us` is passed in so callers and tests
 *                       control Time.now)
 *   ZK_STORE_CASSANDRA  row key = startTime floored to the day (us); a store CLOBBERS that row
 *                       (CassandraAggregates.scala:111-116,122-136). getDependencies walks every
 *                       row and drops a column only if its name -- the index 0, compared with the
 *                       bounds in us (:58-61) -- exceeds a given bound, i.e. it returns every row
 *                       unless a bound is negative; rows in row-key order, Monoid-summed
 *   ZK_STORE_HBASE      row key = Long.MaxValue - startTime in ms, a store replaces a record of the
 *                       same ms (HBaseAggregates.scala:55-60). getDependencies scans row keys
 *                       [MaxValue - start ms, MaxValue - end ms) (:39-53): the records with
 *                       end ms < record start ms <= start ms (no start: from key 0; no end: to the
 *                       last row), newest first, Monoid-summed; start < end scans nothing
 * Monoid-summed = Dependencies monoid left fold in scan order (start = min, end = max, links merged
 * per (parent, child) with MomentsGroup.plus); no record -> the monoid zero (ZK_TIME_TOP,
 * ZK_TIME_BOTTOM, no links). Top-annotation lists: Anorm's are stubs (store ignored, get empty,
 * AnormAggregates.scala:111-137); Cassandra keeps one list per (service, kind), replaced by each
 * store (CassandraAggregates.scala:79-108,119-136); HBase writes both kinds into one family, so its getTopKeyValueAnnotations
 * is always empty and getTopAnnotations falls through to the next service id with a list
 * (HBaseAggregates.scala:62-110). */
#define ZK_STORE_ANORM     0u
#define ZK_STORE_CASSANDRA 1u
#define ZK_STORE_HBASE     2u

/* top-annotation lists (CassandraAggregates.scala:79-108: row "<service>:annotation" / ":kv") */
#define ZK_TOP_ANNOTATIONS    0u
#define ZK_TOP_KV_ANNOTATIONS 1u

typedef struct zk_store zk_store;

zk_status   zk_store_create(uint32_t mode, zk_store** out);
zk_status   zk_store_destroy(zk_store* st);                     /* Aggregates.close() */
const char* zk_store_last_error(const zk_store* st);

/* storeDependencies: one Dependencies record (its links are copied). */
zk_status zk_store_put_dependencies(zk_store* st, int64_t start_us, int64_t end_us, const zk_dep_link* links,
                                    uint64_t n_links);
/* getDependencies(startDate, endDate). start_us/end_us NULL = None. Two-phase: with out == NULL,
 * *n_links receives the number of links; otherwise up to `cap` links are written
 * (ZK_ERR_CAPACITY if cap is too small) together with the result's start/end times. */
zk_status zk_store_get_dependencies(zk_store* st, const int64_t* start_us, const int64_t* end_us, int64_t now_us,
                                    zk_dep_link* out, uint64_t cap, uint64_t* n_links, int64_t* out_start_us,
                                    int64_t* out_end_us);
/* number of stored Dependencies records */
zk_status zk_store_count(zk_store* st, uint64_t* records);
/* The incremental driver's watermark: IFNULL(MAX(end_ts), 0) over every stored row
 * (replaces AnormAggregator.scala:62-66's `SELECT IFNULL(MAX(END_TS), 0) FROM zipkin_dependencies`). */
zk_status zk_store_watermark(zk_store* st, int64_t* end_us);

/* storeTopAnnotations / storeTopKeyValueAnnotations: replace the list of `service` (`kind`
 * ZK_TOP_*); ids are host dictionary ids of the annotation values / keys, in list order. */
zk_status zk_store_put_top(zk_store* st, uint32_t kind, uint32_t service, const uint64_t* ids, uint64_t n);
/* getTopAnnotations / getTopKeyValueAnnotations: two-phase like get_dependencies; a service
 * without a stored list yields 0 entries (Seq.empty). */
zk_status zk_store_get_top(zk_store* st, uint32_t kind, uint32_t service, uint64_t* ids, uint64_t cap, uint64_t* n);

/* algebird MomentsGroup.plus (DependencyLink.sg.plus, Dependencies.scala:38-43) */
zk_status zk_moments_plus(const zk_moments* a, const zk_moments* b, zk_moments* out);

/* The job's output record: the present cells of a finalized HOST link table (zk_deps_finalize
 * with device_ptrs = 0) as DependencyLinks, cell order (parent-major). Two-phase like above.
 * ZipkinAggregateJob.scala:41-43 wraps them in Dependencies(Time(0), Time.now, links); when there
 * is no link the job emits nothing and storeDependencies is not called (:43-45). */
zk_status zk_link_table_compact(const zk_link_table* table, uint32_t num_services, zk_dep_link* out, uint64_t cap,
                                uint64_t* n_links);

#ifdef __cplusplus
}
#endif

#endif /* ZKSTORE_H */
