/*
 * zkcomm.h — the multi-GPU step of libzkagg for hosts without torch.distributed (the JVM drop-in):
 * an RCCL communicator over xGMI and one call per mergeable state.
 *
 * The reference merges the per-reducer partial results of the dependency job with Scalding's
 * cross-reducer `.group.sum` / `.sum`
 *   zipkin-aggregate/src/main/scala/com/twitter/zipkin/aggregate/ZipkinAggregateJob.scala:39-43
 * Here every rank (one process per GPU) aggregates a traceId-disjoint part of the spans -- both
 * shuffle keys of the job contain traceId (:21, :30), so every merge and join is rank-local; a
 * Cassandra/HBase split by row key is traceId-disjoint already, other sources route each span to
 * rank zk_trace_shard(traceId, world) -- and the ranks' states are combined by collectives:
 *
 *   zk_deps_allreduce  zk_deps_partial -> ONE int64 SUM all-reduce of the exchange buffer (56-bit
 *                      limbs + the counter tail, zkagg.h) -> zk_deps_note_merged. Every rank then
 *                      finalizes the same job-wide table and reaches the same status.
 *   zk_rt_allreduce    HyperLogLog registers by u8 MAX, duration histogram bins by u32 SUM.
 *   zk_kv_allreduce    all-gather of every rank's candidate lists, u32 SUM of the count-min
 *                      counters and u64 SUM of the totals, then zk_kv_merge_candidates: every rank
 *                      holds the same top-K lists.
 *
 * All collectives are enqueued on the handle's stream (the ctx's, the sketch's) after its pending
 * work; the calls return without waiting, except zk_deps_allreduce with total_records = 0 (see
 * zk_deps_note_merged). Every rank must make the same calls in the same order, as with any RCCL
 * communicator. RCCL (librccl.so.1 of the ROCm install, or the copy a host process already loaded)
 * is opened at the first zk_comm_* call; without it they return ZK_ERR_UNSUPPORTED.
 *
 * Bootstrap: rank 0 calls zk_comm_unique_id and hands the ZK_COMM_ID_BYTES bytes to the other
 * ranks over the host's own channel (the JVM job's driver, a file, a TCP socket); every rank then
 * calls zk_comm_create with the same bytes. zk_comm_create blocks until all `world` ranks joined.
 */
#ifndef ZKCOMM_H
#define ZKCOMM_H

#include <stdint.h>

#include "zkagg.h"
#include "zksketch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ZK_COMM_ID_BYTES 128

typedef struct zk_comm zk_comm;

zk_status   zk_comm_unique_id(uint8_t* id, uint64_t bytes);  /* bytes >= ZK_COMM_ID_BYTES */
zk_status   zk_comm_create(const uint8_t* id, uint64_t bytes, uint32_t rank, uint32_t world, int32_t device,
                           zk_comm** out);
zk_status   zk_comm_destroy(zk_comm* comm);
/* the handle's last collective error; NULL: why the calling thread's last zk_comm_unique_id /
   zk_comm_create failed (RCCL's message) */
const char* zk_comm_last_error(const zk_comm* comm);

/* total_records: records of the whole job (bounds the capacity check), 0 = read it from the merged
   counter tail (one stream synchronisation). The ctx and the communicator must be on one device. */
zk_status   zk_deps_allreduce(zk_ctx* ctx, zk_comm* comm, uint64_t total_records);
zk_status   zk_rt_allreduce(zk_rt* rt, zk_comm* comm);
zk_status   zk_kv_allreduce(zk_kv* kv, zk_comm* comm);

#ifdef __cplusplus
}
#endif
#endif /* ZKCOMM_H */
