// zk_cluster.h — clustering pass, trace set and stats fold (zk_cluster.hip); internal.
#pragma once
#include "zk_internal.h"

namespace zk {

struct SpanColsMut {
    uint64_t* trace_id;
    uint64_t* span_id;
    uint64_t* parent_id;
    int64_t* first_ts;
    int64_t* last_ts;
    uint32_t* service_id;
    uint32_t* flags;
};

// clustering pass (zk_cluster.hip): b1 + b2 digit bits of the traceId hash (first level P1 global,
// second level P2 per bucket), then P3 per sub-bucket; b1 = 0: P3 alone over the whole batch
constexpr uint64_t kClusterSmall = 4096;
struct ClusterPlan {
    uint64_t n;
    uint32_t b1, b2, nb1, nb2;
    uint32_t grid;  // P0 / P1 workgroups
    uint64_t per;   // records per P0 / P1 workgroup (whole 8192-record chunks)
};
// groups: the plan of the group join (k_group_join), sub-buckets of ~500-1000 records
ClusterPlan cluster_plan(uint64_t n, uint32_t cus, bool groups = false);
uint64_t cluster_scratch_bytes(const ClusterPlan& p);
// the partition's output for the group join: every trace inside one sub-bucket of B
struct ClusterGroups {
    const uint32_t* sub;             // nsub + 1 record bounds
    uint32_t nsub;
    uint32_t* big_list;              // sub-buckets the group join leaves to the fallback
    unsigned int* big_count;
    unsigned long long* out_cursor;  // the fallback's clustered records (its K1's record count)
};
// in (any order) -> trace-clustered columns in A (*result = 0) or B (*result = 1); both hold n records.
// groups != nullptr and a two-level plan: P0-P2 only, B holds the sub-buckets, *groups describes them
// (counters zeroed) and *result = 1.
hipError_t launch_cluster(const ClusterPlan& p, const SpanColsDev& in, const SpanColsMut& A, const SpanColsMut& B,
                          void* scratch, uint32_t cus, hipStream_t s, int* result,
                          unsigned long long* capacity_fail, ClusterGroups* groups = nullptr);
// the group join's fallback: P3 over the listed sub-buckets of B into A[0, *out_cursor), clustered
hipError_t launch_cluster_fallback(const ClusterPlan& p, const ClusterGroups& g, const SpanColsDev& B,
                                   const SpanColsMut& A, void* scratch, uint32_t cus, hipStream_t s,
                                   unsigned long long* capacity_fail);
// insert the traceId of every segment start into `set` (slots: power of two; slot `slots` counts
// traceId 0); *dup += segments whose traceId was already present. Device limits (either may be
// null): only segments starting below *n_dev, and not the one at record 0 when *skip_dev.
hipError_t launch_trace_set_insert(const uint64_t* trace_id, uint64_t n, uint64_t* set, uint64_t slots,
                                   unsigned long long* dup, hipStream_t s,
                                   const unsigned long long* n_dev = nullptr, const uint32_t* skip_dev = nullptr);
hipError_t launch_trace_set_rehash(const uint64_t* old, uint64_t old_slots, uint64_t* set, uint64_t slots,
                                   hipStream_t s);
// out[0..ST_N) = sum over the kStatShards copies of the device counters
hipError_t launch_stat_add(unsigned long long* slot, uint64_t v, hipStream_t s);
hipError_t launch_stats_fold(const unsigned long long* shards, unsigned long long* out, hipStream_t s);
// ZK_BATCH_CONTINUES decided on the device, so a batch costs no host round trip. The held trace
// (the carry: 7 columns of <= max_trace + 2 records) and its state live in HBM; per batch
// k_carry_plan finds the batch's edge runs, mirrors the rules of zkagg.h (the leading run continues
// the held trace when it has its traceId; the held trace is complete once a batch moves on; a held
// trace longer than max_trace_records is dropped and counted once; with CONTINUES the batch's last
// run is held back) and writes the batch's plan, which the trace check, K1 (skip_dev, n_dev = &hi),
// the carry's join (K1 on one workgroup, or the spill kernel) and the tail copy read.
struct CarryState {
    unsigned long long n;         // records held in the carry
    unsigned long long tid;       // their traceId
    unsigned int dropped;         // the held trace outgrew max_trace_records: its rest is skipped
    unsigned int verify;          // a batch that carried it asked for ZK_BATCH_VERIFY_TRACES
    // the current batch's plan
    unsigned long long append_at; // the batch's records [0, append_n) go to carry[append_at, ...)
    unsigned long long append_n;
    unsigned long long flush_n;   // carry records [0, flush_n) are joined now, as one trace (0: none)
    unsigned long long flush_vn;  // ... and inserted into the trace set (flush_n or 0)
    unsigned long long hi;        // K1 and the trace check: the batch's records below hi
    unsigned long long tail_lo;   // the batch's records [tail_lo, n) are the new carry (>= n: none)
    unsigned long long zero;      // the carry join's spill list: one entry, record 0
    unsigned int flush_cnt;       // its length (flush_n > 0)
    unsigned int skip;            // K1: record 0's run belongs to the carry
};
// plan of one batch (batch.n > 0 records, trace-clustered), or with batch.n == 0 a flush: the held
// trace is complete (finalize, a batch in any order, an empty batch without CONTINUES). It also
// appends the batch's leading run to the carry, zeroes *spill_count (the batch's K1 spill list;
// may be null) and, when set != null, inserts the joined carry's traceId into the trace set.
// k1_joins: K1 joins a flushed carry (flush_cnt starts at 0); else the spill kernel (flush_cnt = 1).
hipError_t launch_carry_plan(CarryState* cs, const SpanColsDev& batch, const SpanColsMut& carry, uint64_t max_trace,
                             uint32_t continues, uint32_t verify, uint32_t k1_joins, unsigned long long* too_large,
                             unsigned int* spill_count, uint64_t* set, uint64_t slots, unsigned long long* dup,
                             hipStream_t s);
// the batch's tail -> the carry (the new held trace)
hipError_t launch_carry_tail(const CarryState* cs, const SpanColsDev& batch, const SpanColsMut& carry, hipStream_t s);

}  // namespace zk
