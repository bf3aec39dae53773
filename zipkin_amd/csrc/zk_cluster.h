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

// rocprim scratch for clustering n records
hipError_t cluster_temp_bytes(uint64_t n, size_t* bytes);
// in (any order) -> out (trace-clustered: stable sort by traceId); idx: n u32 scratch
hipError_t launch_cluster(const SpanColsDev& in, const SpanColsMut& out, uint32_t* idx, void* temp, size_t temp_bytes,
                          hipStream_t s);
// insert the traceId of every segment start into `set` (slots: power of two; slot `slots` counts
// traceId 0); *dup += segments whose traceId was already present
hipError_t launch_trace_set_insert(const uint64_t* trace_id, uint64_t n, uint64_t* set, uint64_t slots,
                                   unsigned long long* dup, hipStream_t s);
hipError_t launch_trace_set_rehash(const uint64_t* old, uint64_t old_slots, uint64_t* set, uint64_t slots,
                                   hipStream_t s);
// out[0..ST_N) = sum over the kStatShards copies of the device counters
hipError_t launch_stats_fold(const unsigned long long* shards, unsigned long long* out, hipStream_t s);

}  // namespace zk
