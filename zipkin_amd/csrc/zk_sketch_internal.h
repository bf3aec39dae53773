// zk_sketch_internal.h — shared pieces of the per-service sketches (include/zksketch.h).
//
// Every sketch of this library is per service: count-min + top-K candidates of binary-annotation
// keys (getTopKeyValueAnnotations, Aggregates.scala:34), HyperLogLog of distinct traceIds and a
// t-digest of span durations (RealtimeAggregates.scala:26-38). Updating a sketch of 16-64 KB per
// service with global atomics runs at the memory-side atomic rate (~2e9/s on MI355X, see
// profiles/r01_atomics_microbench.txt) -- three orders of magnitude below HBM streaming. So every
// sketch batch is first PARTITIONED by service (one streaming histogram pass, one scan, one
// scatter pass), after which one workgroup owns a contiguous run of one service's payloads and
// keeps that service's sketch in LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zk {

__host__ __device__ inline uint64_t sk_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Partition of (service, payload) items into service-contiguous order.
struct PartitionPlan {
    uint32_t S = 0;
    uint32_t grid = 0;      // workgroups of the histogram / scatter passes
    uint64_t per_wg = 0;    // items per workgroup (contiguous ranges)
};

PartitionPlan partition_plan(uint64_t n, uint32_t S, uint32_t cus);
// scratch bytes needed for hist (S*grid u32), offsets (S*grid+1 u64) and the scan temp storage
uint64_t partition_scratch_bytes(const PartitionPlan& p);
// svc/payload: device arrays of n items. out: device array of n payloads (service-contiguous).
// seg: device u64[S+1], seg[s]..seg[s+1] is service s's run in `out`. dropped: device u64 counter
// (items with svc >= S are dropped and counted). scratch: partition_scratch_bytes.
hipError_t launch_partition(const PartitionPlan& p, const uint32_t* svc, const uint64_t* payload, uint64_t n,
                            uint64_t* out, uint64_t* seg, unsigned long long* dropped, void* scratch,
                            hipStream_t s);

// Work units: service s's run is cut into ceil(len / unit_items) units. unit_base[s] = first unit
// of service s (exclusive scan), unit_base[S] = total. Computed on device from `seg`.
hipError_t launch_unit_plan(const uint64_t* seg, uint32_t S, uint64_t unit_items, uint32_t* unit_base,
                            hipStream_t s);

// ---- count-min + top-K of keys per service ----------------------------------------------------
constexpr uint32_t kKvMaxWidth = 4096;   // counters per row per service (LDS: depth*width*4 B)
constexpr uint32_t kKvMaxDepth = 8;
constexpr uint32_t kKvMaxCand = 256;     // candidates kept per service
constexpr uint64_t kKvUnitItems = 65536; // keys per workgroup in the sketch / candidate passes

struct KvArgs {
    uint32_t S, width, depth, wbits, cand;
    uint64_t seeds[kKvMaxDepth];
    uint32_t* cm;            // [S][depth][width] u32, accumulated across batches
    const uint64_t* keys;    // service-contiguous batch keys
    const uint64_t* seg;     // [S+1]
    const uint32_t* unit_base;  // [S+1]
    uint64_t unit_items;
    uint32_t max_units;      // grid bound
    uint64_t* unit_key;      // [max_units][cand]
    uint32_t* unit_est;      // [max_units][cand], 0 = empty
    uint64_t* cand_key;      // [S][cand] persistent candidates (sorted: est desc, key asc)
    uint32_t* cand_est;      // [S][cand], 0 = empty
    uint64_t* totals;        // [S] keys counted per service since reset
    // extra lists to merge (multi-GPU all-gather): [lists][S][cand]
    const uint64_t* extra_key;
    const uint32_t* extra_est;
    uint32_t extra_lists;
};

hipError_t launch_kv_sketch(const KvArgs& a, hipStream_t s);
hipError_t launch_kv_candidates(const KvArgs& a, hipStream_t s);
hipError_t launch_kv_merge(const KvArgs& a, hipStream_t s);  // prev cand + unit lists + extra lists
hipError_t launch_kv_estimate(const KvArgs& a, uint32_t svc, const uint64_t* keys, uint64_t n, uint32_t* est,
                              hipStream_t s);

}  // namespace zk
