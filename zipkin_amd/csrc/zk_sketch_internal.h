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
// the inverse of sk_mix64 (the splitmix64 finalizer is a bijection of 64-bit words)
__host__ __device__ inline uint64_t sk_unmix64(uint64_t z) {
    z = z ^ (z >> 31) ^ (z >> 62);
    z *= 0x319642B2D24D8EC3ull;
    z = z ^ (z >> 27) ^ (z >> 54);
    z *= 0x96DE1B173F119089ull;
    z = z ^ (z >> 30) ^ (z >> 60);
    return z;
}

// Partition of (service, payload) items into service-contiguous order.
struct PartitionPlan {
    uint32_t S = 0;
    uint32_t grid = 0;      // workgroups of the histogram / scatter passes
    uint64_t per_wg = 0;    // items per workgroup (contiguous ranges)
};

PartitionPlan partition_plan(uint64_t n, uint32_t S, uint32_t cus);
// which scatter kernel a partition of S services launches: the line scatter when its static LDS plus
// the [S][8] carry fit one CU, else the item scatter, else none (a refusal); *dyn = its dynamic LDS
enum { kScatterNone = -1, kScatterItems = 0, kScatterLines = 1 };
int partition_scatter_choice(uint32_t S, uint64_t static_lines, uint64_t static_items, uint64_t* dyn);
// Partition of per-workgroup lists instead of one flat range: list w is [w*stride, w*stride +
// counts[w]) of svc/payload (the item lists K1 writes), one partition workgroup per list.
PartitionPlan partition_plan_lists(uint32_t lists, uint32_t S);
// scratch bytes needed for hist (S*grid u32), offsets (S*grid+1 u64) and the scan temp storage
uint64_t partition_scratch_bytes(const PartitionPlan& p);
// svc/payload: device arrays of n items. out: device array of n payloads (service-contiguous).
// seg: device u64[S+1], seg[s]..seg[s+1] is service s's run in `out`. dropped: device u64 counter
// (items with svc >= S are dropped and counted). scratch: partition_scratch_bytes.
// hash: every payload is written as sk_mix64(payload ^ hash_seed) (the count-min's key hash,
// computed once here instead of in both sketch passes; sk_unmix64 recovers the key)
hipError_t launch_partition(const PartitionPlan& p, const uint32_t* svc, const uint64_t* payload, uint64_t n,
                            uint64_t* out, uint64_t* seg, unsigned long long* dropped, void* scratch,
                            hipStream_t s, bool hash = false, uint64_t hash_seed = 0);
// lists form: counts[w] items at offset w * stride (plan from partition_plan_lists)
hipError_t launch_partition_lists(const PartitionPlan& p, const uint32_t* svc, const uint64_t* payload,
                                  uint64_t stride, const uint32_t* counts, uint64_t* out, uint64_t* seg,
                                  unsigned long long* dropped, void* scratch, hipStream_t s);

// Work units: service s's run is cut into ceil(len / unit_items) units. unit_base[s] = first unit
// of service s (exclusive scan), unit_base[S] = total. Computed on device from `seg`.
hipError_t launch_unit_plan(const uint64_t* seg, uint32_t S, uint64_t unit_items, uint32_t* unit_base,
                            hipStream_t s);

// ---- count-min + top-K of keys per service ----------------------------------------------------
constexpr uint32_t kKvMaxWidth = 4096;   // counters per row per service (LDS: depth*width*4 B)
constexpr uint32_t kKvMaxDepth = 8;
constexpr uint32_t kKvMaxCand = 256;     // candidates kept per service
constexpr uint64_t kKvUnitItems = 65536;  // keys per workgroup in the sketch / candidate passes

struct KvArgs {
    uint32_t S, width, depth, wbits, cand;
    uint64_t seeds[kKvMaxDepth];
    uint32_t* cm;            // [S][depth][width] u32, accumulated across batches
    const uint64_t* keys;    // service-contiguous batch keys, hashed: sk_mix64(key ^ seeds[0])
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

// small: the counters are read and added in global memory instead of an LDS row block per unit
// (zk_kv_accumulate picks it for batches of fewer than kKvSmallPerService keys per service)
constexpr uint64_t kKvSmallPerService = 8192;
hipError_t launch_kv_sketch(const KvArgs& a, hipStream_t s, bool small);
hipError_t launch_kv_candidates(const KvArgs& a, hipStream_t s, bool small);
hipError_t launch_kv_merge(const KvArgs& a, hipStream_t s, bool small);  // prev cand + unit lists + extra lists
hipError_t launch_kv_estimate(const KvArgs& a, uint32_t svc, const uint64_t* keys, uint64_t n, uint32_t* est,
                              hipStream_t s);

// ---- realtime sketches: HyperLogLog distinct traces + log-linear duration histogram ------------
// item payload: (register index << 46) | (rho << 40) | duration   (p <= 16, rho <= 61, d < 2^40)
constexpr uint32_t kRtMaxP = 16;
constexpr uint32_t kRtPayShiftIdx = 46;
constexpr uint32_t kRtPayShiftRho = 40;
constexpr uint64_t kRtUnitItems = 65536;

__host__ __device__ inline uint32_t rt_nbins(uint32_t m) { return (41u - m) << m; }
// bin of a duration d < 2^40: d itself below 2^m, else (exponent - m + 1, top m mantissa bits)
__host__ __device__ inline uint32_t rt_bin(uint64_t d, uint32_t m) {
    if (d < (1ull << m)) return (uint32_t)d;
    const uint32_t e = 63u - (uint32_t)__builtin_clzll(d);
    return ((e - m + 1u) << m) | (uint32_t)((d >> (e - m)) & ((1ull << m) - 1ull));
}
// The salt decorrelates the register hash from the traceId-hash shard of a span (zk_trace_shard
// also hashes traceIds with splitmix64: a shard's traceIds would otherwise share hash bits).
constexpr uint64_t kRtSalt = 0xD6E8FEB86659FD93ull;
__host__ __device__ inline uint64_t rt_payload(uint64_t trace_id, uint64_t d, uint32_t p, uint64_t seed) {
    const uint64_t h = sk_mix64(trace_id ^ seed ^ kRtSalt);
    const uint64_t idx = h >> (64u - p);
    const uint64_t w = h << p;
    const uint64_t rho = w ? (uint64_t)__builtin_clzll(w) + 1u : (uint64_t)(64u - p + 1u);
    return (idx << kRtPayShiftIdx) | (rho << kRtPayShiftRho) | d;
}

struct RtArgs {
    uint32_t S, p, m, nbins;
    uint8_t* regs;               // [S][2^p] (u32-aligned rows)
    uint32_t* hist;              // [S][nbins]
    const uint64_t* items;       // service-contiguous payloads
    const uint64_t* seg;         // [S+1]
    const uint32_t* unit_base;   // [S+1]
    uint64_t unit_items;
    uint32_t max_units;
};
hipError_t launch_rt_sketch(const RtArgs& a, hipStream_t s);
// per service: [z_lo, z_hi, zero registers, N, the bin of each q[i]] (u64 x (4 + nq)), k_rt_query
constexpr uint32_t kRtQueryMaxQ = 32;
hipError_t launch_rt_query(const uint8_t* regs, const uint32_t* hist, uint32_t S, uint32_t p, uint32_t nbins,
                           const double* q, uint32_t nq, unsigned long long* out, hipStream_t s);
// merged-span input -> (svc, payload) items; invalid items get svc = 0xFFFFFFFF (dropped by the
// partition) and are counted in dropped[0] (service) / dropped[1] (duration)
hipError_t launch_rt_items(const uint32_t* svc, const uint64_t* trace_id, const int64_t* dur, uint64_t n, uint32_t S,
                           uint32_t p, uint64_t seed, uint32_t* out_svc, uint64_t* out_pay,
                           unsigned long long* dropped, hipStream_t s);

}  // namespace zk
