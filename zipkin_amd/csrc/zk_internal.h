// zk_internal.h — shared definitions of the zkagg HIP library (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/zkagg.h"

// roctx ranges around the library's host calls (rocprofv3 --marker-trace shows them next to the
// kernels they enqueue); a scope object so every return path pops
#include <rocprofiler-sdk-roctx/roctx.h>
namespace zk {
struct RoctxRange {
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};
}  // namespace zk

namespace zk {

// ---- exact accumulator layout ----------------------------------------------------------------
// One S x S cell = 16 u64 limbs (128 B). Each limb is a sum of 32-bit chunks, so it absorbs
// 2^32 additions without carrying; the cross-chunk carries are resolved only in finalize.
// With d < 2^40 us:  d: 2 chunks, d^2 (<2^80): 3, d^3 (<2^120): 4, d^4 (<2^160): 5.
constexpr int kLimbs = 16;
constexpr int kLimbM0 = 0;
constexpr int kLimbS1 = 1;   // 2 limbs
constexpr int kLimbS2 = 3;   // 3 limbs
constexpr int kLimbS3 = 6;   // 4 limbs
constexpr int kLimbS4 = 10;  // 5 limbs
constexpr uint64_t kMaxDuration = 1ull << 40;
constexpr uint64_t kMaxRecordsSinceReset = 0xFFFFFFFFull;
constexpr uint32_t kMaxServices = 4096;    // a link packs the cell in 24 bits: (cell << 40) | d
constexpr uint32_t kMaxBuckets = 1024;     // partitioned reduce: <= 1024 buckets of <= 1024 cells

// service key: (kind << 30) | id, kind 0 = server side, 1 = client side, 2 = none.
// atomicMin over fragments picks Span.serviceName's preference (server before client,
// Span.scala:125-131); the lowest id breaks ties between disagreeing fragments (ambiguous).
constexpr uint32_t kSvcKindShift = 30;
constexpr uint32_t kSvcIdMask = (1u << 30) - 1;
constexpr uint32_t kSvcNone = 0xFFFFFFFFu;

// device stats slots (mirror zk_stats field order)
enum Stat : int {
    ST_RECORDS = 0,
    ST_MERGED,
    ST_VALID,
    ST_INVALID,
    ST_CHILD,
    ST_JOINED,
    ST_MISSING_PARENT,
    ST_NO_SERVICE,
    ST_AMBIGUOUS,
    ST_SPILLED,
    ST_DUR_RANGE,
    ST_SVC_RANGE,
    ST_TOO_LARGE,
    ST_RT_DUR_RANGE,     // sketch items dropped for a duration >= 2^40 us (not in zk_stats)
    ST_SPILL_OVERFLOW,   // spill-list pushes past its capacity (cannot happen: one per tile at most)
    ST_NOT_CLUSTERED,    // trace segments whose traceId was already accumulated (ZK_BATCH_VERIFY_TRACES)
    ST_N = 16
};
constexpr int kStatShards = 256;  // stats buffer = kStatShards x ST_N u64
// the exact table is followed by a tail of ST_N u64: the folded counters (zk_deps_partial), so one
// SUM all-reduce of table + tail gives every rank the job-wide counters as well
constexpr uint64_t kTableTailBytes = ST_N * 8;
constexpr uint64_t kStatTailWords = ST_N;
static_assert(ST_NOT_CLUSTERED < ST_N, "stat slots");

struct SpanColsDev {
    const uint64_t* trace_id;
    const uint64_t* span_id;
    const uint64_t* parent_id;
    const int64_t* first_ts;
    const int64_t* last_ts;
    const uint32_t* service_id;
    const uint32_t* flags;
    uint64_t n;
};

// Everything the join kernels need for one accumulate call.
struct JoinArgs {
    SpanColsDev c;
    uint64_t* table;          // S*S*kLimbs
    unsigned long long* stats;  // kStatShards x ST_N
    uint32_t S;
    // spill (giant traces)
    unsigned int* spill_count;
    uint64_t* spill_list;
    uint64_t spill_cap;
    // per-spill-WG global scratch
    uint8_t* spill_scratch;
    uint64_t spill_scratch_stride;  // bytes per WG
    uint32_t max_trace;             // records
    // per-tile link lists written by K1: tile t's links at links[t*link_stride ...], link_count[t]
    uint64_t* links;                // (cell << 40) | duration
    uint32_t* link_count;
    uint64_t link_stride;
    // persistent K1 geometry: workgroup w owns traces starting in [w*per_wg, (w+1)*per_wg)
    uint64_t per_wg;
    uint32_t grid;
    // cell-bucket histogram per K1 workgroup, bucket-major (hist[b * grid + w]); nb = 0 disables it
    uint32_t* hist;
    uint32_t nb;
    uint32_t cb_shift;  // bucket = cell >> cb_shift
    uint32_t join;      // 1: the dependency path (parent join + links); 0: sketch items only
    uint32_t skip;      // 0 or 1: record 0 belongs to a run handled elsewhere (ZK_BATCH_CONTINUES)
    // realtime sketch items (zk_rt.hip), rt_pay == nullptr: none. K1 workgroup w writes rt_count[w]
    // items at w * link_stride; the spill kernel appends to list `grid` (capacity rt_spill_cap).
    uint64_t* rt_pay;
    uint32_t* rt_svc;
    uint32_t* rt_count;
    unsigned long long* rt_dropped;  // [0] spill-list overflow, [1] duration >= 2^40 us
    uint64_t rt_spill_cap;
    uint64_t rt_seed;
    uint32_t rt_p;
    // group join (k_group_join, unclustered batches): the sub-bucket bounds of the clustering pass's
    // partition (every trace inside one sub-bucket), and the list of sub-buckets too long for LDS
    const uint32_t* sub;      // nsub + 1 record bounds
    uint32_t nsub;
    uint32_t* big_list;       // [nsub] sub-bucket indices left to the fallback
    unsigned int* big_count;
    // K1 as the group join's fallback: the record count is on the device (n_dev, <= c.n) and the
    // links append to the lists the group join wrote (append = 1)
    const unsigned long long* n_dev;
    uint32_t append;
    // ZK_BATCH_CONTINUES on the device: skip read from here when set (and n from n_dev)
    const uint32_t* skip_dev;
    // realtime link items (zk_rl, a bound RealtimeAggregates store), lk_key == nullptr: none. One item
    // per emitted link, at the link's own list position: key ((child * S + parent) << 40) | duration,
    // and the child's traceId; the spill kernel appends to list `grid` (lk_spill_count, capacity
    // lk_spill_cap items)
    uint64_t* lk_key;
    uint64_t* lk_tid;
    uint32_t* lk_spill_count;
    uint64_t lk_spill_cap;
};

// host-side launchers (implemented in the .hip files)
// blocks != 0: only workgroups [0, blocks) of the a.grid geometry (K1 joining a held trace)
hipError_t launch_join(const JoinArgs& a, hipStream_t s, uint32_t blocks = 0);
// group join: one workgroup per CU; workgroup w owns the sub-buckets starting in [w*per_wg, (w+1)*per_wg)
hipError_t launch_group_join(const JoinArgs& a, hipStream_t s);
// geometry of the group join and of K1 as its fallback, sharing one set of link lists
void group_join_geometry(uint64_t n, uint32_t cus, uint32_t* grid, uint64_t* per_wg, uint64_t* link_stride);
uint32_t group_join_capacity();  // records of one sub-bucket the group join holds in LDS
uint64_t join_tile_records();   // TILE (records per K1 window)
// K1 launch geometry for n records on a device with `cus` compute units
void join_geometry(uint64_t n, uint32_t cus, uint32_t* grid, uint64_t* per_wg, uint64_t* link_stride);
hipError_t launch_link_reduce(const uint64_t* links, const uint32_t* counts, uint64_t stride, uint64_t tiles,
                              uint64_t* table, hipStream_t s);
// partitioned reduce (no global atomics): hist -> offsets -> bucket-sorted links -> LDS reduce
struct ReduceArgs {
    const uint64_t* links;   // per-workgroup lists from K1
    const uint32_t* counts;
    uint64_t stride;
    uint32_t lists;          // K1 grid
    const uint32_t* hist;    // [nb][lists]
    uint32_t nb, cb_shift;
    uint32_t* col_off;       // [nb][lists] exclusive offsets within each bucket
    uint64_t* bucket_base;   // [nb + 1]
    uint64_t* sorted;        // links grouped by bucket
    uint64_t* table;
    uint64_t cells;
};
hipError_t launch_partitioned_reduce(const ReduceArgs& r, hipStream_t s);
// bucket geometry for S services (nb = 0: use the atomic reduce)
void bucket_geometry(uint32_t S, uint32_t* nb, uint32_t* cb_shift);
uint64_t reduce_scatter_dyn_lds(uint32_t S);  // K2's dynamic LDS for S services (0: atomic reduce)
hipError_t launch_spill(const JoinArgs& a, uint32_t spill_wgs, hipStream_t s);
uint64_t spill_scratch_bytes_per_wg(uint32_t max_trace);
hipError_t launch_finalize(const uint64_t* table, uint32_t S, const zk_link_table* out,
                           hipStream_t s);
// packed exchange form of the table (zk_exchange.hip): S*S cells x 12 u64 (56-bit limbs) + the tail
uint64_t exchange_bytes(uint32_t S);
hipError_t launch_table_pack(const uint64_t* table, uint32_t S, uint64_t* xchg, hipStream_t s);
hipError_t launch_table_unpack(const uint64_t* xchg, uint32_t S, uint64_t* table, hipStream_t s);
hipError_t launch_tracegen(const zk_tracegen_params* p, const zk_span_cols* out, uint64_t cap,
                           uint64_t* n_records, uint64_t* n_traces, hipStream_t s);

}  // namespace zk
