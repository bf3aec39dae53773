// zk_api.cpp — the C ABI of libzkagg (include/zkagg.h): context, memory, launches, status.
//
// Host-side counterpart of the reference's Scalding driver (ZipkinAggregateJob.scala:10-46):
// instead of four Hadoop shuffles it owns one device-resident exact accumulator per context and
// orders every kernel on one HIP stream. There is deliberately no host compute path.
#include <hip/hip_runtime.h>
#include <string.h>

#include <new>
#include <string>
#include <utility>
#include <vector>

#include "zk_cluster.h"
#include "zk_comm.h"

#include "zk_internal.h"
#include "zk_launch.h"
#include "zk_rl_internal.h"
#include "zk_rt_internal.h"

using namespace zk;

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
};

struct zk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t S = 0;
    bool strict = true;
    uint32_t max_trace = 131072;
    bool timing = false;
    // unclustered batches through the group join (k_group_join); zk_config.trace_pass = 1: through
    // P3 + K1 instead (the A/B of profiles/r04/ab_group_join.txt)
    bool group_join = true;
    uint64_t* table = nullptr;            // S*S*kLimbs
    bool own_table = true;
    unsigned long long* stats = nullptr;  // kStatShards*ST_N
    unsigned long long* h_stats = nullptr;  // pinned host copy of stats
    hipEvent_t ev_stats = nullptr;          // recorded after the stats copy (polled, not slept on)
    unsigned int* spill_count = nullptr;
    uint64_t* spill_list = nullptr;
    uint64_t spill_cap = 0;
    uint8_t* spill_scratch = nullptr;
    uint64_t spill_stride = 0;
    uint32_t spill_wgs = 16;
    // per-tile link lists (K1 -> K3)
    uint64_t* links = nullptr;
    uint32_t* link_count = nullptr;
    uint64_t link_slots = 0;  // capacity of `links` in u64
    uint64_t sorted_slots = 0;  // capacity of `sorted` in u64
    uint32_t link_lists = 0;  // capacity of `link_count`
    uint32_t col_off_lists = 0;  // capacity of `col_off` in lists (x nb)
    uint32_t cus = 256;
    // partitioned reduce state (nb = 0: atomic reduce)
    uint32_t nb = 0, cb_shift = 0;
    uint32_t* hist = nullptr;
    uint32_t* col_off = nullptr;
    uint64_t* bucket_base = nullptr;
    uint64_t* sorted = nullptr;
    // host-pointer input staging
    void* stage = nullptr;
    uint64_t stage_cap = 0;
    hipEvent_t ev_stage = nullptr;  // after the staging copies: the call returns once they read the caller's memory
    // finalize staging for host outputs
    void* fin_stage = nullptr;
    uint64_t records_since_reset = 0;
    bool merged = false;                  // the table holds the all-reduced job (zk_deps_note_merged)
    bool continued = false;               // a batch was accumulated into a merged table since the reset
    uint64_t* xchg = nullptr;             // packed exchange form of the table (zk_deps_partial)
    bool aborted = false;                 // zk_deps_abort: the next exchange carries an abort mark
    bool folded = false;                  // zk_deps_partial folded this ctx's counters into the table tail
                                          // since the last reset / accumulate (note_merged requires it)
    // clustering pass for unclustered batches (zk_cluster.hip)
    uint8_t* cl_cols = nullptr;           // 2 x 7 aligned columns of cl_cap records (the passes ping-pong)
    uint64_t cl_cap = 0;
    void* cl_temp = nullptr;              // partition histograms, offsets, bucket bounds, scan scratch
    size_t cl_temp_bytes = 0;
    // traceIds accumulated since reset (ZK_BATCH_VERIFY_TRACES): tset_slots + 1 u64
    uint64_t* tset = nullptr;
    uint64_t tset_slots = 0;
    uint64_t tset_records = 0;
    // ZK_BATCH_CONTINUES: the held-back last trace of the batches so far (7 aligned columns of
    // carry_cap records) and its state, both on the device and decided there (zk_cluster.h
    // CarryState): a batch costs the host no round trip
    uint8_t* carry = nullptr;
    uint64_t carry_cap = 0;
    CarryState* cs = nullptr;
    bool maybe_carry = false;             // a CONTINUES batch since the last flush: the carry may hold records
    bool any_verify = false;              // a batch since the reset asked for ZK_BATCH_VERIFY_TRACES
    std::string err;
    // bound realtime sketch (zk_rt_bind)
    zk_rt* rt = nullptr;
    uint32_t rt_mode = ZK_RT_WITH_DEPS;
    // bound realtime link store (zk_rl_bind): K1 writes an item beside every link
    zk_rl* rl = nullptr;
    // timing
    std::vector<EventPair> ev_free, ev_join, ev_reduce, ev_spill, ev_fin, ev_cluster;
    zk_timing tm{};
};

namespace {

zk_status fail(zk_ctx* c, zk_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

zk_status hip_fail(zk_ctx* c, hipError_t e, const char* where) {
    if (e == hipErrorLaunchOutOfResources && *launch_refusal())  // launch_checked refused a launch
        return fail(c, ZK_ERR_CAPACITY, std::string(where) + ": " + launch_refusal());
    return fail(c, ZK_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define ZK_HIP(ctx, call)                                   \
    do {                                                    \
        hipError_t _e = (call);                             \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #call); \
    } while (0)

#define ZK_ST(call)                        \
    do {                                   \
        const zk_status _s = (call);       \
        if (_s != ZK_OK) return _s;        \
    } while (0)

// No C++ exception crosses the C ABI (zkagg.h: "never throws or aborts").
#define ZK_TRY try {
#define ZK_CATCH(ctx)                                                                      \
    }                                                                                      \
    catch (const std::bad_alloc&) {                                                        \
        return fail(ctx, ZK_ERR_CAPACITY, "host allocation failed");                       \
    }                                                                                      \
    catch (...) {                                                                          \
        return fail(ctx, ZK_ERR_INVALID_ARG, "unexpected host exception");                 \
    }

uint64_t table_bytes(uint32_t S) { return (uint64_t)S * S * kLimbs * 8 + kTableTailBytes; }

EventPair take_pair(zk_ctx* c) {
    EventPair p;
    if (!c->ev_free.empty()) {
        p = c->ev_free.back();
        c->ev_free.pop_back();
    } else {
        hipEventCreate(&p.a);
        hipEventCreate(&p.b);
    }
    return p;
}

uint64_t tiles_for(uint64_t n) { return (n + join_tile_records() - 1) / join_tile_records(); }

zk_status ensure_links(zk_ctx* c, uint32_t grid, uint64_t stride, uint64_t n) {
    const uint64_t slots = (uint64_t)grid * stride;
    // K2's bucket-sorted copy holds every link once: at most one per record
    const uint64_t sorted_slots = n + 64 < slots ? n + 64 : slots;
    const bool set_ok = slots <= c->link_slots && grid <= c->link_lists;
    const bool scratch_ok = !c->nb || (sorted_slots <= c->sorted_slots && grid <= c->col_off_lists);
    if (set_ok && scratch_ok) return ZK_OK;
    if (!set_ok) {  // the link lists
        hipFree(c->links);
        hipFree(c->link_count);
        hipFree(c->hist);
        c->links = nullptr;
        c->link_count = nullptr;
        c->hist = nullptr;
        c->link_slots = 0;
        c->link_lists = 0;
        ZK_HIP(c, hipMalloc(&c->links, slots * sizeof(uint64_t)));
        ZK_HIP(c, hipMalloc(&c->link_count, (uint64_t)grid * sizeof(uint32_t)));
        if (c->nb) ZK_HIP(c, hipMalloc(&c->hist, (uint64_t)grid * c->nb * sizeof(uint32_t)));
        c->link_slots = slots;
        c->link_lists = grid;
    }
    if (!scratch_ok) {  // K2/K3's scratch
        const uint64_t ss = sorted_slots > c->sorted_slots ? sorted_slots : c->sorted_slots;
        const uint32_t gl = grid > c->col_off_lists ? grid : c->col_off_lists;
        hipFree(c->col_off);
        hipFree(c->sorted);
        c->col_off = nullptr;
        c->sorted = nullptr;
        c->sorted_slots = 0;
        c->col_off_lists = 0;
        ZK_HIP(c, hipMalloc(&c->col_off, (uint64_t)gl * c->nb * sizeof(uint32_t)));
        ZK_HIP(c, hipMalloc(&c->sorted, ss * sizeof(uint64_t)));
        c->sorted_slots = ss;
        c->col_off_lists = gl;
        if (!c->bucket_base) ZK_HIP(c, hipMalloc(&c->bucket_base, (c->nb + 1) * sizeof(uint64_t)));
    }
    return ZK_OK;
}

bool aligned(const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; }

zk_status ensure_spill(zk_ctx* c, uint64_t n) {
    const uint64_t need = tiles_for(n) + 1;  // a spilled trace is longer than a tile
    if (need > c->spill_cap) {
        if (c->spill_list) ZK_HIP(c, hipFree(c->spill_list));
        uint64_t cap = need < (1ull << 16) ? (1ull << 16) : need;
        ZK_HIP(c, hipMalloc(&c->spill_list, cap * sizeof(uint64_t)));
        c->spill_cap = cap;
    }
    if (!c->spill_scratch) {
        c->spill_stride = spill_scratch_bytes_per_wg(c->max_trace);
        ZK_HIP(c, hipMalloc(&c->spill_scratch, c->spill_stride * c->spill_wgs));
    }
    return ZK_OK;
}

// zk_deps_abort's mark in the exchange tail's records word (zkagg.h)
constexpr int kAbortShift = 48;
constexpr uint64_t kAbortUnit = 1ull << kAbortShift;

zk_status stats_sum(zk_ctx* c, uint64_t out[ST_N], uint64_t* aborted_ranks = nullptr) {
    // The counters end every finalize (the job's status), so their round trip is on the step's
    // critical path: a pinned destination and a polled event instead of a blocking stream sync
    // (whose wake-up leaves the GPU idle for tens of microseconds before the next step's work).
    const size_t bytes = (size_t)kStatShards * ST_N * 8;
    if (!c->h_stats) ZK_HIP(c, hipHostMalloc((void**)&c->h_stats, bytes, hipHostMallocDefault));
    if (!c->ev_stats) ZK_HIP(c, hipEventCreateWithFlags(&c->ev_stats, hipEventDisableTiming));
    const uint64_t cells = (uint64_t)c->S * c->S;
    if (c->merged)  // the all-reduced job-wide counters in the table's tail
        ZK_HIP(c, hipMemcpyAsync(c->h_stats, c->table + cells * kLimbs, kTableTailBytes, hipMemcpyDeviceToHost,
                                 c->stream));
    else
        ZK_HIP(c, hipMemcpyAsync(c->h_stats, c->stats, bytes, hipMemcpyDeviceToHost, c->stream));
    ZK_HIP(c, hipEventRecord(c->ev_stats, c->stream));
    hipError_t q;
    while ((q = hipEventQuery(c->ev_stats)) == hipErrorNotReady) {
    }
    if (q != hipSuccess) return fail(c, ZK_ERR_HIP, std::string("stats copy: ") + hipGetErrorString(q));
    const unsigned long long* h = c->h_stats;
    for (int s = 0; s < ST_N; ++s) out[s] = 0;
    for (int sh = 0; sh < (c->merged ? 1 : kStatShards); ++sh)
        for (int s = 0; s < ST_N; ++s) out[s] += h[(size_t)sh * ST_N + s];
    if (aborted_ranks) *aborted_ranks = out[ST_RECORDS] >> kAbortShift;
    out[ST_RECORDS] &= kAbortUnit - 1;  // the abort marks of zk_deps_abort ride in the high bits
    return ZK_OK;
}

bool cols_ok(const zk_span_cols* c) {
    return c && c->trace_id && c->span_id && c->parent_id && c->first_ts && c->last_ts && c->service_id && c->flags;
}

// 7 columns of n records carved from one buffer, every column on a 256-byte boundary
uint64_t carved_bytes(uint64_t n) { return 5 * ((n * 8 + 255) & ~255ull) + 2 * ((n * 4 + 255) & ~255ull); }
SpanColsMut carve_cols(uint8_t* p, uint64_t n) {
    auto take = [&](uint64_t bytes) {
        uint8_t* q = p;
        p += (bytes + 255) & ~255ull;
        return q;
    };
    SpanColsMut m;
    m.trace_id = (uint64_t*)take(n * 8);
    m.span_id = (uint64_t*)take(n * 8);
    m.parent_id = (uint64_t*)take(n * 8);
    m.first_ts = (int64_t*)take(n * 8);
    m.last_ts = (int64_t*)take(n * 8);
    m.service_id = (uint32_t*)take(n * 4);
    m.flags = (uint32_t*)take(n * 4);
    return m;
}

// the clustering pass's two column sets and scratch for n records under `plan`
zk_status ensure_cluster(zk_ctx* c, uint64_t n, const ClusterPlan& plan) {
    const uint64_t tb = cluster_scratch_bytes(plan);
    if (n > c->cl_cap) {
        hipFree(c->cl_cols);
        c->cl_cols = nullptr;
        c->cl_cap = 0;
        if (hipMalloc(&c->cl_cols, 2 * carved_bytes(n)) != hipSuccess) {
            (void)hipGetLastError();
            return fail(c, ZK_ERR_CAPACITY, "no device memory for the clustering pass (96 B per record)");
        }
        c->cl_cap = n;
    }
    if (tb > c->cl_temp_bytes) {
        hipFree(c->cl_temp);
        c->cl_temp = nullptr;
        c->cl_temp_bytes = 0;
        ZK_HIP(c, hipMalloc(&c->cl_temp, tb));
        c->cl_temp_bytes = tb;
    }
    return ZK_OK;
}

// clustering pass: d (any order) -> ctx-owned trace-clustered columns
zk_status cluster_batch(zk_ctx* c, SpanColsDev* d) {
    RoctxRange rr("zk_cluster_batch");
    const uint64_t n = d->n;
    if (n > 0xFFFFFFFFull) return fail(c, ZK_ERR_CAPACITY, "an unclustered batch is limited to 2^32-1 records");
    const ClusterPlan plan = cluster_plan(n, c->cus);
    const zk_status es = ensure_cluster(c, n, plan);
    if (es != ZK_OK) return es;
    const SpanColsMut A = carve_cols(c->cl_cols, n);
    const SpanColsMut B = carve_cols(c->cl_cols + carved_bytes(n), n);
    int res = 0;
    ZK_HIP(c, launch_cluster(plan, *d, A, B, c->cl_temp, c->cus, c->stream, &res, c->stats + ST_SPILL_OVERFLOW));
    const SpanColsMut& m = res ? B : A;
    *d = SpanColsDev{m.trace_id, m.span_id, m.parent_id, m.first_ts, m.last_ts, m.service_id, m.flags, n};
    return ZK_OK;
}

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// ZK_BATCH_VERIFY_TRACES: grow the traceId set for `more` records (load <= 1/2 even if every record
// were its own trace)
zk_status ensure_tset(zk_ctx* c, uint64_t more) {
    const uint64_t need = pow2_at_least(2 * (c->tset_records + more) > (1ull << 16) ? 2 * (c->tset_records + more)
                                                                                    : (1ull << 16));
    if (need > c->tset_slots) {
        uint64_t* nt = nullptr;
        if (hipMalloc(&nt, (need + 1) * 8) != hipSuccess) {
            (void)hipGetLastError();  // clear the sticky allocation error
            return fail(c, ZK_ERR_CAPACITY,
                        "ZK_BATCH_VERIFY_TRACES: no device memory for the traceId set (" +
                            std::to_string((need + 1) * 8) + " B; 16 B per record since reset, ~24 B during a rehash)");
        }
        hipError_t e = hipMemsetAsync(nt, 0, (need + 1) * 8, c->stream);
        if (e == hipSuccess && c->tset) {
            e = launch_trace_set_rehash(c->tset, c->tset_slots, nt, need, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        }
        if (e != hipSuccess) {
            hipFree(nt);
            return hip_fail(c, e, "traceId set rehash");
        }
        if (c->tset) hipFree(c->tset);
        c->tset = nt;
        c->tset_slots = need;
    }
    c->tset_records += more;
    return ZK_OK;
}

// ... and insert the batch's trace runs
zk_status verify_batch(zk_ctx* c, const SpanColsDev& d) {
    RoctxRange rr("zk_verify_traces");
    const zk_status st = ensure_tset(c, d.n);
    if (st != ZK_OK) return st;
    ZK_HIP(c, launch_trace_set_insert(d.trace_id, d.n, c->tset, c->tset_slots, &c->stats[ST_NOT_CLUSTERED],
                                      c->stream));
    return ZK_OK;
}

}  // namespace

extern "C" {

uint32_t zk_abi_version(void) { return ZK_ABI_VERSION; }

const char* zk_status_str(zk_status s) {
    switch (s) {
        case ZK_OK: return "ok";
        case ZK_ERR_INVALID_ARG: return "invalid argument";
        case ZK_ERR_HIP: return "HIP runtime error";
        case ZK_ERR_NO_SERVICE: return "joined span without service name (reference: None.get)";
        case ZK_ERR_DURATION_RANGE: return "span duration >= 2^40 us";
        case ZK_ERR_TRACE_TOO_LARGE: return "trace longer than max_trace_records";
        case ZK_ERR_CAPACITY: return "exact accumulator headroom exhausted";
        case ZK_ERR_NOT_CLUSTERED: return "batch is not trace-clustered";
        case ZK_ERR_NO_DEVICE: return "no gfx950 HIP device";
        case ZK_ERR_SERVICE_RANGE: return "service_id >= num_services";
        case ZK_ERR_UNSUPPORTED: return "unsupported";
        case ZK_ERR_INVALID_SPAN: return "invalid or undecodable span";
        case ZK_ERR_RANK_FAILED: return "another rank of the job failed (zk_deps_abort)";
    }
    return "unknown status";
}

const char* zk_last_error(const zk_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

zk_status zk_ctx_create(const zk_config* cfg, zk_ctx** out) {
    ZK_TRY
    if (!cfg || !out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    if (cfg->num_services == 0 || cfg->num_services > kMaxServices) return ZK_ERR_INVALID_ARG;
    if (cfg->max_trace_records > (1u << 20)) return ZK_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ZK_ERR_NO_DEVICE;
    if (cfg->device < 0 || cfg->device >= ndev) return ZK_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return ZK_ERR_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZK_ERR_NO_DEVICE;
    zk_ctx* c = new zk_ctx();
    c->device = cfg->device;
    c->S = cfg->num_services;
    c->strict = cfg->strict != 0;
    c->timing = cfg->timing != 0;
    c->group_join = cfg->trace_pass == 0;
    c->cus = prop.multiProcessorCount > 0 ? (uint32_t)prop.multiProcessorCount : 256;
    bucket_geometry(c->S, &c->nb, &c->cb_shift);
    if (cfg->max_trace_records) c->max_trace = cfg->max_trace_records;
    zk_status st = ZK_OK;
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) {
        if (cfg->stream) {
            c->stream = (hipStream_t)cfg->stream;
        } else {
            e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
            c->own_stream = true;
        }
    }
    if (cfg->table) {
        if (cfg->table_bytes < table_bytes(c->S)) {
            zk_ctx_destroy(c);
            return ZK_ERR_INVALID_ARG;
        }
        c->table = (uint64_t*)cfg->table;
        c->own_table = false;
    } else if (e == hipSuccess) {
        e = hipMalloc(&c->table, table_bytes(c->S));
    }
    if (e == hipSuccess) e = hipMalloc(&c->stats, (size_t)kStatShards * ST_N * 8);
    if (e == hipSuccess) e = hipMalloc(&c->spill_count, 256);
    if (e != hipSuccess) st = ZK_ERR_HIP;
    if (st == ZK_OK) st = zk_deps_reset(c);
    if (st == ZK_OK) st = ensure_spill(c, 1);
    if (st != ZK_OK) {
        zk_ctx_destroy(c);
        return st;
    }
    *out = c;
    return ZK_OK;
    ZK_CATCH(nullptr)
}

zk_status zk_ctx_destroy(zk_ctx* c) {
    if (!c) return ZK_ERR_INVALID_ARG;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->rt) rt_set_stream(c->rt, nullptr);
    if (c->rl) rl_set_stream(c->rl, nullptr);
    if (c->own_table) hipFree(c->table);
    c->table = nullptr;
    hipFree(c->stats);
    if (c->h_stats) hipHostFree(c->h_stats);
    if (c->ev_stats) hipEventDestroy(c->ev_stats);
    if (c->ev_stage) hipEventDestroy(c->ev_stage);
    hipFree(c->spill_count);
    hipFree(c->spill_list);
    hipFree(c->spill_scratch);
    hipFree(c->links);
    hipFree(c->link_count);
    hipFree(c->hist);
    hipFree(c->col_off);
    hipFree(c->bucket_base);
    hipFree(c->sorted);
    hipFree(c->stage);
    hipFree(c->fin_stage);
    hipFree(c->cl_cols);
    hipFree(c->cl_temp);
    hipFree(c->tset);
    hipFree(c->xchg);
    hipFree(c->carry);
    hipFree(c->cs);
    for (auto* v : {&c->ev_free, &c->ev_join, &c->ev_reduce, &c->ev_spill, &c->ev_fin, &c->ev_cluster})
        for (auto& p : *v) {
            hipEventDestroy(p.a);
            hipEventDestroy(p.b);
        }
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    return ZK_OK;
}

zk_status zk_ctx_sync(zk_ctx* c) {
    if (!c) return ZK_ERR_INVALID_ARG;
    ZK_HIP(c, hipSetDevice(c->device));
    ZK_HIP(c, hipStreamSynchronize(c->stream));
    return ZK_OK;
}

// the device-side continuation's batch range for K1 (zk_cluster.h CarryState)
struct DevRange {
    const uint32_t* skip_dev;
    const unsigned long long* n_dev;
};
static zk_status accumulate_dev(zk_ctx* c, SpanColsDev d, uint32_t flags, uint32_t skip,
                                const DevRange* dr = nullptr);
static zk_status continue_batch(zk_ctx* c, const SpanColsDev& d, uint32_t flags);
static zk_status flush_carry(zk_ctx* c);

// the carry state of a fresh job: nothing held
static zk_status carry_state_reset(zk_ctx* c) {
    ZK_HIP(c, hipMemsetAsync(c->cs, 0, sizeof(CarryState), c->stream));
    return ZK_OK;
}

static zk_status ensure_carry(zk_ctx* c) {
    if (!c->carry) {
        c->carry_cap = (uint64_t)c->max_trace + 2;  // a held run has <= max_trace + 1 records
        ZK_HIP(c, hipMalloc(&c->carry, carved_bytes(c->carry_cap)));
    }
    if (!c->cs) {
        ZK_HIP(c, hipMalloc(&c->cs, sizeof(CarryState)));
        ZK_ST(carry_state_reset(c));
    }
    return ZK_OK;
}

zk_status zk_deps_reset(zk_ctx* c) {
    if (!c) return ZK_ERR_INVALID_ARG;
    ZK_HIP(c, hipSetDevice(c->device));
    ZK_HIP(c, hipMemsetAsync(c->table, 0, table_bytes(c->S), c->stream));
    ZK_HIP(c, hipMemsetAsync(c->stats, 0, (size_t)kStatShards * ST_N * 8, c->stream));
    if (c->tset && c->tset_records) ZK_HIP(c, hipMemsetAsync(c->tset, 0, (c->tset_slots + 1) * 8, c->stream));
    c->tset_records = 0;
    c->records_since_reset = 0;
    c->merged = false;
    c->continued = false;
    c->folded = false;
    c->aborted = false;
    // a held-back trace belongs to the job being reset
    c->maybe_carry = false;
    c->any_verify = false;
    if (c->cs) ZK_ST(carry_state_reset(c));
    return ZK_OK;
}


zk_status zk_deps_accumulate(zk_ctx* c, const zk_span_cols* cols, uint32_t flags) {
    if (!c) return ZK_ERR_INVALID_ARG;
    ZK_TRY
    RoctxRange rr("zk_deps_accumulate");
    if (!cols) return fail(c, ZK_ERR_INVALID_ARG, "null columns");
    if (flags & ~(ZK_BATCH_DEVICE_PTRS | ZK_BATCH_TRACE_CLUSTERED | ZK_BATCH_VERIFY_TRACES | ZK_BATCH_CONTINUES))
        return fail(c, ZK_ERR_INVALID_ARG, "unknown batch flag");
    if ((flags & ZK_BATCH_CONTINUES) && !(flags & ZK_BATCH_TRACE_CLUSTERED))
        return fail(c, ZK_ERR_INVALID_ARG, "ZK_BATCH_CONTINUES needs a trace-clustered batch (ZK_BATCH_TRACE_CLUSTERED)");
    const uint64_t n = cols->n;
    if (n == 0) {
        if (!(flags & ZK_BATCH_CONTINUES)) return flush_carry(c);
        return ZK_OK;
    }
    if (!cols_ok(cols)) return fail(c, ZK_ERR_INVALID_ARG, "null column pointer");
    const bool join = !c->rt || c->rt_mode == ZK_RT_WITH_DEPS;
    if (join && c->records_since_reset + n > kMaxRecordsSinceReset)  // (held records counted with their batch)
        return fail(c, ZK_ERR_CAPACITY, "more than 2^32-1 records since reset");
    ZK_HIP(c, hipSetDevice(c->device));
    if (c->merged) {
        // accumulating into a merged table: the table holds the whole job, so the ctx's own counters
        // restart from the merged (job-wide) ones in the tail -- shard 0 takes the tail, the other
        // shards are zeroed -- and finalize then reports the job plus this batch
        ZK_HIP(c, hipMemsetAsync(c->stats, 0, (size_t)kStatShards * ST_N * 8, c->stream));
        ZK_HIP(c, hipMemcpyAsync(c->stats, c->table + (uint64_t)c->S * c->S * kLimbs, kTableTailBytes,
                                 hipMemcpyDeviceToDevice, c->stream));
        c->merged = false;
        c->continued = true;
    }
    c->folded = false;  // the tail no longer holds this ctx's counters once the batch lands
    SpanColsDev d{cols->trace_id, cols->span_id, cols->parent_id, cols->first_ts,
                  cols->last_ts,  cols->service_id, cols->flags,   n};
    if (!(flags & ZK_BATCH_DEVICE_PTRS)) {
        // PCIe path: stage the host columns in HBM (reported separately, never the bench value)
        if (n > c->stage_cap) {
            if (c->stage) ZK_HIP(c, hipFree(c->stage));
            ZK_HIP(c, hipMalloc(&c->stage, n * 48 + 7 * 256));
            c->stage_cap = n;
        }
        uint8_t* p = (uint8_t*)c->stage;
        // every staged column starts on a 256-byte boundary (K1 uses 16-byte pair loads)
        auto carve = [&](uint64_t bytes) {
            uint8_t* q = p;
            p += (bytes + 255) & ~255ull;
            return q;
        };
        uint64_t* tid = (uint64_t*)carve(n * 8);
        uint64_t* sid = (uint64_t*)carve(n * 8);
        uint64_t* pid = (uint64_t*)carve(n * 8);
        int64_t* fts = (int64_t*)carve(n * 8);
        int64_t* lts = (int64_t*)carve(n * 8);
        uint32_t* svc = (uint32_t*)carve(n * 4);
        uint32_t* flg = (uint32_t*)carve(n * 4);
        ZK_HIP(c, hipMemcpyAsync(tid, cols->trace_id, n * 8, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipMemcpyAsync(sid, cols->span_id, n * 8, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipMemcpyAsync(pid, cols->parent_id, n * 8, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipMemcpyAsync(fts, cols->first_ts, n * 8, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipMemcpyAsync(lts, cols->last_ts, n * 8, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipMemcpyAsync(svc, cols->service_id, n * 4, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipMemcpyAsync(flg, cols->flags, n * 4, hipMemcpyHostToDevice, c->stream));
        // host columns are borrowed for the duration of the call only (zkagg.h): from page-locked
        // memory the copies above are DMA reads that run after this call would return, so the call
        // waits until they have consumed the caller's buffers (queued behind the stream's earlier
        // work; the PCIe path, never the bench value)
        if (!c->ev_stage) ZK_HIP(c, hipEventCreateWithFlags(&c->ev_stage, hipEventDisableTiming));
        ZK_HIP(c, hipEventRecord(c->ev_stage, c->stream));
        ZK_HIP(c, hipEventSynchronize(c->ev_stage));
        d = SpanColsDev{tid, sid, pid, fts, lts, svc, flg, n};
    } else if ((flags & ZK_BATCH_TRACE_CLUSTERED) &&
               (!aligned(d.trace_id, 16) || !aligned(d.span_id, 16) || !aligned(d.parent_id, 16) ||
                !aligned(d.first_ts, 16) || !aligned(d.last_ts, 16) || !aligned(d.service_id, 8) ||
                !aligned(d.flags, 8))) {
        // K1 reads two records per lane with one 16-byte (u64 columns) / 8-byte (u32) load
        return fail(c, ZK_ERR_INVALID_ARG, "device columns must be 16-byte (u64) / 8-byte (u32) aligned");
    }
    if (!(flags & ZK_BATCH_TRACE_CLUSTERED)) {
        // a batch in any order ends a held trace (zkagg.h): the held trace is aggregated as it is, the
        // batch as a whole (its first run is not the held trace's continuation)
        ZK_ST(flush_carry(c));
        return accumulate_dev(c, d, flags, 0);
    }
    if (c->maybe_carry || (flags & ZK_BATCH_CONTINUES)) return continue_batch(c, d, flags);
    return accumulate_dev(c, d, flags, 0);
    ZK_CATCH(c)
}

// the join kernels' common arguments for n records of d
static JoinArgs join_args(zk_ctx* c, const SpanColsDev& d) {
    JoinArgs a{};
    a.c = d;
    a.table = c->table;
    a.stats = c->stats;
    a.S = c->S;
    a.spill_count = c->spill_count;
    a.spill_list = c->spill_list;
    a.spill_cap = c->spill_cap;
    a.spill_scratch = c->spill_scratch;
    a.spill_scratch_stride = c->spill_stride;
    a.max_trace = c->max_trace;
    a.links = c->links;
    a.link_count = c->link_count;
    a.hist = c->hist;
    a.nb = c->nb;
    a.cb_shift = c->cb_shift;
    a.join = 1u;
    return a;
}

static zk_status reduce_links(zk_ctx* c, uint32_t grid, uint64_t stride) {
    if (c->nb) {
        ReduceArgs r{};
        r.links = c->links;
        r.counts = c->link_count;
        r.stride = stride;
        r.lists = grid;
        r.hist = c->hist;
        r.nb = c->nb;
        r.cb_shift = c->cb_shift;
        r.col_off = c->col_off;
        r.bucket_base = c->bucket_base;
        r.sorted = c->sorted;
        r.table = c->table;
        r.cells = (uint64_t)c->S * c->S;
        ZK_HIP(c, launch_partitioned_reduce(r, c->stream));
    } else {
        ZK_HIP(c, launch_link_reduce(c->links, c->link_count, stride, grid, c->table, c->stream));
    }
    return ZK_OK;
}

// An unclustered batch through the group join: the clustering pass's partition (P0-P2) leaves every
// trace inside one sub-bucket; k_group_join joins the sub-buckets in LDS, keyed by traceId. The
// sub-buckets too long for it go through P3 (list mode) into the other column set, clustered, and K1
// appends their links to the same lists; then K2/K3 and the spill kernel as for a clustered batch.
static zk_status accumulate_groups(zk_ctx* c, const SpanColsDev& d, const ClusterPlan& plan) {
    RoctxRange rr("zk_group_batch");
    const uint64_t n = d.n;
    ZK_ST(ensure_cluster(c, n, plan));
    const SpanColsMut A = carve_cols(c->cl_cols, n);
    const SpanColsMut B = carve_cols(c->cl_cols + carved_bytes(n), n);
    EventPair ec, ej, er, es;
    if (c->timing) {
        ec = take_pair(c);
        ZK_HIP(c, hipEventRecord(ec.a, c->stream));
    }
    ClusterGroups g{};
    int res = 0;
    ZK_HIP(c, launch_cluster(plan, d, A, B, c->cl_temp, c->cus, c->stream, &res, c->stats + ST_SPILL_OVERFLOW, &g));
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(ec.b, c->stream));
        c->ev_cluster.push_back(ec);
    }
    uint32_t grid = 0;
    uint64_t per = 0, stride = 0;
    group_join_geometry(n, c->cus, &grid, &per, &stride);
    ZK_ST(ensure_spill(c, n));
    ZK_ST(ensure_links(c, grid, stride, n));
    ZK_HIP(c, hipMemsetAsync(c->spill_count, 0, 4, c->stream));
    const SpanColsDev bd{B.trace_id, B.span_id, B.parent_id, B.first_ts, B.last_ts, B.service_id, B.flags, n};
    const SpanColsDev ad{A.trace_id, A.span_id, A.parent_id, A.first_ts, A.last_ts, A.service_id, A.flags, n};
    JoinArgs a = join_args(c, bd);
    a.grid = grid;
    a.per_wg = per;
    a.link_stride = stride;
    a.sub = g.sub;
    a.nsub = g.nsub;
    a.big_list = g.big_list;
    a.big_count = g.big_count;
    if (c->timing) {
        ej = take_pair(c);
        ZK_HIP(c, hipEventRecord(ej.a, c->stream));
    }
    ZK_HIP(c, launch_group_join(a, c->stream));
    ZK_HIP(c, launch_cluster_fallback(plan, g, bd, A, c->cl_temp, c->cus, c->stream, c->stats + ST_SPILL_OVERFLOW));
    JoinArgs f = join_args(c, ad);  // K1 over the fallback's clustered records A[0, *out_cursor)
    f.grid = grid;
    f.per_wg = (per + join_tile_records() - 1) / join_tile_records() * join_tile_records();
    f.link_stride = stride;
    f.n_dev = g.out_cursor;
    f.append = 1u;
    ZK_HIP(c, launch_join(f, c->stream));
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(ej.b, c->stream));
        c->ev_join.push_back(ej);
        er = take_pair(c);
        ZK_HIP(c, hipEventRecord(er.a, c->stream));
    }
    ZK_ST(reduce_links(c, grid, stride));
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(er.b, c->stream));
        c->ev_reduce.push_back(er);
        es = take_pair(c);
        ZK_HIP(c, hipEventRecord(es.a, c->stream));
    }
    ZK_HIP(c, launch_spill(f, c->spill_wgs, c->stream));
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(es.b, c->stream));
        c->ev_spill.push_back(es);
    }
    c->records_since_reset += n;
    return ZK_OK;
}

// One batch already in HBM. skip (0 or 1): the first record belongs to a run handled elsewhere (it
// only keeps the column pointers 16-byte aligned); K1 starts at the trace after it.
static JoinArgs carry_join_args(zk_ctx* c, const JoinArgs* like);

// dr: K1's skip and record count on the device (a batch under ZK_BATCH_CONTINUES); the carry's join
// then follows the batch's spill pass, into the same realtime lists
static zk_status accumulate_dev(zk_ctx* c, SpanColsDev d, uint32_t flags, uint32_t skip, const DevRange* dr) {
    const uint64_t n = d.n;
    if (n <= skip) return ZK_OK;
    const bool join = !c->rt || c->rt_mode == ZK_RT_WITH_DEPS;
    // unclustered, without the trace check or a realtime sketch: the group join (two-level plans)
    // (only when max_trace_records >= the group join's tile: it aggregates every trace of a sub-bucket
    // it holds, so a smaller bound could not be enforced there as K1 enforces it)
    if (!(flags & ZK_BATCH_TRACE_CLUSTERED) && !(flags & ZK_BATCH_VERIFY_TRACES) && !c->rt && !c->rl && c->group_join &&
        c->max_trace >= group_join_capacity() && n <= 0xFFFFFFFFull) {
        const ClusterPlan gp = cluster_plan(n, c->cus, true);
        if (gp.b1 && gp.b2) return accumulate_groups(c, d, gp);
    }
    if (!(flags & ZK_BATCH_TRACE_CLUSTERED)) {
        EventPair ec;
        if (c->timing) {
            ec = take_pair(c);
            ZK_HIP(c, hipEventRecord(ec.a, c->stream));
        }
        const zk_status cs = cluster_batch(c, &d);
        if (cs != ZK_OK) {
            if (c->timing) c->ev_free.push_back(ec);
            return cs;
        }
        if (c->timing) {
            ZK_HIP(c, hipEventRecord(ec.b, c->stream));
            c->ev_cluster.push_back(ec);
        }
    }
    if (flags & ZK_BATCH_VERIFY_TRACES) {
        SpanColsDev v = d;  // (the skipped record's run is verified where it is handled)
        v.trace_id += skip;
        v.n -= skip;
        const zk_status vs = verify_batch(c, v);
        if (vs != ZK_OK) return vs;
    }
        uint32_t grid = 0;
    uint64_t per_wg = 0, stride = 0;
    join_geometry(n, c->cus, &grid, &per_wg, &stride);
    if (dr) stride += join_tile_records();  // list 0 also takes the held trace's links (K1, one workgroup)
    zk_status st = ensure_spill(c, n);
    if (st == ZK_OK) st = ensure_links(c, grid, stride, n);
    if (st != ZK_OK) return st;
    if (!dr) ZK_HIP(c, hipMemsetAsync(c->spill_count, 0, 4, c->stream));  // (else k_carry_plan zeroed it)
    JoinArgs a{};
    a.c = d;
    a.table = c->table;
    a.stats = c->stats;
    a.S = c->S;
    a.spill_count = c->spill_count;
    a.spill_list = c->spill_list;
    a.spill_cap = c->spill_cap;
    a.spill_scratch = c->spill_scratch;
    a.spill_scratch_stride = c->spill_stride;
    a.max_trace = c->max_trace;
    a.links = c->links;
    a.link_count = c->link_count;
    a.link_stride = stride;
    a.per_wg = per_wg;
    a.grid = grid;
    a.hist = c->hist;
    a.nb = c->nb;
    a.cb_shift = c->cb_shift;
    a.join = join ? 1u : 0u;
    a.skip = skip;
    if (dr) {
        a.skip_dev = dr->skip_dev;
        a.n_dev = dr->n_dev;
    }
    if (c->rt) {
        // (the spill list also takes the carry's items under dr)
        st = rt_prepare_lists(c->rt, grid, stride, n + (dr ? c->carry_cap : 0), &a, c->stream);
        if (st != ZK_OK) return fail(c, st, std::string("sketch: ") + rt_error(c->rt));
    }
    if (c->rl && join) {  // realtime link items beside the links (the spill list also takes the carry's)
        st = rl_prepare_lists(c->rl, grid, stride, n + (dr ? c->carry_cap : 0), &a, c->stream);
        if (st != ZK_OK) return fail(c, st, std::string("realtime links: ") + rl_error(c->rl));
    }
    EventPair ej, er, es;
    if (c->timing) {
        ej = take_pair(c);
        ZK_HIP(c, hipEventRecord(ej.a, c->stream));
    }
    ZK_HIP(c, launch_join(a, c->stream));
    JoinArgs f{};
    if (dr) {
        // the held trace joined now (k_carry_plan: flush_n records of the carry, 0: none): by K1 on
        // one workgroup appending to list 0 (its spill list of one entry takes it when it outgrows a
        // window), or with a realtime sketch bound, whose item lists K1 cannot append to, by the spill
        // kernel alone
        f = carry_join_args(c, &a);
        if (!c->rt) ZK_HIP(c, launch_join(f, c->stream, 1));
    }
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(ej.b, c->stream));
        c->ev_join.push_back(ej);
        er = take_pair(c);
        ZK_HIP(c, hipEventRecord(er.a, c->stream));
    }
    if (!join) {
        // sketch-only pass: no links to reduce
    } else if (c->nb) {
        ReduceArgs r{};
        r.links = c->links;
        r.counts = c->link_count;
        r.stride = stride;
        r.lists = grid;
        r.hist = c->hist;
        r.nb = c->nb;
        r.cb_shift = c->cb_shift;
        r.col_off = c->col_off;
        r.bucket_base = c->bucket_base;
        r.sorted = c->sorted;
        r.table = c->table;
        r.cells = (uint64_t)c->S * c->S;
        ZK_HIP(c, launch_partitioned_reduce(r, c->stream));
    } else {
        ZK_HIP(c, launch_link_reduce(c->links, c->link_count, stride, grid, c->table, c->stream));
    }
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(er.b, c->stream));
        c->ev_reduce.push_back(er);
        es = take_pair(c);
        ZK_HIP(c, hipEventRecord(es.a, c->stream));
    }
    ZK_HIP(c, launch_spill(a, c->spill_wgs, c->stream));
    if (dr) ZK_HIP(c, launch_spill(f, 1, c->stream));
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(es.b, c->stream));
        c->ev_spill.push_back(es);
    }
    if (c->rt) {
        st = rt_consume_lists(c->rt, grid, stride, n + (dr ? c->carry_cap : 0));
        if (st != ZK_OK) return fail(c, st, std::string("sketch: ") + rt_error(c->rt));
    }
    if (c->rl && join) {
        st = rl_consume_lists(c->rl, c->link_count, grid, stride, n + (dr ? c->carry_cap : 0));
        if (st != ZK_OK) return fail(c, st, std::string("realtime links: ") + rl_error(c->rl));
    }
    if (join) c->records_since_reset += n - skip;
    return ZK_OK;
}

// The carry's join: one trace of flush_n records of the carry columns, its spill list the one entry
// cs->zero = record 0 of length cs->flush_cnt. `like`: the batch's join arguments, whose geometry,
// link lists (K1 appends to list 0) and realtime lists it shares (nullptr: a flush alone, by the
// spill kernel).
static JoinArgs carry_join_args(zk_ctx* c, const JoinArgs* like) {
    const SpanColsMut m = carve_cols(c->carry, c->carry_cap);
    const SpanColsDev cd{m.trace_id, m.span_id, m.parent_id, m.first_ts, m.last_ts, m.service_id, m.flags,
                         c->carry_cap};
    JoinArgs f = like ? *like : join_args(c, cd);
    f.c = cd;
    f.spill_count = &c->cs->flush_cnt;
    f.spill_list = (uint64_t*)&c->cs->zero;
    f.spill_cap = 1;
    f.n_dev = &c->cs->flush_n;
    f.skip_dev = nullptr;
    f.skip = 0;
    f.append = 1;
    f.join = (!c->rt || c->rt_mode == ZK_RT_WITH_DEPS) ? 1u : 0u;
    return f;
}

// A clustered batch while a trace may be held, or whose last trace may continue: everything is
// decided on the device (k_carry_plan), so nothing waits for the host. The batch's leading run joins
// the held trace when it carries the same traceId; the held trace is joined (the spill kernel) once
// the batch moves on to another trace (or does not continue); with ZK_BATCH_CONTINUES the batch's
// last run becomes the new carry. K1 takes the rest of the batch: records below hi, from the first
// trace boundary after record 0 when record 0's run is the held trace's.
static zk_status continue_batch(zk_ctx* c, const SpanColsDev& d, uint32_t flags) {
    RoctxRange rr("zk_continue_batch");
    ZK_ST(ensure_carry(c));
    const uint64_t n = d.n;
    const uint32_t cont = (flags & ZK_BATCH_CONTINUES) ? 1u : 0u;
    const uint32_t ver = (flags & ZK_BATCH_VERIFY_TRACES) ? 1u : 0u;
    if (ver) c->any_verify = true;
    // (the held trace's records were counted with their batch; its run is checked when it is joined)
    if (c->any_verify) ZK_ST(ensure_tset(c, n));
    const SpanColsMut m = carve_cols(c->carry, c->carry_cap);
    ZK_HIP(c, launch_carry_plan(c->cs, d, m, c->max_trace, cont, ver, c->rt ? 0u : 1u, c->stats + ST_TOO_LARGE,
                                c->spill_count, c->any_verify ? c->tset : nullptr, c->tset_slots,
                                &c->stats[ST_NOT_CLUSTERED], c->stream));
    if (ver)  // the batch's runs below hi (not record 0's when that is the held trace's)
        ZK_HIP(c, launch_trace_set_insert(d.trace_id, n, c->tset, c->tset_slots, &c->stats[ST_NOT_CLUSTERED],
                                          c->stream, &c->cs->hi, &c->cs->skip));
    const DevRange dr{&c->cs->skip, &c->cs->hi};
    zk_status st = accumulate_dev(c, d, flags & ~(ZK_BATCH_CONTINUES | ZK_BATCH_VERIFY_TRACES), 0, &dr);
    if (st == ZK_OK) {
        const hipError_t e = launch_carry_tail(c->cs, d, m, c->stream);  // (after the carry's join read the old one)
        if (e != hipSuccess) st = hip_fail(c, e, "launch_carry_tail");
    }
    if (st != ZK_OK) {
        // the plan already moved the held-trace state past this batch: drop the held trace rather than
        // join a carry whose copy never ran (the batch failed; reset before reusing the job)
        c->maybe_carry = false;
        (void)hipMemsetAsync(c->cs, 0, sizeof(CarryState), c->stream);
        return st;
    }
    c->maybe_carry = cont != 0;
    return ZK_OK;
}

// the held-back trace is complete: join it as a trace of its own
static zk_status flush_carry(zk_ctx* c) {
    if (!c->maybe_carry) return ZK_OK;
    c->maybe_carry = false;
    if (c->any_verify) ZK_ST(ensure_tset(c, 0));
    const SpanColsMut m = carve_cols(c->carry, c->carry_cap);
    ZK_HIP(c, launch_carry_plan(c->cs, SpanColsDev{}, m, c->max_trace, 0, 0, 0, c->stats + ST_TOO_LARGE, nullptr,
                                c->any_verify ? c->tset : nullptr, c->tset_slots, &c->stats[ST_NOT_CLUSTERED],
                                c->stream));
    JoinArgs f = carry_join_args(c, nullptr);
    if (c->rt) {  // its sketch items: one list (list 0 of a zero-width list set)
        f.grid = 0;
        f.link_stride = 0;
        const zk_status st = rt_prepare_lists(c->rt, 0, 0, c->carry_cap, &f, c->stream);
        if (st != ZK_OK) return fail(c, st, std::string("sketch: ") + rt_error(c->rt));
    }
    const bool links = c->rl && f.join;
    if (links) {  // its link items: the spill list of a zero-width list set
        f.grid = 0;
        f.link_stride = 0;
        const zk_status st = rl_prepare_lists(c->rl, 0, 0, c->carry_cap, &f, c->stream);
        if (st != ZK_OK) return fail(c, st, std::string("realtime links: ") + rl_error(c->rl));
    }
    ZK_HIP(c, launch_spill(f, 1, c->stream));
    if (c->rt) {
        const zk_status st = rt_consume_lists(c->rt, 0, 0, c->carry_cap);
        if (st != ZK_OK) return fail(c, st, std::string("sketch: ") + rt_error(c->rt));
    }
    if (links) {
        const zk_status st = rl_consume_lists(c->rl, c->link_count, 0, 0, c->carry_cap);
        if (st != ZK_OK) return fail(c, st, std::string("realtime links: ") + rl_error(c->rl));
    }
    return ZK_OK;
}

zk_status zk_deps_finalize(zk_ctx* c, const zk_link_table* out) {
    if (!c) return ZK_ERR_INVALID_ARG;
    ZK_TRY
    RoctxRange rr("zk_deps_finalize");
    if (!out || !out->m0 || !out->m1 || !out->m2 || !out->m3 || !out->m4 || !out->present)
        return fail(c, ZK_ERR_INVALID_ARG, "null output array");
    ZK_HIP(c, hipSetDevice(c->device));
    ZK_ST(flush_carry(c));  // the job ends here: a held-back trace is complete
    const uint64_t cells = (uint64_t)c->S * c->S;
    zk_link_table dev = *out;
    if (!out->device_ptrs) {
        if (!c->fin_stage) ZK_HIP(c, hipMalloc(&c->fin_stage, cells * 41 + 64));
        uint8_t* p = (uint8_t*)c->fin_stage;
        dev.m0 = (uint64_t*)p;
        dev.m1 = (double*)(p + cells * 8);
        dev.m2 = (double*)(p + cells * 16);
        dev.m3 = (double*)(p + cells * 24);
        dev.m4 = (double*)(p + cells * 32);
        dev.present = p + cells * 40;
    }
    EventPair ef;
    if (c->timing) {
        ef = take_pair(c);
        ZK_HIP(c, hipEventRecord(ef.a, c->stream));
    }
    ZK_HIP(c, launch_finalize(c->table, c->S, &dev, c->stream));
    if (c->timing) {
        ZK_HIP(c, hipEventRecord(ef.b, c->stream));
        c->ev_fin.push_back(ef);
    }
    const uint8_t* h0 = (const uint8_t*)out->m0;
    const bool one_block = !out->device_ptrs && (const uint8_t*)out->m1 == h0 + cells * 8 &&
                           (const uint8_t*)out->m2 == h0 + cells * 16 && (const uint8_t*)out->m3 == h0 + cells * 24 &&
                           (const uint8_t*)out->m4 == h0 + cells * 32 && (const uint8_t*)out->present == h0 + cells * 40;
    if (one_block) {  // the caller's arrays are laid out like the staging block: one copy
        ZK_HIP(c, hipMemcpyAsync(out->m0, dev.m0, cells * 41, hipMemcpyDeviceToHost, c->stream));
    } else if (!out->device_ptrs) {
        ZK_HIP(c, hipMemcpyAsync(out->m0, dev.m0, cells * 8, hipMemcpyDeviceToHost, c->stream));
        ZK_HIP(c, hipMemcpyAsync(out->m1, dev.m1, cells * 8, hipMemcpyDeviceToHost, c->stream));
        ZK_HIP(c, hipMemcpyAsync(out->m2, dev.m2, cells * 8, hipMemcpyDeviceToHost, c->stream));
        ZK_HIP(c, hipMemcpyAsync(out->m3, dev.m3, cells * 8, hipMemcpyDeviceToHost, c->stream));
        ZK_HIP(c, hipMemcpyAsync(out->m4, dev.m4, cells * 8, hipMemcpyDeviceToHost, c->stream));
        ZK_HIP(c, hipMemcpyAsync(out->present, dev.present, cells, hipMemcpyDeviceToHost, c->stream));
    }
    uint64_t s[ST_N], aborted = 0;
    zk_status st = stats_sum(c, s, &aborted);
    if (st != ZK_OK) return st;
    if (aborted)
        return fail(c, ZK_ERR_RANK_FAILED,
                    std::to_string(aborted) + " rank(s) of the job failed before the exchange (zk_deps_abort)");
    if (s[ST_TOO_LARGE]) return fail(c, ZK_ERR_TRACE_TOO_LARGE, "trace longer than max_trace_records skipped");
    if (s[ST_SPILL_OVERFLOW])
        return fail(c, ZK_ERR_CAPACITY,
                    "device capacity exceeded: spill list overflow, or a clustering sub-bucket whose traceIds "
                    "collide in every hash bit the trace pass splits on");
    if (s[ST_NOT_CLUSTERED])
        return fail(c, ZK_ERR_NOT_CLUSTERED, "a trace was split into non-adjacent runs or over two batches");
    if (s[ST_SVC_RANGE]) return fail(c, ZK_ERR_SERVICE_RANGE, "record with service_id >= num_services");
    if (s[ST_DUR_RANGE]) return fail(c, ZK_ERR_DURATION_RANGE, "link with duration >= 2^40 us dropped");
    if (c->strict && s[ST_NO_SERVICE])
        return fail(c, ZK_ERR_NO_SERVICE, "joined span without a service name (reference: None.get)");
    return ZK_OK;
    ZK_CATCH(c)
}

zk_status zk_ctx_stats(zk_ctx* c, zk_stats* out) {
    if (!c || !out) return ZK_ERR_INVALID_ARG;
    ZK_HIP(c, hipSetDevice(c->device));
    uint64_t s[ST_N];
    zk_status st = stats_sum(c, s);
    if (st != ZK_OK) return st;
    memset(out, 0, sizeof(*out));
    uint64_t* o = &out->records;
    for (int i = 0; i < ST_TOO_LARGE + 1; ++i) o[i] = s[i];
    out->not_clustered = s[ST_NOT_CLUSTERED];
    return ZK_OK;
}

zk_status zk_ctx_timing(zk_ctx* c, zk_timing* out) {
    if (!c || !out) return ZK_ERR_INVALID_ARG;
    ZK_TRY
    ZK_HIP(c, hipSetDevice(c->device));
    ZK_HIP(c, hipStreamSynchronize(c->stream));
    auto drain = [&](std::vector<EventPair>& v, double* last, double* total, uint64_t* calls) {
        for (auto& p : v) {
            float ms = 0;
            hipEventElapsedTime(&ms, p.a, p.b);
            *last = ms;
            if (total) *total += ms;
            if (calls) ++*calls;
            c->ev_free.push_back(p);
        }
        v.clear();
    };
    drain(c->ev_join, &c->tm.join_ms, &c->tm.join_ms_total, &c->tm.join_calls);
    drain(c->ev_reduce, &c->tm.reduce_ms, &c->tm.reduce_ms_total, nullptr);
    drain(c->ev_spill, &c->tm.spill_ms, nullptr, nullptr);
    drain(c->ev_fin, &c->tm.finalize_ms, nullptr, nullptr);
    drain(c->ev_cluster, &c->tm.cluster_ms, &c->tm.cluster_ms_total, nullptr);
    *out = c->tm;
    return ZK_OK;
    ZK_CATCH(c)
}

zk_status zk_deps_partial(zk_ctx* c, void** dev_ptr, uint64_t* bytes) {
    if (!c || !dev_ptr || !bytes) return ZK_ERR_INVALID_ARG;
    // a ctx that continued a merged job holds the whole job: a second exchange would add it once per rank
    if (c->continued)
        return fail(c, ZK_ERR_INVALID_ARG, "zk_deps_partial after accumulating into a merged table (reset first)");
    ZK_HIP(c, hipSetDevice(c->device));
    ZK_ST(flush_carry(c));  // the shard's part of the job ends here
    if (!c->merged)  // a merged tail already holds the job-wide counters
        ZK_HIP(c, launch_stats_fold(c->stats, (unsigned long long*)(c->table + (uint64_t)c->S * c->S * kLimbs),
                                    c->stream));
    if (!c->xchg && hipMalloc(&c->xchg, exchange_bytes(c->S)) != hipSuccess) {
        (void)hipGetLastError();
        c->xchg = nullptr;
        return fail(c, ZK_ERR_CAPACITY, "no device memory for the exchange buffer");
    }
    ZK_HIP(c, launch_table_pack(c->table, c->S, c->xchg, c->stream));  // 56-bit limbs + the counter tail
    if (c->aborted) {
        // a failed rank contributes nothing but its abort mark (the exchange still happens, so the
        // other ranks are not left waiting in the collective)
        static const uint64_t mark = kAbortUnit;
        ZK_HIP(c, hipMemsetAsync(c->xchg, 0, exchange_bytes(c->S), c->stream));
        ZK_HIP(c, hipMemcpyAsync((uint8_t*)c->xchg + exchange_bytes(c->S) - kTableTailBytes + ST_RECORDS * 8, &mark,
                                 8, hipMemcpyHostToDevice, c->stream));
        ZK_HIP(c, hipStreamSynchronize(c->stream));  // (`mark` is pageable: nothing reads it later)
    }
    c->folded = true;
    *dev_ptr = c->xchg;
    *bytes = exchange_bytes(c->S);
    return ZK_OK;
}

zk_status zk_deps_note_merged(zk_ctx* c, uint64_t total_records) {
    if (!c) return ZK_ERR_INVALID_ARG;
    // the tail is only meaningful after zk_deps_partial folded this ctx's counters into it (an
    // all-reduce of a stale or zeroed tail would silently drop every error counter on every rank)
    if (!c->folded)
        return fail(c, ZK_ERR_INVALID_ARG, "zk_deps_note_merged without zk_deps_partial since the last reset/accumulate");
    ZK_HIP(c, hipSetDevice(c->device));
    // the all-reduced exchange buffer back into the accumulator's own layout (exact sums, counters)
    ZK_HIP(c, launch_table_unpack(c->xchg, c->S, c->table, c->stream));
    if (total_records == 0) {  // take it from the all-reduced counter tail
        unsigned long long rec = 0;
        ZK_HIP(c, hipMemcpyAsync(&rec, c->table + (uint64_t)c->S * c->S * kLimbs + ST_RECORDS, 8,
                                 hipMemcpyDeviceToHost, c->stream));
        ZK_HIP(c, hipStreamSynchronize(c->stream));
        total_records = rec & (kAbortUnit - 1);  // (abort marks excluded)
    }
    if (total_records > kMaxRecordsSinceReset)
        return fail(c, ZK_ERR_CAPACITY, "merged table exceeds 2^32-1 records");
    c->records_since_reset = total_records;
    c->merged = true;
    return ZK_OK;
}

zk_status zk_deps_abort(zk_ctx* c) {
    if (!c) return ZK_ERR_INVALID_ARG;
    c->aborted = true;
    return ZK_OK;
}

zk_status zk_deps_allreduce(zk_ctx* c, zk_comm* comm, uint64_t total_records) {
    if (!c) return ZK_ERR_INVALID_ARG;
    if (!comm) return fail(c, ZK_ERR_INVALID_ARG, "null communicator");
    ZK_TRY
    RoctxRange rr("zk_deps_allreduce");
    void* x = nullptr;
    uint64_t bytes = 0;
    ZK_ST(zk_deps_partial(c, &x, &bytes));  // counters folded, table packed (ctx stream)
    // ONE int64 SUM over every rank's exchange buffer, ordered after the pack on the ctx stream
    ZK_ST(comm_allreduce(comm, x, bytes / 8, kCommI64, kCommSum, c->device, c->stream, &c->err));
    return zk_deps_note_merged(c, total_records);
    ZK_CATCH(c)
}

zk_status zk_rl_bind(zk_ctx* c, zk_rl* rl) {
    if (!c) return ZK_ERR_INVALID_ARG;
    if (rl && rl_device(rl) != c->device) return fail(c, ZK_ERR_INVALID_ARG, "link store and ctx on different devices");
    if (rl && rl_services(rl) != c->S) return fail(c, ZK_ERR_INVALID_ARG, "link store and ctx differ in num_services");
    if (rl && c->rt && c->rt_mode == ZK_RT_WITH_DEPS)
        return fail(c, ZK_ERR_UNSUPPORTED, "a realtime link store and a ZK_RT_WITH_DEPS sketch on one ctx");
    if (c->rl && c->rl != rl) {
        ZK_HIP(c, hipStreamSynchronize(c->stream));
        rl_set_stream(c->rl, nullptr);
    }
    c->rl = rl;
    if (rl) rl_set_stream(rl, c->stream);  // one stream orders the ctx's and the store's work
    return ZK_OK;
}

zk_status zk_rt_bind(zk_ctx* c, zk_rt* rt, uint32_t mode) {
    if (!c) return ZK_ERR_INVALID_ARG;
    if (mode != ZK_RT_WITH_DEPS && mode != ZK_RT_ONLY) return fail(c, ZK_ERR_INVALID_ARG, "unknown sketch mode");
    if (rt && rt_device(rt) != c->device) return fail(c, ZK_ERR_INVALID_ARG, "sketch and ctx on different devices");
    if (rt && c->rl && mode == ZK_RT_WITH_DEPS)
        return fail(c, ZK_ERR_UNSUPPORTED, "a ZK_RT_WITH_DEPS sketch and a realtime link store on one ctx");
    if (c->rt && c->rt != rt) {
            ZK_HIP(c, hipStreamSynchronize(c->stream));
        rt_set_stream(c->rt, nullptr);
    }
    c->rt = rt;
    c->rt_mode = mode;
    if (rt) rt_set_stream(rt, c->stream);  // one stream orders the ctx's and the sketch's work
    return ZK_OK;
}

zk_status zk_tracegen_device(zk_ctx* c, const zk_tracegen_params* p, const zk_span_cols* out, uint64_t cap,
                             uint64_t* n_records, uint64_t* n_traces) {
    if (!c) return ZK_ERR_INVALID_ARG;
    if (!p || !cols_ok(out) || !n_records || !n_traces || p->max_depth == 0 || p->max_depth > 16 ||
        p->num_services == 0 || (p->world && p->rank >= p->world))
        return fail(c, ZK_ERR_INVALID_ARG, "bad tracegen arguments");
    ZK_HIP(c, hipSetDevice(c->device));
    const hipError_t e = launch_tracegen(p, out, cap, n_records, n_traces, c->stream);
    if (e == hipErrorInvalidValue && p->global_ids)
        return fail(c, ZK_ERR_CAPACITY, "the shard's part of the global trace set exceeds the output capacity");
    ZK_HIP(c, e);
    return ZK_OK;
}

}  // extern "C"
