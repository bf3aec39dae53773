// zk_kv_api.cpp — C ABI of the key-value count-min + top-K sketch (include/zksketch.h).
#include <hip/hip_runtime.h>
#include <string.h>

#include <string>
#include <vector>

#include "zk_comm.h"
#include "zk_guard.h"
#include "zk_launch.h"
#include "zk_internal.h"
#include "zk_sketch_internal.h"
#include "zksketch.h"

using namespace zk;

#ifndef ZK_KV_UNITS_PER_CU
#define ZK_KV_UNITS_PER_CU 2  // sketch units per CU for large batches (A/B knob)
#endif
#ifndef ZK_KV_CAND_ROUNDS
#define ZK_KV_CAND_ROUNDS 2  // candidate-pass units: rounds over its resident workgroups (A/B knob)
#endif

struct zk_kv {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t cus = 256;
    KvArgs a{};
    unsigned long long* dropped = nullptr;
    // batch scratch
    uint64_t* sorted = nullptr;
    uint64_t sorted_cap = 0;
    uint64_t* seg = nullptr;
    uint32_t* unit_base = nullptr;
    uint32_t* cand_base = nullptr;  // the candidate and merge passes' own unit plan
    void* part = nullptr;
    uint64_t part_bytes = 0;
    uint64_t* unit_key = nullptr;
    uint32_t* unit_est = nullptr;
    uint32_t unit_cap = 0;
    void* stage = nullptr;  // host-pointer staging: svc | keys
    uint64_t stage_cap = 0;
    uint64_t* qkeys = nullptr;  // estimate staging
    uint32_t* qest = nullptr;
    uint64_t qcap = 0;
    // pinned host mirror for queries: dropped counter, per-service totals, candidate keys and
    // estimates -- one contiguous copy each instead of strided copies into pageable memory
    uint8_t* hq = nullptr;
    // every rank's candidate lists, gathered by zk_kv_allreduce ([lists][S][cand])
    uint64_t* g_key = nullptr;
    uint32_t* g_est = nullptr;
    uint32_t g_lists = 0;
    bool timing = false;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    bool ev_recorded = false;
    std::string err;
};

namespace {

zk_status kfail(zk_kv* k, zk_status s, const std::string& m) {
    if (k) k->err = m;
    return s;
}

#define KV_HIP(kv, call)                                                                         \
    do {                                                                                         \
        hipError_t _e = (call);                                                                  \
        if (_e != hipSuccess)                                                                          \
            return kfail(kv, is_refusal(_e) ? ZK_ERR_CAPACITY : ZK_ERR_HIP,                          \
                        std::string(#call) + ": " + launch_error_str(_e));                             \
    } while (0)

uint32_t ilog2(uint32_t x) {
    uint32_t r = 0;
    while ((1u << (r + 1)) <= x) ++r;
    return r;
}

// layout of the pinned query mirror: [dropped u64][totals u64 x S][cand keys u64 x S*cand][cand est u32 x S*cand]
uint64_t hq_bytes(const KvArgs& a) { return 8 + (uint64_t)a.S * 8 + (uint64_t)a.S * a.cand * 12; }
uint64_t* hq_totals(zk_kv* k) { return (uint64_t*)(k->hq + 8); }
uint64_t* hq_keys(zk_kv* k) { return (uint64_t*)(k->hq + 8 + (uint64_t)k->a.S * 8); }
uint32_t* hq_est(zk_kv* k) { return (uint32_t*)(k->hq + 8 + (uint64_t)k->a.S * 8 + (uint64_t)k->a.S * k->a.cand * 8); }

// dropped counter + totals (+ the candidate lists) into the pinned mirror, one sync, then the
// state checks every query makes
zk_status check_state(zk_kv* kv, bool need_totals_ok, bool candidates = false) {
    if (!kv->hq) KV_HIP(kv, hipHostMalloc((void**)&kv->hq, hq_bytes(kv->a), hipHostMallocDefault));
    const KvArgs& a = kv->a;
    KV_HIP(kv, hipMemcpyAsync(kv->hq, kv->dropped, 8, hipMemcpyDeviceToHost, kv->stream));
    if (need_totals_ok)
        KV_HIP(kv, hipMemcpyAsync(hq_totals(kv), a.totals, (size_t)a.S * 8, hipMemcpyDeviceToHost, kv->stream));
    if (candidates) {
        KV_HIP(kv, hipMemcpyAsync(hq_keys(kv), a.cand_key, (size_t)a.S * a.cand * 8, hipMemcpyDeviceToHost, kv->stream));
        KV_HIP(kv, hipMemcpyAsync(hq_est(kv), a.cand_est, (size_t)a.S * a.cand * 4, hipMemcpyDeviceToHost, kv->stream));
    }
    KV_HIP(kv, hipStreamSynchronize(kv->stream));
    const uint64_t dropped = *(const uint64_t*)kv->hq;
    if (dropped) return kfail(kv, ZK_ERR_SERVICE_RANGE, std::to_string(dropped) + " items with service_id >= S");
    if (need_totals_ok)
        for (uint32_t s = 0; s < a.S; ++s)
            if (hq_totals(kv)[s] >= (1ull << 32))
                return kfail(kv, ZK_ERR_CAPACITY, "a service counted >= 2^32 keys since reset");
    return ZK_OK;
}

}  // namespace

extern "C" {

zk_status zk_kv_create(const zk_kv_config* cfg, zk_kv** out) {
    ZK_GUARD_BEGIN
    if (!cfg || !out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    const uint32_t S = cfg->num_services;
    if (S == 0 || S > 4096) return ZK_ERR_INVALID_ARG;
    uint32_t width = cfg->width, depth = cfg->depth ? cfg->depth : 4, cand = cfg->candidates ? cfg->candidates : 64;
    if (width == 0) {
        width = 1u << ilog2((1u << 20) / S > 0 ? (1u << 20) / S : 1);
        if (width < 64) width = 64;
        if (width > kKvMaxWidth) width = kKvMaxWidth;
    }
    if (width < 64 || width > kKvMaxWidth || (width & (width - 1))) return ZK_ERR_INVALID_ARG;
    if (depth > kKvMaxDepth || depth * width > 16384) return ZK_ERR_INVALID_ARG;  // LDS: <= 64 KB of rows
    if (cand > kKvMaxCand) return ZK_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ZK_ERR_NO_DEVICE;
    if (cfg->device < 0 || cfg->device >= ndev) return ZK_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return ZK_ERR_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZK_ERR_NO_DEVICE;
    zk_kv* k = new zk_kv();
    k->device = cfg->device;
    k->cus = prop.multiProcessorCount > 0 ? (uint32_t)prop.multiProcessorCount : 256;
    KvArgs& a = k->a;
    a.S = S;
    a.width = width;
    a.wbits = ilog2(width);
    a.depth = depth;
    a.cand = cand;
    for (uint32_t r = 0; r < kKvMaxDepth; ++r) a.seeds[r] = sk_mix64(cfg->seed + 0x9E3779B97F4A7C15ull * (r + 1));
    a.unit_items = kKvUnitItems;
    k->timing = (cfg->reserved[0] & ZK_KV_TIMING) != 0;
    hipError_t e = hipSetDevice(k->device);
    for (int i = 0; i < 5 && k->timing && e == hipSuccess; ++i) e = hipEventCreate(&k->ev[i]);
    if (e == hipSuccess) {
        if (cfg->stream) {
            k->stream = (hipStream_t)cfg->stream;
        } else {
            e = hipStreamCreateWithFlags(&k->stream, hipStreamNonBlocking);
            k->own_stream = true;
        }
    }
    if (e == hipSuccess) e = hipMalloc(&a.cm, (uint64_t)S * depth * width * 4);
    if (e == hipSuccess) e = hipMalloc(&a.totals, (uint64_t)S * 8);
    if (e == hipSuccess) e = hipMalloc(&a.cand_key, (uint64_t)S * cand * 8);
    if (e == hipSuccess) e = hipMalloc(&a.cand_est, (uint64_t)S * cand * 4);
    if (e == hipSuccess) e = hipMalloc(&k->dropped, 8);
    if (e == hipSuccess) e = hipMalloc(&k->seg, (uint64_t)(S + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&k->unit_base, (uint64_t)(S + 1) * 4);
    if (e == hipSuccess) e = hipMalloc(&k->cand_base, (uint64_t)(S + 1) * 4);
    // the pinned query mirror up front: a first query must not pay for a pinned allocation
    if (e == hipSuccess) e = hipHostMalloc((void**)&k->hq, hq_bytes(a), hipHostMallocDefault);
    zk_status st = e == hipSuccess ? zk_kv_reset(k) : ZK_ERR_HIP;
    if (st != ZK_OK) {
        zk_kv_destroy(k);
        return st;
    }
    *out = k;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_destroy(zk_kv* k) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    hipSetDevice(k->device);
    if (k->stream) hipStreamSynchronize(k->stream);
    for (void* p : {(void*)k->a.cm, (void*)k->a.totals, (void*)k->a.cand_key, (void*)k->a.cand_est, (void*)k->dropped,
                    (void*)k->sorted, (void*)k->seg, (void*)k->unit_base, (void*)k->cand_base, k->part, (void*)k->unit_key,
                    (void*)k->unit_est, k->stage, (void*)k->qkeys, (void*)k->qest, (void*)k->g_key, (void*)k->g_est})
        if (p) hipFree(p);
    if (k->hq) hipHostFree(k->hq);
    for (hipEvent_t ev : k->ev)
        if (ev) hipEventDestroy(ev);
    if (k->own_stream && k->stream) hipStreamDestroy(k->stream);
    delete k;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_kv_last_error(const zk_kv* k) { return k ? k->err.c_str() : "null handle"; }

zk_status zk_kv_geometry(const zk_kv* k, uint32_t* width, uint32_t* depth, uint32_t* candidates) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (width) *width = k->a.width;
    if (depth) *depth = k->a.depth;
    if (candidates) *candidates = k->a.cand;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_reset(zk_kv* k) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    const KvArgs& a = k->a;
    KV_HIP(k, hipSetDevice(k->device));
    KV_HIP(k, hipMemsetAsync(a.cm, 0, (uint64_t)a.S * a.depth * a.width * 4, k->stream));
    KV_HIP(k, hipMemsetAsync(a.totals, 0, (uint64_t)a.S * 8, k->stream));
    KV_HIP(k, hipMemsetAsync(a.cand_key, 0, (uint64_t)a.S * a.cand * 8, k->stream));
    KV_HIP(k, hipMemsetAsync(a.cand_est, 0, (uint64_t)a.S * a.cand * 4, k->stream));
    KV_HIP(k, hipMemsetAsync(k->dropped, 0, 8, k->stream));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_accumulate(zk_kv* k, const uint32_t* svc, const uint64_t* keys, uint64_t n, uint32_t flags) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (n == 0) return ZK_OK;
    if (!svc || !keys) return kfail(k, ZK_ERR_INVALID_ARG, "null input");
    if (n >= (1ull << 32)) return kfail(k, ZK_ERR_INVALID_ARG, "batch of >= 2^32 items");
    RoctxRange rr("zk_kv_accumulate");
    KV_HIP(k, hipSetDevice(k->device));
    if (!(flags & ZK_BATCH_DEVICE_PTRS)) {
        if (n > k->stage_cap) {
            if (k->stage) KV_HIP(k, hipFree(k->stage));
            k->stage = nullptr;
            KV_HIP(k, hipMalloc(&k->stage, n * 12 + 256));
            k->stage_cap = n;
        }
        uint64_t* dk = (uint64_t*)k->stage;
        uint32_t* ds = (uint32_t*)((uint8_t*)k->stage + ((n * 8 + 255) & ~255ull));
        KV_HIP(k, hipMemcpyAsync(dk, keys, n * 8, hipMemcpyHostToDevice, k->stream));
        KV_HIP(k, hipMemcpyAsync(ds, svc, n * 4, hipMemcpyHostToDevice, k->stream));
        // host inputs are borrowed for the call only (zkagg.h): wait until the copies (DMA reads of
        // page-locked memory run after an async call returns) have consumed them
        KV_HIP(k, hipStreamSynchronize(k->stream));
        keys = dk;
        svc = ds;
    }
    KvArgs& a = k->a;
    // Units (one workgroup each in the sketch and candidate passes) of at least kKvUnitItems keys,
    // larger for big batches: about 2 units per CU (a service's run is split into equal units).
    // A unit pays a fixed cost (loading its service's rows, two or three top-set sorts), so fewer,
    // longer units are faster as long as they fill the chip (measured on C4: 64 Ki -> 256 Ki keys
    // per unit, candidates 2.40 -> 1.54 ms).
    {
        const uint64_t target = (uint64_t)ZK_KV_UNITS_PER_CU * k->cus;
        uint64_t u = (n + target - 1) / target;
        u = (u + 4095) & ~4095ull;
        a.unit_items = u > kKvUnitItems ? u : kKvUnitItems;
    }
    const PartitionPlan plan = partition_plan(n, a.S, k->cus);
    const uint64_t pb = partition_scratch_bytes(plan);
    if (pb > k->part_bytes) {
        if (k->part) KV_HIP(k, hipFree(k->part));
        k->part = nullptr;
        KV_HIP(k, hipMalloc(&k->part, pb));
        k->part_bytes = pb;
    }
    if (n > k->sorted_cap) {
        if (k->sorted) KV_HIP(k, hipFree(k->sorted));
        k->sorted = nullptr;
        KV_HIP(k, hipMalloc(&k->sorted, n * 8));
        k->sorted_cap = n;
    }
    const uint64_t max_units = (n + a.unit_items - 1) / a.unit_items + a.S;
    // The candidate pass runs ZK_KV_CAND_ROUNDS rounds of units over its resident workgroups (three per
    // CU at 32 KB of rows: its LDS is the rows + 18.5 KB), in units of their own (a service cut into
    // equal parts): two full rounds, where the sketch's units would leave most of a second round idle.
    uint64_t cand_items = a.unit_items;
    {
        const uint64_t rows = (uint64_t)a.depth * a.width * 4;
        uint64_t per_cu = (160ull * 1024) / (rows + 18944);
        per_cu = per_cu < 1 ? 1 : per_cu > 3 ? 3 : per_cu;
        const uint64_t slots = per_cu * k->cus * ZK_KV_CAND_ROUNDS;
        uint64_t u = (n + slots - 1) / slots;
        u += u / 16;  // slack: a service just over a multiple of u is not cut into one more part
        u = (u + 4095) & ~4095ull;
        cand_items = u > kKvUnitItems ? u : kKvUnitItems;
    }
    const uint64_t max_cand = (n + cand_items - 1) / cand_items + a.S;
    const uint64_t max_lists = max_units > max_cand ? max_units : max_cand;
    if (max_lists > k->unit_cap) {
        if (k->unit_key) KV_HIP(k, hipFree(k->unit_key));
        if (k->unit_est) KV_HIP(k, hipFree(k->unit_est));
        k->unit_key = nullptr;
        k->unit_est = nullptr;
        KV_HIP(k, hipMalloc(&k->unit_key, max_lists * a.cand * 8));
        KV_HIP(k, hipMalloc(&k->unit_est, max_lists * a.cand * 4));
        k->unit_cap = (uint32_t)max_lists;
    }
    if (k->timing) KV_HIP(k, hipEventRecord(k->ev[0], k->stream));
    // the partition writes each key's count-min hash sk_mix64(key ^ seeds[0]), not the key itself
    KV_HIP(k, launch_partition(plan, svc, keys, n, k->sorted, k->seg, k->dropped, k->part, k->stream, true,
                               a.seeds[0]));
    KV_HIP(k, launch_unit_plan(k->seg, a.S, a.unit_items, k->unit_base, k->stream));
    KV_HIP(k, launch_unit_plan(k->seg, a.S, cand_items, k->cand_base, k->stream));
    if (k->timing) KV_HIP(k, hipEventRecord(k->ev[1], k->stream));
    a.keys = k->sorted;
    a.seg = k->seg;
    a.unit_base = k->unit_base;
    a.max_units = (uint32_t)max_units;
    a.unit_key = k->unit_key;
    a.unit_est = k->unit_est;
    a.extra_key = nullptr;
    a.extra_est = nullptr;
    a.extra_lists = 0;
    const bool small = n < (uint64_t)a.S * kKvSmallPerService;
    KV_HIP(k, launch_kv_sketch(a, k->stream, small));
    if (k->timing) KV_HIP(k, hipEventRecord(k->ev[2], k->stream));
    a.unit_base = k->cand_base;  // the candidate and merge passes' units
    a.max_units = (uint32_t)max_cand;
    KV_HIP(k, launch_kv_candidates(a, k->stream, small));
    if (k->timing) KV_HIP(k, hipEventRecord(k->ev[3], k->stream));
    KV_HIP(k, launch_kv_merge(a, k->stream, small));
    if (k->timing) {
        KV_HIP(k, hipEventRecord(k->ev[4], k->stream));
        k->ev_recorded = true;
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_phase_ms(zk_kv* k, double out[4]) {
    ZK_GUARD_BEGIN
    if (!k || !out) return ZK_ERR_INVALID_ARG;
    if (!k->timing || !k->ev_recorded) return kfail(k, ZK_ERR_UNSUPPORTED, "create the sketch with ZK_KV_TIMING");
    KV_HIP(k, hipSetDevice(k->device));
    KV_HIP(k, hipEventSynchronize(k->ev[4]));
    for (int i = 0; i < 4; ++i) {
        float ms = 0.f;
        KV_HIP(k, hipEventElapsedTime(&ms, k->ev[i], k->ev[i + 1]));
        out[i] = ms;
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_topk_all(zk_kv* k, uint32_t kk, uint64_t* keys, uint32_t* est, uint32_t* count) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (kk == 0 || kk > k->a.cand || !keys || !est) return kfail(k, ZK_ERR_INVALID_ARG, "k must be in 1..candidates");
    const KvArgs& a = k->a;
    KV_HIP(k, hipSetDevice(k->device));
    zk_status st = check_state(k, true, true);  // syncs; the candidate lists are in the pinned mirror
    if (st != ZK_OK) return st;
    for (uint32_t s = 0; s < a.S; ++s) {
        memcpy(keys + (uint64_t)s * kk, hq_keys(k) + (uint64_t)s * a.cand, (size_t)kk * 8);
        memcpy(est + (uint64_t)s * kk, hq_est(k) + (uint64_t)s * a.cand, (size_t)kk * 4);
    }
    if (count)
        for (uint32_t s = 0; s < a.S; ++s) {
            uint32_t c = 0;
            while (c < kk && est[(uint64_t)s * kk + c]) ++c;
            count[s] = c;
        }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_topk(zk_kv* k, uint32_t svc, uint32_t kk, uint64_t* keys, uint32_t* est, uint32_t* count) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (svc >= k->a.S) return kfail(k, ZK_ERR_SERVICE_RANGE, "service >= S");
    if (kk == 0 || kk > k->a.cand || !keys || !est) return kfail(k, ZK_ERR_INVALID_ARG, "k must be in 1..candidates");
    const KvArgs& a = k->a;
    KV_HIP(k, hipSetDevice(k->device));
    KV_HIP(k, hipMemcpyAsync(keys, a.cand_key + (uint64_t)svc * a.cand, (size_t)kk * 8, hipMemcpyDeviceToHost, k->stream));
    KV_HIP(k, hipMemcpyAsync(est, a.cand_est + (uint64_t)svc * a.cand, (size_t)kk * 4, hipMemcpyDeviceToHost, k->stream));
    zk_status st = check_state(k, true);
    if (st != ZK_OK) return st;
    if (count) {
        uint32_t c = 0;
        while (c < kk && est[c]) ++c;
        *count = c;
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_estimate(zk_kv* k, uint32_t svc, const uint64_t* keys, uint64_t n, uint32_t* est) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (svc >= k->a.S) return kfail(k, ZK_ERR_SERVICE_RANGE, "service >= S");
    if (n == 0) return ZK_OK;
    if (!keys || !est) return kfail(k, ZK_ERR_INVALID_ARG, "null array");
    KV_HIP(k, hipSetDevice(k->device));
    if (n > k->qcap) {
        if (k->qkeys) KV_HIP(k, hipFree(k->qkeys));
        if (k->qest) KV_HIP(k, hipFree(k->qest));
        k->qkeys = nullptr;
        k->qest = nullptr;
        KV_HIP(k, hipMalloc(&k->qkeys, n * 8));
        KV_HIP(k, hipMalloc(&k->qest, n * 4));
        k->qcap = n;
    }
    KV_HIP(k, hipMemcpyAsync(k->qkeys, keys, n * 8, hipMemcpyHostToDevice, k->stream));
    KV_HIP(k, launch_kv_estimate(k->a, svc, k->qkeys, n, k->qest, k->stream));
    KV_HIP(k, hipMemcpyAsync(est, k->qest, n * 4, hipMemcpyDeviceToHost, k->stream));
    KV_HIP(k, hipStreamSynchronize(k->stream));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_totals(zk_kv* k, uint64_t* totals) {
    ZK_GUARD_BEGIN
    if (!k || !totals) return ZK_ERR_INVALID_ARG;
    KV_HIP(k, hipSetDevice(k->device));
    KV_HIP(k, hipMemcpyAsync(totals, k->a.totals, (uint64_t)k->a.S * 8, hipMemcpyDeviceToHost, k->stream));
    KV_HIP(k, hipStreamSynchronize(k->stream));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_partial(zk_kv* k, void** counters, uint64_t* cb, void** totals, uint64_t* tb) {
    ZK_GUARD_BEGIN
    if (!k || !counters || !cb || !totals || !tb) return ZK_ERR_INVALID_ARG;
    *counters = k->a.cm;
    *cb = (uint64_t)k->a.S * k->a.depth * k->a.width * 4;
    *totals = k->a.totals;
    *tb = (uint64_t)k->a.S * 8;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_candidates(zk_kv* k, void** keys, void** est, uint64_t* bk, uint64_t* be) {
    ZK_GUARD_BEGIN
    if (!k || !keys || !est || !bk || !be) return ZK_ERR_INVALID_ARG;
    *keys = k->a.cand_key;
    *est = k->a.cand_est;
    *bk = (uint64_t)k->a.S * k->a.cand * 8;
    *be = (uint64_t)k->a.S * k->a.cand * 4;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_merge_candidates(zk_kv* k, const uint64_t* keys, const uint32_t* est, uint32_t lists) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (lists && (!keys || !est)) return kfail(k, ZK_ERR_INVALID_ARG, "null lists");
    KV_HIP(k, hipSetDevice(k->device));
    KvArgs a = k->a;
    a.max_units = 0;  // no unit lists: previous candidates + gathered lists only
    a.extra_key = keys;
    a.extra_est = est;
    a.extra_lists = lists;
    KV_HIP(k, launch_kv_merge(a, k->stream, false));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_kv_allreduce(zk_kv* k, zk_comm* comm) {
    ZK_GUARD_BEGIN
    if (!k) return ZK_ERR_INVALID_ARG;
    if (!comm) return kfail(k, ZK_ERR_INVALID_ARG, "null communicator");
    KV_HIP(k, hipSetDevice(k->device));
    const KvArgs& a = k->a;
    const uint32_t W = comm_world(comm);
    const uint64_t lk = (uint64_t)a.S * a.cand;
    if (W > k->g_lists) {
        KV_HIP(k, hipStreamSynchronize(k->stream));  // the old buffers may still be read
        hipFree(k->g_key);
        hipFree(k->g_est);
        k->g_key = nullptr;
        k->g_est = nullptr;
        k->g_lists = 0;
        KV_HIP(k, hipMalloc(&k->g_key, W * lk * 8));
        KV_HIP(k, hipMalloc(&k->g_est, W * lk * 4));
        k->g_lists = W;
    }
    // the candidate lists first (the merge overwrites them), then the counters and totals
    zk_status st = comm_allgather(comm, a.cand_key, k->g_key, lk * 8, k->device, k->stream, &k->err);
    if (st == ZK_OK) st = comm_allgather(comm, a.cand_est, k->g_est, lk * 4, k->device, k->stream, &k->err);
    if (st == ZK_OK)
        st = comm_allreduce(comm, a.cm, (uint64_t)a.S * a.depth * a.width, kCommU32, kCommSum, k->device, k->stream,
                            &k->err);
    if (st == ZK_OK) st = comm_allreduce(comm, a.totals, a.S, kCommU64, kCommSum, k->device, k->stream, &k->err);
    if (st == ZK_OK) st = comm_allreduce(comm, k->dropped, 1, kCommU64, kCommSum, k->device, k->stream, &k->err);
    if (st != ZK_OK) return st;
    return zk_kv_merge_candidates(k, k->g_key, k->g_est, W);
    ZK_GUARD_END
}

}  // extern "C"
