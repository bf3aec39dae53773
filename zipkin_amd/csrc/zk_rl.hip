// zk_rl.hip — the realtime link store behind RealtimeAggregates (include/zksketch.h, zk_rl_*).
//
// The reference declares the trait without an implementation (zipkin-common/.../storage/
// RealtimeAggregates.scala:26-38; zipkinQuery.thrift:234-251; QueryService.scala:416-430 answers
// "Not Implemented"). Both queries ask, for a server service, which client services called it and
// with which spans: getSpanDurations the duration of every call, getServiceNamesToTraceIds the
// traceIds. That is the dependency job's join output before its group.sum: one (parent service,
// child service, child duration, traceId) row per joined child span (ZipkinAggregateJob.scala:25-37).
// Bound to a dependency ctx (zk_rl_bind), K1 (kModeLinks) and the spill kernel write one item per
// link they emit -- key ((child * S + parent) << 40) | duration, and the child's traceId -- beside
// the link in the same list position; after the batch, k_rl_gather appends every list to the
// store's window (HBM, 16 B per link, grown as it fills). A query is one filter pass over the window
// for the server's key range (k_rl_count + k_rl_select), then a host sort of that server's rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "zk_guard.h"
#include "zk_internal.h"
#include "zk_launch.h"
#include "zk_rl_internal.h"
#include "zksketch.h"

namespace zk {
namespace {

constexpr int kRlWG = 256;

// list w (w < lists: a K1 list of counts[w] items at w * stride; w == lists: the spill list of
// *spill items) appended to the window at a range claimed with one atomic per workgroup
__global__ __launch_bounds__(kRlWG) void k_rl_gather(const uint64_t* __restrict__ lkey, const uint64_t* __restrict__ ltid,
                                                     const uint32_t* __restrict__ counts, uint32_t lists, uint64_t stride,
                                                     const uint32_t* __restrict__ spill, uint64_t spill_cap,
                                                     uint64_t* __restrict__ wkey, uint64_t* __restrict__ wtid,
                                                     unsigned long long* __restrict__ wcount, uint64_t wcap,
                                                     unsigned long long* __restrict__ dropped) {
    __shared__ unsigned long long s_base;
    const uint32_t w = blockIdx.x;
    uint64_t cnt;
    if (w < lists) {
        cnt = counts[w];
    } else {
        const uint64_t c = *spill;
        cnt = c < spill_cap ? c : spill_cap;
    }
    if (cnt == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(wcount, (unsigned long long)cnt);
    __syncthreads();
    const uint64_t base = s_base;
    if (threadIdx.x == 0 && base + cnt > wcap) atomicAdd(dropped, (unsigned long long)(base + cnt - (base < wcap ? wcap : base)));
    const uint64_t src = (uint64_t)w * stride;
    for (uint64_t i = threadIdx.x; i < cnt; i += kRlWG) {
        if (base + i >= wcap) break;
        wkey[base + i] = lkey[src + i];
        wtid[base + i] = ltid[src + i];
    }
}

// items of the window whose key lies in [lo, hi): counted (k_rl_count), then copied out in any order
// (k_rl_select, one output claim per wave)
__global__ __launch_bounds__(kRlWG) void k_rl_count(const uint64_t* __restrict__ wkey, const unsigned long long* __restrict__ wcount,
                                                    uint64_t wcap, uint64_t lo, uint64_t hi, unsigned long long* __restrict__ out) {
    const uint64_t n = *wcount < wcap ? *wcount : wcap;
    uint32_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kRlWG + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kRlWG) {
        const uint64_t k = wkey[i];
        c += (k >= lo && k < hi) ? 1u : 0u;
    }
    // wave sum, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

__global__ __launch_bounds__(kRlWG) void k_rl_select(const uint64_t* __restrict__ wkey, const uint64_t* __restrict__ wtid,
                                                     const unsigned long long* __restrict__ wcount, uint64_t wcap, uint64_t lo,
                                                     uint64_t hi, uint64_t* __restrict__ okey, uint64_t* __restrict__ otid,
                                                     uint64_t ocap, unsigned long long* __restrict__ ocount) {
    const uint64_t n = *wcount < wcap ? *wcount : wcap;
    const int lane = threadIdx.x & 63;
    const uint64_t step = (uint64_t)gridDim.x * kRlWG;
    for (uint64_t i0 = (uint64_t)blockIdx.x * kRlWG + (threadIdx.x & ~63u); i0 < n; i0 += step) {
        const uint64_t i = i0 + lane;
        const uint64_t k = i < n ? wkey[i] : 0ull;
        const bool take = i < n && k >= lo && k < hi;
        const uint64_t m = __ballot(take);
        if (!m) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(ocount, (unsigned long long)__popcll(m));
        base = __shfl(base, 0);
        if (take) {
            const uint64_t at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (at < ocap) {
                okey[at] = k;
                otid[at] = wtid[i];
            }
        }
    }
}

}  // namespace
}  // namespace zk

using namespace zk;

struct zk_rl {
    int device = 0;
    hipStream_t stream = nullptr;  // the bound ctx's while bound, else `own`
    hipStream_t own = nullptr;
    uint32_t S = 0;
    uint32_t cus = 256;
    // the window: every link item since the last reset
    uint64_t* wkey = nullptr;
    uint64_t* wtid = nullptr;
    uint64_t wcap = 0;              // items
    uint64_t reserved = 0;          // upper bound of the items appended (links <= records)
    unsigned long long* cnt = nullptr;  // device: [0] window items, [1] dropped past capacity, [2] query count
    // one batch's K1 lists (the ctx's link geometry) + the spill list
    uint64_t* lkey = nullptr;
    uint64_t* ltid = nullptr;
    uint64_t lcap = 0;
    uint32_t* lspill = nullptr;
    // query output
    uint64_t* okey = nullptr;
    uint64_t* otid = nullptr;
    uint64_t ocap = 0;
    unsigned long long* h_cnt = nullptr;  // pinned
    std::string err;
};

namespace {

zk_status lfail(zk_rl* r, zk_status s, const std::string& m) {
    if (r) r->err = m;
    return s;
}

#define RL_HIP(r, call)                                                                            \
    do {                                                                                           \
        hipError_t _e = (call);                                                                    \
        if (_e != hipSuccess) return lfail(r, is_refusal(_e) ? ZK_ERR_CAPACITY : ZK_ERR_HIP,       \
                                           std::string(#call) + ": " + launch_error_str(_e));      \
    } while (0)

zk_status grow2(zk_rl* r, uint64_t** a, uint64_t** b, uint64_t* cap, uint64_t need, bool keep, uint64_t keep_n) {
    if (need <= *cap && *a) return ZK_OK;
    uint64_t ncap = need + need / 2 + 1024;
    uint64_t *na = nullptr, *nb = nullptr;
    if (hipMalloc((void**)&na, ncap * 8) != hipSuccess || hipMalloc((void**)&nb, ncap * 8) != hipSuccess) {
        (void)hipGetLastError();
        if (na) (void)hipFree(na);
        return lfail(r, ZK_ERR_CAPACITY, "realtime link store: no device memory for " + std::to_string(ncap) + " items");
    }
    if (keep && keep_n && *a) {
        RL_HIP(r, hipMemcpyAsync(na, *a, keep_n * 8, hipMemcpyDeviceToDevice, r->stream));
        RL_HIP(r, hipMemcpyAsync(nb, *b, keep_n * 8, hipMemcpyDeviceToDevice, r->stream));
        RL_HIP(r, hipStreamSynchronize(r->stream));
    }
    if (*a) RL_HIP(r, hipFree(*a));
    if (*b) RL_HIP(r, hipFree(*b));
    *a = na;
    *b = nb;
    *cap = ncap;
    return ZK_OK;
}

}  // namespace

namespace zk {

zk_status rl_prepare_lists(zk_rl* r, uint32_t grid, uint64_t stride, uint64_t n, JoinArgs* a, hipStream_t s) {
    r->stream = s;
    const uint64_t need = (uint64_t)grid * stride + n;
    zk_status st = grow2(r, &r->lkey, &r->ltid, &r->lcap, need, false, 0);
    if (st != ZK_OK) return st;
    if (!r->lspill) RL_HIP(r, hipMalloc(&r->lspill, 4));
    RL_HIP(r, hipMemsetAsync(r->lspill, 0, 4, s));
    a->lk_key = r->lkey;
    a->lk_tid = r->ltid;
    a->lk_spill_count = r->lspill;
    a->lk_spill_cap = n;
    return ZK_OK;
}

zk_status rl_consume_lists(zk_rl* r, const uint32_t* counts, uint32_t grid, uint64_t stride, uint64_t n) {
    // the window keeps every item; links <= records, so n more records need at most n more slots
    const uint64_t keep = r->reserved < r->wcap ? r->reserved : r->wcap;
    zk_status st = grow2(r, &r->wkey, &r->wtid, &r->wcap, r->reserved + n, true, keep);
    if (st != ZK_OK) return st;
    r->reserved += n;
    RL_HIP(r, launch_checked("k_rl_gather", k_rl_gather, dim3(grid + 1), dim3(kRlWG), 0, r->stream,
                             (const uint64_t*)r->lkey, (const uint64_t*)r->ltid, counts, grid, stride,
                             (const uint32_t*)r->lspill, n, r->wkey, r->wtid, r->cnt, r->wcap, r->cnt + 1));
    return ZK_OK;
}

const char* rl_error(const zk_rl* r) { return r->err.c_str(); }
int rl_device(const zk_rl* r) { return r->device; }
uint32_t rl_services(const zk_rl* r) { return r->S; }
void rl_set_stream(zk_rl* r, hipStream_t s) {
    hipStream_t ns = s ? s : r->own;
    if (ns != r->stream) {
        if (r->stream) (void)hipStreamSynchronize(r->stream);
        r->stream = ns;
    }
}

}  // namespace zk

extern "C" {

zk_status zk_rl_create(const zk_rl_config* cfg, zk_rl** out) {
    ZK_GUARD_BEGIN
    if (!cfg || !out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    if (cfg->num_services == 0 || cfg->num_services > 4096) return ZK_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || cfg->device < 0 || cfg->device >= ndev) return ZK_ERR_NO_DEVICE;
    if (hipSetDevice(cfg->device) != hipSuccess) return ZK_ERR_HIP;
    zk_rl* r = new zk_rl();
    r->device = cfg->device;
    r->S = cfg->num_services;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess && cus > 0)
        r->cus = (uint32_t)cus;
    if (cfg->stream) {
        r->stream = (hipStream_t)cfg->stream;
    } else if (hipStreamCreateWithFlags(&r->own, hipStreamNonBlocking) != hipSuccess) {
        delete r;
        return ZK_ERR_HIP;
    } else {
        r->stream = r->own;
    }
    if (hipMalloc(&r->cnt, 4 * 8) != hipSuccess || hipHostMalloc((void**)&r->h_cnt, 4 * 8, hipHostMallocDefault) != hipSuccess ||
        hipMemsetAsync(r->cnt, 0, 4 * 8, r->stream) != hipSuccess) {
        (void)hipGetLastError();
        zk_rl_destroy(r);
        return ZK_ERR_HIP;
    }
    *out = r;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rl_destroy(zk_rl* r) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    for (void* p : {(void*)r->wkey, (void*)r->wtid, (void*)r->lkey, (void*)r->ltid, (void*)r->lspill, (void*)r->okey,
                    (void*)r->otid, (void*)r->cnt})
        if (p) (void)hipFree(p);
    if (r->h_cnt) (void)hipHostFree(r->h_cnt);
    if (r->own) (void)hipStreamDestroy(r->own);
    delete r;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_rl_last_error(const zk_rl* r) { return r ? r->err.c_str() : "null store"; }

zk_status zk_rl_reset(zk_rl* r) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    RL_HIP(r, hipSetDevice(r->device));
    RL_HIP(r, hipMemsetAsync(r->cnt, 0, 4 * 8, r->stream));
    r->reserved = 0;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rl_count(zk_rl* r, uint64_t* items, uint64_t* dropped) {
    ZK_GUARD_BEGIN
    if (!r || !items) return ZK_ERR_INVALID_ARG;
    RL_HIP(r, hipSetDevice(r->device));
    RL_HIP(r, hipMemcpyAsync(r->h_cnt, r->cnt, 2 * 8, hipMemcpyDeviceToHost, r->stream));
    RL_HIP(r, hipStreamSynchronize(r->stream));
    const uint64_t n = r->h_cnt[0];
    *items = n < r->wcap ? n : r->wcap;
    if (dropped) *dropped = r->h_cnt[1];
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rl_server_links(zk_rl* r, uint32_t server, uint32_t* parent, int64_t* duration, uint64_t* trace_id,
                             uint64_t cap, uint64_t* n) {
    ZK_GUARD_BEGIN
    if (!r || !n) return ZK_ERR_INVALID_ARG;
    if (server >= r->S) return lfail(r, ZK_ERR_SERVICE_RANGE, "server service id >= num_services");
    RL_HIP(r, hipSetDevice(r->device));
    const uint64_t lo = ((uint64_t)server * r->S) << 40, hi = ((uint64_t)(server + 1) * r->S) << 40;
    const uint32_t grid = r->cus * 4;
    RL_HIP(r, hipMemsetAsync(r->cnt + 2, 0, 8, r->stream));
    if (r->wkey)
        RL_HIP(r, launch_checked("k_rl_count", k_rl_count, dim3(grid), dim3(kRlWG), 0, r->stream, (const uint64_t*)r->wkey,
                                 (const unsigned long long*)r->cnt, r->wcap, lo, hi, r->cnt + 2));
    RL_HIP(r, hipMemcpyAsync(r->h_cnt + 2, r->cnt + 2, 8, hipMemcpyDeviceToHost, r->stream));
    RL_HIP(r, hipStreamSynchronize(r->stream));
    const uint64_t m = r->h_cnt[2];
    *n = m;
    if (!parent && !duration && !trace_id) return ZK_OK;
    if (cap < m) return lfail(r, ZK_ERR_CAPACITY, "output capacity < the server's links");
    if (m == 0) return ZK_OK;
    zk_status st = grow2(r, &r->okey, &r->otid, &r->ocap, m, false, 0);
    if (st != ZK_OK) return st;
    RL_HIP(r, hipMemsetAsync(r->cnt + 2, 0, 8, r->stream));
    RL_HIP(r, launch_checked("k_rl_select", k_rl_select, dim3(grid), dim3(kRlWG), 0, r->stream, (const uint64_t*)r->wkey,
                             (const uint64_t*)r->wtid, (const unsigned long long*)r->cnt, r->wcap, lo, hi, r->okey, r->otid,
                             r->ocap, r->cnt + 2));
    std::vector<uint64_t> k(m), t(m);
    RL_HIP(r, hipMemcpyAsync(k.data(), r->okey, m * 8, hipMemcpyDeviceToHost, r->stream));
    RL_HIP(r, hipMemcpyAsync(t.data(), r->otid, m * 8, hipMemcpyDeviceToHost, r->stream));
    RL_HIP(r, hipStreamSynchronize(r->stream));
    // (parent, duration, traceId) order: the key orders parent and duration, the traceId breaks ties
    std::vector<uint64_t> idx(m);
    for (uint64_t i = 0; i < m; ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) { return k[x] != k[y] ? k[x] < k[y] : t[x] < t[y]; });
    const uint64_t dmask = (1ull << 40) - 1;
    for (uint64_t i = 0; i < m; ++i) {
        const uint64_t key = k[idx[i]];
        if (parent) parent[i] = (uint32_t)((key >> 40) - (uint64_t)server * r->S);
        if (duration) duration[i] = (int64_t)(key & dmask);
        if (trace_id) trace_id[i] = t[idx[i]];
    }
    return ZK_OK;
    ZK_GUARD_END
}

}  // extern "C"
