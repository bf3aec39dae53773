// zk_tracegen.hip — device and host drivers of the synthetic zipkin-tracegen workload
// (see zk_tracegen.h for the TraceGen.scala correspondence). Not on the measured path: the bench
// generates its 1e8-record batches here, directly in HBM, before timing starts.
#include <hipcub/hipcub.hpp>

#include "zk_internal.h"
#include "zk_tracegen.h"
#include "zk_launch.h"

namespace zk {
namespace {

struct CountEmit {
    __host__ __device__ void operator()(const zk_tg_rec&) {}
};

struct ColEmit {
    uint64_t* tid;
    uint64_t* sid;
    uint64_t* pid;
    int64_t* first;
    int64_t* last;
    uint32_t* svc;
    uint32_t* flags;
    uint64_t pos;
    __host__ __device__ void operator()(const zk_tg_rec& r) {
        tid[pos] = r.trace_id;
        sid[pos] = r.span_id;
        pid[pos] = r.parent_id;
        first[pos] = r.first_ts;
        last[pos] = r.last_ts;
        svc[pos] = r.service_id;
        flags[pos] = r.flags;
        ++pos;
    }
};

__global__ void k_tg_count(zk_tracegen_params p, uint64_t* counts) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= p.num_traces) return;
    CountEmit e;
    counts[k] = zk_tg_trace(p.seed, k, p.rank, p.world, p.max_depth, p.num_services, p.base_ts, e, p.global_ids != 0);
}

// inclusive prefix -> number of whole traces fitting `target`
__global__ void k_tg_cut(const uint64_t* incl, uint64_t ntr, uint64_t target, uint64_t* out) {
    uint64_t lo = 0, hi = ntr;  // count of k with incl[k] <= target
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (incl[mid] <= target)
            lo = mid + 1;
        else
            hi = mid;
    }
    out[0] = lo;
    out[1] = lo ? incl[lo - 1] : 0;
}

// global set: the record counts of this shard's traces k = k0 + j * step
__global__ void k_tg_gather(const uint64_t* counts, uint64_t k0, uint64_t step, uint64_t L, uint64_t* local) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < L) local[j] = counts[k0 + j * step];
}

__global__ void k_tg_write(zk_tracegen_params p, uint64_t ntr, uint64_t k0, uint64_t step, const uint64_t* incl,
                           const uint64_t* counts, ColEmit cols) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ntr) return;
    ColEmit e = cols;
    e.pos = incl[j] - counts[j];
    zk_tg_trace(p.seed, k0 + j * step, p.rank, p.world, p.max_depth, p.num_services, p.base_ts, e, p.global_ids != 0);
}

}  // namespace

hipError_t launch_tracegen(const zk_tracegen_params* p, const zk_span_cols* out, uint64_t cap,
                           uint64_t* n_records, uint64_t* n_traces, hipStream_t s) {
    const uint64_t T = p->num_traces;
    const bool global = p->global_ids != 0;
    *n_records = 0;
    *n_traces = 0;
    if (T == 0) return hipSuccess;
    uint64_t *counts = nullptr, *incl = nullptr, *cut = nullptr, *lcounts = nullptr, *lincl = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hipError_t e = hipMalloc(&counts, T * 8);
    if (e == hipSuccess) e = hipMalloc(&incl, T * 8);
    if (e == hipSuccess) e = hipMalloc(&cut, 16);
    if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, counts, incl, (int)T, s);
    if (e == hipSuccess) e = hipMalloc(&tmp, tmp_bytes);
    if (e == hipSuccess) {
        e = launch_checked("k_tg_count", k_tg_count, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, s, *p, counts);
    }
    if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, counts, incl, (int)T, s);
    // per-shard traces: the shard's record target, capped by the buffer; the global set: the WHOLE set's
    // target (the same cut on every rank), the shard's part is checked against the buffer below
    const uint64_t target = global ? (p->target_records ? p->target_records : ~0ull)
                                   : p->target_records ? (p->target_records < cap ? p->target_records : cap) : cap;
    if (e == hipSuccess) {
        e = launch_checked("k_tg_cut", k_tg_cut, dim3(1), dim3(1), 0, s, incl, T, target, cut);
    }
    uint64_t hc[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(hc, cut, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    uint64_t L = hc[0], k0 = 0, step = 1, nrec = hc[1];
    const uint64_t* wc = counts;
    const uint64_t* wi = incl;
    if (e == hipSuccess && global && L > 0) {
        step = p->world ? p->world : 1;
        k0 = zk_tg_global_k0(p->seed, p->rank, p->world);
        L = L > k0 ? (L - k0 + step - 1) / step : 0;
        nrec = 0;
        if (L > 0) {
            e = hipMalloc(&lcounts, L * 8);
            if (e == hipSuccess) e = hipMalloc(&lincl, L * 8);
            if (e == hipSuccess)
                e = launch_checked("k_tg_gather", k_tg_gather, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s,
                                   (const uint64_t*)counts, k0, step, L, lcounts);
            if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, lcounts, lincl, (int)L, s);
            if (e == hipSuccess) e = hipMemcpyAsync(&nrec, lincl + (L - 1), 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            wc = lcounts;
            wi = lincl;
        }
        if (e == hipSuccess && nrec > cap) e = hipErrorInvalidValue;  // the shard does not fit the buffer
    }
    if (e == hipSuccess && L > 0) {
        ColEmit c{(uint64_t*)out->trace_id, (uint64_t*)out->span_id, (uint64_t*)out->parent_id, (int64_t*)out->first_ts,
                  (int64_t*)out->last_ts,   (uint32_t*)out->service_id, (uint32_t*)out->flags, 0};
        e = launch_checked("k_tg_write", k_tg_write, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, *p, L, k0, step,
                           wi, wc, c);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    hipFree(counts);
    hipFree(incl);
    hipFree(cut);
    hipFree(lcounts);
    hipFree(lincl);
    hipFree(tmp);
    if (e == hipSuccess) {
        *n_traces = L;
        *n_records = nrec;
    }
    return e;
}

}  // namespace zk

extern "C" uint32_t zk_trace_shard(uint64_t trace_id, uint32_t world) { return zk_shard_of(trace_id, world); }

extern "C" zk_status zk_tracegen_host(const zk_tracegen_params* p, const zk_span_cols* out, uint64_t cap,
                                      uint64_t* n_records, uint64_t* n_traces) {
    if (!p || !n_records || !n_traces || p->max_depth == 0 || p->max_depth > ZK_TG_MAX_DEPTH ||
        p->num_services == 0 || (p->world && p->rank >= p->world))
        return ZK_ERR_INVALID_ARG;
    const bool write = out && out->trace_id;
    const bool global = p->global_ids != 0;
    // per-shard traces: stop at the shard's target (or the buffer); the global set: stop where the
    // WHOLE set reaches its target, keeping only this shard's traces (checked against the buffer)
    const uint64_t target = global ? (p->target_records ? p->target_records : ~0ull)
                            : p->target_records ? (p->target_records < cap || !write ? p->target_records : cap)
                                                : (write ? cap : ~0ull);
    const uint64_t step = global && p->world ? p->world : 1;
    const uint64_t k0 = global ? zk_tg_global_k0(p->seed, p->rank, p->world) : 0;
    uint64_t pos = 0, tot = 0, k = 0, mine = 0;
    for (; k < p->num_traces; ++k) {
        zk::CountEmit ce;
        const uint64_t c = zk_tg_trace(p->seed, k, p->rank, p->world, p->max_depth, p->num_services, p->base_ts, ce, global);
        if (tot + c > target) break;
        tot += c;
        if (global && (k < k0 || (k - k0) % step != 0)) continue;  // another shard's trace
        if (write) {
            if (pos + c > cap) return ZK_ERR_CAPACITY;
            zk::ColEmit e{(uint64_t*)out->trace_id, (uint64_t*)out->span_id, (uint64_t*)out->parent_id,
                          (int64_t*)out->first_ts,  (int64_t*)out->last_ts,  (uint32_t*)out->service_id,
                          (uint32_t*)out->flags,    pos};
            zk_tg_trace(p->seed, k, p->rank, p->world, p->max_depth, p->num_services, p->base_ts, e, global);
        }
        pos += c;
        ++mine;
    }
    *n_records = pos;
    *n_traces = mine;
    return ZK_OK;
}
