// zk_rt_api.cpp — C ABI of the realtime span sketches (include/zksketch.h, zk_rt_*) and the
// K1 glue that feeds them from a bound dependency ctx (zk_rt_bind, zk_api.cpp).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <string>
#include <vector>

#include "zk_comm.h"
#include "zk_guard.h"
#include "zk_launch.h"
#include "zk_internal.h"
#include "zk_rt_internal.h"
#include "zk_sketch_internal.h"
#include "zksketch.h"

using namespace zk;

struct zk_rt {
    int device = 0;
    hipStream_t stream = nullptr;      // current stream (the bound ctx's while bound)
    hipStream_t own = nullptr;         // private stream, if created
    uint32_t S = 0, p = 14, m = 7, nbins = 0;
    uint64_t seed = 0;
    uint32_t cus = 256;
    uint8_t* regs = nullptr;           // [S][2^p]
    uint32_t* hist = nullptr;          // [S][nbins]
    unsigned long long* dropped = nullptr;  // [0] service range, [1] duration range, [2] scratch
    // K1 item lists: list w at w * stride, count[w]; list `grid` = spill items (capacity >= records)
    uint64_t* pay = nullptr;
    uint32_t* svc = nullptr;
    uint32_t* count = nullptr;
    uint64_t list_cap = 0;             // items
    uint32_t count_cap = 0;
    // partition + units
    uint64_t* sorted = nullptr;
    uint64_t sorted_cap = 0;
    uint64_t* seg = nullptr;
    uint32_t* unit_base = nullptr;
    void* part = nullptr;
    uint64_t part_bytes = 0;
    // merged-span staging
    void* stage = nullptr;
    uint64_t stage_cap = 0;
    // all-service queries (k_rt_query): quantiles, its output and the pinned host mirror
    double* q_dev = nullptr;
    unsigned long long* q_out = nullptr;
    unsigned long long* q_host = nullptr;
    std::string err;
};

namespace {

zk_status rfail(zk_rt* r, zk_status s, const std::string& m) {
    if (r) r->err = m;
    return s;
}

#define RT_HIP(rt, call)                                                                                  \
    do {                                                                                                  \
        hipError_t _e = (call);                                                                           \
        if (_e != hipSuccess)                                                                          \
            return rfail(rt, is_refusal(_e) ? ZK_ERR_CAPACITY : ZK_ERR_HIP,                          \
                        std::string(#call) + ": " + launch_error_str(_e));                             \
    } while (0)

template <class T>
zk_status grow(zk_rt* r, T** p, uint64_t* cap, uint64_t need, const char* what) {
    if (need <= *cap && *p) return ZK_OK;
    if (*p) RT_HIP(r, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void**)p, need * sizeof(T) + 256) != hipSuccess) return rfail(r, ZK_ERR_HIP, what);
    *cap = need;
    return ZK_OK;
}

// partition service-contiguous, then one sketch workgroup per unit
zk_status sketch_items(zk_rt* r, const PartitionPlan& plan, bool lists, const uint32_t* svc, const uint64_t* pay,
                       uint64_t n_or_stride, const uint32_t* counts, uint64_t max_items) {
    const uint64_t pb = partition_scratch_bytes(plan);
    if (pb > r->part_bytes) {
        if (r->part) RT_HIP(r, hipFree(r->part));
        r->part = nullptr;
        RT_HIP(r, hipMalloc(&r->part, pb));
        r->part_bytes = pb;
    }
    zk_status st = grow(r, &r->sorted, &r->sorted_cap, max_items ? max_items : 1, "sorted items");
    if (st != ZK_OK) return st;
    if (lists)
        RT_HIP(r, launch_partition_lists(plan, svc, pay, n_or_stride, counts, r->sorted, r->seg, r->dropped + 2, r->part,
                                         r->stream));
    else
        RT_HIP(r, launch_partition(plan, svc, pay, n_or_stride, r->sorted, r->seg, r->dropped + 2, r->part, r->stream));
    RT_HIP(r, launch_unit_plan(r->seg, r->S, kRtUnitItems, r->unit_base, r->stream));
    RtArgs a{};
    a.S = r->S;
    a.p = r->p;
    a.m = r->m;
    a.nbins = r->nbins;
    a.regs = r->regs;
    a.hist = r->hist;
    a.items = r->sorted;
    a.seg = r->seg;
    a.unit_base = r->unit_base;
    a.unit_items = kRtUnitItems;
    a.max_units = (uint32_t)((max_items + kRtUnitItems - 1) / kRtUnitItems + r->S);
    RT_HIP(r, launch_rt_sketch(a, r->stream));
    return ZK_OK;
}

// z = sum of 2^(64 - M[j]) = 2^64 * sum 2^-M[j], exact (k_rt_query counts it on the device)
double hll_estimate(unsigned __int128 z, uint64_t zeros, uint32_t p) {
    const uint32_t mm = 1u << p;
    const double Z = ldexp((double)z, -64);
    const double m = (double)mm;
    double alpha;
    if (mm == 16)
        alpha = 0.673;
    else if (mm == 32)
        alpha = 0.697;
    else if (mm == 64)
        alpha = 0.709;
    else
        alpha = 0.7213 / (1.0 + 1.079 / m);
    double e = alpha * m * m / Z;
    if (e <= 2.5 * m && zeros > 0) e = m * log(m / (double)zeros);  // linear counting
    return e;
}

void bin_bounds(uint32_t b, uint32_t m, int64_t* lo, int64_t* hi) {
    if (b < (1u << m)) {
        *lo = *hi = b;
        return;
    }
    const uint32_t g = b >> m, mant = b & ((1u << m) - 1u);
    const uint32_t e = g + m - 1u;  // exponent of the bin's values
    const uint64_t l = ((1ull << m) | mant) << (e - m);
    *lo = (int64_t)l;
    *hi = (int64_t)(l + (1ull << (e - m)) - 1ull);
}

struct Centroid {
    double mean, weight;
};

// A merging t-digest (Dunning's k1 scale function, compression delta) over one service's histogram:
// the nonzero bins in ascending order, each a point at its midpoint with its count as weight, are
// merged into a centroid while the centroid's quantile span stays within one unit of
// k(q) = delta / (2 pi) * asin(2q - 1). A bin is never split (its values lie in [lo, hi]), so a bin
// heavier than the bound is a centroid of its own. The input is the exact (all-reduced) histogram,
// so the digest is identical on every rank and for every world size and batch order.
void build_tdigest(const std::vector<uint32_t>& h, uint32_t m, double delta, std::vector<Centroid>* out,
                   int64_t* vmin, int64_t* vmax, uint64_t* total) {
    out->clear();
    uint64_t N = 0;
    for (uint32_t c : h) N += c;
    *total = N;
    *vmin = *vmax = 0;
    if (!N) return;
    const double pi = 3.14159265358979323846;
    auto k_of = [&](double q) { return delta / (2.0 * pi) * asin(2.0 * q - 1.0); };
    auto q_of = [&](double k) {
        const double x = 2.0 * pi * k / delta;
        return x >= pi / 2 ? 1.0 : (sin(x) + 1.0) / 2.0;
    };
    bool first = true;
    double before = 0.0, cw = 0.0, cs = 0.0, qlim = 0.0;
    for (uint32_t b = 0; b < (uint32_t)h.size(); ++b) {
        if (!h[b]) continue;
        int64_t lo, hi;
        bin_bounds(b, m, &lo, &hi);
        if (first) *vmin = lo;
        *vmax = hi;
        const double w = (double)h[b], x = 0.5 * ((double)lo + (double)hi);
        if (!first && (before + cw + w) / (double)N <= qlim) {
            cw += w;
            cs += w * x;
            continue;
        }
        if (!first) {
            out->push_back({cs / cw, cw});
            before += cw;
        }
        first = false;
        cw = w;
        cs = w * x;
        qlim = q_of(k_of(before / (double)N) + 1.0);
    }
    out->push_back({cs / cw, cw});
}

// t-digest quantile (nearest centroids' centers, linearly interpolated; the ends interpolate to
// the smallest / largest bin bound)
double tdigest_quantile(const std::vector<Centroid>& c, int64_t vmin, int64_t vmax, uint64_t N, double q) {
    if (c.empty() || !N) return 0.0;
    if (c.size() == 1) return c[0].mean;
    const double idx = q * (double)N;
    if (idx <= c[0].weight / 2) {
        const double t = c[0].weight > 0 ? idx / (c[0].weight / 2) : 0.0;
        return (double)vmin + t * (c[0].mean - (double)vmin);
    }
    double cum = 0.0;
    for (size_t i = 0; i + 1 < c.size(); ++i) {
        const double a = cum + c[i].weight / 2, b = cum + c[i].weight + c[i + 1].weight / 2;
        if (idx <= b) {
            const double t = b > a ? (idx - a) / (b - a) : 0.0;
            return c[i].mean + t * (c[i + 1].mean - c[i].mean);
        }
        cum += c[i].weight;
    }
    const Centroid& l = c.back();
    const double a = (double)N - l.weight / 2;
    const double t = l.weight > 0 ? (idx - a) / (l.weight / 2) : 0.0;
    return l.mean + (t > 1.0 ? 1.0 : t) * ((double)vmax - l.mean);
}

}  // namespace

namespace zk {

zk_status rt_prepare_lists(zk_rt* r, uint32_t grid, uint64_t stride, uint64_t n, JoinArgs* a, hipStream_t s) {
    const uint64_t need = (uint64_t)grid * stride + n;
    if (need > r->list_cap || !r->pay) {
        if (r->pay) RT_HIP(r, hipFree(r->pay));
        if (r->svc) RT_HIP(r, hipFree(r->svc));
        r->pay = nullptr;
        r->svc = nullptr;
        r->list_cap = 0;
        RT_HIP(r, hipMalloc(&r->pay, need * 8));
        RT_HIP(r, hipMalloc(&r->svc, need * 4));
        r->list_cap = need;
    }
    if (grid + 1 > r->count_cap || !r->count) {
        if (r->count) RT_HIP(r, hipFree(r->count));
        r->count = nullptr;
        RT_HIP(r, hipMalloc(&r->count, (uint64_t)(grid + 1) * 4));
        r->count_cap = grid + 1;
    }
    RT_HIP(r, hipMemsetAsync(r->count + grid, 0, 4, s));
    a->rt_pay = r->pay;
    a->rt_svc = r->svc;
    a->rt_count = r->count;
    a->rt_dropped = r->dropped;
    a->rt_spill_cap = n;
    a->rt_seed = r->seed;
    a->rt_p = r->p;
    return ZK_OK;
}

zk_status rt_consume_lists(zk_rt* r, uint32_t grid, uint64_t stride, uint64_t n) {
    const PartitionPlan plan = partition_plan_lists(grid + 1, r->S);
    return sketch_items(r, plan, true, r->svc, r->pay, stride, r->count, n);
}

const char* rt_error(const zk_rt* r) { return r->err.c_str(); }
int rt_device(const zk_rt* r) { return r->device; }
// Moving the sketch to another stream (zk_rt_bind) first drains the one it was on: work queued
// there (the zeroing of zk_rt_create/zk_rt_reset on the private stream) would otherwise race with
// the first kernels on the new one -- a zeroing that lands after the first sketch pass wipes it.
void rt_set_stream(zk_rt* r, hipStream_t s) {
    hipStream_t ns = s ? s : r->own;
    if (ns != r->stream) {
        if (r->stream) (void)hipStreamSynchronize(r->stream);
        r->stream = ns;
    }
}

// every service's HLL sums and the bins of up to kRtQueryMaxQ quantiles, one kernel and one copy
// into the pinned mirror: row s of r->q_host = [z_lo, z_hi, zeros, N, bins...]
zk_status rt_query(zk_rt* r, const double* q, uint32_t nq) {
    if (!r->q_out) {
        RT_HIP(r, hipMalloc(&r->q_dev, kRtQueryMaxQ * sizeof(double)));
        RT_HIP(r, hipMalloc(&r->q_out, (uint64_t)r->S * (4 + kRtQueryMaxQ) * 8));
        RT_HIP(r, hipHostMalloc((void**)&r->q_host, (uint64_t)r->S * (4 + kRtQueryMaxQ) * 8, hipHostMallocDefault));
    }
    if (nq) RT_HIP(r, hipMemcpyAsync(r->q_dev, q, nq * sizeof(double), hipMemcpyHostToDevice, r->stream));
    RT_HIP(r, launch_rt_query(r->regs, r->hist, r->S, r->p, r->nbins, r->q_dev, nq, r->q_out, r->stream));
    RT_HIP(r, hipMemcpyAsync(r->q_host, r->q_out, (uint64_t)r->S * (4 + nq) * 8, hipMemcpyDeviceToHost, r->stream));
    RT_HIP(r, hipStreamSynchronize(r->stream));
    return ZK_OK;
}

}  // namespace zk

extern "C" {

zk_status zk_rt_create(const zk_rt_config* cfg, zk_rt** out) {
    ZK_GUARD_BEGIN
    if (!cfg || !out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    const uint32_t S = cfg->num_services;
    const uint32_t p = cfg->hll_p ? cfg->hll_p : 14, m = cfg->sub_bits ? cfg->sub_bits : 7;
    if (S == 0 || S > 4096 || p < 4 || p > kRtMaxP || m < 2 || m > 8) return ZK_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ZK_ERR_NO_DEVICE;
    if (cfg->device < 0 || cfg->device >= ndev) return ZK_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return ZK_ERR_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZK_ERR_NO_DEVICE;
    zk_rt* r = new zk_rt();
    r->device = cfg->device;
    r->S = S;
    r->p = p;
    r->m = m;
    r->nbins = rt_nbins(m);
    r->seed = cfg->seed;
    r->cus = prop.multiProcessorCount > 0 ? (uint32_t)prop.multiProcessorCount : 256;
    hipError_t e = hipSetDevice(r->device);
    if (e == hipSuccess) {
        if (cfg->stream) {
            r->own = (hipStream_t)cfg->stream;
        } else {
            e = hipStreamCreateWithFlags(&r->own, hipStreamNonBlocking);
        }
        r->stream = r->own;
    }
    if (e == hipSuccess) e = hipMalloc(&r->regs, (uint64_t)S << p);
    if (e == hipSuccess) e = hipMalloc(&r->hist, (uint64_t)S * r->nbins * 4);
    if (e == hipSuccess) e = hipMalloc(&r->dropped, 4 * 8);
    if (e == hipSuccess) e = hipMalloc(&r->seg, (uint64_t)(S + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&r->unit_base, (uint64_t)(S + 1) * 4);
    zk_status st = e == hipSuccess ? zk_rt_reset(r) : ZK_ERR_HIP;
    if (st != ZK_OK) {
        zk_rt_destroy(r);
        return st;
    }
    *out = r;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_destroy(zk_rt* r) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    hipSetDevice(r->device);
    if (r->stream) hipStreamSynchronize(r->stream);
    for (void* q : {(void*)r->regs, (void*)r->hist, (void*)r->dropped, (void*)r->pay, (void*)r->svc, (void*)r->count,
                    (void*)r->sorted, (void*)r->seg, (void*)r->unit_base, r->part, r->stage, (void*)r->q_dev,
                    (void*)r->q_out})
        if (q) hipFree(q);
    if (r->q_host) hipHostFree(r->q_host);
    // a caller-provided stream is not ours to destroy; a private one is
    delete r;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_rt_last_error(const zk_rt* r) { return r ? r->err.c_str() : "null handle"; }

zk_status zk_rt_geometry(const zk_rt* r, uint32_t* registers, uint32_t* bins) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    if (registers) *registers = 1u << r->p;
    if (bins) *bins = r->nbins;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_reset(zk_rt* r) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    RT_HIP(r, hipSetDevice(r->device));
    RT_HIP(r, hipMemsetAsync(r->regs, 0, (uint64_t)r->S << r->p, r->stream));
    RT_HIP(r, hipMemsetAsync(r->hist, 0, (uint64_t)r->S * r->nbins * 4, r->stream));
    RT_HIP(r, hipMemsetAsync(r->dropped, 0, 4 * 8, r->stream));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_accumulate_merged(zk_rt* r, const uint32_t* service_id, const uint64_t* trace_id,
                                  const int64_t* duration, uint64_t n, uint32_t flags) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    if (n == 0) return ZK_OK;
    if (!service_id || !trace_id || !duration) return rfail(r, ZK_ERR_INVALID_ARG, "null input");
    if (n >= (1ull << 32)) return rfail(r, ZK_ERR_INVALID_ARG, "batch of >= 2^32 items");
    RT_HIP(r, hipSetDevice(r->device));
    // staging: [svc u32 n | tid u64 n | dur i64 n] (host input) + items [svc u32 n | pay u64 n]
    const uint64_t a4 = (n * 4 + 255) & ~255ull, a8 = (n * 8 + 255) & ~255ull;
    const uint64_t need = 2 * a4 + 3 * a8;
    if (need > r->stage_cap) {
        if (r->stage) RT_HIP(r, hipFree(r->stage));
        r->stage = nullptr;
        RT_HIP(r, hipMalloc(&r->stage, need));
        r->stage_cap = need;
    }
    uint8_t* base = (uint8_t*)r->stage;
    uint32_t* isvc = (uint32_t*)base;
    uint64_t* ipay = (uint64_t*)(base + a4);
    if (!(flags & ZK_BATCH_DEVICE_PTRS)) {
        uint32_t* ds = (uint32_t*)(base + a4 + a8);
        uint64_t* dt = (uint64_t*)(base + 2 * a4 + a8);
        int64_t* dd = (int64_t*)(base + 2 * a4 + 2 * a8);
        RT_HIP(r, hipMemcpyAsync(ds, service_id, n * 4, hipMemcpyHostToDevice, r->stream));
        RT_HIP(r, hipMemcpyAsync(dt, trace_id, n * 8, hipMemcpyHostToDevice, r->stream));
        RT_HIP(r, hipMemcpyAsync(dd, duration, n * 8, hipMemcpyHostToDevice, r->stream));
        // host inputs are borrowed for the call only (zkagg.h): wait until the copies have read them
        RT_HIP(r, hipStreamSynchronize(r->stream));
        service_id = ds;
        trace_id = dt;
        duration = dd;
    }
    RT_HIP(r, launch_rt_items(service_id, trace_id, duration, n, r->S, r->p, r->seed, isvc, ipay, r->dropped,
                              r->stream));
    const PartitionPlan plan = partition_plan(n, r->S, r->cus);
    return sketch_items(r, plan, false, isvc, ipay, n, nullptr, n);
    ZK_GUARD_END
}

zk_status zk_rt_read(zk_rt* r, uint8_t* registers, uint32_t* histogram) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    RT_HIP(r, hipSetDevice(r->device));
    if (registers) RT_HIP(r, hipMemcpyAsync(registers, r->regs, (uint64_t)r->S << r->p, hipMemcpyDeviceToHost, r->stream));
    if (histogram)
        RT_HIP(r, hipMemcpyAsync(histogram, r->hist, (uint64_t)r->S * r->nbins * 4, hipMemcpyDeviceToHost, r->stream));
    RT_HIP(r, hipStreamSynchronize(r->stream));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_distinct_traces(zk_rt* r, double* estimate) {
    ZK_GUARD_BEGIN
    if (!r || !estimate) return ZK_ERR_INVALID_ARG;
    RT_HIP(r, hipSetDevice(r->device));
    const zk_status st = rt_query(r, nullptr, 0);
    if (st != ZK_OK) return st;
    for (uint32_t s = 0; s < r->S; ++s) {
        const unsigned long long* o = r->q_host + (uint64_t)s * 4;
        estimate[s] = hll_estimate(((unsigned __int128)o[1] << 64) | o[0], o[2], r->p);
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_quantiles_all(zk_rt* r, const double* q, uint32_t nq, int64_t* lo, int64_t* hi, uint64_t* count) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    if (nq && (!q || !lo || !hi)) return rfail(r, ZK_ERR_INVALID_ARG, "null array");
    for (uint32_t i = 0; i < nq; ++i)
        if (!(q[i] >= 0.0 && q[i] <= 1.0)) return rfail(r, ZK_ERR_INVALID_ARG, "quantile outside [0, 1]");
    RT_HIP(r, hipSetDevice(r->device));
    for (uint32_t i0 = 0; i0 < nq || (i0 == 0 && count); i0 += kRtQueryMaxQ) {
        const uint32_t k = nq - i0 < kRtQueryMaxQ ? nq - i0 : kRtQueryMaxQ;
        const zk_status st = rt_query(r, q + i0, k);
        if (st != ZK_OK) return st;
        for (uint32_t s = 0; s < r->S; ++s) {
            const unsigned long long* o = r->q_host + (uint64_t)s * (4 + k);
            if (count) count[s] = o[3];
            for (uint32_t i = 0; i < k; ++i) {
                int64_t* l = lo + (uint64_t)s * nq + i0 + i;
                int64_t* h = hi + (uint64_t)s * nq + i0 + i;
                if (o[3])
                    bin_bounds((uint32_t)o[4 + i], r->m, l, h);
                else
                    *l = *h = 0;
            }
        }
        if (!nq) break;
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_quantiles(zk_rt* r, uint32_t service, const double* q, uint32_t nq, int64_t* lo, int64_t* hi,
                          uint64_t* count) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    if (service >= r->S) return rfail(r, ZK_ERR_SERVICE_RANGE, "service >= S");
    if (nq && (!q || !lo || !hi)) return rfail(r, ZK_ERR_INVALID_ARG, "null array");
    for (uint32_t i = 0; i < nq; ++i)
        if (!(q[i] >= 0.0 && q[i] <= 1.0)) return rfail(r, ZK_ERR_INVALID_ARG, "quantile outside [0, 1]");
    RT_HIP(r, hipSetDevice(r->device));
    std::vector<uint32_t> h(r->nbins);
    RT_HIP(r, hipMemcpyAsync(h.data(), r->hist + (uint64_t)service * r->nbins, (uint64_t)r->nbins * 4,
                             hipMemcpyDeviceToHost, r->stream));
    RT_HIP(r, hipStreamSynchronize(r->stream));
    uint64_t N = 0;
    for (uint32_t c : h) N += c;
    if (count) *count = N;
    for (uint32_t i = 0; i < nq; ++i) {
        lo[i] = hi[i] = 0;
        if (!N) continue;
        uint64_t rank = (uint64_t)ceil(q[i] * (double)N);  // nearest rank, 1-based
        if (rank < 1) rank = 1;
        if (rank > N) rank = N;
        uint64_t cum = 0;
        for (uint32_t b = 0; b < r->nbins; ++b) {
            cum += h[b];
            if (cum >= rank) {
                bin_bounds(b, r->m, &lo[i], &hi[i]);
                break;
            }
        }
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_tdigest(zk_rt* r, uint32_t service, double compression, double* mean, double* weight, uint32_t cap,
                        uint32_t* n, const double* q, uint32_t nq, double* value, uint64_t* count) {
    ZK_GUARD_BEGIN
    if (!r || !n) return ZK_ERR_INVALID_ARG;
    if (service >= r->S) return rfail(r, ZK_ERR_SERVICE_RANGE, "service >= S");
    if (!(compression >= 10.0 && compression <= 10000.0)) return rfail(r, ZK_ERR_INVALID_ARG, "compression outside [10, 10000]");
    if (nq && (!q || !value)) return rfail(r, ZK_ERR_INVALID_ARG, "null array");
    for (uint32_t i = 0; i < nq; ++i)
        if (!(q[i] >= 0.0 && q[i] <= 1.0)) return rfail(r, ZK_ERR_INVALID_ARG, "quantile outside [0, 1]");
    RT_HIP(r, hipSetDevice(r->device));
    std::vector<uint32_t> h(r->nbins);
    RT_HIP(r, hipMemcpyAsync(h.data(), r->hist + (uint64_t)service * r->nbins, (uint64_t)r->nbins * 4,
                             hipMemcpyDeviceToHost, r->stream));
    RT_HIP(r, hipStreamSynchronize(r->stream));
    std::vector<Centroid> c;
    int64_t vmin, vmax;
    uint64_t N;
    build_tdigest(h, r->m, compression, &c, &vmin, &vmax, &N);
    if (count) *count = N;
    *n = (uint32_t)c.size();
    if (mean || weight) {
        if (cap < c.size()) return rfail(r, ZK_ERR_CAPACITY, "centroid capacity smaller than the digest");
        for (size_t i = 0; i < c.size(); ++i) {
            if (mean) mean[i] = c[i].mean;
            if (weight) weight[i] = c[i].weight;
        }
    }
    for (uint32_t i = 0; i < nq; ++i) value[i] = tdigest_quantile(c, vmin, vmax, N, q[i]);
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_partial(zk_rt* r, void** registers, uint64_t* rb, void** histogram, uint64_t* hb) {
    ZK_GUARD_BEGIN
    if (!r || !registers || !rb || !histogram || !hb) return ZK_ERR_INVALID_ARG;
    *registers = r->regs;
    *rb = (uint64_t)r->S << r->p;
    *histogram = r->hist;
    *hb = (uint64_t)r->S * r->nbins * 4;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_dropped(zk_rt* r, uint64_t* service_range, uint64_t* duration_range) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    unsigned long long d[4];
    RT_HIP(r, hipSetDevice(r->device));
    RT_HIP(r, hipMemcpyAsync(d, r->dropped, sizeof(d), hipMemcpyDeviceToHost, r->stream));
    RT_HIP(r, hipStreamSynchronize(r->stream));
    if (service_range) *service_range = d[0];
    if (duration_range) *duration_range = d[1];
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_rt_allreduce(zk_rt* r, zk_comm* comm) {
    ZK_GUARD_BEGIN
    if (!r) return ZK_ERR_INVALID_ARG;
    if (!comm) return rfail(r, ZK_ERR_INVALID_ARG, "null communicator");
    RT_HIP(r, hipSetDevice(r->device));
    // registers by MAX, bins and the two drop counters by SUM, on the sketch's (bound ctx's) stream
    zk_status st = comm_allreduce(comm, r->regs, (uint64_t)r->S << r->p, kCommU8, kCommMax, r->device, r->stream, &r->err);
    if (st == ZK_OK)
        st = comm_allreduce(comm, r->hist, (uint64_t)r->S * r->nbins, kCommU32, kCommSum, r->device, r->stream, &r->err);
    if (st == ZK_OK) st = comm_allreduce(comm, r->dropped, 2, kCommU64, kCommSum, r->device, r->stream, &r->err);
    return st;
    ZK_GUARD_END
}

}  // extern "C"
