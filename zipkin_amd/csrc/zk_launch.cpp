// zk_launch.cpp — kernel attribute cache and launch refusals for launch_checked (zk_launch.h).
#include "zk_launch.h"

#include <stdio.h>

#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "zk_internal.h"
#include "zk_sketch_internal.h"

namespace zk {
namespace {

struct Attr {
    uint32_t static_lds;
    uint32_t max_threads;
};

std::mutex g_mu;
std::unordered_map<const void*, Attr> g_attrs;
std::unordered_set<const void*> g_large_dyn;
thread_local std::string t_refusal;

}  // namespace

hipError_t kernel_attrs(const void* fn, uint32_t* static_lds, uint32_t* max_threads) {
    {
        std::lock_guard<std::mutex> g(g_mu);
        const auto it = g_attrs.find(fn);
        if (it != g_attrs.end()) {
            *static_lds = it->second.static_lds;
            *max_threads = it->second.max_threads;
            return hipSuccess;
        }
    }
    hipFuncAttributes a{};
    const hipError_t e = hipFuncGetAttributes(&a, fn);
    if (e != hipSuccess) return e;
    const Attr x{(uint32_t)a.sharedSizeBytes, a.maxThreadsPerBlock > 0 ? (uint32_t)a.maxThreadsPerBlock : 1024u};
    std::lock_guard<std::mutex> g(g_mu);
    g_attrs[fn] = x;
    *static_lds = x.static_lds;
    *max_threads = x.max_threads;
    return hipSuccess;
}

bool kernel_lds_fits(const void* fn, uint64_t dyn_lds) {
    uint32_t st = 0, mt = 0;
    if (kernel_attrs(fn, &st, &mt) != hipSuccess) return false;
    return lds_fits(st, dyn_lds);
}

hipError_t allow_large_dyn_lds(const void* fn) {
    {
        std::lock_guard<std::mutex> g(g_mu);
        if (g_large_dyn.count(fn)) return hipSuccess;
    }
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPerCU);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(g_mu);
    g_large_dyn.insert(fn);
    return hipSuccess;
}

void set_launch_refusal(const char* kernel, uint64_t static_lds, uint64_t dyn_lds, uint64_t threads,
                        uint32_t max_threads) {
    char buf[320];
    snprintf(buf, sizeof(buf),
             "launch of %s refused: %llu B static + %llu B dynamic LDS (limit %llu B per CU), %llu threads "
             "(limit %u)",
             kernel, (unsigned long long)static_lds, (unsigned long long)dyn_lds, (unsigned long long)kLdsPerCU,
             (unsigned long long)threads, max_threads);
    t_refusal = buf;
}

const char* launch_refusal() { return t_refusal.c_str(); }

void clear_launch_refusal() {
    if (!t_refusal.empty()) t_refusal.clear();
}

}  // namespace zk

// internal (not in include/): the dynamic LDS the library asks for, at the largest configuration it
// accepts, for a CPU test of every dynamic-LDS launch against the kernels' static LDS.
// which: 0 = K2 k_link_scatter at S services; 1 = k_kv_sketch / candidates / merge at the widest
// accepted sketch; 2 = k_rt_sketch at p = kRtMaxP, m = 8
extern "C" uint64_t zk_internal_dyn_lds(uint32_t which, uint32_t S) {
    switch (which) {
        case 0: return zk::reduce_scatter_dyn_lds(S);
        case 1: return 16384ull * 4;  // zk_kv_create: depth * width <= 16384 counters
        case 2: return ((1ull << zk::kRtMaxP) / 4 + (uint64_t)zk::rt_nbins(8)) * 4;
    }
    return 0;
}
