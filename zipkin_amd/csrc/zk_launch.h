// zk_launch.h — every kernel launch of the library goes through launch_checked.
//
// The HIP runtime does not refuse a launch whose static + dynamic LDS exceeds the 160 KiB of a CU
// (round 2: k_part_scatter_lines dispatched with a 163,968-byte group segment at S = 1024 and
// faulted as an illegal memory access). launch_checked reads the kernel's static LDS and thread
// limit from its loaded code object (hipFuncGetAttributes, cached per kernel), refuses a launch
// that does not fit -- hipErrorLaunchOutOfResources, which the C ABI reports as ZK_ERR_CAPACITY
// with the reason from launch_refusal() -- raises the dynamic-LDS limit for launches above the
// runtime's 64 KiB default, launches with hipLaunchKernel and checks the launch status of EACH
// launch. Planners that have a fallback (the partition's line scatter vs item scatter) ask
// kernel_lds_fits() first, with the same attributes, instead of mirroring the kernel's LDS layout
// by hand.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <type_traits>
#include <utility>

namespace zk {

constexpr uint64_t kLdsPerCU = 160ull * 1024;  // MI355X: 160 KiB of LDS per CU (one workgroup may use all of it)

// pure host rule (CPU-tested through zk_internal_lds_plan): a workgroup fits when its static plus
// dynamic LDS fit one CU
inline bool lds_fits(uint64_t static_lds, uint64_t dyn_lds) { return static_lds + dyn_lds <= kLdsPerCU; }

// static LDS (group segment) and max threads per block of a kernel, from the loaded code object;
// cached per kernel pointer after the first query
hipError_t kernel_attrs(const void* fn, uint32_t* static_lds, uint32_t* max_threads);
// whether `fn` launched with `dyn_lds` bytes of dynamic LDS fits a CU (false also when the query fails)
bool kernel_lds_fits(const void* fn, uint64_t dyn_lds);
// the reason of this thread's last refused launch ("" after a launch that was not refused)
const char* launch_refusal();
void clear_launch_refusal();
void set_launch_refusal(const char* kernel, uint64_t static_lds, uint64_t dyn_lds, uint64_t threads,
                        uint32_t max_threads);
// a launch_checked refusal (reported as ZK_ERR_CAPACITY with launch_refusal() as the message)
inline bool is_refusal(hipError_t e) { return e == hipErrorLaunchOutOfResources && *launch_refusal(); }
// the message for a failed HIP call: the refusal's reason, or the runtime's error string
inline const char* launch_error_str(hipError_t e) { return is_refusal(e) ? launch_refusal() : hipGetErrorString(e); }
// raise the kernel's dynamic-LDS limit to 160 KiB once (needed above the runtime's 64 KiB default)
hipError_t allow_large_dyn_lds(const void* fn);

template <typename... P, typename... A>
hipError_t launch_checked(const char* name, void (*kernel)(P...), dim3 grid, dim3 block, size_t dyn_lds,
                          hipStream_t s, A&&... args) {
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    if ((uint64_t)grid.x * grid.y * grid.z == 0) return hipSuccess;  // nothing to run
    clear_launch_refusal();
    uint32_t st = 0, mt = 0;
    hipError_t e = kernel_attrs((const void*)kernel, &st, &mt);
    if (e != hipSuccess) return e;
    const uint64_t threads = (uint64_t)block.x * block.y * block.z;
    if (!lds_fits(st, dyn_lds) || threads > mt || threads == 0) {
        set_launch_refusal(name, st, dyn_lds, threads, mt);
        return hipErrorLaunchOutOfResources;
    }
    if (dyn_lds > 65536) {
        e = allow_large_dyn_lds((const void*)kernel);
        if (e != hipSuccess) return e;
    }
    // the arguments converted to the kernel's own parameter types, one pointer each
    std::tuple<std::decay_t<P>...> held(std::forward<A>(args)...);
    void* argv[sizeof...(P) > 0 ? sizeof...(P) : 1];
    std::apply(
        [&](auto&... x) {
            size_t i = 0;
            ((argv[i++] = (void*)&x), ...);
        },
        held);
    e = hipLaunchKernel((const void*)kernel, grid, block, argv, dyn_lds, s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace zk
