// zk_comm.cpp — the RCCL communicator of include/zkcomm.h.
//
// The library opens RCCL at run time (dlopen) rather than linking it: a JVM host gets the ROCm
// install's librccl.so.1, and a process that already loaded one (torch ships its own copy under the
// same soname) shares it, so one process never holds two RCCL instances. The collectives are plain
// RCCL calls on the caller's stream: one int64 SUM for the dependency table's exchange form (the
// reference's cross-reducer .group.sum / .sum, ZipkinAggregateJob.scala:39-43), MAX/SUM for the
// sketches, an all-gather for the top-K candidate lists.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>
#include <string>

#include "zk_comm.h"
#include "zk_guard.h"

namespace {

struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string err;
};

Rccl& rccl_state() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (!r.h) {
            const char* e = dlerror();
            r.err = std::string("cannot open librccl.so.1: ") + (e ? e : "?");
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
        r.all_gather = (decltype(r.all_gather))dlsym(r.h, "ncclAllGather");
        r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
        if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.all_gather ||
            !r.error_string) {
            r.err = "librccl.so.1 lacks an entry point the library needs";
            r.h = nullptr;
        }
    });
    return r;
}

const Rccl* rccl() {
    const Rccl& r = rccl_state();
    return r.h ? &r : nullptr;
}

std::string nccl_msg(const Rccl* r, const char* what, ncclResult_t e) {
    return std::string(what) + ": " + r->error_string(e);
}

// why the last zk_comm_unique_id / zk_comm_create on this thread failed (no handle to hold it):
// zk_comm_last_error(NULL) returns it
thread_local std::string t_create_err;

}  // namespace

struct zk_comm {
    ncclComm_t comm = nullptr;
    uint32_t rank = 0, world = 0;
    int device = 0;
    std::string err;
};

namespace zk {

uint32_t comm_world(const zk_comm* c) { return c ? c->world : 0; }

zk_status comm_allreduce(zk_comm* c, void* buf, uint64_t count, CommType t, CommOp op, int device, hipStream_t s,
                         std::string* err) {
    const Rccl* r = rccl();
    if (!r) {
        *err = rccl_state().err;
        return ZK_ERR_UNSUPPORTED;
    }
    if (device != c->device) {
        *err = "the handle and the communicator are on different devices";
        return ZK_ERR_INVALID_ARG;
    }
    if (count == 0) return ZK_OK;
    const ncclDataType_t dt = t == kCommU8 ? ncclUint8 : t == kCommU32 ? ncclUint32 : t == kCommI64 ? ncclInt64 : ncclUint64;
    const ncclResult_t e = r->all_reduce(buf, buf, (size_t)count, dt, op == kCommSum ? ncclSum : ncclMax, c->comm, s);
    if (e != ncclSuccess) {
        *err = nccl_msg(r, "ncclAllReduce", e);
        c->err = *err;  // (the handle's zk_comm_last_error as well)
        return ZK_ERR_HIP;
    }
    return ZK_OK;
}

zk_status comm_allgather(zk_comm* c, const void* send, void* recv, uint64_t bytes, int device, hipStream_t s,
                         std::string* err) {
    const Rccl* r = rccl();
    if (!r) {
        *err = rccl_state().err;
        return ZK_ERR_UNSUPPORTED;
    }
    if (device != c->device) {
        *err = "the handle and the communicator are on different devices";
        return ZK_ERR_INVALID_ARG;
    }
    if (bytes == 0) return ZK_OK;
    const ncclResult_t e = r->all_gather(send, recv, (size_t)bytes, ncclUint8, c->comm, s);
    if (e != ncclSuccess) {
        *err = nccl_msg(r, "ncclAllGather", e);
        c->err = *err;
        return ZK_ERR_HIP;
    }
    return ZK_OK;
}

}  // namespace zk

extern "C" {

zk_status zk_comm_unique_id(uint8_t* id, uint64_t bytes) {
    ZK_GUARD_BEGIN
    if (!id || bytes < ZK_COMM_ID_BYTES) return ZK_ERR_INVALID_ARG;
    static_assert(sizeof(ncclUniqueId) == ZK_COMM_ID_BYTES, "RCCL unique id size");
    const Rccl* r = rccl();
    if (!r) {
        t_create_err = rccl_state().err;
        return ZK_ERR_UNSUPPORTED;
    }
    ncclUniqueId u;
    const ncclResult_t e = r->get_unique_id(&u);
    if (e != ncclSuccess) {
        t_create_err = nccl_msg(r, "ncclGetUniqueId", e);
        return ZK_ERR_HIP;
    }
    memcpy(id, &u, ZK_COMM_ID_BYTES);
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_comm_create(const uint8_t* id, uint64_t bytes, uint32_t rank, uint32_t world, int32_t device,
                         zk_comm** out) {
    ZK_GUARD_BEGIN
    if (!out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    if (!id || bytes < ZK_COMM_ID_BYTES || world == 0 || rank >= world || world > 256) return ZK_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device < 0 || device >= ndev) {
        t_create_err = "no HIP device " + std::to_string(device);
        return ZK_ERR_NO_DEVICE;
    }
    const Rccl* r = rccl();
    if (!r) {
        t_create_err = rccl_state().err;
        return ZK_ERR_UNSUPPORTED;
    }
    if (hipSetDevice(device) != hipSuccess) {
        t_create_err = "hipSetDevice failed";
        return ZK_ERR_HIP;
    }
    ncclUniqueId u;
    memcpy(&u, id, ZK_COMM_ID_BYTES);
    zk_comm* c = new zk_comm();
    c->rank = rank;
    c->world = world;
    c->device = device;
    const ncclResult_t e = r->comm_init_rank(&c->comm, (int)world, u, (int)rank);
    if (e != ncclSuccess) {
        t_create_err = nccl_msg(r, "ncclCommInitRank", e) + " (rank " + std::to_string(rank) + " of " +
                       std::to_string(world) + ")";
        delete c;
        return ZK_ERR_HIP;
    }
    *out = c;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_comm_destroy(zk_comm* c) {
    ZK_GUARD_BEGIN
    if (!c) return ZK_ERR_INVALID_ARG;
    const Rccl* r = rccl();
    if (r && c->comm) {
        hipSetDevice(c->device);
        r->comm_destroy(c->comm);
    }
    delete c;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_comm_last_error(const zk_comm* c) {
    if (!c) return !t_create_err.empty() ? t_create_err.c_str() : rccl() ? "null communicator" : rccl_state().err.c_str();
    return c->err.c_str();
}

}  // extern "C"
