// zk_comm.h — collectives on a zk_comm (include/zkcomm.h) for the library's own handles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/zkcomm.h"

namespace zk {

enum CommType : int { kCommU8, kCommU32, kCommI64, kCommU64 };
enum CommOp : int { kCommSum, kCommMax };

// In-place all-reduce of `count` elements at buf, enqueued on s (the handle's stream, on `device`).
// On failure *err says why and the status is returned.
zk_status comm_allreduce(zk_comm* c, void* buf, uint64_t count, CommType t, CommOp op, int device, hipStream_t s,
                         std::string* err);
// recv[r * bytes, (r + 1) * bytes) = rank r's send buffer
zk_status comm_allgather(zk_comm* c, const void* send, void* recv, uint64_t bytes, int device, hipStream_t s,
                         std::string* err);
uint32_t comm_world(const zk_comm* c);

}  // namespace zk
