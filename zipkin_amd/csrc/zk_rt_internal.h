// zk_rt_internal.h — K1 glue of the realtime sketches (zk_rt_api.cpp) used by zk_api.cpp.
#pragma once
#include "zk_internal.h"
#include "zksketch.h"

namespace zk {
// size the item lists for a K1 launch of `grid` workgroups (list stride `stride`) over n records
// and point the JoinArgs at them; zeroes the spill list's count on stream s
zk_status rt_prepare_lists(zk_rt* r, uint32_t grid, uint64_t stride, uint64_t n, JoinArgs* a, hipStream_t s);
// partition the lists K1 (and the spill kernel) wrote and fold them into the sketch
zk_status rt_consume_lists(zk_rt* r, uint32_t grid, uint64_t stride, uint64_t n);
const char* rt_error(const zk_rt* r);
int rt_device(const zk_rt* r);
void rt_set_stream(zk_rt* r, hipStream_t s);  // nullptr: back to the sketch's own stream
}  // namespace zk
