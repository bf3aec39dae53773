// zk_rl_internal.h — K1 glue of the realtime link store (zk_rl.hip) used by zk_api.cpp.
#pragma once
#include "zk_internal.h"
#include "zksketch.h"

namespace zk {
// size the link-item lists for a K1 launch of `grid` workgroups (list stride `stride`) over n
// records, point the JoinArgs at them and zero the spill list's count on stream s
zk_status rl_prepare_lists(zk_rl* r, uint32_t grid, uint64_t stride, uint64_t n, JoinArgs* a, hipStream_t s);
// append the items of the lists (counts: the K1 link counts) and of the spill list to the window
zk_status rl_consume_lists(zk_rl* r, const uint32_t* counts, uint32_t grid, uint64_t stride, uint64_t n);
const char* rl_error(const zk_rl* r);
int rl_device(const zk_rl* r);
uint32_t rl_services(const zk_rl* r);
void rl_set_stream(zk_rl* r, hipStream_t s);  // nullptr: back to the store's own stream
}  // namespace zk
