// kme_internal.h -- what kme_multi.cpp (the N-engine drop-in) needs of an engine beyond kme.h: its
// stream and device, and stream-ordered credit re-splitting that queues behind epochs in flight
// (kme_credit_state / kme_credit_adjust refuse them; these are ordered by the engine stream instead).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "kme.h"

namespace kme {

hipStream_t engine_stream(kme_engine* e);
int engine_device(kme_engine* e);
const kme_config& engine_config(kme_engine* e);
// (bound, demand) per account into dev_out[0, 2A), after everything queued on the engine stream
kme_status credit_state_enqueue(kme_engine* e, int64_t* dev_out);
// the re-split from n blocks of `stride` words (shard-major), before anything queued later
kme_status credit_adjust_enqueue(kme_engine* e, const int64_t* dev_all, uint32_t n, uint32_t me, size_t stride);
// the oids of the resting orders (nothing in flight): a router's directory rebuilt after a restore
kme_status resting_oids(kme_engine* e, std::vector<int64_t>& out);
// a router's oid directory entries: each oid's last BUY/SELL went to `partition` (kme_router.cpp)
void router_seed(kme_router* r, const int64_t* oids, size_t n, uint32_t partition);

}  // namespace kme
