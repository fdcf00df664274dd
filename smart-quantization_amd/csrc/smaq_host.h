// Host-side helpers of smaq.hip shared with the packed codec (smaq_pack.hip). Internal.
#pragma once

#include <hip/hip_runtime.h>

#include "smq.h"

namespace smq {

// Full or sampled statistics of x into the workspace header (SmqSmaqStats at offset 0).
int prepare_stats(const void* x, int dtype, int64_t n, const SmqSmaqParams* p, void* ws,
                  size_t ws_bytes, hipStream_t st);
// Workspace bytes prepare_stats needs for n elements.
size_t smaq_stats_ws_bytes(int64_t n);
// Parameter block + dtype validation (sets the thread's last error).
int smaq_validate(const SmqSmaqParams* p, int dtype);

}  // namespace smq
