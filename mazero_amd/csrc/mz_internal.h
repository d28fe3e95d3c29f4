// mz_internal.h — what the driver-glue and consumer translation units (mzdriver.hip,
// mzconsume.hip) need from the tree library (mzmcts.hip).  Hidden symbols: not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mzmcts.h"

#define MZ_HIDDEN __attribute__((visibility("hidden")))

extern "C" {
// Record `msg` as the calling thread's mz_last_error() and return `code`.
MZ_HIDDEN int mz_internal_fail(int code, const char *msg);
// Make the handle's device current and report its batch size, action count and stream.
MZ_HIDDEN int mz_internal_launch_info(mz_batch *b, int *B, int *A, hipStream_t *stream);
// after a launch on the handle's stream: record its order event (mz_set_stream)
MZ_HIDDEN void mz_internal_enqueued(mz_batch *b);
// agent_num of the handle (0 for a null handle).
MZ_HIDDEN int mz_internal_agent_num(mz_batch *b);
}  // extern "C"
