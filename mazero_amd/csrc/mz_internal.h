// mz_internal.h — what the driver-glue translation unit (mzdriver.hip) needs from the tree
// library (mzmcts.hip).  Hidden symbols: not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mzmcts.h"

#define MZ_HIDDEN __attribute__((visibility("hidden")))

extern "C" {
// Record `msg` as the calling thread's mz_last_error() and return `code`.
MZ_HIDDEN int mz_internal_fail(int code, const char *msg);
// Make the handle's device current and report its batch size, action count and stream.
MZ_HIDDEN int mz_internal_launch_info(mz_batch *b, int *B, int *A, hipStream_t *stream);
}  // extern "C"
