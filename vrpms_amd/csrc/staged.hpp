// Host entry of the LDS-staged row-layout scoring kernels (eval_staged.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ctx.hpp"

#define VRPMS_HOST_DEV_INLINE __host__ __device__ __forceinline__

namespace vrpms {

// True when the staged kernel's LDS tables (depot legs, demands, fleet) and
// one tile fit a workgroup; otherwise vrpms_eval uses eval_generic.
bool staged_fits(const vrpms_ctx* ctx);

// Score C row-layout tours (uint8 / uint16 elements, row stride ld) with the
// staged kernel.  Same outputs and error behaviour as vrpms_eval.
int launch_staged(vrpms_ctx* ctx, const void* perms, int perm_bytes, int64_t C, int n,
                  int64_t ld, uint64_t* keys, int32_t* sums, int32_t* maxs, int32_t* unv,
                  hipStream_t s);

}  // namespace vrpms
