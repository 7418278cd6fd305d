// Workgroup-wide sort of (key, index) pairs in LDS, shared by the pool /
// island kernels (pool.hip) and the fused GA island kernel (ga_fused.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace vrpms {

// ---------------------------------------------------------------------------
// Block bitonic sort of M (power of two) (key, index) pairs in LDS, ascending
// lexicographically.  Every thread of the block must call it.
// ---------------------------------------------------------------------------
VRPMS_DEV void block_sort_pairs(uint64_t* sk, uint32_t* si, int M) {
  for (int size = 2; size <= M; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < M; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const uint64_t ki = sk[i], kj = sk[j];
          const uint32_t ii = si[i], ij = si[j];
          const bool gt = ki > kj || (ki == kj && ii > ij);
          if (gt == up) {
            sk[i] = kj;
            sk[j] = ki;
            si[i] = ij;
            si[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace vrpms
