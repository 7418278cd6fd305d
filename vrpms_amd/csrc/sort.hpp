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

// The same network with the stages of stride < 64 run inside wavefronts:
// wave w (< M / 64) holds elements 64w .. 64w + 63 in registers (lane l
// element 64w + l) and compare-exchanges with __shfl_xor, so only the
// log2(M / 64) * (log2(M / 64) + 1) / 2 stages of stride >= 64 cross the
// LDS with workgroup barriers (M = 512: 6 of 45).  Keys are unique (the
// index breaks ties), so the result equals block_sort_pairs'.  Needs
// 64 <= M <= blockDim.x; every thread of the block must call it.
VRPMS_DEV void block_sort_pairs_waves(uint64_t* sk, uint32_t* si, int M) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int i = (w << 6) | l;
  const bool own = w < (M >> 6);  // wave-uniform
  uint64_t k = 0;
  uint32_t v = 0;
  if (own) {
    k = sk[i];
    v = si[i];
  }
  for (int size = 2; size <= M; size <<= 1) {
    int stride = size >> 1;
    if (stride >= 64) {
      if (own) {
        sk[i] = k;
        si[i] = v;
      }
      __syncthreads();
      for (; stride >= 64; stride >>= 1) {
        for (int x = threadIdx.x; x < M; x += blockDim.x) {
          const int j = x ^ stride;
          if (j > x) {
            const bool up = (x & size) == 0;
            const uint64_t kx = sk[x], kj = sk[j];
            const uint32_t vx = si[x], vj = si[j];
            const bool gt = kx > kj || (kx == kj && vx > vj);
            if (gt == up) {
              sk[x] = kj;
              sk[j] = kx;
              si[x] = vj;
              si[j] = vx;
            }
          }
        }
        __syncthreads();
      }
      if (own) {
        k = sk[i];
        v = si[i];
      }
    }
    if (own) {
      for (; stride > 0; stride >>= 1) {
        const uint64_t ok = __shfl_xor(k, stride, 64);
        const uint32_t ov = __shfl_xor(v, stride, 64);
        const bool lower = (i & stride) == 0, up = (i & size) == 0;
        const bool other_less = ok < k || (ok == k && ov < v);
        if (lower == up ? other_less : !other_less) {
          k = ok;
          v = ov;
        }
      }
    }
  }
  __syncthreads();  // every wave's reads of the last LDS stage are done
  if (own) {
    sk[i] = k;
    si[i] = v;
  }
  __syncthreads();
}

}  // namespace vrpms
