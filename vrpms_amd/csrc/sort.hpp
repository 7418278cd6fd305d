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

// x from lane (lane ^ stride), stride a compile-time power of two after
// unrolling: DPP quad_perm (1, 2) and row_ror:8 (8) ride on a VALU move,
// ds_swizzle's xor mode (4, 16) needs no address; only 32 crosses halves
// through ds_bpermute.
VRPMS_DEV uint32_t xor_lanes(uint32_t x, int stride) {
  switch (stride) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
    case 4: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x101F);
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);
    case 16: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);
    default: return (uint32_t)__shfl_xor((int)x, stride, 64);
  }
}

// Bitonic sort of one (key, index) pair per lane across a wavefront
// (ascending by lane; 21 compare-exchange stages over xor_lanes).  All 64
// lanes must be active.
VRPMS_DEV void wave_sort64(uint64_t& k, uint32_t& v) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint64_t ok = ((uint64_t)xor_lanes((uint32_t)(k >> 32), stride) << 32) |
                          xor_lanes((uint32_t)k, stride);
      const uint32_t ov = xor_lanes(v, stride);
      const bool lower = (l & stride) == 0, up = (l & size) == 0;
      const bool other_less = ok < k || (ok == k && ov < v);
      if (lower == up ? other_less : !other_less) {
        k = ok;
        v = ov;
      }
    }
  }
}

VRPMS_DEV bool pair_less(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// (mu + lambda) selection by merge ranks instead of a full sort of 2P pairs:
// the P parents pk[0..P) are already ascending by (key, slot) (the previous
// selection's output), the P children ck[0..P) (indices P + c) are sorted in
// runs of 64 inside wavefronts, and every pair's final position is its
// position in its own run plus a lower bound in each other run.  Pairs are
// unique (the index breaks ties), so sk[0..P) / si[0..P) equal the first P of
// block_sort_pairs over the 2P pairs.  rk / ri hold the child runs
// (64 * ceil(P / 64) entries); needs blockDim.x >= 64 * ceil(P / 64).
// Every thread of the block must call it.
VRPMS_DEV void merge_select(const uint64_t* pk, const uint64_t* ck, int P, uint64_t* rk,
                            uint32_t* ri, uint64_t* sk, uint32_t* si) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int R = (P + 63) >> 6;
  if (w < R) {  // wave-uniform
    const int c = (w << 6) | l;
    uint64_t k = c < P ? ck[c] : ~0ull;  // padding sorts last (index > 2P)
    uint32_t v = c < P ? (uint32_t)(P + c) : 0xFFFFFFFFu;
    wave_sort64(k, v);
    rk[c] = k;
    ri[c] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * P; e += blockDim.x) {
    const bool child = e >= P;
    const int c = e - P, own = child ? c >> 6 : -1;
    if (child && (c & 63) >= P - (own << 6)) continue;  // run padding
    const uint64_t k = child ? rk[c] : pk[e];
    const uint32_t v = child ? ri[c] : (uint32_t)e;
    int rank = child ? (c & 63) : e;
    if (child) {
      int lo = 0, hi = P;  // lower bound among the parents
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pair_less(pk[mid], (uint32_t)mid, k, v)) lo = mid + 1;
        else hi = mid;
      }
      rank += lo;
    }
    for (int r = 0; r < R; ++r) {  // lower bound in every other run
      if (r == own) continue;
      const uint64_t* rkr = rk + (r << 6);
      const uint32_t* rir = ri + (r << 6);
      int pos = 0;
#pragma unroll
      for (int s = 32; s > 0; s >>= 1)
        if (pair_less(rkr[pos + s - 1], rir[pos + s - 1], k, v)) pos += s;
      if (pair_less(rkr[pos], rir[pos], k, v)) ++pos;
      rank += pos;
    }
    if (rank < P) {
      sk[rank] = k;
      si[rank] = v;
    }
  }
  __syncthreads();
}

// The same selection with the children fully sorted first (M2 = the power of
// two >= max(P, 64), block_sort_pairs_waves: its stride >= 64 stages cross
// the LDS), so every pair's final rank is its position in its own list plus
// ONE lower bound in the other: a child's among the parents, a parent's
// among the sorted children -- one binary search of log2 steps per pair
// instead of one per child run.  Same sk[0..P) / si[0..P) as merge_select.
// rk / ri hold M2 entries; needs M2 <= blockDim.x.  Every thread of the
// block must call it.
VRPMS_DEV void merge_select_sorted(const uint64_t* pk, const uint64_t* ck, int P, int M2,
                                   uint64_t* rk, uint32_t* ri, uint64_t* sk, uint32_t* si) {
  for (int c = threadIdx.x; c < M2; c += blockDim.x) {
    rk[c] = c < P ? ck[c] : ~0ull;  // padding sorts last (index > 2P)
    ri[c] = c < P ? (uint32_t)(P + c) : 0xFFFFFFFFu;
  }
  __syncthreads();
  block_sort_pairs_waves(rk, ri, M2);  // ends with a barrier
  for (int e = threadIdx.x; e < 2 * P; e += blockDim.x) {
    const bool child = e >= P;
    const int j = child ? e - P : e;
    const uint64_t k = child ? rk[j] : pk[j];
    const uint32_t v = child ? ri[j] : (uint32_t)j;
    int pos = 0;
    if (child) {  // lower bound among the P parents
      int hi = P;
      while (pos < hi) {
        const int mid = (pos + hi) >> 1;
        if (pair_less(pk[mid], (uint32_t)mid, k, v)) pos = mid + 1;
        else hi = mid;
      }
    } else {  // lower bound among the M2 sorted children (padding is never less)
      for (int s = M2 >> 1; s > 0; s >>= 1)
        if (pair_less(rk[pos + s - 1], ri[pos + s - 1], k, v)) pos += s;
      if (pair_less(rk[pos], ri[pos], k, v)) ++pos;
    }
    const int rank = j + pos;
    if (rank < P) {
      sk[rank] = k;
      si[rank] = v;
    }
  }
  __syncthreads();
}

}  // namespace vrpms
