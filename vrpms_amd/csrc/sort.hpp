// Workgroup-wide sort of (key, index) pairs in LDS, shared by the pool /
// island kernels (pool.hip) and the fused GA island kernel (ga_fused.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

// hook of the GA phase profile (ga_fused.hip, -DVRPMS_GA_PROF builds)
#ifndef VRPMS_MS_MARK
#define VRPMS_MS_MARK() \
  do {                  \
  } while (0)
#endif

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
// unrolling, all in VALU (no LDS round trip): DPP quad_perm (1, 2) and
// row_ror:8 (8) ride on a move; 4 picks row_shl:4 or row_shr:4 by lane bit
// 2; 16 and 32 are gfx950's v_permlane16_swap / v_permlane32_swap of x with
// itself (the odd 16-lane rows with the even ones, the upper 32 lanes with
// the lower), the partner's copy picked by lane bit 4 / 5.
VRPMS_DEV uint32_t xor_lanes(uint32_t x, int stride) {
  const uint32_t l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  switch (stride) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
    case 4: {
      const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x104, 0xF, 0xF, true);  // lane + 4
      const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xF, 0xF, true);  // lane - 4
      return (l & 4u) ? dn : up;
    }
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);
    case 16: {
      const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
      return (l & 16u) ? r[0] : r[1];
    }
    default: {
      const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
      return (l & 32u) ? r[0] : r[1];
    }
  }
}

// x from lane (lane ^ (size - 1)): the mirror image inside groups of `size`
// lanes (a compile-time power of two after unrolling): DPP quad_perm (2, 4),
// row_half_mirror (8), row_mirror (16), then the 16 / 32 swaps of xor_lanes.
VRPMS_DEV uint32_t mirror_lanes(uint32_t x, int size) {
  switch (size) {
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
    case 4: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, true);
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);
    case 16: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);
    case 32: return xor_lanes((uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true), 16);
    default:
      return xor_lanes(
          xor_lanes((uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true), 16), 32);
  }
}

// Sort of one (key, index) pair per lane across a wavefront (ascending by
// lane; 21 compare-exchange stages).  The bitonic network in its
// mirror form: each merge of two sorted halves of `size` lanes first
// compares lane l with lane l ^ (size - 1), then runs its half-cleaners
// (l ^ stride), every stage ascending -- so the lane keeping the smaller pair
// is always the one with the compared bit clear (six fixed masks instead of
// one direction mask per stage).  All 64 lanes must be active.
VRPMS_DEV void wave_sort64(uint64_t& k, uint32_t& v) {
  const uint32_t l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  auto cx = [&](uint32_t okh, uint32_t okl, uint32_t ov, int bit) __attribute__((always_inline)) {
    const uint64_t ok = ((uint64_t)okh << 32) | okl;
    const bool other_less = ok < k || (ok == k && ov < v);
    const bool low = (l & (uint32_t)bit) == 0;  // keeps the smaller pair
    if (other_less == low) {
      k = ok;
      v = ov;
    }
  };
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
    cx(mirror_lanes((uint32_t)(k >> 32), size), mirror_lanes((uint32_t)k, size),
       mirror_lanes(v, size), size >> 1);
#pragma unroll
    for (int stride = size >> 2; stride > 0; stride >>= 1)
      cx(xor_lanes((uint32_t)(k >> 32), stride), xor_lanes((uint32_t)k, stride),
         xor_lanes(v, stride), stride);
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
// (64 * ceil(P / 64) entries); sk must hold 2P entries (its upper half keeps
// the children's parent ranks meanwhile); needs blockDim.x >= 64 * ceil(P / 64).
// With pmap / cmap, si receives pmap[index] for a parent and
// cmap[index - P] for a child instead of the index (the fused GA's LDS rows
// of the survivors), and lost[rank - P] the row of each pair ranked P .. 2P - 1
// (the rows no survivor holds; lost must not alias cmap).  Every thread of the
// block must call it.
//
// Latency, not issue, bounds the rank searches (each a chain of dependent
// LDS reads): the wavefronts that sort no run search the children's ranks
// among the parents while the others sort, and a lane's searches in two runs
// step together, so a pair waits for one 7-step chain instead of up to three.
//
// IN (merge_select_inplace): the survivors are written over the parents
// (sk aliases pk, orow receives the rows instead of si aliasing pmap); needs
// 4P <= blockDim.x and a wavefront that sorts no run, so each thread holds at
// most one pair, reads its parent's key and row before the run-sort barrier,
// and nothing reads pk / pmap after it.
template <bool IN>
VRPMS_DEV void merge_select_impl(const uint64_t* pk, const uint64_t* ck, int P, uint64_t* rk,
                                 uint32_t* ri, uint64_t* sk, uint32_t* si, const uint16_t* pmap,
                                 const uint16_t* cmap, uint16_t* lost, uint32_t* prank_in,
                                 uint16_t* orow) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int R = (P + 63) >> 6;
  // lower bound of (k, v) among the parents (8 steps for P = 256)
  auto parent_rank = [&](uint64_t k, uint32_t v) {
    int lo = 0, hi = P;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pair_less(pk[mid], (uint32_t)mid, k, v)) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  };
  const int spare = (int)blockDim.x - 64 * R;  // lanes of the waves that sort no run
  // [P] (dead until the writes below)
  uint32_t* prank = IN ? prank_in : reinterpret_cast<uint32_t*>(sk + P);
  uint64_t pkey = 0;  // IN: the parent pair this thread ranks, read before any write
  uint32_t prow_own = 0;
  if (IN && ((int)threadIdx.x >> 1) < P) {
    pkey = pk[threadIdx.x >> 1];
    prow_own = pmap[threadIdx.x >> 1];
  }
  if (w < R) {  // wave-uniform
    const int c = (w << 6) | l;
    uint64_t k = c < P ? ck[c] : ~0ull;  // padding sorts last (index > 2P)
    uint32_t v = c < P ? (uint32_t)(P + c) : 0xFFFFFFFFu;
    wave_sort64(k, v);
    rk[c] = k;
    ri[c] = v;
  } else {
    for (int c = (int)threadIdx.x - 64 * R; c < P; c += spare)
      prank[c] = (uint32_t)parent_rank(ck[c], (uint32_t)(P + c));
  }
  __syncthreads();
  VRPMS_MS_MARK();
  // the lower bounds a pair needs in the other runs are independent
  // searches: with 4P <= blockDim.x two lanes share each pair, lane bit 0
  // choosing the runs of that parity (the even lane also adds the child's
  // parent rank), their counts added by a DPP swap
  const bool two = 4 * P <= (int)blockDim.x;  // block-uniform
  const int step = two ? (int)blockDim.x >> 1 : (int)blockDim.x;
  const int inc = two ? 2 : 1;
  for (int t = two ? (int)threadIdx.x >> 1 : (int)threadIdx.x; t < 2 * P; t += step) {
    const int half = two ? (int)(threadIdx.x & 1u) : -1;
    const int e = t;
    const bool child = e >= P;
    const int c = e - P, own = child ? c >> 6 : -1;
    const bool pad = child && (c & 63) >= P - (own << 6);  // run padding
    const uint64_t k = child ? rk[c] : (IN ? pkey : pk[e]);
    const uint32_t v = child ? ri[c] : (uint32_t)e;
    int part = 0;
    if (child && half <= 0 && !pad)
      part += spare > 0 ? (int)prank[v - (uint32_t)P] : parent_rank(k, v);
    // runs r0, r0 + inc stepped together
    for (int r0 = half < 0 ? 0 : half; r0 < R; r0 += 2 * inc) {
      const int r1 = r0 + inc;
      const bool v0 = r0 != own, v1 = r1 < R && r1 != own;
      const uint64_t* k0 = rk + (r0 << 6);
      const uint32_t* i0 = ri + (r0 << 6);
      const uint64_t* k1 = rk + ((v1 ? r1 : r0) << 6);
      const uint32_t* i1 = ri + ((v1 ? r1 : r0) << 6);
      int p0 = 0, p1 = 0;
#pragma unroll
      for (int s = 32; s > 0; s >>= 1) {
        const bool a0 = pair_less(k0[p0 + s - 1], i0[p0 + s - 1], k, v);
        const bool a1 = pair_less(k1[p1 + s - 1], i1[p1 + s - 1], k, v);
        p0 += a0 ? s : 0;
        p1 += a1 ? s : 0;
      }
      p0 += pair_less(k0[p0], i0[p0], k, v) ? 1 : 0;
      p1 += pair_less(k1[p1], i1[p1], k, v) ? 1 : 0;
      part += (v0 ? p0 : 0) + (v1 ? p1 : 0);
    }
    if (two)  // both lanes of the pair active here (the loop bound is per pair)
      part += __builtin_amdgcn_mov_dpp(part, 0xB1, 0xF, 0xF, false);
    const int rank = part + (child ? (c & 63) : e);
    if (!pad && half <= 0) {
      const uint32_t row =
          pmap ? (uint32_t)(child ? cmap[v - P] : (IN ? prow_own : pmap[v])) : v;
      if (rank < P) {
        sk[rank] = k;
        if (IN) orow[rank] = (uint16_t)row;
        else si[rank] = row;
      } else if (lost) {
        lost[rank - P] = (uint16_t)row;
      }
    }
  }
  __syncthreads();
}

VRPMS_DEV void merge_select(const uint64_t* pk, const uint64_t* ck, int P, uint64_t* rk,
                            uint32_t* ri, uint64_t* sk, uint32_t* si,
                            const uint16_t* pmap = nullptr, const uint16_t* cmap = nullptr,
                            uint16_t* lost = nullptr) {
  merge_select_impl<false>(pk, ck, P, rk, ri, sk, si, pmap, cmap, lost, nullptr, nullptr);
}

// pk / prow <- the survivors' keys and rows (see IN above); prank: P scratch
// words.  Every thread of the block must call it.
VRPMS_DEV void merge_select_inplace(uint64_t* pk, uint16_t* prow, const uint64_t* ck,
                                    const uint16_t* crow, uint16_t* lost, int P, uint64_t* rk,
                                    uint32_t* ri, uint32_t* prank) {
  merge_select_impl<true>(pk, ck, P, rk, ri, pk, nullptr, prow, crow, lost, prank, prow);
}

}  // namespace vrpms
