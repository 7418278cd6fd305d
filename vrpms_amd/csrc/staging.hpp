// Instance staging shared by the search kernels (search.hip, sa_seg.hip):
// the matrix in LDS when it fits (<= 64 KB), else read from L2; demand,
// capacities and start times always in LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"
#include "ctx.hpp"
#include "tour.hpp"

namespace vrpms {

VRPMS_DEV int lane_id() { return (int)(threadIdx.x & 63u); }

// Instance staged for a search kernel: matrix in LDS when it fits, else L2.
struct SearchInst {
  const void* mat;   // u16 or i32 [H][N][N] (global)
  int N, H, K, problem, objective;
  const int32_t* dem;
  const int32_t* cap;
  const int32_t* start;
  int mat_lds;       // 1: stage the matrix into LDS (only when mat_bytes <= 64 KB)
  uint64_t mat_bytes; // H*N*N*elem: 64-bit, an int32 matrix can exceed 4 GB
  int symmetric;     // hour slice 0 symmetric (O(1) 2-opt delta)
};

inline SearchInst search_inst(const vrpms_ctx* ctx) {
  const Instance& in = ctx->inst;
  SearchInst s;
  s.mat = in.use16 ? static_cast<const void*>(in.mat16) : static_cast<const void*>(in.mat32);
  s.N = in.N;
  s.H = in.H;
  s.K = in.K;
  s.problem = in.problem;
  s.objective = in.objective;
  s.dem = in.dem;
  s.cap = in.cap;
  s.start = in.start;
  s.mat_bytes = (uint64_t)in.H * (uint64_t)in.N * (uint64_t)in.N * (in.use16 ? 2u : 4u);
  s.mat_lds = s.mat_bytes <= 64u * 1024u ? 1 : 0;
  s.symmetric = in.symmetric ? 1 : 0;
  return s;
}

// LDS carve for the instance part: [matrix][dem N][cap K][start K], 16-B aligned.
VRPMS_DEV uint32_t inst_lds_bytes(const SearchInst& si) {
  const uint32_t m = si.mat_lds ? (((uint32_t)si.mat_bytes + 15u) & ~15u) : 0u;
  return m + (((uint32_t)(si.N + 2 * si.K) * 4u + 15u) & ~15u);
}

inline size_t inst_lds_bytes_host(const SearchInst& si) {
  const size_t m = si.mat_lds ? (((size_t)si.mat_bytes + 15u) & ~(size_t)15u) : 0u;
  return m + ((((size_t)si.N + 2 * si.K) * 4u + 15u) & ~(size_t)15u);
}

template <typename MatT, int HM>
struct StagedInst {
  MatView<MatT, HM> D;
  SplitParams sp;
};

template <typename MatT, int HM>
VRPMS_DEV StagedInst<MatT, HM> stage_inst(const SearchInst& si, unsigned char* smem) {
  const uint32_t NN = (uint32_t)si.N * si.N;
  const MatT* M = static_cast<const MatT*>(si.mat);
  uint32_t off = 0;
  if (si.mat_lds) {
    const uint32_t mb = (uint32_t)si.mat_bytes;  // <= 64 KB when staged
    const uint32_t* s = static_cast<const uint32_t*>(si.mat);
    uint32_t* d = reinterpret_cast<uint32_t*>(smem);
    for (uint32_t i = threadIdx.x; i < mb / 4; i += blockDim.x) d[i] = s[i];
    if ((mb & 2u) && threadIdx.x == 0)
      reinterpret_cast<uint16_t*>(smem)[mb / 2 - 1] = static_cast<const uint16_t*>(si.mat)[mb / 2 - 1];
    M = reinterpret_cast<const MatT*>(smem);
    off = (mb + 15u) & ~15u;
  }
  int32_t* dem = reinterpret_cast<int32_t*>(smem + off);
  int32_t* cap = dem + si.N;
  int32_t* st = cap + si.K;
  for (int i = threadIdx.x; i < si.N; i += blockDim.x) dem[i] = si.dem[i];
  for (int i = threadIdx.x; i < si.K; i += blockDim.x) {
    cap[i] = si.cap[i];
    st[i] = si.start[i];
  }
  __syncthreads();
  return {{M, (uint32_t)si.N, NN, si.H}, {dem, cap, st, si.K, si.objective}};
}

}  // namespace vrpms
