// Row-layout scoring for everything the LDS-packed kernels do not cover:
// hour-indexed matrices (cfg 3, H = 24), L2-resident matrices (cfg 4,
// N = 1001), uint16 tours, heterogeneous fleets, time-dependent TSP.
//
// Bound: random 2-byte gathers into an L2-resident (uint16) matrix, one per
// customer.  Everything else a lane needs is moved out of that path:
//   * tours are staged through LDS in 32-byte chunks per candidate, loaded
//     cooperatively (8 consecutive lanes read one row's chunk, so a wave
//     load touches 8 rows instead of 64) -- a lane never reads its own row
//     from global memory;
//   * the depot legs D[h][a][0] / D[h][0][b] (route close / route open),
//     the demands, capacities and start times sit in LDS tables, so a route
//     closure costs no extra global gather;
//   * static matrices (H = 1): the gather of position i reads
//     D[tour[i-1]][tour[i]], independent of the split state, so a lane
//     issues the gathers of 16 positions before the 16 split steps;
//   * hour-indexed matrices: the gather address depends on the clock, a
//     true dependency chain; 2048 lanes per CU hide it (an M = 2 variant,
//     two interleaved candidates per lane, measured slower and is kept for
//     A/B runs only).
// Semantics are exactly eval_tour (tour.hpp) / oracle/spec.py eval_cvrp,
// eval_tsp, bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "ctx.hpp"
#include "staged.hpp"
#include "tour.hpp"

namespace vrpms {

struct StagedArgs {
  const void* mat;  // [H][N][N] MatT (global)
  int N, H, K;
  const int32_t* dem;
  const int32_t* cap;
  const int32_t* start;
  const unsigned char* perms;
  int64_t C;
  int n;
  int64_t ld;  // elements
  int objective;
  uint64_t* keys;
  int32_t* sums;
  int32_t* maxs;
  int32_t* unv;
};

constexpr int kStBlock = 512;
constexpr int kChunkBytes = 32;                // tour bytes per candidate per chunk
constexpr int kChunkDw = kChunkBytes / 4;      // 8 dwords
constexpr int kRowDw = kChunkDw + 1;           // odd LDS row stride: conflict-free b32 reads
constexpr int kGroup = 16;                     // static path: gathers issued per batch

VRPMS_HOST_DEV_INLINE size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS carve-up shared by host (size) and device (offsets).
struct StagedLds {
  size_t mat, ret, out, dem, cap, st, tile, total;
  VRPMS_HOST_DEV_INLINE StagedLds(int N, int H, int K, size_t elem, bool mlds, int rows) {
    size_t o = 0;
    mat = o;
    o += mlds ? align16((size_t)H * N * N * elem) : 0;
    ret = o;
    o += align16((size_t)H * N * elem);
    out = o;
    o += align16((size_t)H * N * elem);
    dem = o;
    o += align16((size_t)N * 4);
    cap = o;
    o += align16((size_t)K * 4);
    st = o;
    o += align16((size_t)K * 4);
    tile = o;
    o += (size_t)rows * kRowDw * 4;
    total = o;
  }
};

struct StState {
  int t, load, k, capk;
  uint32_t prev, dsum, dmax, unv;
};

template <typename MatT, int HM, bool CVRP, bool FLEX, typename PermT, int M, bool ALIGNED,
          bool MLDS>
__global__ __launch_bounds__(kStBlock) void eval_staged(StagedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int R = kStBlock * M;                       // tile rows (candidates)
  constexpr int EPC = kChunkBytes / (int)sizeof(PermT);  // tour elements per chunk
  constexpr int RPP = kStBlock / kChunkDw;              // rows covered per staging pass
  constexpr int UPT = R / RPP;                          // dwords per thread per chunk
  const int N = a.N, H = a.H, K = a.K, n = a.n;
  const uint32_t NN = (uint32_t)N * (uint32_t)N, Nm1 = (uint32_t)N - 1;
  const StagedLds L(N, H, K, sizeof(MatT), MLDS, R);
  const MatT* Mg = static_cast<const MatT*>(a.mat);
  MatT* retT = reinterpret_cast<MatT*>(smem + L.ret);
  MatT* outT = reinterpret_cast<MatT*>(smem + L.out);
  int32_t* demT = reinterpret_cast<int32_t*>(smem + L.dem);
  int32_t* capT = reinterpret_cast<int32_t*>(smem + L.cap);
  int32_t* stT = reinterpret_cast<int32_t*>(smem + L.st);
  uint32_t* tile = reinterpret_cast<uint32_t*>(smem + L.tile);
  const MatT* Mx = Mg;
  if constexpr (MLDS) {
    MatT* Ml = reinterpret_cast<MatT*>(smem + L.mat);
    for (uint32_t i = threadIdx.x; i < NN * (uint32_t)H; i += kStBlock) Ml[i] = Mg[i];
    Mx = Ml;
  }
  for (int i = threadIdx.x; i < H * N; i += kStBlock) {
    const int h = i / N, x = i - h * N;
    retT[i] = Mg[(size_t)h * NN + (size_t)x * N];
    outT[i] = Mg[(size_t)h * NN + x];
  }
  if constexpr (CVRP)
    for (int i = threadIdx.x; i < N; i += kStBlock) demT[i] = a.dem[i];
  for (int i = threadIdx.x; i < K; i += kStBlock) {
    capT[i] = CVRP ? a.cap[i] : 0;
    stT[i] = a.start[i];
  }

  const int64_t C = a.C;
  const int nchunks = (n + EPC - 1) / EPC;
  const size_t ldb = (size_t)a.ld * sizeof(PermT);
  const size_t nbytes = (size_t)n * sizeof(PermT);
  const int64_t tstride = (int64_t)gridDim.x * R;

  // ---- tour staging: 8 consecutive lanes read one row's 32-byte chunk -----
  const int prow = threadIdx.x / kChunkDw, piece = threadIdx.x % kChunkDw;
  uint32_t pf[ALIGNED ? UPT : 1];
  auto prefetch = [&](int64_t base, int q) {
    if constexpr (ALIGNED) {
      const size_t o = (size_t)q * kChunkBytes + (size_t)piece * 4;
      const bool ok = o < nbytes;
      const unsigned char* p0 = a.perms + (size_t)(base + prow) * ldb + o;
#pragma unroll
      for (int v = 0; v < UPT; ++v)
        pf[v] = (ok && base + prow + v * RPP < C)
                    ? *reinterpret_cast<const uint32_t*>(p0 + (size_t)v * RPP * ldb)
                    : 0u;
    }
  };
  auto commit = [&](int64_t base, int q) {
    if constexpr (ALIGNED) {
#pragma unroll
      for (int v = 0; v < UPT; ++v) tile[(prow + v * RPP) * kRowDw + piece] = pf[v];
    } else {  // unaligned rows: element loads straight into the tile
      const PermT* P = reinterpret_cast<const PermT*>(a.perms);
      for (int e = threadIdx.x; e < R * EPC; e += kStBlock) {
        const int row = e / EPC, k = e - row * EPC;
        const int pos = q * EPC + k;
        const int64_t c = base + row;
        const PermT v = (c < C && pos < n) ? P[c * a.ld + pos] : (PermT)0;
        reinterpret_cast<PermT*>(tile + row * kRowDw)[k] = v;
      }
    }
  };

  auto hour = [&](int t) -> uint32_t { return hour_of<HM>(t, H); };
  // route k returns to the depot; vehicle k + 1 (if any) opens empty
  auto close_route = [&](StState& s) {
    if (s.prev) {
      s.t += (int)retT[hour(s.t) * N + s.prev];
      const uint32_t rd = (uint32_t)(s.t - stT[s.k]);
      s.dsum += rd;
      s.dmax = max(s.dmax, rd);
    }
    ++s.k;
    if (s.k < K) {
      s.load = 0;
      s.t = stT[s.k];
      s.prev = 0;
      s.capk = capT[s.k];
    }
  };
  // One greedy-split step for customer cc; g = D(t, prev, cc) gathered
  // before the step (used unless the step closes a route).
  auto step = [&](StState& s, uint32_t cc, int g) {
    if constexpr (CVRP) {
      if (cc == 0) {  // A10 separator: close route k (if any), open vehicle k + 1
        if (s.k < K) close_route(s);
        return;
      }
      const int dc = demT[cc];
      bool closed = false;
      if (s.k < K && s.load + dc > s.capk) {
        closed = true;
        close_route(s);
        // FLEX: skip vehicles too small for this customer (A6); without it
        // the host has checked min(cap) >= max(demand), so one close suffices
        if constexpr (FLEX)
          while (s.k < K && dc > s.capk) close_route(s);
      }
      if (s.k < K) {
        s.t += closed ? (int)outT[hour(s.t) * N + cc] : g;
        s.load += dc;
        s.prev = cc;
      } else {
        ++s.unv;
      }
    } else {
      s.t += g;
      s.prev = cc;
    }
  };
  // customer j (0 <= j < EPC) of tile row r
  auto tour_at = [&](int r, int j) -> uint32_t {
    const uint32_t w = tile[r * kRowDw + j * (int)sizeof(PermT) / 4];
    const uint32_t v = sizeof(PermT) == 1 ? (w >> (8 * (j & 3))) & 0xffu
                                          : (w >> (16 * (j & 1))) & 0xffffu;
    return min(v, Nm1);
  };

  // customer g0 + j of tile row r, g0 a multiple of kGroup (compile-time lane shifts)
  auto tour_at_g = [&](int r, int g0, int j) -> uint32_t {
    const uint32_t w = tile[r * kRowDw + (g0 * (int)sizeof(PermT)) / 4 + j * (int)sizeof(PermT) / 4];
    const uint32_t v = sizeof(PermT) == 1 ? (w >> (8 * (j & 3))) & 0xffu
                                          : (w >> (16 * (j & 1))) & 0xffffu;
    return min(v, Nm1);
  };

  __syncthreads();  // tables staged
  int64_t base = blockIdx.x * (int64_t)R;
  if (base < C && nchunks > 0) prefetch(base, 0);
  for (; base < C; base += tstride) {
    StState st[M];
    uint32_t last[M];  // tour[i-1] (the depot before the first customer)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      st[m] = {stT[0], 0, 0, CVRP ? capT[0] : 0, 0u, 0u, 0u, 0u};
      last[m] = 0;
    }
    for (int q = 0; q < nchunks; ++q) {
      __syncthreads();  // previous chunk consumed
      commit(base, q);
      __syncthreads();
      if (q + 1 < nchunks) prefetch(base, q + 1);
      else if (base + tstride < C) prefetch(base + tstride, 0);
      const int cnt = min(EPC, n - q * EPC);
      if constexpr (HM == 1) {
        // static: gathers depend on the tour only -- issue a group, then step
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int r = m * kStBlock + threadIdx.x;
          for (int g0 = 0; g0 < cnt; g0 += kGroup) {
            uint32_t ids[kGroup];
            int gv[kGroup];
#pragma unroll
            for (int j = 0; j < kGroup; ++j) ids[j] = tour_at_g(r, g0, j);
#pragma unroll
            for (int j = 0; j < kGroup; ++j)
              gv[j] = (int)Mx[(j ? ids[j - 1] : last[m]) * (uint32_t)N + ids[j]];
            const int lim = min(kGroup, cnt - g0);
#pragma unroll
            for (int j = 0; j < kGroup; ++j)
              if (j < lim) step(st[m], ids[j], gv[j]);
#pragma unroll
            for (int j = 0; j < kGroup; ++j)
              if (j == lim - 1) last[m] = ids[j];
          }
        }
      } else {
        // hour-indexed: the clock feeds the address; interleave M chains
        for (int j = 0; j < cnt; ++j) {
          uint32_t ids[M];
          int gv[M];
#pragma unroll
          for (int m = 0; m < M; ++m) ids[m] = tour_at(m * kStBlock + threadIdx.x, j);
#pragma unroll
          for (int m = 0; m < M; ++m)
            gv[m] = (int)Mx[(size_t)hour(st[m].t) * NN + st[m].prev * (uint32_t)N + ids[m]];
#pragma unroll
          for (int m = 0; m < M; ++m) step(st[m], ids[m], gv[m]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int64_t c = base + m * kStBlock + threadIdx.x;
      StState& s = st[m];
      TourCost tc;
      if constexpr (CVRP) {
        if (s.k < K && s.prev) {
          s.t += (int)retT[hour(s.t) * N + s.prev];
          const uint32_t rd = (uint32_t)(s.t - stT[s.k]);
          s.dsum += rd;
          s.dmax = max(s.dmax, rd);
        }
        tc = {cvrp_key(s.unv, s.dsum, s.dmax, a.objective), (int32_t)s.dsum, (int32_t)s.dmax,
              (int32_t)s.unv};
      } else {
        s.t += (int)retT[hour(s.t) * N + s.prev];
        const int d = s.t - stT[0];
        tc = {pack_key(0, (uint32_t)d, 0), d, d, 0};
      }
      if (c < C) {
        a.keys[c] = tc.key;
        if (a.sums) a.sums[c] = tc.sum;
        if (a.maxs) a.maxs[c] = tc.max;
        if (a.unv) a.unv[c] = tc.unv;
      }
    }
  }
}

template <typename K>
static void allow_lds_st(K kern, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <typename MatT, int HM, bool CVRP, bool FLEX, typename PermT, int M, bool ALIGNED,
          bool MLDS>
static int go_staged(const vrpms_ctx* ctx, const StagedArgs& a, hipStream_t s) {
  const Instance& in = ctx->inst;
  const StagedLds L(in.N, in.H, in.K, sizeof(MatT), MLDS, kStBlock * M);
  if (L.total > ctx->max_lds) return fail(VRPMS_EINVAL, "staged eval: LDS layout too large");
  const int per_cu = std::max<int>(1, std::min<int>(2048 / kStBlock, (int)(ctx->max_lds / L.total)));
  const int64_t tiles = (a.C + kStBlock * M - 1) / (kStBlock * M);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(tiles, (int64_t)ctx->num_cus * per_cu));
  auto kern = eval_staged<MatT, HM, CVRP, FLEX, PermT, M, ALIGNED, MLDS>;
  allow_lds_st(kern, L.total);
  kern<<<grid, kStBlock, L.total, s>>>(a);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

struct StagedSel {
  bool aligned, mlds, flex;
  int M;
};

// Instantiated variants: M = 2 only for the clock-dependent (H > 1) chains,
// the LDS matrix only for uint8 tours (uint16 tours mean N > 256, whose
// matrix never fits), FLEX only with M = 1.
template <typename MatT, int HM, bool CVRP, typename PermT>
static int pick_staged(const vrpms_ctx* ctx, const StagedArgs& a, const StagedSel& v,
                       hipStream_t s) {
  constexpr bool U8 = sizeof(PermT) == 1;
  if (v.flex && CVRP) {
    if (v.aligned) return v.mlds && U8 ? go_staged<MatT, HM, CVRP, true, PermT, 1, true, U8>(ctx, a, s)
                                       : go_staged<MatT, HM, CVRP, true, PermT, 1, true, false>(ctx, a, s);
    return v.mlds && U8 ? go_staged<MatT, HM, CVRP, true, PermT, 1, false, U8>(ctx, a, s)
                        : go_staged<MatT, HM, CVRP, true, PermT, 1, false, false>(ctx, a, s);
  }
  if constexpr (HM != 1) {
    if (v.M == 2) {
      if (v.aligned) return v.mlds && U8 ? go_staged<MatT, HM, CVRP, false, PermT, 2, true, U8>(ctx, a, s)
                                         : go_staged<MatT, HM, CVRP, false, PermT, 2, true, false>(ctx, a, s);
      return v.mlds && U8 ? go_staged<MatT, HM, CVRP, false, PermT, 2, false, U8>(ctx, a, s)
                          : go_staged<MatT, HM, CVRP, false, PermT, 2, false, false>(ctx, a, s);
    }
  }
  if (v.aligned) return v.mlds && U8 ? go_staged<MatT, HM, CVRP, false, PermT, 1, true, U8>(ctx, a, s)
                                     : go_staged<MatT, HM, CVRP, false, PermT, 1, true, false>(ctx, a, s);
  return v.mlds && U8 ? go_staged<MatT, HM, CVRP, false, PermT, 1, false, U8>(ctx, a, s)
                      : go_staged<MatT, HM, CVRP, false, PermT, 1, false, false>(ctx, a, s);
}

template <typename MatT, typename PermT>
static int staged_mat(const vrpms_ctx* ctx, const StagedArgs& a, const StagedSel& v,
                      hipStream_t s) {
  const Instance& in = ctx->inst;
  const bool cvrp = in.problem == VRPMS_CVRP;
  if (in.H == 1)
    return cvrp ? pick_staged<MatT, 1, true, PermT>(ctx, a, v, s)
                : pick_staged<MatT, 1, false, PermT>(ctx, a, v, s);
  if (in.H == 24)
    return cvrp ? pick_staged<MatT, 24, true, PermT>(ctx, a, v, s)
                : pick_staged<MatT, 24, false, PermT>(ctx, a, v, s);
  return cvrp ? pick_staged<MatT, 0, true, PermT>(ctx, a, v, s)
              : pick_staged<MatT, 0, false, PermT>(ctx, a, v, s);
}

int launch_staged(vrpms_ctx* ctx, const void* perms, int perm_bytes, int64_t C, int n,
                  int64_t ld, uint64_t* keys, int32_t* sums, int32_t* maxs, int32_t* unv,
                  hipStream_t s) {
  const Instance& in = ctx->inst;
  const size_t elem = in.use16 ? 2 : 4;
  StagedArgs a{in.use16 ? static_cast<const void*>(in.mat16) : static_cast<const void*>(in.mat32),
               in.N, in.H, in.K, in.dem, in.cap, in.start,
               static_cast<const unsigned char*>(perms), C, n, ld, in.objective,
               keys, sums, maxs, unv};
  StagedSel v;
  v.aligned = ((uintptr_t)perms & 3u) == 0 && ((size_t)ld * perm_bytes) % 4 == 0;
  // matrix in LDS when small (the old LDS tier), else L2-resident gathers
  v.mlds = perm_bytes == 1 && (size_t)in.H * in.N * in.N * elem <= 64 * 1024;
  v.flex = in.problem == VRPMS_CVRP && in.min_cap < in.max_dem;
  // Chains per lane.  Measured on MI355X (tools/l2_probe.py): TD-200 x 24 h
  // 1.24 G evals/s with M = 1 vs 1.09 G with M = 2 -- at 2048 lanes per CU
  // the L2 request rate, not the per-lane dependency chain, is the bound,
  // and M = 2 costs occupancy -- so M = 1 unless forced (A/B tests).
  v.M = 1;
  if (in.H > 1 && !v.flex && ctx->opt_staged_m == 2) v.M = 2;
  // fall back to one chain per lane when two do not fit the LDS
  if (v.M == 2 && StagedLds(in.N, in.H, in.K, elem, v.mlds, kStBlock * 2).total > ctx->max_lds)
    v.M = 1;
  if (perm_bytes == 1)
    return in.use16 ? staged_mat<uint16_t, uint8_t>(ctx, a, v, s)
                    : staged_mat<int32_t, uint8_t>(ctx, a, v, s);
  return in.use16 ? staged_mat<uint16_t, uint16_t>(ctx, a, v, s)
                  : staged_mat<int32_t, uint16_t>(ctx, a, v, s);
}

bool staged_fits(const vrpms_ctx* ctx) {
  const Instance& in = ctx->inst;
  const size_t elem = in.use16 ? 2 : 4;
  const bool mlds = (size_t)in.H * in.N * in.N * elem <= 64 * 1024;
  return StagedLds(in.N, in.H, in.K, elem, mlds, kStBlock).total <= ctx->max_lds;
}

}  // namespace vrpms
