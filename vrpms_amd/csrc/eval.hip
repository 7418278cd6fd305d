// Batched candidate scoring: the first half of the vrpms hot path.
//
// One LANE evaluates one candidate giant tour (lane-per-candidate): the
// greedy capacity split (A6) and the time-dependent clock (A3) are
// sequential, non-associative recurrences, so parallelism comes from the
// thousands of independent candidates, 64 per wavefront.
//
// Kernels (all integer; costs bit-exact with oracle/spec.py):
//   eval_cvrp_packed  static CVRP, N <= ~120: the packed u64 matrix
//                     E[a][b] = dur(a,b) | {ret(b), out(b), dem(b)} << 32 is
//                     LDS-resident and the candidate tile is staged through
//                     LDS with coalesced 16-B loads.  One ds_read_b64 gather
//                     per customer carries the edge, the demand test and
//                     both depot legs of a route closure.
//   eval_tsp_staged   static TSP with the (u16/i32) matrix LDS-resident.
//   eval_generic      everything else: hour-indexed matrices (H = 24),
//                     uint16 tours, L2-resident matrices (N >= ~180),
//                     heterogeneous fleets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "common.hpp"
#include "ctx.hpp"

namespace vrpms {

struct EvalArgs {
  const void* mat;
  int N, H, K;
  const int32_t* dem;
  const int32_t* cap;
  const int32_t* start;
  const void* perms;
  int64_t C;
  int n;
  int64_t ld;
  int objective;
  uint64_t* keys;
  int32_t* sums;
  int32_t* maxs;
  int32_t* unv;
};

// A3: hour slice of an edge departing at minute t.  HM = 1 static,
// HM = 24 hour-indexed (constant divisor), HM = 0 runtime H.
template <int HM>
VRPMS_DEV uint32_t hour_of(int t, int H) {
  if constexpr (HM == 1) {
    return 0;
  } else if constexpr (HM == 24) {
    return ((uint32_t)t / 60u) % 24u;
  } else {
    return ((uint32_t)t / 60u) % (uint32_t)H;
  }
}

VRPMS_DEV void write_out(const EvalArgs& a, int64_t c, uint64_t key, int32_t s, int32_t m,
                         int32_t u) {
  a.keys[c] = key;
  if (a.sums) a.sums[c] = s;
  if (a.maxs) a.maxs[c] = m;
  if (a.unv) a.unv[c] = u;
}

// ---------------------------------------------------------------------------
// Generic lane-per-candidate evaluation (any tier / H / perm width).
// ---------------------------------------------------------------------------
template <typename MatT, bool LDS, bool CVRP, int HM, typename PermT>
__global__ __launch_bounds__(256) void eval_generic(EvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N;
  const uint32_t NN = (uint32_t)N * (uint32_t)N;
  const MatT* M = static_cast<const MatT*>(a.mat);
  if constexpr (LDS) {
    const uint32_t bytes = NN * (uint32_t)a.H * sizeof(MatT);
    const uint32_t words = bytes / 4;
    const uint32_t* src = static_cast<const uint32_t*>(a.mat);
    uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) dst[i] = src[i];
    if ((bytes & 2u) && threadIdx.x == 0)
      reinterpret_cast<uint16_t*>(smem)[bytes / 2 - 1] =
          static_cast<const uint16_t*>(a.mat)[bytes / 2 - 1];
    __syncthreads();
    M = reinterpret_cast<const MatT*>(smem);
  }
  const PermT* P = static_cast<const PermT*>(a.perms);
  const uint32_t Nm1 = (uint32_t)N - 1;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < a.C;
       c += (int64_t)gridDim.x * blockDim.x) {
    const PermT* row = P + c * a.ld;
    if constexpr (!CVRP) {
      const int t0 = a.start[0];
      int t = t0;
      uint32_t prev = 0;
      for (int i = 0; i < a.n; ++i) {
        const uint32_t cc = min((uint32_t)row[i], Nm1);
        t += (int)M[hour_of<HM>(t, a.H) * NN + prev * N + cc];
        prev = cc;
      }
      t += (int)M[hour_of<HM>(t, a.H) * NN + prev * N];
      const int d = t - t0;
      write_out(a, c, pack_key(0, (uint32_t)d, 0), d, d, 0);
    } else {
      const int K = a.K;
      int k = 0, load = 0, t = a.start[0], capk = a.cap[0];
      uint32_t prev = 0, unv = 0, dsum = 0, dmax = 0;
      for (int i = 0; i < a.n; ++i) {
        const uint32_t cc = min((uint32_t)row[i], Nm1);
        const int dc = a.dem[cc];
        if (k < K && load + dc > capk) {
          do {
            if (prev) {
              t += (int)M[hour_of<HM>(t, a.H) * NN + prev * N];
              const uint32_t rd = (uint32_t)(t - a.start[k]);
              dsum += rd;
              dmax = max(dmax, rd);
            }
            ++k;
            if (k < K) {
              load = 0;
              t = a.start[k];
              prev = 0;
              capk = a.cap[k];
            }
          } while (k < K && load + dc > capk);
        }
        if (k < K) {
          t += (int)M[hour_of<HM>(t, a.H) * NN + prev * N + cc];
          load += dc;
          prev = cc;
        } else {
          ++unv;
        }
      }
      if (k < K && prev) {
        t += (int)M[hour_of<HM>(t, a.H) * NN + prev * N];
        const uint32_t rd = (uint32_t)(t - a.start[k]);
        dsum += rd;
        dmax = max(dmax, rd);
      }
      write_out(a, c, cvrp_key(unv, dsum, dmax, a.objective), (int32_t)dsum, (int32_t)dmax,
                (int32_t)unv);
    }
  }
}

// ---------------------------------------------------------------------------
// Candidate tiles staged through LDS: BLOCK rows of `ld` bytes are one
// contiguous HBM range, copied with 16-byte loads (fully coalesced), then
// each lane walks its own row with ds_read_b32 (4 customers per read; with
// ld/4 odd the 64 lanes hit distinct banks).
// ---------------------------------------------------------------------------
template <int BLOCK>
VRPMS_DEV void stage_tile(unsigned char* tile, const unsigned char* g, uint32_t bytes) {
  const uint32_t nvec = bytes / 16;
  const uint4* gs = reinterpret_cast<const uint4*>(g);
  uint4* ts = reinterpret_cast<uint4*>(tile);
  for (uint32_t i = threadIdx.x; i < nvec; i += BLOCK) ts[i] = gs[i];
  const uint32_t* gw = reinterpret_cast<const uint32_t*>(g);
  uint32_t* tw = reinterpret_cast<uint32_t*>(tile);
  for (uint32_t i = nvec * 4 + threadIdx.x; i < bytes / 4; i += BLOCK) tw[i] = gw[i];
}

struct PackedArgs {
  const uint64_t* pack;
  int N, K, w;
  int uniform_cap, cap0;
  const int32_t* cap;
  const uint8_t* perms;
  int64_t C;
  int n, ld;
  int objective;
  uint64_t* keys;
  int32_t* sums;
  int32_t* maxs;
  int32_t* unv;
};

// Static CVRP, packed u64 matrix in LDS (tier 0).  Per customer c after
// prev: e = E[prev][c]; if dem(c) fits the remaining capacity the route
// grows by dur(prev,c), else the route closes with ret(prev) (kept from the
// previous gather) and vehicle k+1 opens with out(c).  Static H = 1, so a
// route's duration is the sum of its legs (A7, start time cancels).
template <int BLOCK, bool UNIFORM>
__global__ __launch_bounds__(BLOCK) void eval_cvrp_packed(PackedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N;
  const uint32_t ebytes = (uint32_t)N * N * 8;
  const uint32_t ebytes16 = (ebytes + 15) & ~15u;
  unsigned char* tile = smem + ebytes16;
  int32_t* capL = reinterpret_cast<int32_t*>(tile + (uint32_t)BLOCK * a.ld);
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.pack);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    for (uint32_t i = threadIdx.x; i < ebytes / 16; i += BLOCK) dst[i] = src[i];
    if ((ebytes & 8u) && threadIdx.x == 0)
      reinterpret_cast<uint64_t*>(smem)[ebytes / 8 - 1] = a.pack[ebytes / 8 - 1];
    if constexpr (!UNIFORM)
      for (int i = threadIdx.x; i < a.K; i += BLOCK) capL[i] = a.cap[i];
  }
  const uint64_t* E = reinterpret_cast<const uint64_t*>(smem);
  const int K = a.K, n = a.n, ld = a.ld;
  const uint32_t w = (uint32_t)a.w, wmask = (1u << w) - 1u, dshift = 2u * w;
  const int cap0 = a.cap0;

  for (int64_t base = blockIdx.x * (int64_t)BLOCK; base < a.C; base += (int64_t)gridDim.x * BLOCK) {
    const int rows = (int)min<int64_t>(BLOCK, a.C - base);
    __syncthreads();  // previous tile fully consumed (and E/capL staged on entry)
    stage_tile<BLOCK>(tile, a.perms + base * ld, (uint32_t)rows * ld);
    __syncthreads();
    if ((int)threadIdx.x >= rows) continue;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(tile + threadIdx.x * (uint32_t)ld);

    int k = 0;
    int rcap = UNIFORM ? cap0 : capL[0];
    uint32_t cur = 0, prow = 0, hprev = 0, dsum = 0, dmax = 0, unv = 0;
    auto visit = [&](uint32_t c) {
      const uint64_t e = E[prow + c];
      const uint32_t dur = (uint32_t)e, hi = (uint32_t)(e >> 32);
      const int dem = (int)(hi >> dshift);
      if (dem <= rcap) {
        cur += dur;
        rcap -= dem;
        prow = c * (uint32_t)N;
        hprev = hi;
      } else if (k >= K) {
        ++unv;
      } else {
        if (prow) {  // close the open route: prev -> depot
          const uint32_t rd = cur + (hprev & wmask);
          dsum += rd;
          dmax = max(dmax, rd);
        }
        ++k;
        while (k < K && dem > (UNIFORM ? cap0 : capL[k])) ++k;  // empty vehicles: unused
        if (k < K) {
          cur = (hi >> w) & wmask;  // depot -> c
          rcap = (UNIFORM ? cap0 : capL[k]) - dem;
          prow = c * (uint32_t)N;
          hprev = hi;
        } else {
          ++unv;
          rcap = INT_MIN;
          prow = 0;
        }
      }
    };
    const int n4 = n >> 2;
    for (int j = 0; j < n4; ++j) {
      const uint32_t w4 = row[j];
      visit(w4 & 0xffu);
      visit((w4 >> 8) & 0xffu);
      visit((w4 >> 16) & 0xffu);
      visit(w4 >> 24);
    }
    if (n & 3) {
      const uint32_t w4 = row[n4];
      for (int q = 0; q < (n & 3); ++q) visit((w4 >> (8 * q)) & 0xffu);
    }
    if (k < K && prow) {
      const uint32_t rd = cur + (hprev & wmask);
      dsum += rd;
      dmax = max(dmax, rd);
    }
    const int64_t c = base + threadIdx.x;
    a.keys[c] = cvrp_key(unv, dsum, dmax, a.objective);
    if (a.sums) a.sums[c] = (int32_t)dsum;
    if (a.maxs) a.maxs[c] = (int32_t)dmax;
    if (a.unv) a.unv[c] = (int32_t)unv;
  }
}

struct TspArgs {
  const void* mat;
  int N;
  const uint8_t* perms;
  int64_t C;
  int n, ld;
  uint64_t* keys;
  int32_t* sums;
  int32_t* maxs;
  int32_t* unv;
};

// Static TSP with the matrix LDS-resident and the tile staged through LDS.
template <int BLOCK, typename MatT>
__global__ __launch_bounds__(BLOCK) void eval_tsp_staged(TspArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N;
  const uint32_t mbytes = (uint32_t)N * N * sizeof(MatT);
  const uint32_t mbytes16 = (mbytes + 15) & ~15u;
  unsigned char* tile = smem + mbytes16;
  {
    const uint32_t* src = static_cast<const uint32_t*>(a.mat);
    uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
    for (uint32_t i = threadIdx.x; i < mbytes / 4; i += BLOCK) dst[i] = src[i];
    if ((mbytes & 2u) && threadIdx.x == 0)
      reinterpret_cast<uint16_t*>(smem)[mbytes / 2 - 1] =
          static_cast<const uint16_t*>(a.mat)[mbytes / 2 - 1];
  }
  const MatT* M = reinterpret_cast<const MatT*>(smem);
  const int n = a.n, ld = a.ld;
  for (int64_t base = blockIdx.x * (int64_t)BLOCK; base < a.C; base += (int64_t)gridDim.x * BLOCK) {
    const int rows = (int)min<int64_t>(BLOCK, a.C - base);
    __syncthreads();
    stage_tile<BLOCK>(tile, a.perms + base * ld, (uint32_t)rows * ld);
    __syncthreads();
    if ((int)threadIdx.x >= rows) continue;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(tile + threadIdx.x * (uint32_t)ld);
    uint32_t prow = 0, d = 0;
    auto visit = [&](uint32_t c) {
      d += (uint32_t)M[prow + c];
      prow = c * (uint32_t)N;
    };
    const int n4 = n >> 2;
    for (int j = 0; j < n4; ++j) {
      const uint32_t w4 = row[j];
      visit(w4 & 0xffu);
      visit((w4 >> 8) & 0xffu);
      visit((w4 >> 16) & 0xffu);
      visit(w4 >> 24);
    }
    if (n & 3) {
      const uint32_t w4 = row[n4];
      for (int q = 0; q < (n & 3); ++q) visit((w4 >> (8 * q)) & 0xffu);
    }
    d += (uint32_t)M[prow];
    const int64_t c = base + threadIdx.x;
    a.keys[c] = pack_key(0, d, 0);
    if (a.sums) a.sums[c] = (int32_t)d;
    if (a.maxs) a.maxs[c] = (int32_t)d;
    if (a.unv) a.unv[c] = 0;
  }
}

// ---------------------------------------------------------------------------
// Decode one giant tour (single lane; runs once per solve).
// ---------------------------------------------------------------------------
template <typename PermT>
__global__ void decode_kernel(const int32_t* __restrict__ M, int N, int H, int problem,
                              const int32_t* __restrict__ dem, const int32_t* __restrict__ cap,
                              const int32_t* __restrict__ start, int K, const PermT* perm, int n,
                              int32_t* vehicle_of, int32_t* route_dur) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t NN = (uint32_t)N * N;
  auto hr = [&](int t) { return (((uint32_t)t / 60u) % (uint32_t)H) * NN; };
  for (int k = 0; k < K; ++k) route_dur[k] = 0;
  if (problem == VRPMS_TSP) {
    int t = start[0];
    uint32_t prev = 0;
    for (int i = 0; i < n; ++i) {
      const uint32_t cc = min((uint32_t)perm[i], (uint32_t)N - 1);
      t += M[hr(t) + prev * N + cc];
      prev = cc;
      vehicle_of[i] = 0;
    }
    t += M[hr(t) + prev * N];
    route_dur[0] = t - start[0];
    return;
  }
  int k = 0, load = 0, t = start[0];
  uint32_t prev = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t cc = min((uint32_t)perm[i], (uint32_t)N - 1);
    const int dc = dem[cc];
    while (k < K && load + dc > cap[k]) {
      if (prev) {
        t += M[hr(t) + prev * N];
        route_dur[k] = t - start[k];
      }
      ++k;
      if (k < K) {
        load = 0;
        t = start[k];
        prev = 0;
      }
    }
    if (k < K) {
      t += M[hr(t) + prev * N + cc];
      load += dc;
      prev = cc;
      vehicle_of[i] = k;
    } else {
      vehicle_of[i] = -1;
    }
  }
  if (k < K && prev) {
    t += M[hr(t) + prev * N];
    route_dur[k] = t - start[k];
  }
}

// ---------------------------------------------------------------------------
// Argmin over keys: pass 1 min key, pass 2 smallest index holding it.
// ---------------------------------------------------------------------------
__global__ void min_key_kernel(const uint64_t* __restrict__ keys, int64_t C, uint64_t* out) {
  uint64_t v = ~0ull;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < C;
       i += (int64_t)gridDim.x * blockDim.x)
    v = min(v, keys[i]);
  v = wave_min_u64(v);
  if ((threadIdx.x & 63) == 0) atomicMin(reinterpret_cast<unsigned long long*>(out), v);
}

__global__ void min_index_kernel(const uint64_t* __restrict__ keys, int64_t C, uint64_t* out) {
  const uint64_t best = out[0];
  uint64_t idx = ~0ull;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < C;
       i += (int64_t)gridDim.x * blockDim.x)
    if (keys[i] == best) {
      idx = (uint64_t)i;
      break;
    }
  idx = wave_min_u64(idx);
  if ((threadIdx.x & 63) == 0) atomicMin(reinterpret_cast<unsigned long long*>(out + 1), idx);
}

template <typename K>
static void allow_lds(K kern, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <typename MatT, bool LDS, bool CVRP, typename PermT>
static int launch_generic_h(vrpms_ctx* ctx, const EvalArgs& a, hipStream_t s) {
  const Instance& in = ctx->inst;
  const int64_t blocks_needed = (a.C + 255) / 256;
  size_t lds = 0;
  int per_cu = 8;
  if (LDS) {
    lds = ((size_t)in.N * in.N * in.H * sizeof(MatT) + 15) & ~(size_t)15;
    per_cu = std::max<int>(1, std::min<int>(8, (int)(ctx->max_lds / std::max<size_t>(lds, 1))));
  }
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks_needed, (int64_t)ctx->num_cus * per_cu));
#define VRPMS_LAUNCH_G(HM)                                                     \
  do {                                                                         \
    auto kern = eval_generic<MatT, LDS, CVRP, HM, PermT>;                      \
    if (lds > 65536) allow_lds(kern, lds);                                     \
    kern<<<grid, 256, lds, s>>>(a);                                            \
  } while (0)
  if (in.H == 1)
    VRPMS_LAUNCH_G(1);
  else if (in.H == 24)
    VRPMS_LAUNCH_G(24);
  else
    VRPMS_LAUNCH_G(0);
#undef VRPMS_LAUNCH_G
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

template <typename PermT>
static int launch_generic(vrpms_ctx* ctx, EvalArgs a, hipStream_t s) {
  const Instance& in = ctx->inst;
  const bool lds = in.tier != kTierGlobal &&
                   (size_t)in.N * in.N * in.H * (in.use16 ? 2 : 4) <= 64 * 1024;
  const bool cvrp = in.problem == VRPMS_CVRP;
  a.mat = in.use16 ? static_cast<const void*>(in.mat16) : static_cast<const void*>(in.mat32);
  if (in.use16) {
    if (lds) return cvrp ? launch_generic_h<uint16_t, true, true, PermT>(ctx, a, s)
                         : launch_generic_h<uint16_t, true, false, PermT>(ctx, a, s);
    return cvrp ? launch_generic_h<uint16_t, false, true, PermT>(ctx, a, s)
                : launch_generic_h<uint16_t, false, false, PermT>(ctx, a, s);
  }
  if (lds) return cvrp ? launch_generic_h<int32_t, true, true, PermT>(ctx, a, s)
                       : launch_generic_h<int32_t, true, false, PermT>(ctx, a, s);
  return cvrp ? launch_generic_h<int32_t, false, true, PermT>(ctx, a, s)
              : launch_generic_h<int32_t, false, false, PermT>(ctx, a, s);
}

}  // namespace vrpms

using namespace vrpms;

// Which kernel vrpms_eval will use (exposed for tests and the bench).
extern "C" int vrpms_eval_path(vrpms_ctx* ctx, int32_t perm_bytes, int64_t ld, const void* d_perms) {
  if (!ctx || !ctx->has_instance) return -1;
  const Instance& in = ctx->inst;
  const bool aligned = ((uintptr_t)d_perms & 15u) == 0;
  const bool staged_ok = perm_bytes == 1 && (ld & 3) == 0 && aligned && in.N <= 256;
  if (in.problem == VRPMS_CVRP && in.tier == kTierLdsPacked && staged_ok) {
    const size_t need256 = (((size_t)in.N * in.N * 8 + 15) & ~(size_t)15) + 256 * (size_t)ld + 4 * in.K;
    if (need256 <= ctx->max_lds) return 0;
  }
  if (in.problem == VRPMS_TSP && in.H == 1 && staged_ok) {
    const size_t need = (((size_t)in.N * in.N * (in.use16 ? 2 : 4) + 15) & ~(size_t)15) + 256 * (size_t)ld;
    if (need <= ctx->max_lds) return 1;
  }
  return 2;
}

extern "C" int vrpms_eval(vrpms_ctx* ctx, const void* d_perms, int32_t perm_bytes, int64_t C,
                          int32_t n, int64_t ld, uint64_t* d_keys, int32_t* d_sum, int32_t* d_max,
                          int32_t* d_unv, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_eval: ctx is NULL");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_eval: no instance loaded");
  if (perm_bytes != 1 && perm_bytes != 2)
    return fail(VRPMS_EINVAL, "vrpms_eval: perm_bytes must be 1 or 2");
  if (C < 0 || n < 0 || ld < n) return fail(VRPMS_EINVAL, "vrpms_eval: need C >= 0, 0 <= n <= ld");
  if (C == 0) return VRPMS_OK;
  if (!d_perms || !d_keys) return fail(VRPMS_EINVAL, "vrpms_eval: d_perms/d_keys NULL");
  const Instance& in = ctx->inst;
  if (perm_bytes == 1 && in.N > 256)
    return fail(VRPMS_EINVAL, "vrpms_eval: uint8 tours need N <= 256");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  const int path = vrpms_eval_path(ctx, perm_bytes, ld, d_perms);
  if (path == 0) {
    PackedArgs p{in.pack64, in.N, in.K, in.pack_w, in.uniform_cap ? 1 : 0, in.cap0, in.cap,
                 static_cast<const uint8_t*>(d_perms), C, n, (int)ld, in.objective, d_keys, d_sum,
                 d_max, d_unv};
    const size_t e16 = ((size_t)in.N * in.N * 8 + 15) & ~(size_t)15;
    const bool big = e16 + 512 * (size_t)ld + 4 * in.K <= ctx->max_lds;
    const int block = big ? 512 : 256;
    const size_t lds = e16 + (size_t)block * ld + 4 * (size_t)in.K;
    const int per_cu = std::max<int>(1, (int)(ctx->max_lds / lds));
    const int64_t tiles = (C + block - 1) / block;
    const int grid = (int)std::min<int64_t>(tiles, (int64_t)ctx->num_cus * per_cu);
#define VRPMS_LAUNCH_P(B, U)                                \
  do {                                                      \
    auto kern = eval_cvrp_packed<B, U>;                     \
    allow_lds(kern, lds);                                   \
    kern<<<grid, B, lds, s>>>(p);                           \
  } while (0)
    if (big) {
      if (in.uniform_cap) VRPMS_LAUNCH_P(512, true); else VRPMS_LAUNCH_P(512, false);
    } else {
      if (in.uniform_cap) VRPMS_LAUNCH_P(256, true); else VRPMS_LAUNCH_P(256, false);
    }
#undef VRPMS_LAUNCH_P
    VRPMS_HIP(hipGetLastError());
    return VRPMS_OK;
  }
  if (path == 1) {
    TspArgs t{in.use16 ? static_cast<const void*>(in.mat16) : static_cast<const void*>(in.mat32),
              in.N, static_cast<const uint8_t*>(d_perms), C, n, (int)ld, d_keys, d_sum, d_max,
              d_unv};
    const size_t m16 = ((size_t)in.N * in.N * (in.use16 ? 2 : 4) + 15) & ~(size_t)15;
    const size_t lds = m16 + 256 * (size_t)ld;
    const int per_cu = std::max<int>(1, std::min<int>(8, (int)(ctx->max_lds / lds)));
    const int64_t tiles = (C + 255) / 256;
    const int grid = (int)std::min<int64_t>(tiles, (int64_t)ctx->num_cus * per_cu);
    if (in.use16) {
      auto kern = eval_tsp_staged<256, uint16_t>;
      allow_lds(kern, lds);
      kern<<<grid, 256, lds, s>>>(t);
    } else {
      auto kern = eval_tsp_staged<256, int32_t>;
      allow_lds(kern, lds);
      kern<<<grid, 256, lds, s>>>(t);
    }
    VRPMS_HIP(hipGetLastError());
    return VRPMS_OK;
  }
  EvalArgs a{nullptr, in.N, in.H, in.K, in.dem, in.cap, in.start, d_perms, C, n, ld,
             in.objective, d_keys, d_sum, d_max, d_unv};
  return perm_bytes == 1 ? launch_generic<uint8_t>(ctx, a, s) : launch_generic<uint16_t>(ctx, a, s);
}

extern "C" int vrpms_decode(vrpms_ctx* ctx, const void* d_perm, int32_t perm_bytes, int32_t n,
                            int32_t* d_vehicle_of, int32_t* d_route_dur, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_decode: ctx is NULL");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_decode: no instance loaded");
  if (perm_bytes != 1 && perm_bytes != 2) return fail(VRPMS_EINVAL, "vrpms_decode: perm_bytes");
  if (n < 0 || (n > 0 && (!d_perm || !d_vehicle_of)) || !d_route_dur)
    return fail(VRPMS_EINVAL, "vrpms_decode: bad buffers");
  VRPMS_HIP(hipSetDevice(ctx->device));
  const Instance& in = ctx->inst;
  hipStream_t s = (hipStream_t)stream;
  if (perm_bytes == 1)
    decode_kernel<uint8_t><<<1, 64, 0, s>>>(in.mat32, in.N, in.H, in.problem, in.dem, in.cap,
                                            in.start, in.K, static_cast<const uint8_t*>(d_perm), n,
                                            d_vehicle_of, d_route_dur);
  else
    decode_kernel<uint16_t><<<1, 64, 0, s>>>(in.mat32, in.N, in.H, in.problem, in.dem, in.cap,
                                             in.start, in.K, static_cast<const uint16_t*>(d_perm),
                                             n, d_vehicle_of, d_route_dur);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

extern "C" int vrpms_argmin(vrpms_ctx* ctx, const uint64_t* d_keys, int64_t C, uint64_t* d_out,
                            void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_argmin: ctx is NULL");
  if (!d_keys || !d_out || C <= 0) return fail(VRPMS_EINVAL, "vrpms_argmin: bad arguments");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  VRPMS_HIP(hipMemsetAsync(d_out, 0xff, 16, s));
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((C + 255) / 256, (int64_t)ctx->num_cus * 4));
  min_key_kernel<<<grid, 256, 0, s>>>(d_keys, C, d_out);
  min_index_kernel<<<grid, 256, 0, s>>>(d_keys, C, d_out);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}
