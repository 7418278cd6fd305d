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
//   (the headline uniform-fleet kernels eval_cvrp_words2 / eval_cvrp_rows2
//   live in eval_words.hip)
//   eval_generic      everything else: hour-indexed matrices (H = 24),
//                     uint16 tours, L2-resident matrices (N >= ~180),
//                     heterogeneous fleets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "common.hpp"
#include "ctx.hpp"
#include "split.hpp"
#include "staged.hpp"
#include "words.hpp"
#include "tour.hpp"

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

VRPMS_DEV void write_out(const EvalArgs& a, int64_t c, const TourCost& r) {
  a.keys[c] = r.key;
  if (a.sums) a.sums[c] = r.sum;
  if (a.maxs) a.maxs[c] = r.max;
  if (a.unv) a.unv[c] = r.unv;
}

// ---------------------------------------------------------------------------
// Generic lane-per-candidate evaluation (any tier / H / perm width / layout).
// ---------------------------------------------------------------------------
// Tour element i of candidate c in either layout.
template <typename PermT, bool WORDS>
struct TourAccess {
  const PermT* row;
  const uint32_t* w;
  int64_t C, c;
  VRPMS_DEV uint32_t operator()(int i) const {
    if constexpr (WORDS) return (w[(int64_t)(i >> 2) * C + c] >> (8 * (i & 3))) & 0xffu;
    else return (uint32_t)row[i];
  }
};

// Copy `bytes` (a multiple of 2) from global to LDS with dword moves.
VRPMS_DEV void stage_to_lds(unsigned char* dst, const void* src, uint32_t bytes) {
  const uint32_t* s = static_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (uint32_t i = threadIdx.x; i < bytes / 4; i += blockDim.x) d[i] = s[i];
  if ((bytes & 2u) && threadIdx.x == 0)
    reinterpret_cast<uint16_t*>(dst)[bytes / 2 - 1] = static_cast<const uint16_t*>(src)[bytes / 2 - 1];
}

template <typename MatT, bool LDS, bool CVRP, int HM, typename PermT, bool WORDS = false>
__global__ __launch_bounds__(256) void eval_generic(EvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t NN = (uint32_t)a.N * (uint32_t)a.N;
  const MatT* M = static_cast<const MatT*>(a.mat);
  if constexpr (LDS) {
    stage_to_lds(smem, a.mat, NN * (uint32_t)a.H * sizeof(MatT));
    __syncthreads();
    M = reinterpret_cast<const MatT*>(smem);
  }
  const MatView<MatT, HM> D{M, (uint32_t)a.N, NN, a.H};
  const SplitParams sp{a.dem, a.cap, a.start, a.K, a.objective};
  const PermT* P = static_cast<const PermT*>(a.perms);
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < a.C;
       c += (int64_t)gridDim.x * blockDim.x) {
    const TourAccess<PermT, WORDS> tour{P + c * a.ld, static_cast<const uint32_t*>(a.perms), a.C, c};
    write_out(a, c, eval_tour<CVRP>(D, sp, tour, a.n));
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
  const v4u* gs = reinterpret_cast<const v4u*>(g);
  v4u* ts = reinterpret_cast<v4u*>(tile);
  for (uint32_t i = threadIdx.x; i < nvec; i += BLOCK) ts[i] = gs[i];
  const uint32_t* gw = reinterpret_cast<const uint32_t*>(g);
  uint32_t* tw = reinterpret_cast<uint32_t*>(tile);
  for (uint32_t i = nvec * 4 + threadIdx.x; i < bytes / 4; i += BLOCK) tw[i] = gw[i];
}

struct PackedArgs {
  const uint64_t* pack;
  int N, K, w;
  int uniform_cap, cap0;
  uint32_t lim, smask;  // MODE 1: (cap0 + 1) << S and (1 << S) - 1
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
//
// Address chain: the gather for position i reads E[p(i-1)][p(i)], which
// depends only on the tour -- never on the split state -- because a
// visited customer always becomes `prev` and, once every vehicle is closed
// (k == K), `prev` is never read again.  So the gathers of a whole perm
// word (4 customers) are issued one word ahead of the split arithmetic and
// the LDS latency overlaps the VALU work instead of serialising it.
//
// Tile pipeline: the next tile's tours are loaded into registers (16-B
// coalesced loads) while the current tile is scored, then written to the
// LDS tile between two barriers.
template <int NV>
VRPMS_DEV void prefetch_tile(v4u (&pf)[NV], const unsigned char* g, uint32_t bytes, int block) {
  // unconditional (clamped) loads keep pf[] in registers
  const uint32_t last = bytes >= 16 ? bytes / 16 - 1 : 0;
  const v4u* gs = reinterpret_cast<const v4u*>(g);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const uint32_t idx = threadIdx.x + (uint32_t)v * block;
    pf[v] = gs[min(idx, last)];
  }
}

template <int NV>
VRPMS_DEV void commit_tile(const v4u (&pf)[NV], unsigned char* tile, const unsigned char* g,
                           uint32_t bytes, int block) {
  const uint32_t nvec = bytes / 16;
  v4u* ts = reinterpret_cast<v4u*>(tile);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const uint32_t idx = threadIdx.x + (uint32_t)v * block;
    if (idx < nvec) ts[idx] = pf[v];
  }
  // ragged last tile: the few trailing dwords are copied directly
  const uint32_t* gw = reinterpret_cast<const uint32_t*>(g);
  uint32_t* tw = reinterpret_cast<uint32_t*>(tile);
  for (uint32_t i = nvec * 4 + threadIdx.x; i < bytes / 4; i += block) tw[i] = gw[i];
}

// MODE 0: heterogeneous fleet (capacities from LDS, branchy split)
// MODE 1: uniform fleet, "prefix-ret" layout (branch-free split, see step())
// MODE 2: uniform fleet, branchy split (when the prefix-ret fields do not fit)
template <int BLOCK, int MODE, int NV>
__global__ __launch_bounds__(BLOCK) void eval_cvrp_packed(PackedArgs a) {
  constexpr bool UNIFORM = MODE != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N;
  const uint32_t ebytes = (uint32_t)N * N * 8;
  const uint32_t ebytes16 = (ebytes + 15) & ~15u;
  unsigned char* tile = smem + ebytes16;
  int32_t* capL = reinterpret_cast<int32_t*>(tile + (uint32_t)BLOCK * a.ld + 16);
  {
    const v4u* src = reinterpret_cast<const v4u*>(a.pack);
    v4u* dst = reinterpret_cast<v4u*>(smem);
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
  const uint32_t lim = a.lim, smask = a.smask;
  const int64_t stride = (int64_t)gridDim.x * BLOCK;
  const int nwords = (n + 3) >> 2;

  v4u pf[NV];
  int64_t base = blockIdx.x * (int64_t)BLOCK;
  if (base < a.C)
    prefetch_tile<NV>(pf, a.perms + base * ld, (uint32_t)min<int64_t>(BLOCK, a.C - base) * ld,
                      BLOCK);
  for (; base < a.C; base += stride) {
    const int rows = (int)min<int64_t>(BLOCK, a.C - base);
    __syncthreads();  // previous tile consumed (and E / capL staged on entry)
    commit_tile<NV>(pf, tile, a.perms + base * ld, (uint32_t)rows * ld, BLOCK);
    __syncthreads();
    const int64_t nbase = base + stride;
    if (nbase < a.C)
      prefetch_tile<NV>(pf, a.perms + nbase * ld, (uint32_t)min<int64_t>(BLOCK, a.C - nbase) * ld,
                        BLOCK);
    if ((int)threadIdx.x >= rows) continue;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(tile + threadIdx.x * (uint32_t)ld);

    uint32_t dsum = 0, dmax = 0, unv = 0;
    int k = 0;
    // MODE 1 state (prefix-ret): acc = load << S | (cur + ret(prev))
    uint32_t acc = 0;
    bool dead = false;  // all K vehicles closed: customers unvisited, separators ignored
    // MODE 0/2 state
    int rcap = MODE == 0 ? capL[0] : cap0;
    // hprev is held in 64 bits (only its low word is read): as a uint32_t,
    // SimplifyCFG merged the separator branch's "rcap = ...; return" with the
    // customer path's "hprev = hi" into one store through a phi of their
    // addresses, and both stayed in scratch memory (MODE 0 / 2); stores of
    // different types are never merged
    uint32_t cur = 0;
    uint64_t hprev = 0;
    bool open = false;  // the current route holds a customer
    // one split step for token c (A10: c == 0 is a route separator)
    auto step = [&](uint64_t e, uint32_t c) {
      const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
      if constexpr (MODE == 1) {
        // one add + one unsigned compare is the capacity test (the load sits
        // above bit S); closing a route reads its duration straight out of
        // the low field because ret(prev) is pre-added
        if (dead) {
          unv += c != 0u;
          return;
        }
        const uint32_t t = acc + lo;
        if (c != 0u && t < lim) {
          acc = t;
          return;
        }
        const uint32_t rd = acc & smask;  // close route k (0 when empty)
        dsum += rd;
        dmax = max(dmax, rd);
        ++k;
        if (c == 0u) {
          dead = k >= K;
          acc = 0;
        } else if (k >= K || hi >= lim) {  // no vehicle left / c fits no empty vehicle
          dead = true;
          ++unv;
        } else {
          acc = hi;  // hi = open'(c): a fresh route holding c
        }
      } else {
        if (c == 0u) {  // separator: close route k (if any), open vehicle k + 1
          if (k < K) {
            if (open) {
              const uint32_t rd = cur + (hprev & wmask);
              dsum += rd;
              dmax = max(dmax, rd);
            }
            ++k;
            open = false;
            cur = 0;
            rcap = k < K ? (MODE == 2 ? cap0 : capL[k]) : INT_MIN;
          }
          return;
        }
        const int dem = (int)(hi >> dshift);
        if (dem <= rcap) {
          cur += lo;
          rcap -= dem;
          open = true;
        } else if (k >= K) {
          ++unv;
        } else {
          if (open) {  // close the open route: prev -> depot
            const uint32_t rd = cur + (hprev & wmask);
            dsum += rd;
            dmax = max(dmax, rd);
          }
          ++k;
          if constexpr (MODE == 2) {
            if (dem > cap0) k = K;  // fits no (empty) vehicle: all remaining ones unused
          } else {
            while (k < K && dem > capL[k]) ++k;
          }
          if (k < K) {
            cur = (hi >> w) & wmask;  // depot -> c
            rcap = (MODE == 2 ? cap0 : capL[k]) - dem;
            open = true;
          } else {
            ++unv;
            rcap = INT_MIN;
            open = false;
          }
        }
        hprev = hi;
      }
    };
    // byte offsets of E[a][b]: a * 8N + 8b with 24-bit multiplies
    const uint32_t N8 = 8u * (uint32_t)N;
    const unsigned char* Eb = reinterpret_cast<const unsigned char*>(E);
    auto gat = [&](uint32_t a_, uint32_t b_) {
      return *reinterpret_cast<const uint64_t*>(Eb + (__umul24(a_, N8) + (b_ << 3)));
    };
    uint32_t wd = row[0];
    uint32_t c0 = wd & 0xffu, c1 = (wd >> 8) & 0xffu, c2 = (wd >> 16) & 0xffu, c3 = wd >> 24;
    uint64_t e0 = gat(0, c0), e1 = gat(c0, c1), e2 = gat(c1, c2), e3 = gat(c2, c3);
    for (int j = 0; j < nwords; ++j) {
      // issue the next word's gathers before consuming this word's
      const uint32_t wn = row[j + 1];
      const uint32_t n0 = wn & 0xffu, n1 = (wn >> 8) & 0xffu, n2 = (wn >> 16) & 0xffu,
                     n3 = wn >> 24;
      const uint64_t f0 = gat(c3, n0), f1 = gat(n0, n1), f2 = gat(n1, n2), f3 = gat(n2, n3);
      const int pos = 4 * j;
      step(e0, c0);
      if (pos + 1 < n) step(e1, c1);
      if (pos + 2 < n) step(e2, c2);
      if (pos + 3 < n) step(e3, c3);
      c0 = n0;
      c1 = n1;
      c2 = n2;
      c3 = n3;
      e0 = f0;
      e1 = f1;
      e2 = f2;
      e3 = f3;
    }
    if constexpr (MODE == 1) {
      if (!dead && n > 0) {
        const uint32_t rd = acc & smask;
        dsum += rd;
        dmax = max(dmax, rd);
      }
    } else {
      if (k < K && open) {
        const uint32_t rd = cur + (hprev & wmask);
        dsum += rd;
        dmax = max(dmax, rd);
      }
    }
    const int64_t c = base + threadIdx.x;
    a.keys[c] = cvrp_key(unv, dsum, dmax, a.objective);
    if (a.sums) a.sums[c] = (int32_t)dsum;
    if (a.maxs) a.maxs[c] = (int32_t)dmax;
    if (a.unv) a.unv[c] = (int32_t)unv;
  }
}

// rows (uint8 [C][ld]) -> words (uint32 [ceil(n/4)][C]); one lane per (word, candidate)
__global__ void rows_to_words_kernel(const uint8_t* __restrict__ rows, int64_t C, int n,
                                     int64_t ld, uint32_t* __restrict__ words) {
  const int nw = (n + 3) >> 2;
  const int64_t total = (int64_t)nw * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i / C);
    const int64_t c = i - (int64_t)w * C;
    const uint8_t* r = rows + c * ld + 4 * w;
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * w + q < n) v |= (uint32_t)r[q] << (8 * q);
    words[i] = v;
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
    if (cc == 0) {  // A10 separator
      vehicle_of[i] = -2;
      if (k < K) {
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
      continue;
    }
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

template <typename MatT, bool LDS, bool CVRP, typename PermT, bool WORDS>
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
    auto kern = eval_generic<MatT, LDS, CVRP, HM, PermT, WORDS>;               \
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

template <typename PermT, bool WORDS = false>
static int launch_generic(vrpms_ctx* ctx, EvalArgs a, hipStream_t s) {
  const Instance& in = ctx->inst;
  const bool lds = in.tier != kTierGlobal &&
                   (size_t)in.N * in.N * in.H * (in.use16 ? 2 : 4) <= 64 * 1024;
  const bool cvrp = in.problem == VRPMS_CVRP;
  a.mat = in.use16 ? static_cast<const void*>(in.mat16) : static_cast<const void*>(in.mat32);
  if (in.use16) {
    if (lds) return cvrp ? launch_generic_h<uint16_t, true, true, PermT, WORDS>(ctx, a, s)
                         : launch_generic_h<uint16_t, true, false, PermT, WORDS>(ctx, a, s);
    return cvrp ? launch_generic_h<uint16_t, false, true, PermT, WORDS>(ctx, a, s)
                : launch_generic_h<uint16_t, false, false, PermT, WORDS>(ctx, a, s);
  }
  if (lds) return cvrp ? launch_generic_h<int32_t, true, true, PermT, WORDS>(ctx, a, s)
                       : launch_generic_h<int32_t, true, false, PermT, WORDS>(ctx, a, s);
  return cvrp ? launch_generic_h<int32_t, false, true, PermT, WORDS>(ctx, a, s)
              : launch_generic_h<int32_t, false, false, PermT, WORDS>(ctx, a, s);
}

// words-layout fast path available? (uniform fleet, prefix-ret layout, matrix fits LDS)
static bool words_fast_ok(const vrpms_ctx* ctx) {
  const Instance& in = ctx->inst;
  return in.problem == VRPMS_CVRP && in.pack64p && ctx->opt_split_mode != 2 &&
         (size_t)in.N * in.N * 8 <= ctx->max_lds;
}

// Exactness conditions of the branch-free split (split.hpp): every demand fits
// an empty vehicle, the vehicle counter fits above the duration sum in dsum,
// and DEAD stays below 2^32.
bool fast_split_params(const vrpms_ctx* ctx, int n, FastSplit* out) {
  const Instance& in = ctx->inst;
  if (!words_fast_ok(ctx) || !in.pack64w || in.max_dem > in.cap0) return false;
  const int64_t sum_bound = (int64_t)(n + in.K + 1) * std::max(in.max_dur, 1);
  int ks = 1;
  while (ks < 31 && ((int64_t)1 << ks) <= sum_bound) ++ks;
  const int B = 31 - ks;  // width of dsum's vehicle counter (bit 31 = exhausted)
  if (B < 1 || ((int64_t)1 << B) <= std::max<int64_t>(in.K, n)) return false;
  if ((((int64_t)in.cap0 + in.max_dem + 3) << in.pref_S) > ((int64_t)1 << 31)) return false;
  out->pack = in.pack64w;
  out->N = in.N;
  out->K = in.K;
  out->objective = in.objective;
  out->lim = in.pref_lim;
  out->smask = in.pref_smask;
  out->ks = (uint32_t)ks;
  out->klim = (uint32_t)((((int64_t)1 << B) - in.K) << ks);
  out->dead = (uint32_t)1u << in.pref_S;
  out->carry = in.min_dem >= 1;
  return true;
}

template <int NV>
static int launch_packed(const PackedArgs& p, bool big, int mode, int grid, size_t lds,
                         hipStream_t s) {
  auto go = [&](auto kern, int block) {
    allow_lds(kern, lds);
    kern<<<grid, block, lds, s>>>(p);
  };
  if (big) {
    if (mode == 1) go(eval_cvrp_packed<512, 1, NV>, 512);
    else if (mode == 2) go(eval_cvrp_packed<512, 2, NV>, 512);
    else go(eval_cvrp_packed<512, 0, NV>, 512);
  } else {
    if (mode == 1) go(eval_cvrp_packed<256, 1, NV>, 256);
    else if (mode == 2) go(eval_cvrp_packed<256, 2, NV>, 256);
    else go(eval_cvrp_packed<256, 0, NV>, 256);
  }
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

// Split variant for the packed path: 1 (prefix-ret) whenever its layout was
// built, unless a test forced 2 through vrpms_set_option.
static int packed_mode(const vrpms_ctx* ctx) {
  const Instance& in = ctx->inst;
  if (!in.uniform_cap) return 0;
  if (in.pack64p && ctx->opt_split_mode != 2) return 1;
  return 2;
}

}  // namespace vrpms

using namespace vrpms;

// Which kernel vrpms_eval will use (exposed for tests and the bench).
extern "C" int vrpms_eval_path(vrpms_ctx* ctx, int32_t perm_bytes, int64_t ld, const void* d_perms) {
  if (!ctx || !ctx->has_instance) return -1;
  const Instance& in = ctx->inst;
  const bool aligned = ((uintptr_t)d_perms & 15u) == 0;
  const bool staged_ok = perm_bytes == 1 && (ld & 3) == 0 && aligned && in.N <= 256;
  if (in.problem == VRPMS_CVRP && in.tier == kTierLdsPacked && staged_ok && ld <= 128) {
    const size_t need256 =
        (((size_t)in.N * in.N * 8 + 15) & ~(size_t)15) + 256 * (size_t)ld + 16 + 4 * in.K;
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
    FastSplit f;
    if (ctx->opt_words_kernel != 1 && fast_split_params(ctx, n, &f) &&
        rows2_chunk_words(ctx, f, n) > 0) {
      RowsArgs r{f, static_cast<const unsigned char*>(d_perms), C, n, (int)ld,
                 d_keys, d_sum, d_max, d_unv};
      return launch_rows2(ctx, r, s);
    }
    const int mode = packed_mode(ctx);
    PackedArgs p{mode == 1 ? in.pack64p : in.pack64, in.N, in.K, in.pack_w,
                 in.uniform_cap ? 1 : 0, in.cap0, in.pref_lim, in.pref_smask, in.cap,
                 static_cast<const uint8_t*>(d_perms), C, n, (int)ld, in.objective, d_keys, d_sum,
                 d_max, d_unv};
    const size_t e16 = ((size_t)in.N * in.N * 8 + 15) & ~(size_t)15;
    const bool big = e16 + 512 * (size_t)ld + 16 + 4 * in.K <= ctx->max_lds;
    const int block = big ? 512 : 256;
    const size_t lds = e16 + (size_t)block * ld + 16 + 4 * (size_t)in.K;
    const int per_cu = std::max<int>(1, (int)(ctx->max_lds / lds));
    const int64_t tiles = (C + block - 1) / block;
    const int grid = (int)std::min<int64_t>(tiles, (int64_t)ctx->num_cus * per_cu);
    return ld <= 32 ? launch_packed<2>(p, big, mode, grid, lds, s)
         : ld <= 64 ? launch_packed<4>(p, big, mode, grid, lds, s)
                    : launch_packed<8>(p, big, mode, grid, lds, s);
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
  if (staged_fits(ctx))
    return launch_staged(ctx, d_perms, perm_bytes, C, n, ld, d_keys, d_sum, d_max, d_unv, s);
  EvalArgs a{nullptr, in.N, in.H, in.K, in.dem, in.cap, in.start, d_perms, C, n, ld,
             in.objective, d_keys, d_sum, d_max, d_unv};
  return perm_bytes == 1 ? launch_generic<uint8_t>(ctx, a, s) : launch_generic<uint16_t>(ctx, a, s);
}

extern "C" int vrpms_eval_words(vrpms_ctx* ctx, const uint32_t* d_words, int64_t C, int32_t n,
                                uint64_t* d_keys, int32_t* d_sum, int32_t* d_max, int32_t* d_unv,
                                void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_eval_words: ctx is NULL");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_eval_words: no instance loaded");
  if (C < 0 || n < 0) return fail(VRPMS_EINVAL, "vrpms_eval_words: need C >= 0, n >= 0");
  if (C == 0) return VRPMS_OK;
  if (!d_words || !d_keys) return fail(VRPMS_EINVAL, "vrpms_eval_words: d_words/d_keys NULL");
  const Instance& in = ctx->inst;
  if (in.N > 256) return fail(VRPMS_EINVAL, "vrpms_eval_words: uint8 tours need N <= 256");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  FastSplit f;
  if (fast_split_params(ctx, n, &f)) {
    // ring depth: the R in [4, 8] that wastes the fewest slots on ceil(n/4) words
    WordsArgs w{f, d_words, C, n, d_keys, d_sum, d_max, d_unv, C, 1u};
    return launch_words2(ctx, w, words2_ring(n), s);
  }
  EvalArgs a{nullptr, in.N, in.H, in.K, in.dem, in.cap, in.start, d_words, C, n, 0,
             in.objective, d_keys, d_sum, d_max, d_unv};
  return launch_generic<uint8_t, true>(ctx, a, s);
}

extern "C" int vrpms_rows_to_words(vrpms_ctx* ctx, const uint8_t* d_rows, int64_t C, int32_t n,
                                   int64_t ld, uint32_t* d_words, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_rows_to_words: ctx is NULL");
  if (C < 0 || n < 0 || ld < n) return fail(VRPMS_EINVAL, "vrpms_rows_to_words: bad shape");
  if (C == 0 || n == 0) return VRPMS_OK;
  if (!d_rows || !d_words) return fail(VRPMS_EINVAL, "vrpms_rows_to_words: NULL buffer");
  VRPMS_HIP(hipSetDevice(ctx->device));
  const int64_t total = (int64_t)((n + 3) / 4) * C;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, (int64_t)ctx->num_cus * 8));
  rows_to_words_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(d_rows, C, n, ld, d_words);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
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
