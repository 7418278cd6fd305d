// SA on hour-indexed matrices (A3: time_of_day, src/solver.py:7 -- the
// reference's normal VRP request, api/vrp/sa/index.py:40-45, with
// per-vehicle capacities and start times, api/parameters.py:11-12) by full
// walks whose matrix reads are LDS reads.
//
// On an hour-indexed matrix a move's price depends on the clock at every
// position after it, so every candidate is walked in full (the greedy split
// with per-vehicle capacities and start times, eval_tour).  What bounds that
// walk on the L2 tier (sa_kernel) is one dependent L2 gather per token: the
// hour of an edge is known only when the clock reaches it.  Here the clock
// does not decide WHICH entry is read, only which of an edge's 24 hourly
// values: every edge of the current tour keeps its 24 durations in LDS
// (48 bytes, hour-minor rows of the [N][N][24] copy the context builds), so
// a token costs one dependent ds_read_u16 at row + 2 hour(t).
//
//   F[q]   row of the edge tour[q-1] -> tour[q] (tour[-1] = the depot)
//   R[q]   row of tour[q+1] -> tour[q] (asymmetric matrices only; on a
//          symmetric one it is F[q+1])
//   LEG[c] depot legs 0 -> c and c -> 0 (two rows, shared by the workgroup)
//   J      each lane's four junction rows: every adjacency of the moved tour
//          except at positions lo, lo+1, hi, hi+1 is one of the current
//          tour's, forward or reversed; those four are fetched per step from
//          the hour-minor copy in L2 (12 independent 16-byte loads).
//
// An accepted move rewrites F (and R) over its span [lo-1, hi+1] from the
// old rows (shifted / reversed) and the new junctions (L2), through the J
// area as a temporary.  W wavefronts per chain price 64 W moves per step
// (move index lane + 64 w, (key, index) minimum across wavefronts), as in
// sa_route_kernel.  The arithmetic is eval_tour's on the same values, so the
// trajectories equal sa_kernel's and the C restatement's full re-evaluation.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "ctx.hpp"
#include "staging.hpp"
#include "tour.hpp"

namespace vrpms {

constexpr int kTdH = 24;
constexpr uint32_t kTdRow = 48;  // bytes: one edge's 24 hourly u16 durations
constexpr int kTdMaxWaves = 4;
constexpr uint32_t kTdXBytes = 2 * kTdMaxWaves * 32;
constexpr int kTdUnroll = 8;  // tokens whose addresses / demands are read ahead of the clock

typedef __attribute__((address_space(3))) const uint16_t td_lds_u16;
typedef __attribute__((address_space(3))) const unsigned char td_lds_uc;
typedef __attribute__((address_space(3))) const v4u td_lds_v4u;

struct TdArgs {
  SearchInst si;       // matrix not staged (mat_lds = 0): dem / cap / start in LDS
  const uint16_t* mh;  // [N][N][24] hour-minor copy of the u16 matrix
  int chains, n, steps, window;
  uint32_t window_types;
  float inv_t0, inv_alpha;
  uint32_t seed_lo, seed_hi;
  uint64_t step0;
  uint16_t* cur;
  uint64_t* cur_key;
  uint16_t* best;
  uint64_t* best_key;
  int W, CPW, sym;
  uint32_t legs_off, veh_off, chains_off, chain_bytes, npad, jbytes;
};

// per-chain LDS: tours (current, next, best), F, R (asymmetric), J / temp, exchange
__host__ __device__ inline uint32_t td_tours_bytes(uint32_t npad) { return (6u * npad + 15u) & ~15u; }
__host__ __device__ inline uint32_t td_rows_bytes(uint32_t npad, bool sym) {
  return npad * kTdRow * (sym ? 1u : 2u);
}
// shared LDS after the instance: LEG rows (OUT | RET per node), a zero row, vehicles
__host__ __device__ inline uint32_t td_legs_bytes(int N) { return (uint32_t)N * 2u * kTdRow + 2u * kTdRow; }
__host__ __device__ inline uint32_t td_veh_bytes(int K) { return ((uint32_t)K + 1u) * 16u; }

// 48-byte row of edge (x, y) in the hour-minor copy, as three 16-byte words
VRPMS_DEV const v4u* td_grow(const uint16_t* mh, uint32_t N, uint32_t x, uint32_t y) {
  return reinterpret_cast<const v4u*>(mh + ((size_t)x * N + y) * kTdH);
}

struct TdChain {
  uint32_t A;         // LDS byte address of the current tour (u16 tokens)
  uint32_t F, R;      // LDS byte addresses of the row caches (R == F + 48 on a symmetric matrix)
  uint32_t LEG, ZR;   // depot legs (OUT at +0, RET at +48, 96 bytes per node), a zero row
  uint32_t VEH;       // vehicles: {capacity, start minute of the day, 2 hour(start), valid}
  uint32_t DEM;       // demands (i32)
  const int32_t* cap;
  const int32_t* start;
  int K, objective;
  uint32_t Nm1;
  uint32_t ncust;     // customer tokens of the tour (moves permute them)
  bool sym;
};

VRPMS_DEV int td_rd(uint32_t addr) { return (int)*(td_lds_u16*)(uintptr_t)addr; }
VRPMS_DEV uint32_t td_rd32(uint32_t addr) {
  return *(__attribute__((address_space(3))) const uint32_t*)(uintptr_t)addr;
}

// Minute of the day (t mod 1440) after adding a duration e <= 65535 to a
// minute of the day: floor(x / 1440) = hi32(x * 2982617) for x < 2^17 (one
// full-rate 24-bit multiply), so the clock's hour never needs a 32-bit divide.
VRPMS_DEV uint32_t td_day_add(uint32_t tm, uint32_t e) {
  const uint32_t x = (tm + e) & 0x1ffffu;  // < 1440 + 65536; the mask lets LLVM pick v_mul_hi_u32_u24
  const int d = (int)(((uint64_t)x * 2982617u) >> 32);
  return (uint32_t)(__mul24(d, -1440) + (int)x);  // v_mad_i32_i24
}
// byte offset of the hour of minute-of-day tm (< 1440) in a 24-entry u16 row:
// floor(tm / 60) = (tm * 1093) >> 16 on [0, 1440)
VRPMS_DEV uint32_t td_hoff(uint32_t tm) { return (__umul24(tm, 1093u) >> 15) & ~1u; }

// Per-token addresses of the moved tour, read ahead of the clock: the row of
// the edge into position q and the token there.  All U positions first (VALU
// only), then the U token reads, so their LDS round trips overlap.
struct TdAhead {
  uint32_t wbr, F48, jA, jB;
  int wsr;
  MoveMap mm;
  int lo, hi;
  template <int U>
  VRPMS_DEV void block(const TdChain& C, int base, int n, uint32_t (&ra)[U], uint32_t (&tk)[U]) const {
    uint32_t pa[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = min(base + u, n - 1);  // past the end: the last token again (not walked)
      const bool inw = (uint32_t)(q - mm.lo) < (uint32_t)mm.len;
      const int pw = mm.a + __mul24(mm.s, q);
      int p = inw ? pw : q;
      p = q == mm.p1 ? mm.v1 : p;
      p = q == mm.p2 ? mm.v2 : p;
      pa[u] = C.A + 2u * (uint32_t)p;
      // a window's adjacencies run forward (relocate) or reversed (2-opt);
      // the four junction positions read the lane's J rows
      const uint32_t wq = wbr + (uint32_t)__mul24(wsr, q), fq = F48 + 48u * (uint32_t)q;
      const uint32_t ja = jA + 48u * (uint32_t)q, jbq = jB + 48u * (uint32_t)q;
      uint32_t r = inw ? wq : fq;
      r = (uint32_t)(q - lo) < 2u ? ja : r;
      r = (uint32_t)(q - hi) < 2u ? jbq : r;
      ra[u] = r;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) tk[u] = min((uint32_t)td_rd(pa[u]), C.Nm1);
  }
};

// The moved tour (identity map and no junctions for the current tour) walked
// with eval_tour's arithmetic; every duration is read from an LDS row at the
// hour of the clock.  jb: LDS address of the lane's four junction rows
// (positions lo, lo + 1, hi, hi + 1).  FAST (every demand fits every
// vehicle) runs each token without a branch: a wavefront whose lanes close
// routes at different tokens would otherwise run every path at every token.
// The state is the route's elapsed time el (a route lasts el + its return
// leg), the clock's minute of the day tm and its hour offset h; the next
// vehicle's record is read ahead, and a route with no customer yet points
// its return leg at the zero row.  The clock's critical chain per token:
// h -> ds_read_u16 -> tm + e (mod 1440) -> h.
template <bool CVRP, bool FAST>
VRPMS_DEV TourCost td_walk(const TdChain& C, const MoveMap& mm, int lo, int hi, uint32_t jb, int n) {
  TdAhead ah;
  ah.F48 = C.F;
  ah.jA = jb - (uint32_t)__mul24(48, lo);
  ah.jB = jb + 96u - (uint32_t)__mul24(48, hi);
  ah.wsr = 48 * mm.s;
  ah.mm = mm;
  ah.lo = lo;
  ah.hi = hi;
  ah.wbr = mm.s > 0 ? C.F + (uint32_t)__mul24(48, mm.a)
                    : (C.sym ? C.F + (uint32_t)__mul24(48, mm.a + 1) : C.R + (uint32_t)__mul24(48, mm.a));
  const v4u v0 = *(td_lds_v4u*)(uintptr_t)C.VEH;
  uint32_t tm = v0.y, h = v0.z;
  int capk = (int)v0.x;
  uint32_t el = 0, dsum = 0, dmax = 0, unv = 0;
  int load = 0;
  if constexpr (!CVRP) {
    uint32_t last = 0;
    for (int base = 0; base < n; base += kTdUnroll) {
      uint32_t ra[kTdUnroll], tk[kTdUnroll];
      ah.block(C, base, n, ra, tk);
#pragma unroll
      for (int u = 0; u < kTdUnroll; ++u) {
        const bool v = base + u < n;
        const uint32_t e = v ? (uint32_t)td_rd(ra[u] + h) : 0u;
        el += e;
        tm = td_day_add(tm, e);
        h = td_hoff(tm);
        last = v ? tk[u] : last;
      }
    }
    el += (uint32_t)td_rd(C.LEG + (uint32_t)__mul24(96, last) + 48u + h);
    const int d = (int)el;
    return {pack_key(0, (uint32_t)d, 0), d, d, 0};
  } else if constexpr (FAST) {
    // no loop-carried booleans (LLVM keeps those as 0/1 VGPRs re-tested
    // every token): a dead fleet is capk = -1 (the sentinel vehicle's
    // capacity), so every customer then "closes" onto the sentinel, which
    // links to itself; an empty route is pret == ZR; unv = customers - served
    uint32_t vaddr = C.VEH + 16u;
    v4u rec = *(td_lds_v4u*)(uintptr_t)vaddr;  // the next vehicle
    uint32_t pret = C.ZR, served = 0;
    for (int base = 0; base < n; base += kTdUnroll) {
      uint32_t ra[kTdUnroll], tk[kTdUnroll];
      int dm[kTdUnroll];
      ah.block(C, base, n, ra, tk);
#pragma unroll
      for (int u = 0; u < kTdUnroll; ++u) dm[u] = (int)td_rd32(C.DEM + 4u * tk[u]);
#pragma unroll
      for (int u = 0; u < kTdUnroll; ++u) {
        const bool v = base + u < n;  // wave-uniform
        const uint32_t cc = tk[u];
        const int dc = dm[u];
        const bool sep = cc == 0;     // A10 separator: closes route k, opens vehicle k + 1
        const bool close = v && (sep || load + dc > capk);
        const uint32_t rdur = el + (uint32_t)td_rd(pret + h);
        const uint32_t dv = close ? rdur : 0u;
        dsum += dv;
        dmax = max(dmax, dv);
        capk = close ? (int)rec.x : capk;
        tm = close ? rec.y : tm;
        h = close ? rec.z : h;
        vaddr = close ? rec.w : vaddr;
        el = close ? 0u : el;
        load = close ? 0 : load;
        pret = close ? C.ZR : pret;
        rec = *(td_lds_v4u*)(uintptr_t)vaddr;
        const bool serve = v && !sep && capk >= 0;
        const uint32_t lg = C.LEG + (uint32_t)__mul24(96, (int)cc);
        uint32_t row = pret != C.ZR ? ra[u] : lg;
        row = serve ? row : C.ZR;
        const uint32_t e = (uint32_t)td_rd(row + h);
        el += e;
        tm = td_day_add(tm, e);
        h = td_hoff(tm);
        load += serve ? dc : 0;
        pret = serve ? lg + 48u : pret;
        served += serve ? 1u : 0u;
      }
    }
    if (capk >= 0) {
      const uint32_t rdur = el + (uint32_t)td_rd(pret + h);
      dsum += rdur;
      dmax = max(dmax, rdur);
    }
    unv = C.ncust - served;
    return {cvrp_key(unv, dsum, dmax, C.objective), (int32_t)dsum, (int32_t)dmax, (int32_t)unv};
  } else {
    // a demand may exceed a vehicle's capacity: eval_tour's per-token
    // branches (empty vehicles close until one takes the customer)
    int t = C.start[0], stk = t;
    tm = (uint32_t)t % 1440u;
    int k = 0;
    uint32_t prev = 0;
    const int K = C.K;
    for (int base = 0; base < n; base += kTdUnroll) {
      uint32_t ra[kTdUnroll], tk[kTdUnroll];
      ah.block(C, base, n, ra, tk);
#pragma unroll
      for (int u = 0; u < kTdUnroll; ++u) {
        if (base + u >= n) break;
        const uint32_t cc = tk[u];
        auto close_route = [&]() {
          if (prev) {
            t += td_rd(C.LEG + (uint32_t)__mul24(96, prev) + 48u + td_hoff(tm));
            const uint32_t rd = (uint32_t)(t - stk);
            dsum += rd;
            dmax = max(dmax, rd);
          }
          ++k;
          if (k < K) {
            load = 0;
            stk = C.start[k];
            t = stk;
            tm = (uint32_t)stk % 1440u;
            prev = 0;
            capk = C.cap[k];
          }
        };
        if (cc == 0) {
          if (k < K) close_route();
          continue;
        }
        const int dc = (int)td_rd32(C.DEM + 4u * cc);
        if (k < K && load + dc > capk) {
          do close_route();
          while (k < K && load + dc > capk);
        }
        if (k < K) {
          const uint32_t row = prev ? ra[u] : C.LEG + (uint32_t)__mul24(96, cc);
          const int e = td_rd(row + td_hoff(tm));
          t += e;
          tm = td_day_add(tm, (uint32_t)e);
          load += dc;
          prev = cc;
        } else {
          ++unv;
        }
      }
    }
    if (k < K && prev) {
      t += td_rd(C.LEG + (uint32_t)__mul24(96, prev) + 48u + td_hoff(tm));
      const uint32_t rd = (uint32_t)(t - stk);
      dsum += rd;
      dmax = max(dmax, rd);
    }
    return {cvrp_key(unv, dsum, dmax, C.objective), (int32_t)dsum, (int32_t)dmax, (int32_t)unv};
  }
}

template <bool CVRP, bool FAST>
__global__ __launch_bounds__(256) void sa_td_kernel(TdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StagedInst<uint16_t, 24> I = stage_inst<uint16_t, 24>(a.si, smem);  // dem / cap / start
  const uint32_t N = (uint32_t)a.si.N, Nm1 = N - 1;
  const int K = a.si.K;
  const uint32_t sbase = (uint32_t)(uintptr_t)(td_lds_uc*)smem;
  {  // depot legs: row 2c = edge (0, c) (OUT), row 2c + 1 = edge (c, 0) (RET); then a zero row
    v4u* d = reinterpret_cast<v4u*>(smem + a.legs_off);
    const v4u* g = reinterpret_cast<const v4u*>(a.mh);
    for (uint32_t i = threadIdx.x; i < 6 * N; i += blockDim.x) {
      const uint32_t r = i / 3, part = i - 3 * r, c = r >> 1;
      const size_t e = (r & 1u) ? (size_t)c * N : (size_t)c;
      d[i] = g[e * 3 + part];
    }
    if (threadIdx.x < 6) d[6 * N + threadIdx.x] = v4u{0u, 0u, 0u, 0u};
    // vehicles 0..K-1 {capacity, start minute of the day, its hour offset,
    // LDS address of the next record}, then a sentinel (capacity -1, linked
    // to itself): the fleet is exhausted
    v4u* veh = reinterpret_cast<v4u*>(smem + a.veh_off);
    const uint32_t vbase = sbase + a.veh_off;
    for (int k = threadIdx.x; k <= K; k += blockDim.x) {
      const int st = k < K ? a.si.start[k] : 0;
      const uint32_t tm = (uint32_t)st % 1440u;
      veh[k] = v4u{k < K ? (uint32_t)a.si.cap[k] : 0xffffffffu, tm, td_hoff(tm),
                   vbase + 16u * (uint32_t)min(k + 1, K)};
    }
  }
  __syncthreads();
  const int W = a.W, n = a.n;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int cw = W > 1 ? wave : 0;    // wavefront within the chain
  const int slot = W > 1 ? 0 : wave;  // chain within the workgroup (W = 1)
  const int chain = (int)blockIdx.x * a.CPW + slot;
  if (chain >= a.chains) return;  // W > 1: the whole workgroup is one chain
  const int ct = cw * 64 + lane, CT = 64 * W;  // thread within the chain
  const uint32_t npad = a.npad;
  const bool sym = a.sym != 0;
  unsigned char* cb = smem + a.chains_off + (uint32_t)slot * a.chain_bytes;
  uint16_t* tA = reinterpret_cast<uint16_t*>(cb);
  uint16_t* tB = tA + npad;
  uint16_t* tBest = tB + npad;
  unsigned char* Fp = cb + td_tours_bytes(npad);
  unsigned char* Rp = sym ? Fp + kTdRow : Fp + npad * kTdRow;
  unsigned char* Jp = Fp + td_rows_bytes(npad, sym);
  struct XSlot {
    uint64_t key;
    uint32_t idx, u, typ;
    int i, j, pad;
  };
  XSlot* xs = reinterpret_cast<XSlot*>(Jp + a.jbytes);
  auto lds = [&](const unsigned char* p) { return sbase + (uint32_t)(p - smem); };
  auto csync = [&]() {
    if (W > 1) __syncthreads();
    else wave_sync();
  };
  auto row_copy = [&](unsigned char* dst, const v4u* src) {  // 48 bytes
    const v4u x0 = src[0], x1 = src[1], x2 = src[2];
    v4u* d = reinterpret_cast<v4u*>(dst);
    d[0] = x0;
    d[1] = x1;
    d[2] = x2;
  };
  auto tokA = [&](int p) { return min((uint32_t)tA[p], Nm1); };

  const uint16_t* gcur = a.cur + (int64_t)chain * n;
  for (int q = ct; q < n; q += CT) tA[q] = gcur[q];
  csync();
  // the current tour's rows: F[q] = (tour[q-1], tour[q]), R[q] = (tour[q+1], tour[q])
  for (int q = ct; q < n; q += CT) {
    const uint32_t y = tokA(q);
    row_copy(Fp + (uint32_t)q * kTdRow, td_grow(a.mh, N, q ? tokA(q - 1) : 0u, y));
    if (!sym) row_copy(Rp + (uint32_t)q * kTdRow, td_grow(a.mh, N, q + 1 < n ? tokA(q + 1) : 0u, y));
  }
  csync();
  TdChain C;
  C.A = lds(reinterpret_cast<unsigned char*>(tA));
  C.F = lds(Fp);
  C.R = lds(Rp);
  C.LEG = sbase + a.legs_off;
  C.ZR = C.LEG + 2u * N * kTdRow;
  C.VEH = sbase + a.veh_off;
  C.DEM = lds(reinterpret_cast<const unsigned char*>(I.sp.dem));
  C.cap = I.sp.cap;
  C.start = I.sp.start;
  C.K = K;
  C.objective = a.si.objective;
  C.Nm1 = Nm1;
  C.sym = sym;
  {
    uint32_t nc = 0;
    for (int q = lane; q < n; q += 64) nc += tA[q] != 0 ? 1u : 0u;
    for (int off = 32; off > 0; off >>= 1) nc += (uint32_t)__shfl_xor((int)nc, off, 64);
    C.ncust = nc;
  }
  // the lane's junction rows
  unsigned char* jrow = Jp + ((uint32_t)cw * 64u + (uint32_t)lane) * 4u * kTdRow;
  const uint32_t jb = lds(jrow);
  uint64_t ck = td_walk<CVRP, FAST>(C, identity_map(), n + 2, n + 2, jb, n).key;
  uint64_t bk = a.best_key[chain];
  bool best_in_lds = false;
  if (ck < bk) {
    bk = ck;
    for (int q = ct; q < n; q += CT) tBest[q] = tA[q];
    best_in_lds = true;
  }
  const uint32_t mlane = (uint32_t)ct;
  float invT = a.inv_t0;
  for (int st = 0; st < a.steps && n >= 2; ++st) {
    const uint64_t step = a.step0 + (uint64_t)st;
    const u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)chain, mlane,
                           a.seed_lo, a.seed_hi);
    const Move m = decode_move_window(r.x, r.y, r.z, n, a.window, a.window_types);
    const MoveMap mm = move_map(m);
    const int lo = min(m.i, m.j), hi = max(m.i, m.j);
    {  // junction rows: (moved[c - 1], moved[c]) at c = lo, lo + 1, hi, hi + 1 (12 loads in flight)
      const int cs[4] = {lo, lo + 1, hi, hi + 1};
      v4u g[4][3];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int c = min(cs[s], n - 1);
        const uint32_t x = c >= 1 ? tokA(map_src(mm, c - 1)) : 0u, y = tokA(map_src(mm, c));
        const v4u* src = td_grow(a.mh, N, x, y);
        g[s][0] = src[0];
        g[s][1] = src[1];
        g[s][2] = src[2];
      }
      v4u* d = reinterpret_cast<v4u*>(jrow);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        d[3 * s] = g[s][0];
        d[3 * s + 1] = g[s][1];
        d[3 * s + 2] = g[s][2];
      }
      wave_sync();
    }
    uint64_t k = td_walk<CVRP, FAST>(C, mm, lo, hi, jb, n).key;
    int bl;
    k = wave_argmin_lane(k, bl);  // wave-uniform (key, lane) minimum
    uint32_t uw = (uint32_t)wave_bcast((int)r.w, bl);
    Move mb;
    mb.typ = (uint32_t)wave_bcast((int)m.typ, bl);
    mb.i = wave_bcast(m.i, bl);
    mb.j = wave_bcast(m.j, bl);
    if (W > 1) {
      // the chain's (key, move index) minimum over its wavefronts; two slot
      // buffers by step parity, so a slot is rewritten only after the next
      // step's barrier
      XSlot* xb = xs + (st & 1) * kTdMaxWaves;
      if (lane == 0) xb[cw] = XSlot{k, (uint32_t)(64 * cw + bl), uw, mb.typ, mb.i, mb.j, 0};
      __syncthreads();
      XSlot b = xb[0];
      for (int v = 1; v < W; ++v) {
        const XSlot o = xb[v];
        if (o.key < b.key) b = o;  // equal keys: the lower index (earlier slot) stays
      }
      k = b.key;
      uw = b.u;
      mb.typ = b.typ;
      mb.i = b.i;
      mb.j = b.j;
    }
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      accept = (uw >> 8) < accept_threshold(dp, invT);
    }
    if (accept) {
      // every thread of the chain: the next tour, then the changed rows into
      // the J area (free once every wavefront has priced), then back into F / R
      const MoveMap mmb = move_map(mb);
      const int blo = min(mb.i, mb.j), bhi = max(mb.i, mb.j);
      if (W == 1) wave_sync();  // W > 1: the exchange barrier ordered the walks' reads
      for (int q = ct; q < n; q += CT) tB[q] = tA[map_src(mmb, q)];
      const int f0 = blo, f1 = min(bhi + 1, n - 1);
      for (int q = f0 + ct; q <= f1; q += CT) {
        const int x = map_src(mmb, q), xp = q ? map_src(mmb, q - 1) : -1;
        unsigned char* dst = Jp + (uint32_t)(q - f0) * kTdRow;
        if (x == xp + 1) {
          row_copy(dst, reinterpret_cast<const v4u*>(Fp + (uint32_t)x * kTdRow));
        } else if (x == xp - 1) {
          row_copy(dst, reinterpret_cast<const v4u*>(sym ? Fp + (uint32_t)xp * kTdRow
                                                         : Rp + (uint32_t)x * kTdRow));
        } else {
          row_copy(dst, td_grow(a.mh, N, xp >= 0 ? tokA(xp) : 0u, tokA(x)));
        }
      }
      const int r0 = max(blo - 1, 0), r1 = min(bhi, n - 2);
      unsigned char* J2 = Jp + npad * kTdRow;
      if (!sym) {
        for (int q = r0 + ct; q <= r1; q += CT) {
          const int x = map_src(mmb, q), y = map_src(mmb, q + 1);
          unsigned char* dst = J2 + (uint32_t)(q - r0) * kTdRow;
          if (y == x + 1) row_copy(dst, reinterpret_cast<const v4u*>(Rp + (uint32_t)x * kTdRow));
          else if (y == x - 1) row_copy(dst, reinterpret_cast<const v4u*>(Fp + (uint32_t)x * kTdRow));
          else row_copy(dst, td_grow(a.mh, N, tokA(y), tokA(x)));
        }
      }
      csync();
      for (int q = f0 + ct; q <= f1; q += CT)
        row_copy(Fp + (uint32_t)q * kTdRow, reinterpret_cast<const v4u*>(Jp + (uint32_t)(q - f0) * kTdRow));
      if (!sym)
        for (int q = r0 + ct; q <= r1; q += CT)
          row_copy(Rp + (uint32_t)q * kTdRow, reinterpret_cast<const v4u*>(J2 + (uint32_t)(q - r0) * kTdRow));
      uint16_t* t = tA;
      tA = tB;
      tB = t;
      C.A = lds(reinterpret_cast<unsigned char*>(tA));
      ck = k;
      if (ck < bk) {
        bk = ck;
        for (int q = ct; q < n; q += CT) tBest[q] = tA[q];
        best_in_lds = true;
      }
      csync();
    }
    invT = invT * a.inv_alpha;
  }
  csync();
  uint16_t* gout = a.cur + (int64_t)chain * n;
  for (int q = ct; q < n; q += CT) gout[q] = tA[q];
  if (best_in_lds) {
    uint16_t* gb = a.best + (int64_t)chain * n;
    for (int q = ct; q < n; q += CT) gb[q] = tBest[q];
  }
  if (ct == 0) {
    a.cur_key[chain] = ck;
    a.best_key[chain] = bk;
  }
}

// Launch when the instance is hour-indexed (H = 24) with a u16 matrix and the
// hour-minor copy, and one chain's rows fit the LDS.  Returns 1 when it does
// not apply (the caller falls back), else a VRPMS status.
int launch_sa_td(const vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur,
                 uint64_t* d_cur_key, uint16_t* d_best, uint64_t* d_best_key, int n,
                 uint32_t wtypes, int moves, hipStream_t s) {
  const Instance& in = ctx->inst;
  if (in.H != kTdH || !in.mat16h || n < 1) return 1;
  const int W = moves / 64;
  if (W < 1 || W > kTdMaxWaves) return 1;
  SearchInst si = search_inst(ctx);
  si.mat_lds = 0;
  const bool sym = in.sym_all;
  const uint32_t npad = ((uint32_t)n + 7u) & ~7u;
  const uint32_t legs_off = (uint32_t)inst_lds_bytes_host(si);
  const uint32_t veh_off = legs_off + td_legs_bytes(in.N);
  const uint32_t chains_off = (veh_off + td_veh_bytes(in.K) + 15u) & ~15u;
  const uint32_t rows = td_rows_bytes(npad, sym);
  const uint32_t jbytes = std::max((uint32_t)W * 64u * 4u * kTdRow, rows);  // junction rows / accept temp
  const uint32_t chain_bytes = td_tours_bytes(npad) + rows + jbytes + kTdXBytes;
  if ((size_t)chains_off + chain_bytes > ctx->max_lds) return 1;
  // one chain per workgroup spreads small launches over every CU; four per
  // workgroup (sharing the depot legs) once the chains outnumber what
  // one-chain workgroups keep resident
  int CPW = 1;
  if (W == 1) {
    const size_t per_cu1 = ctx->max_lds / ((size_t)chains_off + chain_bytes);
    if ((size_t)p->chains > per_cu1 * (size_t)ctx->num_cus) {
      for (int c = 4; c > 1; c >>= 1)
        if ((size_t)chains_off + (size_t)c * chain_bytes <= ctx->max_lds) {
          CPW = c;
          break;
        }
    }
  }
  const size_t lds = (size_t)chains_off + (size_t)CPW * chain_bytes;
  TdArgs a{si, in.mat16h, p->chains, n, p->steps, p->window, wtypes, p->inv_t0, p->inv_alpha,
           (uint32_t)p->seed, (uint32_t)(p->seed >> 32), p->step0, d_cur, d_cur_key, d_best,
           d_best_key, W, CPW, sym ? 1 : 0, legs_off, veh_off, chains_off, chain_bytes, npad,
           jbytes};
  // FAST: every demand fits every vehicle (no empty vehicle is ever skipped)
  const bool fast = in.max_dem <= in.min_cap;
  auto kern = in.problem != VRPMS_CVRP ? sa_td_kernel<false, true>
                                       : (fast ? sa_td_kernel<true, true> : sa_td_kernel<true, false>);
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int grid = (p->chains + CPW - 1) / CPW;
  kern<<<grid, 64 * W * CPW, lds, s>>>(a);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

}  // namespace vrpms
