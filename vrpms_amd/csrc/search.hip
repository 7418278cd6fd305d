// The neighbourhood / search half of the vrpms hot path: the algorithms the
// reference exposes as endpoints (api/{tsp,vrp}/{sa,ga,aco,bf}/index.py) but
// never implements (each stops at `# TODO: Run algorithm`).  Every random
// choice comes from Philox4x32-10 keyed by (seed) with counters naming
// (step/generation, chain/island/child, lane, stream), so oracle/spec.py
// replays the exact same trajectory on the CPU; every tour is scored by
// eval_tour (tour.hpp), the same arithmetic vrpms_eval uses.
//
//   sa_kernel           one wavefront per SA chain; each step the 64 lanes
//                       score 64 sampled moves of the chain's tour (LDS),
//                       a wave argmin picks the best, Metropolis accepts.
//   ga_breed_kernel     one wavefront per child: tournament selection,
//                       wave-parallel OX crossover (ballot + popcount
//                       compaction), Philox-gated mutation.
//   ga_select_kernel    one workgroup per island: (mu + lambda) survivors by
//                       a bitonic sort of (key, index) in LDS.
//   aco_construct_kernel  one wavefront per ant: integer roulette over
//                       tau * eta with a wave prefix scan (exact, so the
//                       choice is order-independent and reproducible).
//   aco_update_kernel   integer evaporation + iteration-best deposit.
//   bf_kernel           lexicographic rank ranges of nibble-packed tours.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <vector>

#include "common.hpp"
#include "ctx.hpp"
#include "split.hpp"
#include "staging.hpp"
#include "tour.hpp"
#include "words.hpp"

namespace vrpms {

// ===========================================================================
// Simulated annealing: one wavefront per chain.
// ===========================================================================
struct SaArgs {
  SearchInst si;
  int chains, n, steps, window;
  uint32_t window_types;
  float inv_t0, inv_alpha;
  uint32_t seed_lo, seed_hi;
  uint64_t step0;
  uint16_t* cur;        // [chains][n]
  uint64_t* cur_key;    // [chains]
  uint16_t* best;       // [chains][n]
  uint64_t* best_key;   // [chains]
  int wpc;              // sa_route_kernel: wavefronts per chain (1: 4 chains per workgroup)
};

template <typename MatT, int HM, bool CVRP>
__global__ __launch_bounds__(256) void sa_kernel(SaArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StagedInst<MatT, HM> I = stage_inst<MatT, HM>(a.si, smem);
  const int n = a.n;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int chain = blockIdx.x * 4 + wave;
  const uint32_t npad = ((uint32_t)n + 7u) & ~7u;
  uint16_t* buf = reinterpret_cast<uint16_t*>(smem + inst_lds_bytes(a.si)) + wave * 3 * npad;
  if (chain >= a.chains) return;  // no block-wide barrier after this point
  uint16_t* A = buf;              // current tour
  uint16_t* B = buf + npad;       // scratch for the accepted move
  uint16_t* Best = buf + 2 * npad;
  const uint16_t* gcur = a.cur + (int64_t)chain * n;
  for (int q = lane; q < n; q += 64) A[q] = gcur[q];
  wave_sync();
  // Static TSP prices a move by its exact O(1) integer delta (tsp_move_delta);
  // everything else re-evaluates the moved tour (the split / departure-time
  // dependence makes a CVRP or time-dependent delta non-local).
  constexpr bool kDelta = !CVRP && HM == 1;
  const uint32_t Nm1 = (uint32_t)a.si.N - 1;
  int dur;
  uint64_t ck;
  {
    auto tour = [&](int i) { return (uint32_t)A[i]; };
    const TourCost c0 = eval_tour<CVRP>(I.D, I.sp, tour, n);
    ck = c0.key;
    dur = c0.sum;
  }
  uint64_t bk = a.best_key[chain];
  bool best_in_lds = false;
  if (ck < bk) {
    bk = ck;
    for (int q = lane; q < n; q += 64) Best[q] = A[q];
    best_in_lds = true;
  }
  float invT = a.inv_t0;
  for (int s = 0; s < a.steps && n >= 2; ++s) {
    const uint64_t step = a.step0 + (uint64_t)s;
    const u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)chain,
                           (uint32_t)lane, a.seed_lo, a.seed_hi);
    const Move m = decode_move_window(r.x, r.y, r.z, n, a.window, a.window_types);
    uint64_t k;
    int nd = 0;
    if constexpr (kDelta) {
      auto dist = [&](uint32_t x, uint32_t y) { return I.D(0, x, y); };
      auto tourA = [&](int q) { return min((uint32_t)A[q], Nm1); };
      nd = dur + (a.si.symmetric ? tsp_move_delta_sym(dist, tourA, n, m)
                                 : tsp_move_delta(dist, tourA, n, m, false));
      k = pack_key(0, (uint32_t)nd, 0);
    } else {
      auto moved = [&](int q) { return (uint32_t)A[moved_index(q, m)]; };
      k = eval_tour<CVRP>(I.D, I.sp, moved, n).key;
    }
    int bl;
    k = wave_argmin_lane(k, bl);  // wave-uniform (key, lane) minimum
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      const uint32_t u = (uint32_t)wave_bcast((int)r.w, bl) >> 8;
      accept = u < accept_threshold(dp, invT);
    }
    if (accept) {
      Move mb;
      mb.typ = (uint32_t)wave_bcast((int)m.typ, bl);
      mb.i = wave_bcast(m.i, bl);
      mb.j = wave_bcast(m.j, bl);
      if constexpr (kDelta) dur = wave_bcast(nd, bl);
      for (int q = lane; q < n; q += 64) B[q] = A[moved_index(q, mb)];
      wave_sync();
      uint16_t* t = A;
      A = B;
      B = t;
      ck = k;
      if (ck < bk) {
        bk = ck;
        for (int q = lane; q < n; q += 64) Best[q] = A[q];
        best_in_lds = true;
      }
      wave_sync();
    }
    invT = invT * a.inv_alpha;
  }
  uint16_t* gout = a.cur + (int64_t)chain * n;
  for (int q = lane; q < n; q += 64) gout[q] = A[q];
  if (best_in_lds) {
    uint16_t* gb = a.best + (int64_t)chain * n;
    for (int q = lane; q < n; q += 64) gb[q] = Best[q];
  }
  if (lane == 0) {
    a.cur_key[chain] = ck;
    a.best_key[chain] = bk;
  }
}

// ===========================================================================
// Route-local SA (CVRP tours with A10 separators, exchangeable vehicles: one
// capacity and one start time for the whole fleet, every demand fits an
// empty vehicle).  Same chain, moves and acceptance as sa_kernel; what
// changes is how a move is priced.
//
// Every route of the greedy split starts from the same state (empty
// vehicle at the depot at the common start time), whether a separator or a
// customer that did not fit opened it.  So a move touching positions lo..hi
// leaves the split before the route holding lo untouched; a lane walks the
// moved tour from that route's start, and stops as soon as its walk is back
// in step with the current tour: at a position where the current tour
// starts a route and the walk is also at a route start (fresh, or the
// token there does not fit).  From there on the two splits coincide.  Swap
// and relocate leave the tokens between their two ends in order (a
// relocate shifts them by one), so the walk re-synchronises between the
// ends too and prices the second end as its own zone; a 2-opt reverses the
// span and is walked through it.  The key is composed from the walked
// zones and per-route totals of the current tour kept in LDS (prefix sums
// of durations, prefix / suffix maxima, a sparse table for the maximum
// between the zones, the last route holding a customer).
//
// Exact: a composed tour that serves every customer (fewer closures before
// its last customer than vehicles) gets its exact key; one that cannot is
// re-evaluated in full, or -- when the current tour serves everyone and
// 2^28 * invT makes accepting an unserved customer impossible -- given the
// largest key, so the trajectory equals full re-evaluation.  An accepted
// move re-walks its zones once, recording their routes, and the per-route
// tables are rebuilt around them.
// ===========================================================================
#ifndef VRPMS_KBLK
#define VRPMS_KBLK 8
#endif
constexpr int kBlk = VRPMS_KBLK;  // tokens a pricing walk reads (and gathers edges for) at once
constexpr int kTourRegs = 18;   // tour positions per lane held in registers on an accept

__host__ __device__ inline int route_max(int K) { return 2 * K + 2; }  // routes stored
__host__ __device__ inline int route_rm(int K) { return (route_max(K) + 1 + 7) & ~7; }
__host__ __device__ inline int route_levels(int rm) {
  int lv = 1;
  while ((2 << (lv - 1)) <= rm) ++lv;
  return lv;
}
__host__ __device__ inline int route_segs(int K) { return (K + 2 + 7) & ~7; }
// per-chain LDS: u32 [tour | demand], u32 tables, u32 route-start bits,
// then u16 route starts / separator positions, then u8 route ids / flags,
// then (16-byte aligned) the cross-wavefront exchange of a multi-wave chain
constexpr int kRouteMaxWaves = 8;
constexpr uint32_t kRouteXBytes = 2 * kRouteMaxWaves * 16 + 16;
__host__ __device__ inline uint32_t route_wave_bytes(int npad, int K) {
  const uint32_t rm = (uint32_t)route_rm(K), lv = (uint32_t)route_levels(route_rm(K));
  const uint32_t words = (uint32_t)npad / 32u + 4u;
  const uint32_t u32s = (uint32_t)npad + (6u + (lv - 1u)) * rm + words;
  const uint32_t u16s = rm + (uint32_t)route_segs(K);
  const uint32_t u8s = (uint32_t)npad + rm;
  return ((4u * u32s + 2u * u16s + u8s + 15u) & ~15u) + kRouteXBytes;
}

// LDS after the per-chain tables: the depot legs (static matrix), then per
// chain the edge cache ein (+ erev on an asymmetric matrix)
__host__ __device__ inline uint32_t route_legs_bytes(int hm, int N, int elem) {
  return hm == 1 ? ((uint32_t)(2 * N * elem) + 15u) & ~15u : 0u;
}
__host__ __device__ inline uint32_t route_edge_bytes(int hm, int npad, int elem, bool sym) {
  return hm == 1 ? ((uint32_t)(npad * elem * (sym ? 1 : 2)) + 15u) & ~15u : 0u;
}

struct RouteTabs {
  uint32_t* at;      // [npad] token | demand << 16 of each position (the current tour)
  uint32_t *dur, *dsp, *pmx, *smx, *lnea;  // per route; prefix sum / max, suffix max, customers >= r
  int32_t* lnb;      // last route < r holding a customer (-1: none)
  uint32_t* sp;      // sparse table of dur, level l >= 1 at sp + (l - 1) * rm
  uint32_t* bits;    // bit q: a route starts at position q
  uint16_t* rs;      // first position of route r (rs[R] = n)
  uint16_t* send;    // separator positions (full builds only)
  uint8_t* rid;      // route of each position
  uint8_t* cus;      // route holds a customer
};

// Wave-wide inclusive scan (add or max) of v over lanes (shuffle steps).
template <bool MAX>
VRPMS_DEV uint32_t wave_scan_incl(uint32_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, off, 64);
    if (lane >= off) v = MAX ? (o > v ? o : v) : v + o;
  }
  return v;
}

#ifdef VRPMS_ROUTE_DUMP
// (debug builds only: tools/route_dump.py) each chain's route tables at the
// end of a call: R, route_ok, then dur / rs / dsp [RM] and rid [n]
constexpr int kRouteDumpInts = 4096;
__device__ int g_route_dump[kRouteDumpInts * 64];
#endif

#ifdef VRPMS_ROUTE_PROF
// per-chain counters (A/B builds only: tools/route_prof.py): pricing and
// accept ticks (wall_clock64, 100 MHz), steps, accepts, walked tokens (wave
// max, lane sum), lanes re-evaluated in full, walk ticks (wave max), walk
// blocks (wave max)
__device__ unsigned long long g_route_prof[12 * 8192];
#endif

// HV: a fleet of different vehicles (per-vehicle capacities or start
// times, api/parameters.py:11-12).  Route r of the split runs on vehicle
// min(r, K - 1) (past the fleet the routes serve no one and the fleet count
// rejects the tour), so a walk is back in step only at a route start of the
// current tour that it reaches on the same vehicle: from there both run on
// the same vehicles from the same state.  A zone that re-synchronises then
// keeps its route count (d = 0); one that does not is walked to the end of
// the tour.  The tables of a full build come from one lane's walk (a
// segment's routes depend on the vehicles before it).
template <typename MatT, int HM, bool HV = false>
__global__ __launch_bounds__(512) void sa_route_kernel(SaArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#ifdef VRPMS_ROUTE_PROF
  const unsigned long long pk0 = wall_clock64();
#endif
  const StagedInst<MatT, HM> I = stage_inst<MatT, HM>(a.si, smem);
  const int n = a.n;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  // W = 1: four chains per workgroup, one wavefront each.  W > 1: one chain
  // per workgroup, its W wavefronts price 64 W moves per step (move index
  // lane + 64 cw), the (key, index) minimum meets in LDS, and the winning
  // wavefront applies an accepted move to the chain's tables.
  const int W = a.wpc;
  const int cw = W > 1 ? wave : 0;  // wavefront within the chain
  const int slot = W > 1 ? 0 : wave;
  const int CPW = W > 1 ? 1 : 4;    // chains per workgroup
  const int chain = W > 1 ? (int)blockIdx.x : (int)blockIdx.x * 4 + wave;
  const uint32_t mlane = (uint32_t)(lane + 64 * cw);
  const int K = a.si.K;
  const int RMAX = route_max(K), RM = route_rm(K), LV = route_levels(RM);
  const int SEGS = route_segs(K);
  const uint32_t npad = ((uint32_t)n + 7u) & ~7u;
  const uint32_t wbytes = (route_wave_bytes((int)npad, K) + 15u) & ~15u;
  unsigned char* wb = smem + inst_lds_bytes(a.si) + slot * wbytes;
  // cross-wavefront exchange (W > 1): two buffers of W (key, index, u) slots
  // (by step parity), then R and route_ok after an accept
  struct XSlot {
    uint64_t key;
    uint32_t idx, u;
  };
  XSlot* xs = reinterpret_cast<XSlot*>(wb + wbytes - kRouteXBytes);
  int32_t* xr = reinterpret_cast<int32_t*>(xs + 2 * kRouteMaxWaves);
  const uint32_t N = (uint32_t)a.si.N;
  // static matrix: the depot legs out(c) = D(0, c) and ret(c) = D(c, 0) in
  // LDS (one u32 per node for a u16 matrix), so a pricing walk gathers one
  // matrix entry per token from L2
  MatT* legs = reinterpret_cast<MatT*>(smem + inst_lds_bytes(a.si) + CPW * wbytes);
  const MatT* M0 = static_cast<const MatT*>(a.si.mat);  // hour 0 in global memory (L2)
  if constexpr (HM == 1) {
    const MatT* M = M0;
    for (uint32_t c = threadIdx.x; c < N; c += blockDim.x) {
      legs[2 * c] = M[c];
      legs[2 * c + 1] = M[(size_t)c * N];
    }
    __syncthreads();
  }
  if (chain >= a.chains) return;  // no block-wide barrier after this point
  RouteTabs T;
  {
    uint32_t* u = reinterpret_cast<uint32_t*>(wb);
    T.at = u;
    u += npad;
    T.dur = u;
    T.dsp = u + RM;
    T.pmx = u + 2 * RM;
    T.smx = u + 3 * RM;
    T.lnea = u + 4 * RM;
    T.lnb = reinterpret_cast<int32_t*>(u + 5 * RM);
    T.sp = u + 6 * RM;
    T.bits = u + (6 + LV - 1) * RM;
    uint16_t* h = reinterpret_cast<uint16_t*>(T.bits + npad / 32u + 4u);
    T.rs = h;
    T.send = h + RM;
    uint8_t* b = reinterpret_cast<uint8_t*>(T.send + SEGS);
    T.rid = b;
    T.cus = b + npad;
  }
  const uint32_t Nm1 = N - 1;
  const int cap0 = I.sp.cap[0], st0 = I.sp.start[0];
  const int32_t* dem = I.sp.dem;
  // vehicle v's capacity and start time (HV; past the fleet: the last vehicle's)
  auto capv = [&](int v) -> int { return HV ? I.sp.cap[v < K ? v : K - 1] : cap0; };
  auto stv = [&](int v) -> int { return HV ? I.sp.start[v < K ? v : K - 1] : st0; };
  if (cw == 0) {  // the chain's first wavefront owns every table write outside an accept
    const uint16_t* gcur = a.cur + (int64_t)chain * n;
    for (int q = lane; q < n; q += 64) {
      const uint32_t c = min((uint32_t)gcur[q], Nm1);
      T.at[q] = c | ((uint32_t)dem[c] << 16);
    }
    wave_sync();
  }
  auto tokA = [&](int q) { return T.at[q] & 0xffffu; };
  // static matrix: the edge into each position from the token before it
  // (ein; erev = the reverse edge, its own array on an asymmetric matrix),
  // kept with the tour, so a pricing walk reads the edges of every adjacency
  // the move keeps (forward or reversed) from LDS and gathers only the <= 4
  // junction edges it creates from L2
  const bool sym = a.si.symmetric != 0;
  MatT* ein = reinterpret_cast<MatT*>(smem + inst_lds_bytes(a.si) + CPW * wbytes +
                                      route_legs_bytes(HM, (int)N, (int)sizeof(MatT)) +
                                      slot * route_edge_bytes(HM, (int)npad, (int)sizeof(MatT), sym));
  MatT* erev = sym ? ein : ein + npad;
  auto edge_cache = [&]() {
    if constexpr (HM == 1) {
      for (int q = lane; q < n; q += 64) {
        const uint32_t c = tokA(q), p = q ? tokA(q - 1) : 0u;
        ein[q] = M0[(size_t)p * N + c];
        if (!sym) erev[q] = M0[(size_t)c * N + p];
      }
      wave_sync();
    }
  };
  if (cw == 0) edge_cache();
  if (W > 1) __syncthreads();
  auto SP = [&](int l) { return l ? T.sp + (l - 1) * RM : T.dur; };

  // greedy split state of one walk and what it has closed so far
  struct Walk {
    int load, t;
    uint32_t prev, cnt, ds, dm;
    int xs;    // closures before the last customer (-1: none yet)
    int pret;  // return leg of prev (static matrix)
    int v, cap, st;  // (HV) the open route's vehicle, its capacity and start time
  };
  auto fresh = [&](Walk& w, int v) {  // a route start on vehicle v (HV)
    w.load = 0;
    w.v = v;
    w.cap = capv(v);
    w.st = stv(v);
    w.t = HV ? w.st : st0;
    w.prev = 0;
    w.cnt = w.ds = w.dm = 0;
    w.xs = -1;
    w.pret = 0;
  };
  auto leg_out = [&](uint32_t c) -> int {
    if constexpr (HM == 1) return (int)legs[2 * c];
    else return 0;
  };
  auto leg_ret = [&](uint32_t c) -> int {
    if constexpr (HM == 1) return (int)legs[2 * c + 1];
    else return 0;
  };
  auto close = [&](Walk& w) -> uint32_t {  // returns the closed route's duration
    uint32_t rd = 0;
    const int s0 = HV ? w.st : st0;
    if constexpr (HM == 1) {  // branch-free: the return leg rides in pret
      rd = w.prev ? (uint32_t)(w.t + w.pret - s0) : 0u;
      w.ds += rd;
      w.dm = max(w.dm, rd);
    } else if (w.prev) {
      w.t += I.D(w.t, w.prev, 0);
      rd = (uint32_t)(w.t - s0);
      w.ds += rd;
      w.dm = max(w.dm, rd);
    }
    ++w.cnt;
    w.load = 0;
    if (HV) {
      ++w.v;
      w.cap = capv(w.v);
      w.st = stv(w.v);
    }
    w.t = HV ? w.st : st0;
    w.prev = 0;
    return rd;
  };
  // customer c with demand d, entered from prev (edge e_in when prev is the
  // token before it on a static matrix, else the depot leg)
  auto add = [&](Walk& w, uint32_t c, int d, int e_in) {
    if constexpr (HM == 1) {
      w.t += w.prev ? e_in : leg_out(c);
      w.pret = leg_ret(c);
    } else {
      w.t += I.D(w.t, w.prev, c);
    }
    w.load += d;
    w.prev = c;
    w.xs = (int)w.cnt;
  };
  auto edge = [&](uint32_t x, uint32_t y) -> int {  // static matrix entry (L2)
    if constexpr (HM == 1) return I.D(0, x, y);
    else return 0;
  };
  // the current tour's edge into position q (static matrix, LDS)
  auto ein_q = [&](int q) -> int {
    if constexpr (HM == 1) return (int)ein[q];
    else return 0;
  };

  // per-route prefix tables over routes 0..R-1 (entries 0..R)
  auto derive = [&](int R) {
    uint32_t cds = 0, cmx = 0;
    int clnb = -1;
    for (int base = 0; base <= R; base += 64) {
      const int r = base + lane;
      const bool in = r < R;
      const uint32_t d = in ? T.dur[r] : 0u;
      const int nb = in && T.cus[r] ? r : -1;
      const uint32_t ids = wave_scan_incl<false>(d), imx = wave_scan_incl<true>(d);
      const int ilnb = (int)wave_scan_incl<true>((uint32_t)(nb + 1)) - 1;
      const uint32_t ex_mx = (uint32_t)__shfl_up((int)imx, 1, 64);
      const int ex_lnb = __shfl_up(ilnb, 1, 64);
      if (r <= R) {
        T.dsp[r] = cds + ids - d;
        T.pmx[r] = max(cmx, lane ? ex_mx : 0u);
        T.lnb[r] = max(clnb, lane ? ex_lnb : -1);
      }
      cds += (uint32_t)__shfl((int)ids, 63, 64);
      cmx = max(cmx, (uint32_t)__shfl((int)imx, 63, 64));
      clnb = max(clnb, __shfl(ilnb, 63, 64));
    }
    uint32_t smx = 0, sne = 0;
    for (int top = R; top >= 0; top -= 64) {
      const int r = top - lane;
      const bool in = r >= 0 && r < R;
      const uint32_t d = in ? T.dur[r] : 0u, ne = in ? (uint32_t)T.cus[r] : 0u;
      const uint32_t imx = wave_scan_incl<true>(d), ine = wave_scan_incl<true>(ne);
      if (r >= 0) {
        T.smx[r] = max(smx, imx);
        T.lnea[r] = max(sne, ine);
      }
      smx = max(smx, (uint32_t)__shfl((int)imx, 63, 64));
      sne = max(sne, (uint32_t)__shfl((int)ine, 63, 64));
    }
    wave_sync();
    for (int l = 1; l < LV; ++l) {
      const int w = 1 << (l - 1);
      const uint32_t* src = SP(l - 1);
      uint32_t* dst = SP(l);
      for (int r = lane; r + 2 * w <= R; r += 64) dst[r] = max(src[r], src[r + w]);
      wave_sync();
    }
  };
  auto range_max = [&](int r0, int r1) -> uint32_t {  // max dur over routes r0..r1
    if (r0 > r1) return 0u;
    const int l = 31 - __builtin_clz((uint32_t)(r1 - r0 + 1));
    const uint32_t* t = SP(l);
    return max(t[r0], t[r1 - (1 << l) + 1]);
  };
  // route-start bits from the route ids (a route starts where the id changes)
  auto build_bits = [&]() {
    for (int base = 0; base < (int)npad + 64; base += 64) {
      const int q = base + lane;
      const bool s = q < n && (q == 0 || T.rid[q] != T.rid[q - 1]);
      const uint64_t ball = __ballot(s);
      if (lane < 2 && (base >> 5) + lane < (int)(npad / 32u + 4u))
        T.bits[(base >> 5) + lane] = (uint32_t)(lane ? ball >> 32 : ball);
    }
    wave_sync();
  };

  // Full route tables of the current tour: separators cut it into segments
  // the lanes split in parallel (two passes: route counts, then routes at
  // their global index).  Returns R, or -1 when the tables cannot hold it.
  auto full_build = [&]() -> int {
    if constexpr (HV) {
      // the vehicles of a segment's routes depend on every route before it:
      // one lane walks the tour (full builds are rare: the start of a call
      // and accepts whose routes no longer fit the incremental update)
      int r = 0;
      if (lane == 0) {
        Walk w;
        fresh(w, 0);
        int start = 0;
        for (int q = 0; q < n && r <= RMAX; ++q) {
          const uint32_t at = T.at[q], c = at & 0xffffu;
          const int d = (int)(at >> 16);
          if (c == 0 || w.load + d > w.cap) {
            const bool cu = w.prev != 0;
            if (c == 0) T.rid[q] = (uint8_t)r;  // a separator belongs to the route it ends
            T.dur[r] = close(w);
            T.cus[r] = cu ? 1 : 0;
            T.rs[r] = (uint16_t)start;
            ++r;
            start = c == 0 ? q + 1 : q;
            if (c == 0 || r > RMAX) continue;
          }
          add(w, c, d, w.prev ? ein_q(q) : 0);
          T.rid[q] = (uint8_t)r;
        }
        if (r <= RMAX) {
          const bool cu = w.prev != 0;
          T.dur[r] = close(w);
          T.cus[r] = cu ? 1 : 0;
          T.rs[r] = (uint16_t)start;
          ++r;
          if (r <= RMAX) T.rs[r] = (uint16_t)n;
        }
      }
      const int R = __builtin_amdgcn_readfirstlane(r);
      wave_sync();
      if (R > RMAX) return -1;
      // route starts past the last route read a fixed value (the tour's end),
      // never what the LDS held before (a stale start was a bug)
      for (int x = R + 1 + lane; x < RM; x += 64) T.rs[x] = (uint16_t)n;
      derive(R);
      build_bits();
      return R;
    }
    int S = 0;
    for (int base = 0; base < n; base += 64) {
      const int q = base + lane;
      const bool z = q < n && tokA(q) == 0;
      const uint64_t ball = __ballot(z);
      const int pre = S + __popcll(ball & ((1ull << lane) - 1ull));
      if (z && pre < SEGS - 1) T.send[pre] = (uint16_t)q;
      S += __popcll(ball);
    }
    if (S > SEGS - 2) return -1;
    if (lane == 0) T.send[S] = (uint16_t)n;
    wave_sync();
    // pass 1: routes per segment (T.smx as scratch), exclusive prefix (T.pmx)
    for (int s = lane; s <= S; s += 64) {
      const int from = s ? T.send[s - 1] + 1 : 0, to = T.send[s];
      Walk w;
      fresh(w, 0);
      for (int q = from; q < to; ++q) {
        const uint32_t at = T.at[q], c = at & 0xffffu;
        const int d = (int)(at >> 16);
        if (w.load + d > cap0) close(w);
        add(w, c, d, w.prev ? ein_q(q) : 0);
      }
      close(w);
      T.smx[s] = w.cnt;
    }
    wave_sync();
    uint32_t carry = 0;
    for (int base = 0; base <= S; base += 64) {
      const int s = base + lane;
      const uint32_t v = s <= S ? T.smx[s] : 0u;
      const uint32_t inc = wave_scan_incl<false>(v);
      if (s <= S) T.pmx[s] = carry + inc - v;
      carry += (uint32_t)__shfl((int)inc, 63, 64);
    }
    const int R = (int)carry;
    if (R > RMAX) return -1;
    wave_sync();
    // pass 2: each segment's routes at their global index, the route of each position
    for (int s = lane; s <= S; s += 64) {
      const int from = s ? T.send[s - 1] + 1 : 0, to = T.send[s];
      int r = (int)T.pmx[s], start = from;
      Walk w;
      fresh(w, 0);
      for (int q = from; q < to; ++q) {
        const uint32_t at = T.at[q], c = at & 0xffffu;
        const int d = (int)(at >> 16);
        if (w.load + d > cap0) {
          const bool cu = w.prev != 0;
          T.dur[r] = close(w);
          T.cus[r] = cu ? 1 : 0;
          T.rs[r] = (uint16_t)start;
          ++r;
          start = q;
        }
        add(w, c, d, w.prev ? ein_q(q) : 0);
        T.rid[q] = (uint8_t)r;
      }
      const bool cu = w.prev != 0;
      T.dur[r] = close(w);
      T.cus[r] = cu ? 1 : 0;
      T.rs[r] = (uint16_t)start;
      if (to < n) T.rid[to] = (uint8_t)r;
    }
    if (lane == 0) T.rs[R] = (uint16_t)n;
    for (int x = R + 1 + lane; x < RM; x += 64) T.rs[x] = (uint16_t)n;
    wave_sync();
    derive(R);
    build_bits();
    return R;
  };

  // the current tour
  uint64_t ck;
  {
    auto tour = [&](int i) { return tokA(i); };
    ck = eval_tour<true>(I.D, I.sp, tour, n).key;
  }
  int R = 0;
  if (cw == 0) {
    R = full_build();
    if (lane == 0) xr[0] = R;
  }
  if (W > 1) {
    __syncthreads();
    R = xr[0];
  }
  bool route_ok = R >= 0;
  uint16_t* gbest = a.best + (int64_t)chain * n;
  uint64_t bk = a.best_key[chain];
  if (ck < bk) {
    bk = ck;
    if (cw == 0)
      for (int q = lane; q < n; q += 64) gbest[q] = (uint16_t)tokA(q);
  }
  float invT = a.inv_t0;
#ifdef VRPMS_ROUTE_PROF
  unsigned long long pf[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  pf[10] = wall_clock64() - pk0;
#endif
  for (int st = 0; st < a.steps && n >= 2; ++st) {
#ifdef VRPMS_ROUTE_PROF
    const unsigned long long pt0 = wall_clock64();
    int wtok = 0, wblk = 0;
    unsigned long long pwalk = 0;
#endif
    const uint64_t step = a.step0 + (uint64_t)st;
    const u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)chain, mlane,
                           a.seed_lo, a.seed_hi);
    const Move m = decode_move_window(r.x, r.y, r.z, n, a.window, a.window_types);
    const MoveMap mm = move_map(m);
    auto moved = [&](int q) { return tokA(map_src(mm, q)); };
    uint64_t k = 0;
    // an unserved customer cannot be accepted from a tour serving everyone
    // when 2^28 * invT puts the acceptance threshold at 0 (tour.hpp)
    const bool shortcut = (ck >> 56) == 0 && invT >= 0x1p-20f;
    bool full = !route_ok;
    // zone bookkeeping and the routes each zone closes (for an accept)
    int r1s = 0, r1e = 0, r2s = 0, r2e = 0, P1 = 0, Z2 = 0, q1 = 0, q2 = 0, dl = 0;
    // junction edges: every adjacency of the moved tour except at positions
    // lo, lo + 1, hi, hi + 1 is one of the current tour's (forward or
    // reversed), read from the edge cache; these four are gathered here
    int jx0 = 0, jx1 = 0, jx2 = 0, jx3 = 0;
    uint32_t c1 = 0, c2 = 0;
    // route starts of each zone as bits over its positions (zone start = bit
    // 0; bits at or past the zone's end are ignored); zones of more than 128
    // positions are re-walked on an accept
    uint64_t zm[4] = {1ull, 0ull, 1ull, 0ull};
    bool zovf = false;
    if (route_ok) {
      const int lo = min(m.i, m.j), hi = max(m.i, m.j);
      if constexpr (HM == 1) {
        auto jedge = [&](int p) { return p >= 1 && p < n ? edge(moved(p - 1), moved(p)) : 0; };
        jx0 = jedge(lo);
        jx1 = jedge(lo + 1);
        jx2 = jedge(hi);
        jx3 = jedge(hi + 1);
      }
      int bq0 = lo + 1;  // first moved position of the shifted middle
      if (m.typ == kMoveRelocate && m.i < m.j) {
        dl = -1;
        bq0 = lo;
      } else if (m.typ == kMoveRelocate) {
        dl = 1;
      }
      // a changed token also decides whether the route before it closes
      // there, so each zone starts at the route holding the position before
      // its first change (a relocate to j > i inserts after A[hi], which stays)
      r1s = lo > 0 ? T.rid[lo - 1] : 0;
      P1 = T.rs[r1s];
      r2s = (m.typ == kMoveRelocate && m.i < m.j) || m.typ == kMove2Opt ? T.rid[hi] : T.rid[hi - 1];
      Z2 = (int)T.rs[r2s] + dl;
      const bool two = m.typ != kMove2Opt && Z2 > bq0;
      int phase = two ? 1 : 3;  // 1: first zone, 2: second zone, 3: one merged zone
      Walk w, w1;
      fresh(w, r1s);
      fresh(w1, r1s);
      r2e = R;
      int q = P1;
      int zbase = P1;  // first position of the zone being walked
      bool z2 = false;
      // close the walk's route; the next route starts at `next`
      auto close_rec = [&](Walk& ww, int next) {
        close(ww);
        const uint32_t off = (uint32_t)(next - zbase);
        zovf = zovf || off >= 128u;
        const uint64_t b = off < 128u ? 1ull << (off & 63u) : 0ull;
        const uint64_t bl0 = off < 64u ? b : 0ull, bh0 = off < 64u ? 0ull : b;
        zm[0] |= z2 ? 0ull : bl0;
        zm[1] |= z2 ? 0ull : bh0;
        zm[2] |= z2 ? bl0 : 0ull;
        zm[3] |= z2 ? bh0 : 0ull;
      };
      // The walk goes in blocks of kBlk tokens: their tokens and demands,
      // depot legs and route-start bits are read from LDS, and on a static
      // matrix their edges from the token before (which depend only on the
      // tokens) are gathered from L2 together, so a block costs one round
      // trip instead of one per token.  A time-dependent matrix reads each
      // edge at the clock.
      bool fin = false;
#ifdef VRPMS_ROUTE_PROF
      const unsigned long long pw0 = wall_clock64();
#endif
      while (!fin) {
#ifdef VRPMS_ROUTE_PROF
        ++wblk;
#endif
        uint32_t cb[kBlk];
        int db[kBlk], eb[kBlk], ob[kBlk], rb[kBlk];
#pragma unroll
        for (int i = 0; i < kBlk; ++i) {
          const int qq = q + i;
          const int sq = map_src(mm, qq), sp = map_src(mm, qq - 1);
          const uint32_t at = qq < n ? T.at[sq] : 0u;
          cb[i] = at & 0xffffu;
          db[i] = (int)(at >> 16);
          if constexpr (HM == 1) {
            // forward adjacency: the current edge into sq; reversed (sp ==
            // sq + 1): the reverse of the current edge into sp
            int e = qq < n ? (sp + 1 == sq ? (int)ein[sq] : (int)erev[max(sp, 0)]) : 0;
            e = qq == lo ? jx0 : e;
            e = qq == lo + 1 ? jx1 : e;
            e = qq == hi ? jx2 : e;
            e = qq == hi + 1 ? jx3 : e;
            eb[i] = e;
            ob[i] = leg_out(cb[i]);
            rb[i] = leg_ret(cb[i]);
          } else {
            eb[i] = ob[i] = rb[i] = 0;
          }
        }
        // route-start bits at the current tour's positions of the middle
        // (q + i - dl) and of the rest (q + i), as 8-bit windows
        const int bm = q - dl;
        const uint64_t wm = bm >= 0 ? (((uint64_t)T.bits[(bm >> 5) + 1] << 32) | T.bits[bm >> 5]) >> (bm & 31)
                                    : 0ull;
        const uint64_t wa = (((uint64_t)T.bits[(q >> 5) + 1] << 32) | T.bits[q >> 5]) >> (q & 31);
        // (HV) the current tour's routes at the window bases: the route
        // starting at base + i is that plus the starts in (base, base + i];
        // and the capacities / start times of the next two vehicles (a block
        // closing a third route stops before it and resumes in the next)
        int ridm = 0, rida = 0, cap1 = 0, st1 = 0, cap2 = 0, st2 = 0, ncl = 0;
        if constexpr (HV) {
          ridm = bm >= 0 && bm < n ? (int)T.rid[bm] : 0;
          rida = (int)T.rid[q < n ? q : n - 1];
          if (HM == 1) {
            cap1 = capv(w.v + 1);
            st1 = stv(w.v + 1);
            cap2 = capv(w.v + 2);
            st2 = stv(w.v + 2);
          }
        }
        int adv = kBlk;
        // Each token is straight-line predicated code: a lane that leaves the
        // block early sets `stop`, and the rare events that end a zone (back
        // in step in the middle: the second zone starts; back in step after
        // both ends: the walk is done) are applied after the block, so the
        // unrolled tokens carry no loop exits and no copies of the walk state.
        bool stop = false;
        int ev = 0, evq = 0;  // event (1: zone switch, 2: done) and its position
        uint32_t blk = 0;     // route starts closed in this block, bit i = offset q - zbase + i
#pragma unroll
        for (int i = 0; i < kBlk; ++i) {
          const int qq = q + i;
          const uint32_t c = cb[i];
          if (!stop && qq >= n) {  // blocks start at or before n: qq == n here
            fin = true;
            adv = i;
            stop = true;
          }
          // back in step at a route start of the current tour: the walk's
          // route is fresh there, or the customer there does not fit (a
          // separator would close the walk's route, not the tour's empty one)
          // -- and (HV) the walk's next route there is that route
          const bool nofit = c != 0 && w.load + db[i] > (HV ? w.cap : cap0);
          bool insm = w.prev == 0 || nofit, insa = insm;
          if constexpr (HV) {
            const int vw = w.prev == 0 ? w.v : w.v + 1;
            const uint32_t below = (1u << i) - 1u;
            insm = insm && vw == ridm + __popc((uint32_t)(wm >> 1) & below);
            insa = insa && vw == rida + __popc((uint32_t)(wa >> 1) & below);
          }
          const bool mid = !stop && phase == 1 && qq >= bq0;  // moved(qq) = A[qq - dl]
          const bool sw = mid && ((wm >> i) & 1u) && insm;
          phase = mid && !sw && qq == Z2 ? 3 : phase;  // never back in step before the second end
          const bool done = !stop && !sw && phase >= 2 && qq > hi && ((wa >> i) & 1u) && insa;
          ev = sw ? 1 : done ? 2 : ev;
          evq = sw || done ? qq : evq;
          // (HV, static matrix) a third closure in the block: resume there
          const bool over = HV && HM == 1 && !stop && !sw && !done && (c == 0 || nofit) && ncl >= 2;
          adv = over ? i : adv;
          const bool act = !stop && !sw && !done && !over;
          stop = stop || sw || done || over;
          // a separator ends the walk's route (the next one starts after it);
          // a customer that does not fit closes it and opens the next
          if constexpr (HM == 1) {
            const bool closing = act && (c == 0 || nofit);
            const uint32_t rd =
                closing && w.prev ? (uint32_t)(w.t + w.pret - (HV ? w.st : st0)) : 0u;
            w.ds += rd;
            w.dm = max(w.dm, rd);
            w.cnt += closing ? 1u : 0u;
            if constexpr (HV) {  // the next vehicle opens
              w.v += closing ? 1 : 0;
              w.cap = closing ? cap1 : w.cap;
              w.st = closing ? st1 : w.st;
              cap1 = closing ? cap2 : cap1;
              st1 = closing ? st2 : st1;
              ncl += closing ? 1 : 0;
            }
            // the next route starts at block offset i (i + 1 after a
            // separator); zbase and z2 are fixed inside a block, so the bits
            // go to the zone's mask once, after the block
            blk |= closing ? (c == 0 ? 2u << i : 1u << i) : 0u;
            const int t0 = closing ? (HV ? w.st : st0) : w.t, l0 = closing ? 0 : w.load;
            const uint32_t p0 = closing ? 0u : w.prev;
            const bool addf = act && c != 0;
            w.t = addf ? t0 + (p0 ? eb[i] : ob[i]) : t0;
            w.load = addf ? l0 + db[i] : l0;
            w.prev = addf ? c : p0;
            w.pret = addf ? rb[i] : w.pret;
            w.xs = addf ? (int)w.cnt : w.xs;
          } else if (act) {
            if (c == 0 || nofit) close_rec(w, c == 0 ? qq + 1 : qq);
            if (c != 0) add(w, c, db[i], eb[i]);
          }
#ifdef VRPMS_ROUTE_PROF
          if (act) ++wtok;
#endif
        }
        if (blk) {  // as close_rec per bit: offsets >= 128 overflow the zone's mask
          const uint32_t base = (uint32_t)(q - zbase);
          zovf = zovf || base + 31u - (uint32_t)__builtin_clz(blk) >= 128u;
          const uint64_t b = blk;
          const uint64_t lo = base < 64u ? b << base : 0ull;
          const uint64_t hi = base == 0u ? 0ull
                              : base < 64u ? b >> (64u - base)
                              : base < 128u ? b << (base - 64u) : 0ull;
          zm[0] |= z2 ? 0ull : lo;
          zm[1] |= z2 ? 0ull : hi;
          zm[2] |= z2 ? lo : 0ull;
          zm[3] |= z2 ? hi : 0ull;
        }
        if (ev == 1) {  // back in step in the middle: the second zone starts fresh at Z2
          if (w.prev != 0) close_rec(w, evq);  // the token opens a route in both tours
          w1 = w;
          r1e = T.rid[evq - dl];
          q1 = evq;
          fresh(w, r2s + (int)w1.cnt - (r1e - r1s));  // (HV: back in step on r1e, so r2s)
          phase = 2;
          z2 = true;
          zbase = Z2;
          adv = Z2 - q;
        } else if (ev == 2) {  // back in step after both ends
          if (w.prev != 0) close_rec(w, evq);
          r2e = T.rid[evq];
          fin = true;
          adv = evq - q;
        }
        q += adv;
      }
      if (q >= n) close_rec(w, n);  // the tour end closes the last route
#ifdef VRPMS_ROUTE_PROF
      pwalk = wall_clock64() - pw0;
#endif
      q2 = q;
      if (phase != 2) {  // one zone: routes r1s .. r2e - 1
        w1 = w;
        fresh(w, R);
        r1e = r2s = r2e;
        q1 = Z2 = q2;
      }
      c1 = w1.cnt;
      c2 = w.cnt;
      const int d1 = (int)w1.cnt - (r1e - r1s), d2 = (int)w.cnt - (r2e - r2s);
      int X;  // closures before the moved tour's last customer
      if (T.lnea[r2e]) X = T.lnb[R] + d1 + d2;
      else if (w.xs >= 0) X = r2s + d1 + w.xs;
      else if (T.lnb[r2s] >= r1e) X = T.lnb[r2s] + d1;
      else if (w1.xs >= 0) X = r1s + w1.xs;
      else X = T.lnb[r1s];
      if (X < K) {
        const uint32_t dsum = T.dsp[R] - (T.dsp[r1e] - T.dsp[r1s]) - (T.dsp[r2e] - T.dsp[r2s]) +
                              w1.ds + w.ds;
        const uint32_t dmax = max(max(max(T.pmx[r1s], T.smx[r2e]), max(w1.dm, w.dm)),
                                  range_max(r1e, r2s - 1));
        k = cvrp_key(0, dsum, dmax, I.sp.objective);
      } else if (shortcut) {
        k = ~0ull;
      } else {
        full = true;
      }
    }
    if (full) k = eval_tour<true>(I.D, I.sp, moved, n).key;
    int bl;
    k = wave_argmin_lane(k, bl);  // wave-uniform (key, lane) minimum
    uint32_t uw = (uint32_t)wave_bcast((int)r.w, bl);
    int ww = 0;  // winning wavefront of the chain
    if (W > 1) {
      // the chain's (key, move index) minimum over its wavefronts; two slot
      // buffers by step parity, so a slot is rewritten only after the next
      // step's barrier
      XSlot* xb = xs + (st & 1) * kRouteMaxWaves;
      if (lane == 0) xb[cw] = XSlot{k, (uint32_t)(64 * cw + bl), uw};
      __syncthreads();
      XSlot b = xb[0];
      for (int v = 1; v < W; ++v) {
        const XSlot o = xb[v];
        if (o.key < b.key) b = o;  // equal keys: the lower index (earlier slot) stays
      }
      k = b.key;
      uw = b.u;
      ww = (int)(b.idx >> 6);
    }
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      accept = (uw >> 8) < accept_threshold(dp, invT);
    }
#ifdef VRPMS_ROUTE_PROF
    const unsigned long long pt1 = wall_clock64();
    {
      int mx = wtok, sm = wtok, bx = wblk;
      unsigned long long wx = pwalk;
      for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, __shfl_xor(mx, off, 64));
        sm += __shfl_xor(sm, off, 64);
        bx = max(bx, __shfl_xor(bx, off, 64));
        wx = max(wx, (unsigned long long)__shfl_xor((long long)wx, off, 64));
      }
      pf[0] += pt1 - pt0;
      pf[2] += 1;
      pf[3] += accept ? 1 : 0;
      pf[4] += (unsigned long long)mx;
      pf[5] += (unsigned long long)sm;
      pf[6] += (unsigned long long)__popcll(__ballot(full));
      pf[8] += wx;
      pf[9] += (unsigned long long)bx;
    }
#endif
    if (accept && cw != ww) {  // another wavefront applies it: wait for its tables
      __syncthreads();
      R = xr[0];
      route_ok = xr[1] != 0;
      ck = k;
      bk = ck < bk ? ck : bk;
    } else if (accept) {
      Move mb;
      mb.typ = (uint32_t)wave_bcast((int)m.typ, bl);
      mb.i = wave_bcast(m.i, bl);
      mb.j = wave_bcast(m.j, bl);
      const MoveMap mmb = move_map(mb);
      const bool regs = n <= 64 * kTourRegs;
      // the accepted lane's zones, in positions of the new tour
      const int br1s = wave_bcast(r1s, bl), br1e = wave_bcast(r1e, bl);
      const int br2s = wave_bcast(r2s, bl), br2e = wave_bcast(r2e, bl);
      const int bP1 = wave_bcast(P1, bl), bZ2 = wave_bcast(Z2, bl);
      const int bq1 = wave_bcast(q1, bl), bq2 = wave_bcast(q2, bl), bdl = wave_bcast(dl, bl);
      const int bc1 = wave_bcast((int)c1, bl), bc2 = wave_bcast((int)c2, bl);
      const bool bovf = wave_bcast(zovf ? 1 : 0, bl) != 0 || bc1 + bc2 > 64;
      uint64_t bm[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t lo = (uint32_t)wave_bcast((int)(uint32_t)zm[i], bl);
        const uint32_t hi = (uint32_t)wave_bcast((int)(uint32_t)(zm[i] >> 32), bl);
        bm[i] = ((uint64_t)hi << 32) | lo;
      }
      const int d1 = bc1 - (br1e - br1s), d2 = bc2 - (br2e - br2s);
      const int R2 = R + d1 + d2;
      const bool incremental = route_ok && regs && R2 <= RMAX;
#ifdef VRPMS_ROUTE_PROF
      pf[7] += incremental ? (bovf ? 1 : 0) : 1000000;
#endif
      // route starts of zone z (bits over its positions) at or before offset off
      auto starts_upto = [&](int z, int off) {
        const uint64_t lo = bm[2 * z], hi = bm[2 * z + 1];
        if (off < 64) return __popcll(lo & (off == 63 ? ~0ull : ((2ull << off) - 1ull)));
        return __popcll(lo) + __popcll(hi & (off >= 127 ? ~0ull : ((2ull << (off - 64)) - 1ull)));
      };
      // apply the move in place: each lane holds its positions' new entries
      // (and, incrementally, their new route ids) in registers over one sync
      if (regs) {
        {
          // the new tour's entries and its edge cache: kept adjacencies come
          // from the current cache, the four junction edges from the winner's
          // gathers (or from L2 when it priced in full)
          const int blo = min(mb.i, mb.j), bhi = max(mb.i, mb.j);
          const int bj0 = wave_bcast(jx0, bl), bj1 = wave_bcast(jx1, bl);
          const int bj2 = wave_bcast(jx2, bl), bj3 = wave_bcast(jx3, bl);
          // one register per position: the entry, and the new cache entries
          // packed (u16 matrix: ein | erev << 16; int32 symmetric: ein; an
          // int32 asymmetric matrix rebuilds its cache from L2 instead)
          constexpr bool kPack = sizeof(MatT) == 2;
          const bool regcache = HM == 1 && (kPack || sym);
          uint32_t v[kTourRegs], fr[kTourRegs];
#pragma unroll
          for (int i = 0; i < kTourRegs; ++i) {
            const int q = lane + 64 * i;
            const int sq = map_src(mmb, q), sp = map_src(mmb, q - 1);
            v[i] = q < n ? T.at[sq] : 0u;
            fr[i] = 0;
            if (regcache && q < n) {
              const bool fwd = sp + 1 == sq;
              const int spc = max(sp, 0);
              uint32_t fe = fwd ? (uint32_t)ein[sq] : (uint32_t)erev[spc];
              uint32_t re = fwd ? (uint32_t)erev[sq] : (uint32_t)ein[spc];
              const uint32_t c = v[i] & 0xffffu;
              if (q == 0) {
                fe = (uint32_t)legs[2 * c];
                re = (uint32_t)legs[2 * c + 1];
              } else if (q == blo || q == blo + 1 || q == bhi || q == bhi + 1) {
                const uint32_t pc = tokA(sp);
                fe = route_ok ? (uint32_t)(q == blo ? bj0 : q == blo + 1 ? bj1 : q == bhi ? bj2 : bj3)
                              : (uint32_t)M0[(size_t)pc * N + c];
                re = sym ? fe : (uint32_t)M0[(size_t)c * N + pc];
              }
              fr[i] = kPack ? (fe | (re << 16)) : fe;
            }
          }
          wave_sync();
#pragma unroll
          for (int i = 0; i < kTourRegs; ++i) {
            const int q = lane + 64 * i;
            if (q < n) {
              T.at[q] = v[i];
              if (regcache) {
                ein[q] = (MatT)(kPack ? (fr[i] & 0xffffu) : fr[i]);
                if (!sym) erev[q] = (MatT)(fr[i] >> 16);
              }
            }
          }
          if (HM == 1 && !regcache) {
            wave_sync();
            edge_cache();
          }
        }
        if (incremental) {
          uint32_t rv[kTourRegs];
#pragma unroll
          for (int i = 0; i < kTourRegs; ++i) {
            const int q = lane + 64 * i;
            rv[i] = 0;
            if (q >= n) continue;
            if (q < bP1) rv[i] = T.rid[q];
            else if (q < bq1) rv[i] = bovf ? 0u : (uint32_t)(br1s + starts_upto(0, q - bP1) - 1);
            else if (q < bZ2) rv[i] = (uint32_t)((int)T.rid[q - bdl] + d1);  // the middle, shifted
            else if (q < bq2) rv[i] = bovf ? 0u : (uint32_t)(br2s + d1 + starts_upto(1, q - bZ2) - 1);
            else rv[i] = (uint32_t)((int)T.rid[q] + d1 + d2);
          }
          wave_sync();
#pragma unroll
          for (int i = 0; i < kTourRegs; ++i) {
            const int q = lane + 64 * i;
            if (q < n) T.rid[q] = (uint8_t)rv[i];
          }
          if (bovf) {
            // one lane re-walks the zones of the new tour, writing their
            // positions' route ids and their routes into scratch (the
            // derived tables smx / lnea / lnb, rebuilt by derive below)
            wave_sync();
            if (lane == 0) {
              int zi = 0;
              auto rec = [&](int from, int to, int r0) {
                Walk w;
                fresh(w, r0);
                int start = from, rr = r0;
                auto put = [&](int next) {
                  const bool cu = w.prev != 0;
                  T.smx[zi] = close(w);
                  T.lnea[zi] = (uint32_t)start;
                  T.lnb[zi] = cu ? 1 : 0;
                  ++zi;
                  ++rr;
                  start = next;
                };
                for (int q = from; q < to; ++q) {
                  const uint32_t at = T.at[q], c = at & 0xffffu;
                  const int d = (int)(at >> 16);
                  if (c == 0) {  // the separator ends this route: it belongs to it
                    T.rid[q] = (uint8_t)rr;
                    put(q + 1);
                    continue;
                  }
                  if (w.load + d > (HV ? w.cap : cap0)) put(q);
                  add(w, c, d, w.prev ? ein_q(q) : 0);
                  T.rid[q] = (uint8_t)rr;
                }
                if (w.prev != 0 || to >= n) put(to);  // back in step right after a closure: none
              };
              rec(bP1, bq1, br1s);
              if (bq1 < bq2) rec(bZ2, bq2, br2s + d1);
            }
          }
        }
        wave_sync();
      } else {  // tours too long for registers: stage the new tour in HBM (the cur row)
        uint16_t* gscr = a.cur + (int64_t)chain * n;
        for (int q = lane; q < n; q += 64) gscr[q] = (uint16_t)tokA(map_src(mmb, q));
        __threadfence_block();
        wave_sync();
        for (int q = lane; q < n; q += 64) {
          const uint32_t c = gscr[q];
          T.at[q] = c | ((uint32_t)dem[c] << 16);
        }
        wave_sync();
        edge_cache();
      }
      ck = k;
      if (ck < bk) {
        bk = ck;
        for (int q = lane; q < n; q += 64) gbest[q] = (uint16_t)tokA(q);
      }
      if (incremental) {
        // the routes: before the first zone, the first zone's, the middle's
        // (shifted by dl positions), the second zone's, the rest
        uint32_t vd[4], vs[4], vc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lane + 64 * i;
          vd[i] = vs[i] = vc[i] = 0;
          if (rr >= R2) continue;
          int src = -1, sh = 0, zr = -1;  // zr: scratch row of a re-walked zone route
          if (rr < br1s) src = rr;
          else if (rr < br1s + bc1) zr = rr - br1s;
          else if (rr < br2s + d1) src = rr - d1, sh = bdl;
          else if (rr < br2s + d1 + bc2) zr = bc1 + (rr - br2s - d1);
          else src = rr - d1 - d2;
          if (src >= 0) {
            vd[i] = T.dur[src];
            vs[i] = (uint32_t)((int)T.rs[src] + sh);
            vc[i] = T.cus[src];
          } else if (bovf) {
            vd[i] = T.smx[zr];
            vs[i] = T.lnea[zr];
            vc[i] = (uint32_t)T.lnb[zr];
          } else {
            vs[i] = 0xffffffffu;  // a zone route: start from the bits, duration walked below
          }
        }
        wave_sync();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = lane + 64 * i;
          if (rr < R2 && vs[i] != 0xffffffffu) {
            T.dur[rr] = vd[i];
            T.rs[rr] = (uint16_t)vs[i];
            T.cus[rr] = (uint8_t)vc[i];
          }
        }
        if (!bovf) {
          // zone route starts: the set bits below each zone's length, in order
#pragma unroll
          for (int z = 0; z < 2; ++z) {
            const int len = z ? bq2 - bZ2 : bq1 - bP1, base = z ? bZ2 : bP1;
            const int r0 = z ? br2s + d1 : br1s;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int off = 64 * h + lane;
              if (off < len && ((bm[2 * z + h] >> lane) & 1ull))
                T.rs[r0 + starts_upto(z, off) - 1] = (uint16_t)(base + off);
            }
            // routes of the zone past its set bits start at its end: the
            // empty route a walk that reaches the tour end closes after a
            // trailing separator (its start bit is the zone's length)
            const int cz = z ? bc2 : bc1, nb = len > 0 ? starts_upto(z, len - 1) : 0;
            if (lane < cz - nb) T.rs[r0 + nb + lane] = (uint16_t)(base + len);
          }
        }
        if (lane == 0) T.rs[R2] = (uint16_t)n;
        wave_sync();
        if (!bovf) {
          // one lane per zone route walks it (a single route: no closure
          // before its end) for its duration and whether it serves anyone
          const int nz = bc1 + bc2;
          if (lane < nz) {
            const int rr = lane < bc1 ? br1s + lane : br2s + d1 + (lane - bc1);
            const int from = T.rs[rr], to = T.rs[rr + 1];
            Walk w;
            fresh(w, rr);
            for (int q = from; q < to; ++q) {
              const uint32_t at = T.at[q], c = at & 0xffffu;
              if (c == 0) break;  // a separator ends the route
              add(w, c, (int)(at >> 16), w.prev ? ein_q(q) : 0);
            }
            const bool cu = w.prev != 0;
            T.dur[rr] = close(w);
            T.cus[rr] = cu ? 1 : 0;
          }
          wave_sync();
        }
        R = R2;
        derive(R);
        build_bits();
      } else {
        R = full_build();
        route_ok = R >= 0;
      }
      if (W > 1) {  // publish the tables' route count to the chain's other wavefronts
        if (lane == 0) {
          xr[0] = R;
          xr[1] = route_ok ? 1 : 0;
        }
        __syncthreads();
      }
    }
#ifdef VRPMS_ROUTE_PROF
    pf[1] += wall_clock64() - pt1;
#endif
    invT = invT * a.inv_alpha;
  }
  if (cw != 0) return;
#ifdef VRPMS_ROUTE_DUMP
  if (chain < 64 && 2 + 3 * RM + n <= kRouteDumpInts) {
    int* d = g_route_dump + chain * kRouteDumpInts;
    if (lane == 0) {
      d[0] = R;
      d[1] = route_ok ? 1 : 0;
    }
    for (int r = lane; r < RM; r += 64) {
      d[2 + r] = (int)T.dur[r];
      d[2 + RM + r] = (int)T.rs[r];
      d[2 + 2 * RM + r] = (int)T.dsp[r];
    }
    for (int q = lane; q < n; q += 64) d[2 + 3 * RM + q] = (int)T.rid[q];
  }
#endif
  uint16_t* gout = a.cur + (int64_t)chain * n;
  for (int q = lane; q < n; q += 64) gout[q] = (uint16_t)tokA(q);
  if (lane == 0) {
    a.cur_key[chain] = ck;
    a.best_key[chain] = bk;
#ifdef VRPMS_ROUTE_PROF
    pf[11] = wall_clock64() - pk0;
    if (chain < 8192)
      for (int i = 0; i < 12; ++i) g_route_prof[12 * chain + i] += pf[i];
#endif
  }
}

// ===========================================================================
// SA fast path (static CVRP, uniform fleet, every demand fits an empty
// vehicle): the same chain, moves and acceptance as sa_kernel, but each
// candidate is priced with the branch-free split of split.hpp over the
// biased prefix-ret matrix (one ds_read_b64 per customer carries the edge,
// the demand and both depot legs).  One 1024-lane workgroup = 16 chains
// share the LDS-resident matrix; tours are u8 in LDS.  Each lane reads its
// moved tour through the select-chain map (move_map), software-pipelined two
// blocks of 4 customers ahead: tour bytes of block b+2 and matrix gathers of
// block b+1 are in flight while block b's split steps run.
// ===========================================================================
constexpr int kSaPackedWaves = 16;

struct SaPackedArgs {
  FastSplit f;
  int chains, n, steps, window;
  uint32_t window_types;
  float inv_t0, inv_alpha;
  uint32_t seed_lo, seed_hi;
  uint64_t step0;
  uint32_t tb;          // bytes per LDS tour buffer (>= n + 12, zero padded)
  uint16_t* cur;
  uint64_t* cur_key;
  uint16_t* best;
  uint64_t* best_key;
};

// Key of tour T (u8, LDS, zero padded to n + 12) read through map mm.
VRPMS_DEV uint64_t eval_mapped(const FastSplit& f, const unsigned char* E, uint32_t N8,
                               const uint8_t* T, int n, const MoveMap& mm) {
  // E[x][y] at x * 8N + 8y: the pair laid out as u16 halves (one v_lshl_or)
  // and v_dot2_u32_u16 against (8N, 8) with the LDS base as accumulator
  typedef unsigned short us2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const uint64_t lds_u64v;
  const uint32_t ebase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const unsigned char*)E;
  const us2v w8 = {(unsigned short)N8, (unsigned short)8};
  auto gat = [&](uint32_t x, uint32_t y) {
    const uint32_t addr =
        __builtin_amdgcn_udot2(__builtin_bit_cast(us2v, x | (y << 16)), w8, ebase, false);
    return *(lds_u64v*)(uintptr_t)addr;
  };
  auto rd = [&](int q) { return (uint32_t)T[map_src(mm, q)]; };
  const uint32_t smask = f.smask, kinc = 1u << f.ks;
  SplitAcc sa;
  sa.init(f);
  const int nfull = n >> 2;
  uint32_t b0 = rd(4), b1 = rd(5), b2 = rd(6), b3 = rd(7);
  uint32_t last;
  uint64_t e0, e1, e2, e3;
  {
    const uint32_t a0 = rd(0), a1 = rd(1), a2 = rd(2), a3 = rd(3);
    e0 = gat(0, a0);
    e1 = gat(a0, a1);
    e2 = gat(a1, a2);
    e3 = gat(a2, a3);
    last = a3;
  }
  for (int b = 0; b < nfull; ++b) {
    const int q = 4 * b + 8;
    const uint32_t c0 = rd(q), c1 = rd(q + 1), c2 = rd(q + 2), c3 = rd(q + 3);
    const uint64_t f0 = gat(last, b0), f1 = gat(b0, b1), f2 = gat(b1, b2), f3 = gat(b2, b3);
    sa.step_fast(e0, smask, kinc);
    sa.step_fast(e1, smask, kinc);
    sa.step_fast(e2, smask, kinc);
    sa.step_fast(e3, smask, kinc);
    last = b3;
    b0 = c0;
    b1 = c1;
    b2 = c2;
    b3 = c3;
    e0 = f0;
    e1 = f1;
    e2 = f2;
    e3 = f3;
  }
  const int rem = n & 3;  // e0..e(rem-1): the ragged last block
  if (rem > 0) sa.step_fast(e0, smask, kinc);
  if (rem > 1) sa.step_fast(e1, smask, kinc);
  if (rem > 2) sa.step_fast(e2, smask, kinc);
  if (sa.hit_fleet_limit())  // rare: exact re-walk (fleet limit, separators)
    return exact_split(f, n, rd, gat).key;
  return sa.finish(f, n).key;
}

__global__ __launch_bounds__(1024) void sa_packed_kernel(SaPackedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.f.N;
  const uint32_t ebytes = (uint32_t)N * N * 8;
  {
    const v4u* src = reinterpret_cast<const v4u*>(a.f.pack);
    v4u* dst = reinterpret_cast<v4u*>(smem);
    for (uint32_t i = threadIdx.x; i < ebytes / 16; i += blockDim.x) dst[i] = src[i];
    if ((ebytes & 8u) && threadIdx.x == 0)
      reinterpret_cast<uint64_t*>(smem)[ebytes / 8 - 1] = a.f.pack[ebytes / 8 - 1];
  }
  __syncthreads();
  const int n = a.n;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int chain = blockIdx.x * kSaPackedWaves + wave;
  if (chain >= a.chains) return;  // no block-wide barrier after this point
  const uint32_t N8 = 8u * (uint32_t)N, tb = a.tb;
  uint8_t* A = smem + ((ebytes + 15u) & ~15u) + (uint32_t)wave * 3u * tb;
  uint8_t* B = A + tb;
  uint8_t* Best = B + tb;
  const uint16_t* gcur = a.cur + (int64_t)chain * n;
  for (uint32_t q = lane; q < tb; q += 64) {
    A[q] = q < (uint32_t)n ? (uint8_t)min((uint32_t)gcur[q], (uint32_t)N - 1) : 0;
    B[q] = 0;
  }
  wave_sync();
  uint64_t ck = eval_mapped(a.f, smem, N8, A, n, identity_map());
  uint64_t bk = a.best_key[chain];
  bool best_in_lds = false;
  if (ck < bk) {
    bk = ck;
    for (int q = lane; q < n; q += 64) Best[q] = A[q];
    best_in_lds = true;
  }
  float invT = a.inv_t0;
  for (int s = 0; s < a.steps && n >= 2; ++s) {
    const uint64_t step = a.step0 + (uint64_t)s;
    const u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)chain,
                           (uint32_t)lane, a.seed_lo, a.seed_hi);
    const Move m = decode_move_window(r.x, r.y, r.z, n, a.window, a.window_types);
    uint64_t k = eval_mapped(a.f, smem, N8, A, n, move_map(m));
    int bl;
    k = wave_argmin_lane(k, bl);  // wave-uniform (key, lane) minimum
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      accept = ((uint32_t)wave_bcast((int)r.w, bl) >> 8) < accept_threshold(dp, invT);
    }
    if (accept) {
      Move mb;
      mb.typ = (uint32_t)wave_bcast((int)m.typ, bl);
      mb.i = wave_bcast(m.i, bl);
      mb.j = wave_bcast(m.j, bl);
      const MoveMap mm = move_map(mb);
      for (int q = lane; q < n; q += 64) B[q] = A[map_src(mm, q)];
      wave_sync();
      uint8_t* t = A;
      A = B;
      B = t;
      ck = k;
      if (ck < bk) {
        bk = ck;
        for (int q = lane; q < n; q += 64) Best[q] = A[q];
        best_in_lds = true;
      }
      wave_sync();
    }
    invT = invT * a.inv_alpha;
  }
  uint16_t* gout = a.cur + (int64_t)chain * n;
  for (int q = lane; q < n; q += 64) gout[q] = A[q];
  if (best_in_lds) {
    uint16_t* gb = a.best + (int64_t)chain * n;
    for (int q = lane; q < n; q += 64) gb[q] = Best[q];
  }
  if (lane == 0) {
    a.cur_key[chain] = ck;
    a.best_key[chain] = bk;
  }
}

// ===========================================================================
// Genetic algorithm: breed (one wavefront per child) + select (one block per island).
// ===========================================================================
struct GaBreedArgs {
  int islands, pop, n, N;
  uint32_t pmut;        // mutation iff philox word < pmut
  uint32_t seed_lo, seed_hi;
  uint64_t gen;
  const uint16_t* pop_tours;  // [islands][pop][n]
  const uint64_t* pop_keys;   // [islands][pop]
  uint16_t* child;            // rows [islands][pop][n]            (WORDS == false)
  uint32_t* child_w;          // words [ceil(n/4)][islands * pop]  (WORDS == true)
};

// Tournament of two: the lower (key, index) wins.
VRPMS_DEV int tourney(const uint64_t* keys, int pop, uint32_t r0, uint32_t r1) {
  const int x = (int)(r0 % (uint32_t)pop), y = (int)(r1 % (uint32_t)pop);
  const uint64_t kx = keys[x], ky = keys[y];
  return (ky < kx || (ky == kx && y < x)) ? y : x;
}

// One child per wavefront.  WORDS (n <= 255): the child is assembled in a
// wave-private LDS byte buffer and leaves as ceil(n/4) words of the
// word-interleaved layout, which eval_cvrp_words2 -- the headline scoring
// kernel -- reads with one coalesced wave load per word.  Otherwise the
// child is written straight into its uint16 row.
template <bool WORDS>
__global__ __launch_bounds__(256) void ga_breed_kernel(GaBreedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int64_t gid = (int64_t)blockIdx.x * 4 + wave;  // child id = island * pop + i
  const int n = a.n;
  const uint32_t words = ((uint32_t)a.N + 31u) / 32u;
  uint32_t* used = reinterpret_cast<uint32_t*>(smem) + wave * words;
  uint8_t* cbuf = smem + ((4u * words * 4u + 15u) & ~15u) + wave * 256;
  const int64_t members = (int64_t)a.islands * a.pop;
  if (gid >= members) return;
  const int island = (int)(gid / a.pop), child = (int)(gid % a.pop);
  const uint16_t* P = a.pop_tours + (int64_t)island * a.pop * n;
  const uint64_t* Kk = a.pop_keys + (int64_t)island * a.pop;
  uint16_t* out = a.child + gid * n;
  auto put = [&](int q, uint32_t g) {
    if constexpr (WORDS) cbuf[q] = (uint8_t)g;
    else out[q] = (uint16_t)g;
  };
  auto get = [&](int q) -> uint32_t {
    if constexpr (WORDS) return cbuf[q];
    else return out[q];
  };
  const uint32_t cid = (uint32_t)(island * a.pop + child);
  const u32x4 r = philox((uint32_t)a.gen, (uint32_t)(a.gen >> 32), cid, 0u, a.seed_lo, a.seed_hi);
  const u32x4 r2 = philox((uint32_t)a.gen, (uint32_t)(a.gen >> 32), cid, 1u, a.seed_lo, a.seed_hi);
  const int pa = tourney(Kk, a.pop, r.x, r.y), pb = tourney(Kk, a.pop, r.z, r.w);
  const uint16_t* A = P + (int64_t)pa * n;
  const uint16_t* B = P + (int64_t)pb * n;
  if constexpr (WORDS) {
    for (int q = n + lane; q < 256; q += 64) cbuf[q] = 0;  // zero pad of the last word
  }
  if (n < 2) {
    for (int q = lane; q < n; q += 64) put(q, A[q]);
  } else {
    // OX1: child[lo..hi] = A[lo..hi]; the rest, in order from position hi+1
    // (wrapping), are B's genes from B[hi+1] onwards (wrapping) not yet used.
    int lo = (int)(r2.x % (uint32_t)n), hi = (int)(r2.y % (uint32_t)n);
    if (lo > hi) {
      const int t = lo;
      lo = hi;
      hi = t;
    }
    for (uint32_t w = lane; w < words; w += 64) used[w] = 0u;
    wave_sync();
    for (int q = lo + lane; q <= hi; q += 64) {
      const uint32_t g = A[q];
      put(q, g);
      atomicOr(&used[g >> 5], 1u << (g & 31u));
    }
    wave_sync();
    const int seg = hi - lo + 1, rest = n - seg;
    int filled = 0;
    for (int base = 0; base < n; base += 64) {
      const int q = base + lane;
      uint32_t g = 0;
      bool keep = false;
      if (q < n) {
        g = B[(hi + 1 + q) % n];
        keep = ((used[g >> 5] >> (g & 31u)) & 1u) == 0u;
      }
      const uint64_t ball = __ballot(keep);
      const int before = __popcll(ball & ((1ull << lane) - 1ull));
      if (keep) {
        const int slot = filled + before;  // slot-th free position after hi
        if (slot < rest) put((hi + 1 + slot) % n, g);
      }
      filled += __popcll(ball);
    }
    wave_sync();
    // mutation: one sampled move, applied by lane 0 (rare, O(n))
    if (r2.z < a.pmut && lane == 0) {
      const Move m = decode_move(r2.w, r.x ^ r2.x, r.y ^ r2.y, n);
      if (m.typ == kMoveSwap) {
        const uint32_t t = get(m.i);
        put(m.i, get(m.j));
        put(m.j, t);
      } else if (m.typ == kMove2Opt) {
        for (int x = m.i, y = m.j; x < y; ++x, --y) {
          const uint32_t t = get(x);
          put(x, get(y));
          put(y, t);
        }
      } else if (m.i < m.j) {
        const uint32_t v = get(m.i);
        for (int x = m.i; x < m.j; ++x) put(x, get(x + 1));
        put(m.j, v);
      } else {
        const uint32_t v = get(m.i);
        for (int x = m.i; x > m.j; --x) put(x, get(x - 1));
        put(m.j, v);
      }
    }
  }
  if constexpr (WORDS) {
    wave_sync();
    const int nw = (n + 3) >> 2;
    for (int w = lane; w < nw; w += 64)
      a.child_w[(int64_t)w * members + gid] = reinterpret_cast<const uint32_t*>(cbuf)[w];
  }
}

struct GaSelectArgs {
  int islands, pop, n;
  const uint16_t* pop_tours;   // [islands][pop][n]
  const uint64_t* pop_keys;
  const uint16_t* child;       // rows [islands][pop][n]            (WORDS == false)
  const uint32_t* child_w;     // words [ceil(n/4)][islands * pop]  (WORDS == true)
  const uint64_t* child_keys;
  uint16_t* out_tours;         // [islands][pop][n]
  uint64_t* out_keys;
};

// (mu + lambda): the pop best of parents (index i) and children (index pop + i)
// by (key, index); bitonic sort over the next power of two >= 2 * pop.
template <bool WORDS>
__global__ __launch_bounds__(1024) void ga_select_kernel(GaSelectArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* sk = reinterpret_cast<uint64_t*>(smem);
  const int island = blockIdx.x, pop = a.pop, n = a.n;
  int M = 1;
  while (M < 2 * pop) M <<= 1;
  uint32_t* si = reinterpret_cast<uint32_t*>(sk + M);
  const uint64_t* pk = a.pop_keys + (int64_t)island * pop;
  const uint64_t* ck = a.child_keys + (int64_t)island * pop;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    sk[i] = i < pop ? pk[i] : (i < 2 * pop ? ck[i - pop] : ~0ull);
    si[i] = (uint32_t)i;
  }
  __syncthreads();
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
  const uint16_t* P = a.pop_tours + (int64_t)island * pop * n;
  const int64_t members = (int64_t)a.islands * pop;
  uint16_t* O = a.out_tours + (int64_t)island * pop * n;
  for (int i = threadIdx.x; i < pop; i += blockDim.x) a.out_keys[(int64_t)island * pop + i] = sk[i];
  for (int64_t e = threadIdx.x; e < (int64_t)pop * n; e += blockDim.x) {
    const int i = (int)(e / n), q = (int)(e % n);
    const uint32_t src = si[i];
    uint32_t g;
    if (src < (uint32_t)pop) {
      g = P[(int64_t)src * n + q];
    } else {
      const int64_t c = (int64_t)island * pop + (src - pop);
      if constexpr (WORDS) g = (a.child_w[(int64_t)(q >> 2) * members + c] >> (8 * (q & 3))) & 0xffu;
      else g = a.child[c * n + q];
    }
    O[e] = (uint16_t)g;
  }
}

// ===========================================================================
// Integer ant colony: tau (uint32 fixed point) per colony, eta2 = floor(2^24 / (1 + d)^2).
// ===========================================================================
struct AcoArgs {
  int colonies, ants, n, N;
  uint32_t seed_lo, seed_hi;
  uint64_t iter;
  const uint32_t* tau;   // [colonies][N][N]
  const uint32_t* eta;   // [N][N] (static part of the weight)
  uint16_t* tours;       // [colonies][ants][n]
  uint32_t* words;       // WORDS: the same tours, word-interleaved [ceil(n/4)][colonies * ants]
};

// Ant: starts at node 0; each step picks j among unvisited customers with
// probability w_j / sum w, w_j = (tau[i][j] >> 8) * eta[i][j] (uint64, exact),
// r = philox64 % sum, the smallest j (index order) whose prefix sum exceeds r.
// WORDS (n <= 255): the ant's tour is also kept in a wave-private LDS byte
// buffer and written out in the word-interleaved layout, so the colony is
// scored by eval_cvrp_words2 (the headline kernel).
//
// CH > 0 (N <= 64 CH): lane l owns nodes l + 64c (c < CH) -- their visited
// bits in a register mask and their weights in registers -- so a step is ONE
// gather round trip for the tau / eta row (the LDS path below gathers the row
// twice, once per pass), one DPP scan per chunk whose row totals give the
// colony total, and ballots for the first free node and the pick: no LDS
// visited set, no atomics, no wave barriers inside the construction.  Same
// weights, same sums (exact integers), same pick as the LDS path.
template <bool WORDS, int CH>
__global__ __launch_bounds__(256) void aco_construct_kernel(AcoArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  // wave-uniform in SGPRs (threadIdx.x >> 6 is not uniform to the compiler),
  // so the ant's Philox blocks and row addresses run on the scalar unit
  const int64_t gid = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(wave);
  const int N = a.N, n = a.n;
  const uint32_t words = ((uint32_t)N + 31u) / 32u;
  uint32_t* vis = reinterpret_cast<uint32_t*>(smem) + wave * words;
  uint8_t* tbuf = smem + ((4u * words * 4u + 15u) & ~15u) + wave * 256;
  const int64_t total_ants = (int64_t)a.colonies * a.ants;
  if (gid >= total_ants) return;
  if constexpr (WORDS) {
    for (int q = n + lane; q < 256; q += 64) tbuf[q] = 0;
  }
  const int colony = (int)(gid / a.ants), ant = (int)(gid % a.ants);
  const uint32_t* T = a.tau + (int64_t)colony * N * N;
  uint16_t* out = a.tours + gid * n;
  if constexpr (CH > 0) {
    uint32_t vm = lane == 0 ? 1u : 0u;  // bit c: node lane + 64c visited (or past N); depot
#pragma unroll
    for (int c = 0; c < CH; ++c)
      if (lane + 64 * c >= N) vm |= 1u << c;
    uint32_t cur = 0;
    uint32_t rx = 0, ry = 0;  // lane l: Philox block (iter, ant, s0 + l), words x / y
    for (int s = 0; s < n; ++s) {
      if ((s & 63) == 0) {  // the next 64 steps' draws, one per lane, in VALU
        const u32x4 r = philox((uint32_t)a.iter, (uint32_t)(a.iter >> 32),
                               (uint32_t)(colony * a.ants + ant), (uint32_t)(s + lane), a.seed_lo,
                               a.seed_hi);
        rx = r.x;
        ry = r.y;
      }
      const uint32_t r_x = (uint32_t)__builtin_amdgcn_readlane((int)rx, s & 63);
      const uint32_t r_y = (uint32_t)__builtin_amdgcn_readlane((int)ry, s & 63);
      const uint32_t* Tr = T + (int64_t)cur * N;
      const uint32_t* Er = a.eta + (int64_t)cur * N;
      uint32_t tv[CH], ev[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const bool fr = !((vm >> c) & 1u);
        tv[c] = fr ? Tr[lane + 64 * c] : 0u;
        ev[c] = fr ? Er[lane + 64 * c] : 0u;
      }
      uint64_t w[CH], inc[CH], ct[CH], tot = 0;
      uint32_t pick = 0xffffffffu;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        w[c] = (uint64_t)(tv[c] >> 8) * ev[c];
        inc[c] = w[c];
        ct[c] = wave_scan_add_u64(inc[c]);
        tot += ct[c];
        const uint64_t fb = __ballot(!((vm >> c) & 1u));
        if (pick == 0xffffffffu && fb) pick = (uint32_t)(64 * c + __ffsll((long long)fb) - 1);
      }
      if (tot != 0) {  // else: the first free node
        const uint64_t rr = umod64(((uint64_t)r_y << 32) | r_x, tot);
        uint64_t run = 0;
        uint32_t hp = 0xffffffffu;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const uint64_t ball = __ballot(w[c] > 0 && run + inc[c] > rr);
          if (hp == 0xffffffffu && ball) hp = (uint32_t)(64 * c + __ffsll((long long)ball) - 1);
          run += ct[c];
        }
        if (hp != 0xffffffffu) pick = hp;  // always: tot > rr
      }
      if (lane == 0) {
        out[s] = (uint16_t)pick;
        if constexpr (WORDS) tbuf[s] = (uint8_t)pick;
      }
      if (lane == (int)(pick & 63u)) vm |= 1u << (pick >> 6);
      cur = pick;
    }
    if constexpr (WORDS) {
      wave_sync();
      const int nw = (n + 3) >> 2;
      for (int w = lane; w < nw; w += 64)
        a.words[(int64_t)w * total_ants + gid] = reinterpret_cast<const uint32_t*>(tbuf)[w];
    }
  } else {  // LDS path (N > 256): visited bits in LDS, the row gathered once per pass
    for (uint32_t w = lane; w < words; w += 64) vis[w] = 0u;
    wave_sync();
    if (lane == 0) atomicOr(&vis[0], 1u);  // depot
    wave_sync();
    uint32_t cur = 0;
    for (int s = 0; s < n; ++s) {
      const u32x4 r = philox((uint32_t)a.iter, (uint32_t)(a.iter >> 32),
                             (uint32_t)(colony * a.ants + ant), (uint32_t)s, a.seed_lo, a.seed_hi);
      const uint32_t* Tr = T + (int64_t)cur * N;
      const uint32_t* Er = a.eta + (int64_t)cur * N;
      // pass 1: total weight (integer, so the order of summation is irrelevant)
      uint64_t tot = 0;
      int first_free = INT_MAX;
      for (int j = lane; j < N; j += 64) {
        if (!((vis[j >> 5] >> (j & 31)) & 1u)) {
          tot += (uint64_t)(Tr[j] >> 8) * Er[j];
          first_free = min(first_free, j);
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        tot += __shfl_xor(tot, off, 64);
        first_free = min(first_free, __shfl_xor(first_free, off, 64));
      }
      uint32_t pick;
      if (tot == 0) {
        pick = (uint32_t)first_free;
      } else {
        const uint64_t rr = (((uint64_t)r.y << 32) | r.x) % tot;
        // pass 2: scan chunks of 64 consecutive j; lane-level inclusive prefix
        uint64_t run = 0;
        pick = 0xffffffffu;
        for (int base = 0; base < N && pick == 0xffffffffu; base += 64) {
          const int j = base + lane;
          uint64_t w = 0;
          if (j < N && !((vis[j >> 5] >> (j & 31)) & 1u)) w = (uint64_t)(Tr[j] >> 8) * Er[j];
          uint64_t inc = w;
          for (int off = 1; off < 64; off <<= 1) {
            const uint64_t o = __shfl_up(inc, off, 64);
            if (lane >= off) inc += o;
          }
          const bool hit = w > 0 && run + inc > rr;
          const uint64_t ball = __ballot(hit);
          if (ball) pick = (uint32_t)(base + __ffsll((long long)ball) - 1);
          run += __shfl(inc, 63, 64);
        }
        if (pick == 0xffffffffu) pick = (uint32_t)first_free;  // unreachable: tot > rr
      }
      if (lane == 0) {
        out[s] = (uint16_t)pick;
        if constexpr (WORDS) tbuf[s] = (uint8_t)pick;
        atomicOr(&vis[pick >> 5], 1u << (pick & 31u));
      }
      wave_sync();
      cur = pick;
    }
    if constexpr (WORDS) {
      const int nw = (n + 3) >> 2;
      for (int w = lane; w < nw; w += 64)
        a.words[(int64_t)w * total_ants + gid] = reinterpret_cast<const uint32_t*>(tbuf)[w];
    }
  }
}

// The register path with the colony's weights staged in LDS (N * N * 8 bytes
// fit beside the tour buffers): a workgroup is up to 16 ants of ONE colony
// (wpg wavefronts), which first forms w[i][j] = (tau[i][j] >> 8) * eta[i][j]
// -- the same uint64 products the L2 path forms at every step -- for the
// whole colony, coalesced, once per iteration; then each step of each ant
// reads its row with one ds_read_b64 per chunk (conflict-free: consecutive
// lanes, consecutive entries) instead of a dependent tau + eta round trip to
// L2 and a 64-bit multiply.  Philox streams (colony * ants + ant, step), the
// roulette and the pick are the register path's, so the tours are the same.
// (Both paths draw the Philox blocks of 64 steps at once, lane l computing
// step s0 + l's in VALU and each step reading its own with v_readlane: the
// per-step block on the scalar unit made the construction SALU-issue bound,
// ~142 SALU per wave-step beside ~136 VALU, profiles/round6_aco_lds_*.)
template <bool WORDS, int CH>
__global__ __launch_bounds__(1024) void aco_construct_lds_kernel(AcoArgs a, int wpg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N, n = a.n;
  // [N][NS] weights, NS = N rounded up to even: a row starts 16-byte aligned,
  // so lane l's CH consecutive entries are whole ds_read_b128s (conflict-free)
  const int NS = (N + 1) & ~1;
  uint64_t* Wt = reinterpret_cast<uint64_t*>(smem);
  uint8_t* tbuf = smem + (((size_t)N * NS * 8 + 15) & ~(size_t)15);
  const int groups = (a.ants + wpg - 1) / wpg;
  const int colony = (int)blockIdx.x / groups;
  const int ant0 = ((int)blockIdx.x % groups) * wpg;
  {
    const uint32_t* T = a.tau + (int64_t)colony * N * N;
    for (int e = threadIdx.x; e < N * NS; e += blockDim.x) {
      const int i = e / NS, j = e - i * NS;
      Wt[e] = j < N ? (uint64_t)(T[i * N + j] >> 8) * a.eta[i * N + j] : 0ull;
    }
  }
  __syncthreads();
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int ant = ant0 + wave;
  if (ant >= a.ants) return;  // (no barrier after this point)
  uint8_t* tb = tbuf + wave * 256;
  const int64_t gid = (int64_t)colony * a.ants + ant;
  const int64_t total_ants = (int64_t)a.colonies * a.ants;
  if constexpr (WORDS) {
    for (int q = n + lane; q < 256; q += 64) tb[q] = 0;
  }
  uint16_t* out = a.tours + gid * n;
  // Lane l owns the CH consecutive nodes CH l .. CH l + CH - 1, so the
  // roulette's prefix sums in node order are the lanes' prefix (ONE 64-bit
  // wave scan of each lane's sum, not one per 64-node chunk) followed by the
  // lane's own running sum: the first lane whose inclusive prefix passes r
  // holds the pick, the first of its nodes whose running sum passes r.  (The
  // first node j with prefix P_j > r has w_j > 0, the register path's rule.)
  uint32_t vm = lane == 0 ? 1u : 0u;  // bit c: node CH lane + c visited (or past N); depot
#pragma unroll
  for (int c = 0; c < CH; ++c)
    if (CH * lane + c >= N) vm |= 1u << c;
  constexpr uint32_t kAll = (1u << CH) - 1u;
  uint32_t cur = 0;
  uint32_t rx = 0, ry = 0;  // lane l: Philox block (iter, gid, s0 + l), words x / y
  for (int s = 0; s < n; ++s) {
    if ((s & 63) == 0) {  // the next 64 steps' draws, one per lane, in VALU
      const u32x4 r = philox((uint32_t)a.iter, (uint32_t)(a.iter >> 32), (uint32_t)gid,
                             (uint32_t)(s + lane), a.seed_lo, a.seed_hi);
      rx = r.x;
      ry = r.y;
    }
    const uint32_t r_x = (uint32_t)__builtin_amdgcn_readlane((int)rx, s & 63);
    const uint32_t r_y = (uint32_t)__builtin_amdgcn_readlane((int)ry, s & 63);
    const uint64_t* Wr = Wt + cur * (uint32_t)NS + CH * lane;
    uint64_t w[CH], sum = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      w[c] = !((vm >> c) & 1u) ? Wr[c] : 0ull;
      sum += w[c];
    }
    uint64_t incl = sum;
    const uint64_t tot = wave_scan_add_u64(incl);
    uint32_t mine, L;  // this lane's candidate node, the lane that holds the pick
    if (tot != 0) {
      const uint64_t rr = umod64(((uint64_t)r_y << 32) | r_x, tot);
      L = (uint32_t)__ffsll((long long)__ballot(incl > rr)) - 1u;  // exists: the last lane's is tot
      uint64_t run = incl - sum;
      uint32_t cc = CH - 1;
      bool found = false;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        run += w[c];
        if (!found && run > rr) {
          cc = (uint32_t)c;
          found = true;
        }
      }
      mine = CH * (uint32_t)lane + cc;
    } else {  // every free weight is 0: the first free node
      L = (uint32_t)__ffsll((long long)__ballot(vm != kAll)) - 1u;
      mine = CH * (uint32_t)lane + (uint32_t)__builtin_ctz((~vm & kAll) | (1u << CH));
    }
    const uint32_t pick = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)L);
    if (lane == 0) {
      out[s] = (uint16_t)pick;
      if constexpr (WORDS) tb[s] = (uint8_t)pick;
    }
    if ((uint32_t)lane == pick / CH) vm |= 1u << (pick % CH);
    cur = pick;
  }
  if constexpr (WORDS) {
    wave_sync();
    const int nw = (n + 3) >> 2;
    for (int w = lane; w < nw; w += 64)
      a.words[(int64_t)w * total_ants + gid] = reinterpret_cast<const uint32_t*>(tb)[w];
  }
}

// LDS bytes of aco_construct_lds_kernel (weights + a 256-byte tour buffer per wavefront)
static size_t aco_lds_bytes(int N, int wpg) {
  return (((size_t)N * ((N + 1) & ~1) * 8 + 15) & ~(size_t)15) + 256 * (size_t)wpg;
}

struct AcoUpdateArgs {
  int colonies, ants, n, N;
  uint32_t evap_shift, tau_min, tau_max;
  uint32_t* tau;                 // [colonies][N][N]
  const uint16_t* tours;         // [colonies][ants][n]
  const uint64_t* ib;            // [colonies][2] iteration-best (key, ant)
  int bsf;                       // this iteration the best-so-far deposits
};

// The end of an iteration for small matrices (N <= 256), one workgroup per
// colony instead of four launches: the colony's iteration-best (key, ant)
// (lowest ant on ties, as segment_argmin_kernel), its best-so-far when
// strictly better (aco_track_best_kernel), evaporation of its tau, then the
// deposit on the iteration-best tour, or on a best-so-far iteration the
// best-so-far's (aco_deposit_kernel) -- colonies share nothing, so the
// per-colony order is the whole order.
__global__ __launch_bounds__(1024) void aco_update_fused_kernel(AcoUpdateArgs a, const uint64_t* __restrict__ keys,
                                                               uint64_t* ib, uint16_t* best_tours,
                                                               uint64_t* best_keys) {
  const int c = blockIdx.x;
  uint64_t k = ~0ull, idx = ~0ull;
  for (int i = threadIdx.x; i < a.ants; i += blockDim.x) {
    const uint64_t v = keys[(int64_t)c * a.ants + i];
    if (v < k || (v == k && (uint64_t)i < idx)) {
      k = v;
      idx = (uint64_t)i;
    }
  }
  wave_argmin(k, idx);
  __shared__ uint64_t wk[16], wi[16];
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    wk[w] = k;
    wi[w] = idx;
  }
  __syncthreads();
  k = wk[0];
  idx = wi[0];
  for (int x = 1; x < (int)(blockDim.x >> 6); ++x)
    if (wk[x] < k || (wk[x] == k && wi[x] < idx)) {
      k = wk[x];
      idx = wi[x];
    }
  const uint16_t* t = a.tours + ((int64_t)c * a.ants + (int64_t)idx) * a.n;
  if (threadIdx.x == 0) {
    ib[2 * c] = k;
    ib[2 * c + 1] = idx;
  }
  const bool tracked = best_tours && best_keys;
  const uint64_t bsf_key = tracked ? best_keys[c] : ~0ull;  // block-uniform
  __syncthreads();
  if (tracked && k < bsf_key) {
    for (int q = threadIdx.x; q < a.n; q += blockDim.x) best_tours[(int64_t)c * a.n + q] = t[q];
    __syncthreads();
    if (threadIdx.x == 0) best_keys[c] = k;
  } else if (tracked && a.bsf) {  // the (unchanged) best-so-far deposits
    t = best_tours + (int64_t)c * a.n;
    k = bsf_key;
  }
  // evaporation: 8 loads in flight per thread before the stores
  uint32_t* T = a.tau + (int64_t)c * a.N * a.N;
  const int NN = a.N * a.N, B = (int)blockDim.x;
  for (int base = (int)threadIdx.x; base < NN; base += 8 * B) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base + u * B < NN ? T[base + u * B] : 0u;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (base + u * B < NN) T[base + u * B] = min(a.tau_max, max(a.tau_min, v[u] - (v[u] >> a.evap_shift)));
  }
  __syncthreads();
  const uint32_t primary = (uint32_t)((k >> 28) & ((1u << 28) - 1u));
  const uint32_t dep = (uint32_t)((1u << 30) / (1ull + primary));
  for (int q = threadIdx.x; q <= a.n; q += blockDim.x) {
    const uint32_t from = q == 0 ? 0u : t[q - 1];
    const uint32_t to = q == a.n ? 0u : t[q];
    atomicAdd(&T[(uint64_t)from * a.N + to], dep);
  }
}

__global__ void aco_evaporate_kernel(AcoUpdateArgs a) {
  const int64_t total = (int64_t)a.colonies * a.N * a.N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t t = a.tau[i];
    a.tau[i] = min(a.tau_max, max(a.tau_min, t - (t >> a.evap_shift)));
  }
}

// deposit floor(2^30 / (1 + primary)) on every edge of the iteration-best
// tour, or on a best-so-far iteration (a.bsf) of the colony's best-so-far
// (already updated by aco_track_best_kernel)
__global__ void aco_deposit_kernel(AcoUpdateArgs a, const uint16_t* best_tours,
                                   const uint64_t* best_keys) {
  const int colony = blockIdx.x;
  const bool bsf = a.bsf && best_tours && best_keys;
  const uint64_t key = bsf ? best_keys[colony] : a.ib[2 * colony];
  const int ant = (int)a.ib[2 * colony + 1];
  const uint32_t primary = (uint32_t)((key >> 28) & ((1u << 28) - 1u));
  const uint32_t dep = (uint32_t)((1u << 30) / (1ull + primary));
  const uint16_t* t = bsf ? best_tours + (int64_t)colony * a.n
                          : a.tours + ((int64_t)colony * a.ants + ant) * a.n;
  uint32_t* T = a.tau + (int64_t)colony * a.N * a.N;
  for (int q = threadIdx.x; q <= a.n; q += blockDim.x) {
    const uint32_t from = q == 0 ? 0u : t[q - 1];
    const uint32_t to = q == a.n ? 0u : t[q];
    const uint64_t idx = (uint64_t)from * a.N + to;
    const uint32_t old = atomicAdd(&T[idx], dep);
    (void)old;
  }
}

// colony c's best-so-far <- its iteration-best ant when strictly better
__global__ void aco_track_best_kernel(const uint16_t* __restrict__ tours, int ants, int n,
                                      const uint64_t* __restrict__ ib, uint16_t* best_tours,
                                      uint64_t* best_keys) {
  const int c = blockIdx.x;
  const uint64_t key = ib[2 * c];
  if (!(key < best_keys[c])) return;  // block-uniform
  const uint16_t* t = tours + ((int64_t)c * ants + (int64_t)ib[2 * c + 1]) * n;
  for (int q = threadIdx.x; q < n; q += blockDim.x) best_tours[(int64_t)c * n + q] = t[q];
  __syncthreads();
  if (threadIdx.x == 0) best_keys[c] = key;
}

// per-colony argmin over ant keys -> ib[2c] = key, ib[2c+1] = ant
__global__ void segment_argmin_kernel(const uint64_t* __restrict__ keys, int seg, int nseg,
                                      uint64_t* out) {
  const int s = blockIdx.x;
  if (s >= nseg) return;
  uint64_t k = ~0ull, idx = ~0ull;
  for (int i = threadIdx.x; i < seg; i += blockDim.x) {
    const uint64_t v = keys[(int64_t)s * seg + i];
    if (v < k || (v == k && (uint64_t)i < idx)) {
      k = v;
      idx = (uint64_t)i;
    }
  }
  wave_argmin(k, idx);
  __shared__ uint64_t wk[16], wi[16];
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    wk[w] = k;
    wi[w] = idx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int x = 1; x < (int)(blockDim.x >> 6); ++x)
      if (wk[x] < k || (wk[x] == k && wi[x] < idx)) {
        k = wk[x];
        idx = wi[x];
      }
    out[2 * s] = k;
    out[2 * s + 1] = idx;
  }
}

// ===========================================================================
// Brute force: lexicographic ranks [r0, r1) of permutations of 1..n (n <= 15),
// nibble-packed (element i in bits 4i..4i+3).
// ===========================================================================
struct BfArgs {
  SearchInst si;
  int n;
  uint64_t r0, r1, chunk;
  uint64_t* block_best;  // [gridDim.x][2] (key, rank)
};

VRPMS_DEV uint32_t nib(uint64_t p, int i) { return (uint32_t)(p >> (4 * i)) & 15u; }

VRPMS_DEV uint64_t unrank(uint64_t r, int n) {
  uint64_t fact[16];
  fact[0] = 1;
  for (int i = 1; i < 16; ++i) fact[i] = fact[i - 1] * (uint64_t)i;
  uint32_t avail = (1u << n) - 1u;  // bit v-1 = value v available
  uint64_t p = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t f = fact[n - 1 - i];
    int d = (int)(r / f);
    r %= f;
    // d-th smallest available value
    uint32_t m = avail;
    for (int x = 0; x < d; ++x) m &= m - 1u;
    const int v = __ffs((int)m);  // 1-based bit position = value
    avail &= ~(1u << (v - 1));
    p |= (uint64_t)v << (4 * i);
  }
  return p;
}

VRPMS_DEV uint64_t next_perm(uint64_t p, int n) {
  int i = n - 2;
  while (i >= 0 && nib(p, i) >= nib(p, i + 1)) --i;
  if (i < 0) return p;
  int j = n - 1;
  while (nib(p, j) <= nib(p, i)) --j;
  const uint64_t a = nib(p, i), b = nib(p, j);
  p &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
  p |= (b << (4 * i)) | (a << (4 * j));
  for (int x = i + 1, y = n - 1; x < y; ++x, --y) {
    const uint64_t vx = nib(p, x), vy = nib(p, y);
    p &= ~((15ull << (4 * x)) | (15ull << (4 * y)));
    p |= (vy << (4 * x)) | (vx << (4 * y));
  }
  return p;
}

template <typename MatT, int HM, bool CVRP>
__global__ __launch_bounds__(256) void bf_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StagedInst<MatT, HM> I = stage_inst<MatT, HM>(a.si, smem);
  const int n = a.n;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t bk = ~0ull, br = ~0ull;
  const uint64_t lo = a.r0 + tid * a.chunk;
  if (lo < a.r1) {
    const uint64_t hi = min(a.r1, lo + a.chunk);
    uint64_t p = unrank(lo, n);
    for (uint64_t rk = lo; rk < hi; ++rk) {
      auto tour = [&](int i) { return nib(p, i); };
      const uint64_t k = eval_tour<CVRP>(I.D, I.sp, tour, n).key;
      if (k < bk) {
        bk = k;
        br = rk;
      }
      p = next_perm(p, n);
    }
  }
  wave_argmin(bk, br);
  __shared__ uint64_t wk[4], wr[4];
  if (lane_id() == 0) {
    wk[threadIdx.x >> 6] = bk;
    wr[threadIdx.x >> 6] = br;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (wk[w] < bk || (wk[w] == bk && wr[w] < br)) {
        bk = wk[w];
        br = wr[w];
      }
    a.block_best[2 * blockIdx.x] = bk;
    a.block_best[2 * blockIdx.x + 1] = br;
  }
}

__global__ void reduce_pairs_kernel(const uint64_t* in, int count, uint64_t* out) {
  uint64_t k = ~0ull, r = ~0ull;
  for (int i = threadIdx.x; i < count; i += blockDim.x) {
    const uint64_t kk = in[2 * i], rr = in[2 * i + 1];
    if (kk < k || (kk == k && rr < r)) {
      k = kk;
      r = rr;
    }
  }
  wave_argmin(k, r);
  __shared__ uint64_t wk[16], wr[16];
  if (lane_id() == 0) {
    wk[threadIdx.x >> 6] = k;
    wr[threadIdx.x >> 6] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (wk[w] < k || (wk[w] == k && wr[w] < r)) {
        k = wk[w];
        r = wr[w];
      }
    out[0] = k;
    out[1] = r;
  }
}

// ===========================================================================
// Throughput mode (BASELINE.json config 5): a batch of independent static TSP
// requests, each with its own matrix, ONE WORKGROUP PER REQUEST.  The
// request's matrix is staged in LDS; its 4 wavefronts run 4 SA chains from
// Philox Fisher-Yates starts; candidate moves are priced by the exact O(1)
// integer delta (tsp_move_delta), so a step costs ~8 LDS gathers per lane
// instead of n; the best (key, wave) of the 4 chains is the answer.
// ===========================================================================
struct TspBatchArgs {
  const int32_t* mats;   // [R][N][N]
  int R, N, steps;
  float inv_t0, inv_alpha;
  uint32_t seed_lo, seed_hi;
  uint16_t* best_tours;  // [R][N-1]
  uint64_t* best_keys;   // [R]
};

// One request's 4 chains over its LDS-resident matrix D (MatT = uint16_t when
// every entry fits, int32_t otherwise); `work` is the LDS after the matrix.
template <typename MatT, bool symmetric, bool small>
VRPMS_DEV void tsp_batch_body(const TspBatchArgs& a, const MatT* D, unsigned char* work) {
  const int N = a.N, n = N - 1, r = blockIdx.x;
  // each tour buffer holds the depot (0) at positions -1 and n, so a move's
  // six tour reads need no bounds test
  const uint32_t npad = ((uint32_t)n + 2u + 7u) & ~7u;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  uint16_t* buf = reinterpret_cast<uint16_t*>(work) + wave * 3 * npad;
  uint64_t* wbest = reinterpret_cast<uint64_t*>(work + 4 * 3 * npad * 2);
  for (uint32_t q = lane; q < 3 * npad; q += 64) buf[q] = 0;
  wave_sync();
  uint16_t* A = buf + 1;
  uint16_t* B = buf + npad + 1;
  uint16_t* Best = buf + 2 * npad + 1;
  const uint32_t cid = (uint32_t)(r * 4 + wave);
  // Philox Fisher-Yates start: for i = n-1..1 swap t[i], t[x % (i+1)].  Lane
  // l draws i = 64c + l's block for a chunk c of 64 steps at once (VALU, not
  // 49 scalar Philox blocks in a row); lane 0 swaps, reading each j by
  // v_readlane.
  for (int q = lane; q < n; q += 64) A[q] = (uint16_t)(q + 1);
  wave_sync();
  uint32_t jv = 0;
  for (int i = n - 1; i >= 1; --i) {
    if (i == n - 1 || (i & 63) == 63) {
      const uint32_t il = (uint32_t)(i & ~63) + (uint32_t)lane;
      const u32x4 x = philox(0xffffffffu, 0xffffffffu, cid, il, a.seed_lo, a.seed_hi);
      jv = x.x % (il + 1u);
    }
    const int j = __builtin_amdgcn_readlane((int)jv, i & 63);
    if (lane == 0) {
      const uint16_t t = A[i];
      A[i] = A[j];
      A[j] = t;
    }
  }
  wave_sync();
  auto dist = [&](uint32_t x, uint32_t y) { return (int)D[__umul24(x, (uint32_t)N) + y]; };
  // symmetric matrix: the current tour's edges E[q] = D(A[q-1], A[q]), q = 0..n
  // (the depot at both ends), kept with the tour -- a move's removed edges
  // are tour edges at positions i, i+1, j, j+1, so they are read from E
  // (a few dwords, no bank conflicts) and only its added edges are random
  // matrix gathers; E is rebuilt on an accept
  const uint32_t epad = npad + 8u;
  MatT* E = reinterpret_cast<MatT*>(work + 4 * 3 * npad * 2 + 4 * 8) + wave * epad;
  auto build_E = [&]() {
    for (int q = lane; q <= n; q += 64)
      E[q] = (MatT)dist(q ? (uint32_t)A[q - 1] : 0u, q < n ? (uint32_t)A[q] : 0u);
    wave_sync();
  };
  if constexpr (symmetric) build_E();
  auto full = [&](const uint16_t* T) {
    int s = 0;
    uint32_t prev = 0;
    for (int q = 0; q < n; ++q) {
      s += dist(prev, T[q]);
      prev = T[q];
    }
    return s + dist(prev, 0);
  };
  int dur = full(A);
  uint64_t ck = pack_key(0, (uint32_t)dur, 0), bk = ck;
  for (int q = lane; q < n; q += 64) Best[q] = A[q];
  float invT = a.inv_t0;
  // one SA step: xm = the lane's move word, xa = the chain's acceptance draw
  auto step = [&](uint32_t xm, uint32_t xa) __attribute__((always_inline)) {
    const Move m = decode_move1(xm, n);
    auto tourA = [&](int q) { return (uint32_t)A[q]; };
    int delta;
    if constexpr (symmetric)
      delta = tsp_move_delta_sym_cached<true>(dist, tourA, [&](int q) { return (int)E[q]; }, n, m);
    else delta = tsp_move_delta(dist, tourA, n, m, false);
    const int nd = dur + delta;
    uint64_t k;
    int bl;
#if VRPMS_TSPB_AB == 2  // timing attribution only (wrong search): no argmin, lane 0's move
    if (true) {
      bl = 0;
      k = pack_key(0, (uint32_t)wave_bcast(nd, 0), 0);
    } else
#endif
    if constexpr (small) {  // (duration << 6 | lane): the same order as (key, lane)
      const uint32_t v = wave_min_u32_uniform(((uint32_t)nd << 6) | (uint32_t)lane);
      bl = (int)(v & 63u);
      k = pack_key(0, v >> 6, 0);
    } else {
      k = wave_argmin_lane(pack_key(0, (uint32_t)nd, 0), bl);
    }
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      accept = accept_test(dp, invT, xa >> 8);
    }
#if VRPMS_TSPB_AB >= 1  // timing attribution only (wrong search): the tour never moves
    if (xa != 0xFFFFFFFFu) accept = false;
#endif
    if (accept) {  // bl is wave-uniform: the winner's move by v_readlane
      Move mb;
      mb.typ = (uint32_t)wave_bcast((int)m.typ, bl);
      mb.i = wave_bcast(m.i, bl);
      mb.j = wave_bcast(m.j, bl);
      dur = wave_bcast(nd, bl);
      if (n < 64) {  // one position per lane: the moved tour stays in registers
        const uint32_t v = lane < n ? (uint32_t)A[moved_index(lane, mb)] : 0u;  // 0: the depot
        if (lane < n) B[lane] = (uint16_t)v;
        if constexpr (symmetric) {  // E from the moved tour: the predecessor by wave_shr:1
          const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
          if (lane <= n) E[lane] = (MatT)dist(lane ? prev : 0u, v);
        }
        uint16_t* t = A;
        A = B;
        B = t;
        ck = k;
        if (ck < bk) {
          bk = ck;
          if (lane < n) Best[lane] = (uint16_t)v;
        }
      } else {
        for (int q = lane; q < n; q += 64) B[q] = A[moved_index(q, mb)];
        wave_sync();
        uint16_t* t = A;
        A = B;
        B = t;
        if constexpr (symmetric) build_E();
        ck = k;
        if (ck < bk) {
          bk = ck;
          for (int q = lane; q < n; q += 64) Best[q] = A[q];
        }
      }
      wave_sync();
    }
    invT = invT * a.inv_alpha;
  };
  // A13: one Philox block per lane serves four steps (word s & 3 is step s's
  // move) and one per chain -- wave-uniform counters, so the scalar unit
  // computes it -- the four steps' acceptance draws.  Unrolled by four, so
  // each step reads its words without a select.
  int s = 0;
  if (n >= 2) {
    for (; s + 4 <= a.steps; s += 4) {
      const u32x4 rb = philox((uint32_t)(s >> 2), 0u, cid, (uint32_t)lane, a.seed_lo, a.seed_hi);
      const u32x4 ra = philox((uint32_t)(s >> 2), 1u, cid, 0u, a.seed_lo, a.seed_hi);
      step(rb.x, ra.x);
      step(rb.y, ra.y);
      step(rb.z, ra.z);
      step(rb.w, ra.w);
    }
    if (s < a.steps) {  // the last 1..3 steps
      const u32x4 rb = philox((uint32_t)(s >> 2), 0u, cid, (uint32_t)lane, a.seed_lo, a.seed_hi);
      const u32x4 ra = philox((uint32_t)(s >> 2), 1u, cid, 0u, a.seed_lo, a.seed_hi);
      for (int h = 0; s + h < a.steps; ++h)
        step(h == 0 ? rb.x : h == 1 ? rb.y : rb.z, h == 0 ? ra.x : h == 1 ? ra.y : ra.z);
    }
  }
  if (lane == 0) wbest[wave] = bk;
  __syncthreads();
  int bw = 0;
  for (int w = 1; w < 4; ++w)
    if (wbest[w] < wbest[bw]) bw = w;
  if (wave == bw) {
    uint16_t* out = a.best_tours + (int64_t)r * n;
    for (int q = lane; q < n; q += 64) out[q] = Best[q];
    if (lane == 0) a.best_keys[r] = bk;
  }
}

// The request's matrix is checked in HBM (symmetric? every entry below
// 2^26 / N, so the one-dword argmin applies? every entry below 2^16?) and
// staged into LDS as uint16 when it fits -- half the LDS bytes per request
// and two entries per dword for the 8 random gathers of each move -- else
// as int32.
__global__ __launch_bounds__(256) void tsp_batch_sa_kernel(TspBatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.N, r = blockIdx.x;
  const uint32_t NN = (uint32_t)N * N;
  const int32_t* src = a.mats + (int64_t)r * NN;
  int asym = 0, big = 0, wide = 0;
  // tour durations < 2^26 when every entry is below 2^26 / N: the 64-lane
  // argmin of (duration, lane) then fits one dword
  const int32_t lim26 = (int32_t)((1u << 26) / (uint32_t)N);
  for (uint32_t i = threadIdx.x; i < NN; i += blockDim.x) {
    const uint32_t x = i / N, y = i % N;
    const int32_t v = src[i];
    asym |= v != src[y * N + x];
    big |= v < 0 || v >= lim26;
    wide |= v < 0 || v > 65535;
  }
  const bool symmetric = __syncthreads_or(asym) == 0;
  const bool small = __syncthreads_or(big) == 0;
  const bool narrow = __syncthreads_or(wide) == 0;
  unsigned char* work = smem + ((NN * 4 + 15u) & ~15u);
  // block-uniform flags as template arguments: one straight step loop each
  auto run = [&](auto* D) {
    using MT = std::remove_pointer_t<decltype(D)>;
    if (symmetric) {
      if (small) tsp_batch_body<MT, true, true>(a, D, work);
      else tsp_batch_body<MT, true, false>(a, D, work);
    } else {
      if (small) tsp_batch_body<MT, false, true>(a, D, work);
      else tsp_batch_body<MT, false, false>(a, D, work);
    }
  };
  if (narrow) {
    uint16_t* D = reinterpret_cast<uint16_t*>(smem);
    for (uint32_t i = threadIdx.x; i < NN; i += blockDim.x) D[i] = (uint16_t)src[i];
    __syncthreads();
    run(D);
  } else {
    int32_t* D = reinterpret_cast<int32_t*>(smem);
    for (uint32_t i = threadIdx.x; i < NN; i += blockDim.x) D[i] = src[i];
    __syncthreads();
    run(D);
  }
}

// ---------------------------------------------------------------------------
// dispatch helpers: <MatT, HM, CVRP> from the loaded instance
// ---------------------------------------------------------------------------
template <template <typename, int, bool> class K, typename Args>
static int launch_inst(const vrpms_ctx* ctx, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                       const Args& args) {
  const Instance& in = ctx->inst;
  const bool cvrp = in.problem == VRPMS_CVRP;
  auto go = [&](auto kern) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, block, lds, s>>>(args);
  };
#define VRPMS_SEL(MT)                                                            \
  if (in.H == 1) {                                                               \
    if (cvrp) go(K<MT, 1, true>::kernel()); else go(K<MT, 1, false>::kernel());  \
  } else if (in.H == 24) {                                                       \
    if (cvrp) go(K<MT, 24, true>::kernel()); else go(K<MT, 24, false>::kernel());\
  } else {                                                                       \
    if (cvrp) go(K<MT, 0, true>::kernel()); else go(K<MT, 0, false>::kernel());  \
  }
  if (in.use16) {
    VRPMS_SEL(uint16_t)
  } else {
    VRPMS_SEL(int32_t)
  }
#undef VRPMS_SEL
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

template <typename MatT, int HM, bool CVRP>
struct SaK {
  static auto kernel() { return sa_kernel<MatT, HM, CVRP>; }
};
template <typename MatT, int HM, bool CVRP>
struct RouteK {
  static auto kernel() { return sa_route_kernel<MatT, HM>; }
};
template <typename MatT, int HM, bool CVRP>
struct RouteHK {  // per-vehicle capacities / start times
  static auto kernel() { return sa_route_kernel<MatT, HM, true>; }
};
template <typename MatT, int HM, bool CVRP>
struct BfK {
  static auto kernel() { return bf_kernel<MatT, HM, CVRP>; }
};

int launch_ga_fused(const vrpms_ctx* ctx, const vrpms_ga_params* p, uint16_t* d_pop,
                    uint64_t* d_keys, int n, hipStream_t s);  // ga_fused.hip
int launch_sa_seg(const vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur,
                  uint64_t* d_cur_key, uint16_t* d_best, uint64_t* d_best_key, int n,
                  uint32_t wtypes, int moves, hipStream_t s);  // sa_seg.hip
int launch_sa_td(const vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur,
                 uint64_t* d_cur_key, uint16_t* d_best, uint64_t* d_best_key, int n,
                 uint32_t wtypes, int moves, hipStream_t s);  // sa_td.hip

static void ensure_scratch(vrpms_ctx* ctx, size_t bytes, int* err) {
  if (ctx->search_scratch_bytes >= bytes) return;
  (void)hipFree(ctx->search_scratch);
  ctx->search_scratch = nullptr;
  ctx->search_scratch_bytes = 0;
  if (hipMalloc(&ctx->search_scratch, bytes) != hipSuccess) {
    *err = fail(VRPMS_ENOMEM, "search scratch allocation failed");
    return;
  }
  ctx->search_scratch_bytes = bytes;
}

}  // namespace vrpms

using namespace vrpms;

extern "C" int vrpms_sa_run(vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur,
                            uint64_t* d_cur_key, uint16_t* d_best, uint64_t* d_best_key,
                            int32_t n, void* stream) {
  if (!ctx || !p) return fail(VRPMS_EINVAL, "vrpms_sa_run: NULL ctx/params");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_sa_run: no instance loaded");
  // tours: customers, plus (CVRP) A10 separator tokens, fewer than K of
  // them useful; at most N - 1 + K tokens
  const int max_tokens = ctx->inst.N - 1 + (ctx->inst.problem == VRPMS_CVRP ? ctx->inst.K : 0);
  if (p->chains <= 0 || p->steps < 0 || n < 0 || n > max_tokens)
    return fail(VRPMS_EINVAL, "vrpms_sa_run: need chains > 0, steps >= 0, 0 <= n <= N-1 (+K for CVRP)");
  if (!d_cur || !d_cur_key || !d_best || !d_best_key)
    return fail(VRPMS_EINVAL, "vrpms_sa_run: NULL state buffer");
  if (p->window_types > 7u) return fail(VRPMS_EINVAL, "vrpms_sa_run: window_types is a 3-bit mask");
  const uint32_t wtypes = p->window_types ? p->window_types : 7u;
  // moves per step: 64 (one wavefront per chain) or 64 W, W = 2..8 wavefronts
  // per chain (route-local kernel only)
  const int moves = p->moves ? p->moves : 64;
  if (moves % 64 != 0 || moves < 64 || moves > 64 * kRouteMaxWaves)
    return fail(VRPMS_EINVAL, "vrpms_sa_run: moves must be 64 * W, W = 1..8");
  const int wpc = moves / 64;
  VRPMS_HIP(hipSetDevice(ctx->device));
  if (ctx->opt_sa_route == 4) {  // force the hour-row kernel (sa_td.hip)
    const int rc = launch_sa_td(ctx, p, d_cur, d_cur_key, d_best, d_best_key, n, wtypes, moves,
                                (hipStream_t)stream);
    if (rc <= 0) return rc;
    return fail(VRPMS_EINVAL,
                "vrpms_sa_run: the hour-row kernel needs H = 24, a u16 matrix, moves <= 256 and "
                "LDS room for one chain's rows");
  }
  FastSplit f;
  if (wpc == 1 && ctx->inst.H == 1 && fast_split_params(ctx, n, &f)) {
    const uint32_t tb = ((uint32_t)n + 12u + 15u) & ~15u;
    const size_t lds = (((size_t)f.N * f.N * 8 + 15) & ~(size_t)15) +
                       (size_t)kSaPackedWaves * 3 * tb;
    if (lds <= ctx->max_lds) {
      SaPackedArgs pa{f, p->chains, n, p->steps, p->window, wtypes, p->inv_t0, p->inv_alpha, (uint32_t)p->seed,
                      (uint32_t)(p->seed >> 32), p->step0, tb, d_cur, d_cur_key, d_best,
                      d_best_key};
      if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(sa_packed_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      const int grid = (p->chains + kSaPackedWaves - 1) / kSaPackedWaves;
      sa_packed_kernel<<<grid, 64 * kSaPackedWaves, lds, (hipStream_t)stream>>>(pa);
      VRPMS_HIP(hipGetLastError());
      return VRPMS_OK;
    }
  }
  // segment pricing (sa_seg_kernel, sa_seg.hip): static symmetric matrix,
  // one capacity, every demand fits a vehicle -- any move span, any start times
  if (ctx->opt_sa_route == 0) {
    const int rc = launch_sa_seg(ctx, p, d_cur, d_cur_key, d_best, d_best_key, n, wtypes, moves,
                                 (hipStream_t)stream);
    if (rc <= 0) return rc;
  }
  // hour-indexed matrices (H = 24): full walks over LDS hour rows, any fleet
  // (sa_td.hip) -- except a uniform fleet's long tours, where the route-local
  // walks are faster: sa_td / sa_route 1.08x at 419 tokens, 0.85x at 629
  // (TD-400 / TD-600 x 24, tools/td_large_rate.py FLEET=uniform,
  // profiles/round6_td_large_rate_uniform.log), so past 480 tokens the
  // route kernel takes them when it applies
  const Instance& in0 = ctx->inst;
  const bool uniform_fleet = in0.uniform_cap && in0.min_start == in0.max_start;
  const bool route_applies = p->window > 0 && in0.problem == VRPMS_CVRP &&
                             in0.max_dem <= in0.min_cap && in0.max_dem <= 65535 &&
                             route_max(in0.K) <= 255 && n <= 65535;
  if (ctx->opt_sa_route == 0 && !(uniform_fleet && route_applies && n > 480)) {
    const int rc = launch_sa_td(ctx, p, d_cur, d_cur_key, d_best, d_best_key, n, wtypes, moves,
                                (hipStream_t)stream);
    if (rc <= 0) return rc;
  }
  SaArgs a{search_inst(ctx), p->chains, n, p->steps, p->window, wtypes, p->inv_t0, p->inv_alpha,
           (uint32_t)p->seed, (uint32_t)(p->seed >> 32), p->step0, d_cur, d_cur_key, d_best,
           d_best_key, wpc};
  // route-local pricing (sa_route_kernel) for windowed SA, every demand
  // fitting the smallest vehicle: an exchangeable fleet (one capacity, one
  // start time) or not (HV: walks re-synchronise on the same vehicle only)
  const Instance& in = ctx->inst;
  const bool hv = !(in.uniform_cap && in.min_start == in.max_start);
  // Hour-indexed (H = 24) requests with per-vehicle capacities or start times
  // that sa_td_kernel cannot hold (its LDS rows: large n) go to sa_kernel's
  // full L2 walks when one wavefront prices a chain's moves: measured faster
  // than the route-local walks there, 1.15-1.21x at TD-400 .. TD-1000 x 24
  // (tools/td_large_rate.py, profiles/round6_td_large_rate.log; same
  // trajectories).  Option 3 still forces the route kernel.
  const bool td_full_walk = ctx->opt_sa_route == 0 && in.H == 24 && hv && wpc == 1;
  if (p->window > 0 && in.problem == VRPMS_CVRP && in.max_dem <= in.min_cap &&
      in.max_dem <= 65535 && route_max(in.K) <= 255 && !td_full_walk &&
      n <= 65535 && ctx->opt_sa_route != 2) {  // (0 auto, 3 force this kernel)
    const size_t npad = ((size_t)n + 7) & ~(size_t)7;
    const size_t wbytes = ((size_t)route_wave_bytes((int)npad, in.K) + 15) & ~(size_t)15;
    const int elem = in.use16 ? 2 : 4;
    const size_t cpw = wpc > 1 ? 1 : 4;  // chains per workgroup
    const size_t legs = route_legs_bytes(in.H, in.N, elem) +
                        cpw * (size_t)route_edge_bytes(in.H, (int)npad, elem, a.si.symmetric != 0);
    size_t lds = inst_lds_bytes_host(a.si) + cpw * wbytes + legs;
    if (lds > ctx->max_lds) {
      a.si.mat_lds = 0;
      lds = inst_lds_bytes_host(a.si) + cpw * wbytes + legs;
    }
    if (lds <= ctx->max_lds) {
      // one workgroup per CU: request more than half the CU's LDS
      const int per_cu = ctx->opt_route_wg_per_cu ? ctx->opt_route_wg_per_cu : (wpc > 1 ? 1 : 2);
      if (per_cu == 1) lds = std::max(lds, ctx->max_lds / 2 + 16);
      const dim3 grid(wpc > 1 ? p->chains : (p->chains + 3) / 4), block(wpc > 1 ? 64 * wpc : 256);
      if (hv) return launch_inst<RouteHK>(ctx, grid, block, lds, (hipStream_t)stream, a);
      return launch_inst<RouteK>(ctx, grid, block, lds, (hipStream_t)stream, a);
    }
  }
  if (wpc > 1)
    return fail(VRPMS_EINVAL,
                "vrpms_sa_run: moves > 64 needs the route-local kernel (window > 0, CVRP, every "
                "demand fits the smallest vehicle, at most 126 vehicles)");
  const size_t npad = ((size_t)n + 7) & ~(size_t)7;
  size_t lds = inst_lds_bytes_host(a.si) + 4 * 3 * npad * 2;
  if (lds > ctx->max_lds) {
    a.si.mat_lds = 0;
    lds = inst_lds_bytes_host(a.si) + 4 * 3 * npad * 2;
  }
  if (lds > ctx->max_lds) return fail(VRPMS_EINVAL, "vrpms_sa_run: tours too long for LDS");
  return launch_inst<SaK>(ctx, dim3((p->chains + 3) / 4), dim3(256), lds, (hipStream_t)stream, a);
}

extern "C" int vrpms_ga_generation(vrpms_ctx* ctx, const vrpms_ga_params* p, uint16_t* d_pop,
                                   uint64_t* d_keys, int32_t n, void* stream) {
  if (!ctx || !p) return fail(VRPMS_EINVAL, "vrpms_ga_generation: NULL ctx/params");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_ga_generation: no instance loaded");
  if (p->islands <= 0 || p->pop <= 1 || p->pop > 4096 || n < 0 || n > ctx->inst.N - 1)
    return fail(VRPMS_EINVAL, "vrpms_ga_generation: need islands > 0, 2 <= pop <= 4096, n <= N-1");
  if (!d_pop || !d_keys) return fail(VRPMS_EINVAL, "vrpms_ga_generation: NULL population");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  // one workgroup per island for the whole call when the island fits the LDS
  const int fused = launch_ga_fused(ctx, p, d_pop, d_keys, n, s);
  if (fused < 0) return fused;
  if (fused) return VRPMS_OK;
  const int64_t members = (int64_t)p->islands * p->pop;
  const size_t tour_bytes = (size_t)members * n * 2;
  // Children are scored by the headline kernel (eval_cvrp_words2) whenever
  // its packed layout applies: the breed kernel then emits them in the
  // word-interleaved layout directly.  Otherwise uint16 rows + vrpms_eval.
  FastSplit f;
  const bool words = n <= 255 && fast_split_params(ctx, n, &f);
  const int nw = (n + 3) / 4;
  const size_t child_bytes = words ? (size_t)nw * members * 4 : tour_bytes;
  const size_t a16 = 255;
  auto up = [&](size_t x) { return (x + a16) & ~a16; };
  const size_t need = up(child_bytes) + up(tour_bytes) + 2 * up((size_t)members * 8);
  int err = VRPMS_OK;
  ensure_scratch(ctx, need, &err);
  if (err) return err;
  unsigned char* sp = static_cast<unsigned char*>(ctx->search_scratch);
  void* child = sp;
  uint16_t* next = reinterpret_cast<uint16_t*>(sp + up(child_bytes));
  uint64_t* ckeys = reinterpret_cast<uint64_t*>(sp + up(child_bytes) + up(tour_bytes));
  uint64_t* nkeys = reinterpret_cast<uint64_t*>(reinterpret_cast<unsigned char*>(ckeys) +
                                                up((size_t)members * 8));
  int M = 1;
  while (M < 2 * p->pop) M <<= 1;
  const size_t lds_s = (size_t)M * 12;
  const uint32_t bw = ((uint32_t)ctx->inst.N + 31u) / 32u;
  const size_t lds_b = ((4 * (size_t)bw * 4 + 15) & ~(size_t)15) + (words ? 4 * 256 : 0);
  if (lds_s > ctx->max_lds || lds_b > ctx->max_lds)
    return fail(VRPMS_EINVAL, "vrpms_ga_generation: population too large for LDS");
  auto breed = words ? ga_breed_kernel<true> : ga_breed_kernel<false>;
  auto select = words ? ga_select_kernel<true> : ga_select_kernel<false>;
  if (lds_b > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(breed),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_b);
  if (lds_s > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(select),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_s);
  // ping-pong between the caller's population and the scratch one: no copy
  // per generation, one at the end when the result landed in scratch
  uint16_t* src_t = d_pop;
  uint64_t* src_k = d_keys;
  uint16_t* dst_t = next;
  uint64_t* dst_k = nkeys;
  for (int g = 0; g < p->generations; ++g) {
    const uint64_t gen = p->gen0 + (uint64_t)g;
    GaBreedArgs b{p->islands, p->pop, n, ctx->inst.N, p->pmut, (uint32_t)p->seed,
                  (uint32_t)(p->seed >> 32), gen, src_t, src_k,
                  static_cast<uint16_t*>(child), static_cast<uint32_t*>(child)};
    breed<<<(unsigned)((members + 3) / 4), 256, lds_b, s>>>(b);
    VRPMS_HIP(hipGetLastError());
    if (words) {
      WordsArgs w{f, static_cast<const uint32_t*>(child), members, n, ckeys, nullptr, nullptr,
                  nullptr, members, 1u};
      int rc = launch_words2(ctx, w, words2_ring(n), s);
      if (rc) return rc;
    } else {
      int rc = vrpms_eval(ctx, child, 2, members, n, n, ckeys, nullptr, nullptr, nullptr, stream);
      if (rc) return rc;
    }
    GaSelectArgs sa{p->islands, p->pop, n, src_t, src_k, static_cast<const uint16_t*>(child),
                    static_cast<const uint32_t*>(child), ckeys, dst_t, dst_k};
    select<<<p->islands, 1024, lds_s, s>>>(sa);
    VRPMS_HIP(hipGetLastError());
    std::swap(src_t, dst_t);
    std::swap(src_k, dst_k);
  }
  if (src_t != d_pop) {
    VRPMS_HIP(hipMemcpyAsync(d_pop, src_t, tour_bytes, hipMemcpyDeviceToDevice, s));
    VRPMS_HIP(hipMemcpyAsync(d_keys, src_k, (size_t)members * 8, hipMemcpyDeviceToDevice, s));
  }
  return VRPMS_OK;
}

extern "C" int vrpms_aco_init(vrpms_ctx* ctx, int32_t colonies, uint32_t tau0, uint32_t* d_tau,
                              uint32_t* d_eta, void* stream);

extern "C" int vrpms_aco_iteration(vrpms_ctx* ctx, const vrpms_aco_params* p, uint32_t* d_tau,
                                   const uint32_t* d_eta, uint16_t* d_tours, uint64_t* d_keys,
                                   uint64_t* d_iter_best, uint16_t* d_best_tours,
                                   uint64_t* d_best_keys, int32_t n, void* stream) {
  if (!ctx || !p) return fail(VRPMS_EINVAL, "vrpms_aco_iteration: NULL ctx/params");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_aco_iteration: no instance loaded");
  const Instance& in = ctx->inst;
  if (p->colonies <= 0 || p->ants <= 0 || n != in.N - 1)
    return fail(VRPMS_EINVAL, "vrpms_aco_iteration: need colonies, ants > 0 and n == N-1");
  if (!d_tau || !d_eta || !d_tours || !d_keys || !d_iter_best)
    return fail(VRPMS_EINVAL, "vrpms_aco_iteration: NULL buffer");
  if (p->tau_max > (1u << 31) || p->tau_min > p->tau_max)
    return fail(VRPMS_EINVAL, "vrpms_aco_iteration: need tau_min <= tau_max <= 2^31");
  if (p->evap_shift < 1 || p->evap_shift > 31)
    return fail(VRPMS_EINVAL, "vrpms_aco_iteration: evap_shift must be in [1, 31]");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t ants = (int64_t)p->colonies * p->ants;
  FastSplit f;
  const bool words = n <= 255 && fast_split_params(ctx, n, &f);
  uint32_t* wbuf = nullptr;
  if (words) {
    int err = VRPMS_OK;
    ensure_scratch(ctx, (size_t)((n + 3) / 4) * ants * 4, &err);
    if (err) return err;
    wbuf = static_cast<uint32_t*>(ctx->search_scratch);
  }
  AcoArgs c{p->colonies, p->ants, n, in.N, (uint32_t)p->seed, (uint32_t)(p->seed >> 32), p->iter,
            d_tau, d_eta, d_tours, wbuf};
  const size_t lds = ((4 * (((size_t)in.N + 31) / 32) * 4 + 15) & ~(size_t)15) + (words ? 4 * 256 : 0);
  const dim3 grid((unsigned)((ants + 3) / 4));
  // LDS-staged weights (one workgroup = up to 16 ants of one colony) when the
  // colony's N x N uint64 weights fit; VRPMS_OPT_ACO_CONSTRUCT 2 forces the L2 path
  const int wpg = std::min(16, p->ants);
  const bool staged = ctx->opt_aco_construct != 2 && in.N <= 256 &&
                      aco_lds_bytes(in.N, wpg) <= ctx->max_lds;
  auto construct = [&](auto wtag) {
    constexpr bool WD = decltype(wtag)::value;
    if (staged) {
      const size_t l2 = aco_lds_bytes(in.N, wpg);
      const dim3 g2((unsigned)(p->colonies * ((p->ants + wpg - 1) / wpg)));
      auto go = [&](auto kern) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2);
        kern<<<g2, 64 * wpg, l2, s>>>(c, wpg);
      };
      if (in.N <= 64) go(aco_construct_lds_kernel<WD, 1>);
      else if (in.N <= 128) go(aco_construct_lds_kernel<WD, 2>);
      else go(aco_construct_lds_kernel<WD, 4>);
      return;
    }
    if (in.N <= 64) aco_construct_kernel<WD, 1><<<grid, 256, lds, s>>>(c);
    else if (in.N <= 128) aco_construct_kernel<WD, 2><<<grid, 256, lds, s>>>(c);
    else if (in.N <= 256) aco_construct_kernel<WD, 4><<<grid, 256, lds, s>>>(c);
    else aco_construct_kernel<WD, 0><<<grid, 256, lds, s>>>(c);
  };
  if (words) construct(std::true_type{});
  else construct(std::false_type{});
  VRPMS_HIP(hipGetLastError());
  if (words) {
    WordsArgs w{f, wbuf, ants, n, d_keys, nullptr, nullptr, nullptr, ants, 1u};
    int rc = launch_words2(ctx, w, words2_ring(n), s);
    if (rc) return rc;
  } else {
    int rc = vrpms_eval(ctx, d_tours, 2, ants, n, n, d_keys, nullptr, nullptr, nullptr, stream);
    if (rc) return rc;
  }
  const int bsf = p->bsf_period > 0 && (p->iter + 1) % p->bsf_period == 0 ? 1 : 0;
  AcoUpdateArgs u{p->colonies, p->ants, n, in.N, (uint32_t)p->evap_shift, p->tau_min, p->tau_max,
                  d_tau, d_tours, d_iter_best, bsf};
  if (in.N <= 256) {
    aco_update_fused_kernel<<<p->colonies, 1024, 0, s>>>(
        u, d_keys, d_iter_best, d_best_keys ? d_best_tours : nullptr, d_best_tours ? d_best_keys : nullptr);
    VRPMS_HIP(hipGetLastError());
    return VRPMS_OK;
  }
  segment_argmin_kernel<<<p->colonies, 256, 0, s>>>(d_keys, p->ants, p->colonies, d_iter_best);
  if (d_best_tours && d_best_keys)
    aco_track_best_kernel<<<p->colonies, 128, 0, s>>>(d_tours, p->ants, n, d_iter_best,
                                                      d_best_tours, d_best_keys);
  const int64_t total = (int64_t)p->colonies * in.N * in.N;
  aco_evaporate_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, ctx->num_cus * 8), 256, 0,
                         s>>>(u);
  aco_deposit_kernel<<<p->colonies, 256, 0, s>>>(u, d_best_keys ? d_best_tours : nullptr,
                                                 d_best_tours ? d_best_keys : nullptr);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

__global__ void aco_init_kernel(const int32_t* __restrict__ D, int N, int colonies, uint32_t tau0,
                                uint32_t* tau, uint32_t* eta) {
  const int64_t NN = (int64_t)N * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)colonies * NN;
       i += (int64_t)gridDim.x * blockDim.x) {
    tau[i] = tau0;
    if (i < NN) {
      const uint64_t d1 = 1ull + (uint64_t)(uint32_t)D[i];  // static slice (hour 0)
      eta[i] = (uint32_t)((1ull << 24) / (d1 * d1));
    }
  }
}

extern "C" int vrpms_aco_init(vrpms_ctx* ctx, int32_t colonies, uint32_t tau0, uint32_t* d_tau,
                              uint32_t* d_eta, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_aco_init: ctx is NULL");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_aco_init: no instance loaded");
  if (colonies <= 0 || !d_tau || !d_eta) return fail(VRPMS_EINVAL, "vrpms_aco_init: bad args");
  VRPMS_HIP(hipSetDevice(ctx->device));
  const Instance& in = ctx->inst;
  const int64_t total = (int64_t)colonies * in.N * in.N;
  aco_init_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, ctx->num_cus * 8), 256, 0,
                    (hipStream_t)stream>>>(in.mat32, in.N, colonies, tau0, d_tau, d_eta);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

extern "C" int vrpms_bf_run(vrpms_ctx* ctx, int32_t n, uint64_t rank_begin, uint64_t rank_end,
                            uint64_t* d_out, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_bf_run: ctx is NULL");
  if (!ctx->has_instance) return fail(VRPMS_ESTATE, "vrpms_bf_run: no instance loaded");
  if (n < 1 || n > 15 || n > ctx->inst.N - 1)
    return fail(VRPMS_EINVAL, "vrpms_bf_run: brute force needs 1 <= n <= min(15, N-1)");
  if (!d_out || rank_end < rank_begin) return fail(VRPMS_EINVAL, "vrpms_bf_run: bad range/out");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  VRPMS_HIP(hipMemsetAsync(d_out, 0xff, 16, s));
  const uint64_t count = rank_end - rank_begin;
  if (count == 0) return VRPMS_OK;
  const uint64_t threads_max = (uint64_t)ctx->num_cus * 8 * 256;
  uint64_t chunk = std::max<uint64_t>(64, (count + threads_max - 1) / threads_max);
  const uint64_t threads = (count + chunk - 1) / chunk;
  const int blocks = (int)((threads + 255) / 256);
  int err = VRPMS_OK;
  ensure_scratch(ctx, (size_t)blocks * 16, &err);
  if (err) return err;
  BfArgs a{search_inst(ctx), n, rank_begin, rank_end, chunk,
           static_cast<uint64_t*>(ctx->search_scratch)};
  size_t lds = inst_lds_bytes_host(a.si);
  if (lds > ctx->max_lds) {
    a.si.mat_lds = 0;
    lds = inst_lds_bytes_host(a.si);
  }
  int rc = launch_inst<BfK>(ctx, dim3(blocks), dim3(256), lds, s, a);
  if (rc) return rc;
  reduce_pairs_kernel<<<1, 1024, 0, s>>>(static_cast<uint64_t*>(ctx->search_scratch), blocks,
                                         d_out);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

extern "C" int vrpms_tsp_batch_sa(vrpms_ctx* ctx, const int32_t* d_mats, int32_t R, int32_t N,
                                  const vrpms_sa_params* p, uint16_t* d_best_tours,
                                  uint64_t* d_best_keys, void* stream) {
  if (!ctx || !p) return fail(VRPMS_EINVAL, "vrpms_tsp_batch_sa: NULL ctx/params");
  if (R < 0 || N < 2 || p->steps < 0) return fail(VRPMS_EINVAL, "vrpms_tsp_batch_sa: bad shape");
  if (R == 0) return VRPMS_OK;
  if (!d_mats || !d_best_tours || !d_best_keys)
    return fail(VRPMS_EINVAL, "vrpms_tsp_batch_sa: NULL buffer");
  const size_t npad = ((size_t)N - 1 + 2 + 7) & ~(size_t)7;   // tours padded with the depot
  // matrix, 4 chains x (current / next / best tour), their best keys, their edge caches E
  const size_t lds = (((size_t)N * N * 4 + 15) & ~(size_t)15) + 4 * 3 * npad * 2 + 4 * 8 +
                     4 * (npad + 8) * 4;
  if (lds > ctx->max_lds) return fail(VRPMS_EINVAL, "vrpms_tsp_batch_sa: request too large for LDS");
  VRPMS_HIP(hipSetDevice(ctx->device));
  TspBatchArgs a{d_mats, R, N, p->steps, p->inv_t0, p->inv_alpha, (uint32_t)p->seed,
                 (uint32_t)(p->seed >> 32), d_best_tours, d_best_keys};
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(tsp_batch_sa_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  tsp_batch_sa_kernel<<<R, 256, lds, (hipStream_t)stream>>>(a);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

#ifdef VRPMS_ROUTE_DUMP
extern "C" int vrpms_debug_route_dump(int* out, int count) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vrpms::g_route_dump), sizeof(int) * count) ==
                 hipSuccess ? 0 : -2;
}
#endif

#ifdef VRPMS_ROUTE_PROF
extern "C" int vrpms_debug_route_prof(unsigned long long* out, int count, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vrpms::g_route_prof),
                          sizeof(unsigned long long) * count) != hipSuccess)
    return -2;
  if (reset) {
    static unsigned long long zero[12 * 8192];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(vrpms::g_route_prof), zero, sizeof(zero));
  }
  return 0;
}
#endif
