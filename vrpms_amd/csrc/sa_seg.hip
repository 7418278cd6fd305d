// Segment-priced SA (the SA endpoints api/{vrp}/sa/index.py:40-45 on large
// static instances; model: oracle/route_model.py SegTables / price_seg, host
// restatement: oracle/oracle_c.c seg_key).
//
// Same chain, moves, Philox streams and acceptance as sa_kernel /
// sa_route_kernel, so the trajectories are the same bit for bit; what
// changes is how a sampled move is priced.  On a fleet of one capacity
// (start times do not enter a static route's duration), a static symmetric
// matrix and demands that each fit an empty vehicle, the greedy split with
// unlimited vehicles is the concatenation, over the separator-delimited
// segments of the giant tour, of each segment's own split from an empty
// vehicle.  A route's duration is then a sum of consecutive edges of the
// tour (an A10 separator standing for the depot), so with prefix sums over
// the positions (edges PE, demands PD, separators SC) every run of the moved
// tour that reads the current tour contiguously -- forward, or reversed on
// the symmetric matrix -- is priced in O(1); a capacity cut inside a run is
// a binary search on PD; whole segments between a piece's separators come
// from per-route tables (prefix sums, prefix / suffix maxima, a sparse
// table).  The fleet limit is one count: R routes (empty segments included)
// and T separators after the last customer serve everyone iff R - T <= K.
// A move's only matrix gathers are its <= 4 junction edges (L2), issued
// together; everything else is LDS.  Pricing does not walk the tour, so a
// step costs the same whatever the move's span (the route-local kernel's
// step is set by the longest walk of its 64 lanes).
//
// A moved tour that leaves a customer unserved gets the largest key when
// the current tour serves everyone and 2^28 invT makes accepting it
// impossible (the same rule as sa_route_kernel), else it is re-evaluated in
// full.  An accepted move rebuilds the tables in parallel (one pass of DPP
// scans over the positions, one lane per segment, per-route scans).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "ctx.hpp"
#include "staging.hpp"
#include "tour.hpp"

namespace vrpms {

constexpr int kSegRegs = 20;      // positions per lane in registers on an accept: n < 64 * 20
constexpr int kSegMaxMoves = 8;   // moves per lane per step (64 M per step)
#ifndef VRPMS_SEG_SHIFT
#define VRPMS_SEG_SHIFT 8  // (A/B builds may set another)
#endif
constexpr int kSegShift = VRPMS_SEG_SHIFT;  // heterogeneous fleets: shifts |delta| <= 8 from tables

struct SegArgs {
  SearchInst si;
  int chains, n, steps, window;
  uint32_t window_types;
  float inv_t0, inv_alpha;
  uint32_t seed_lo, seed_hi;
  uint64_t step0;
  uint16_t* cur;
  uint64_t* cur_key;
  uint16_t* best;
  uint64_t* best_key;
  int M;        // moves per lane per step
  int cpw;      // chains (wavefronts) per workgroup
  int segs;     // separator slots per chain
  int rm, lv;   // route slots, sparse-table levels
  uint32_t chain_bytes;
  int W;        // wavefronts per chain (W > 1: one chain per workgroup, cpw = 1)
};

// The cross-wavefront exchange of a multi-wavefront chain: each wavefront's
// best (key, move index) with what applying it needs, two buffers by step
// parity, then the table scalars wavefront 0 publishes after a rebuild.
struct SegXSlot {
  uint64_t key;
  uint32_t idx, w, typ;
  int32_t i, j;
  uint32_t jx[4];
  uint32_t pad;
};
constexpr int kSegMaxWaves = 4;
constexpr uint32_t kSegXBytes = 2 * kSegMaxWaves * sizeof(SegXSlot) + 32;

// per-chain LDS: u32 [PE n+2 | PD n+2 | LG n+2 | dur rm+1 | dsp, pmx, smx rm+1
// each | sparse (lv-1) x rm | (het) need, allow rm+1 each], then u16 [tok n+2 |
// SC n+2 | SP, RB, FNE, LNE1 segs+2 | RS rm+1 | (het) NB 2 kSegShift x (rm+1) |
// SEGR rm+1 | cend K]
__host__ __device__ inline uint32_t seg_chain_bytes(int n, int segs, int rm, int lv, bool het, int K) {
  const uint32_t np2 = ((uint32_t)n + 2u + 1u) & ~1u;
  const uint32_t u32s = 3u * np2 + 4u * (uint32_t)(rm + 1) + (uint32_t)(lv - 1) * (uint32_t)rm +
                        (het ? 2u * (uint32_t)(rm + 1) : 0u);
  const uint32_t u16s = 2u * np2 + 4u * (uint32_t)(segs + 2) + (uint32_t)(rm + 1) +
                        (het ? (2u * kSegShift + 1u) * (uint32_t)(rm + 1) + (uint32_t)K : 0u);
  return ((4u * u32s + 2u * u16s + 15u) & ~15u) + kSegXBytes;
}

__host__ __device__ inline int seg_levels(int rm) {
  int lv = 1;
  while ((2 << (lv - 1)) <= rm) ++lv;
  return lv;
}

// Wave64 inclusive scans in VALU (every lane active): Hillis-Steele inside
// each 16-lane row by DPP row_shr 1, 2, 4, 8 (a lane shifted in from outside
// the row reads 0), then the row totals (v_readlane) folded into the rows
// above.  MAX needs values >= 0 (0 is its identity).  `total` = the wave's.
template <bool MAX>
VRPMS_DEV uint32_t dpp_scan(uint32_t v, uint32_t& total) {
  auto op = [](uint32_t x, uint32_t y) { return MAX ? (x > y ? x : y) : x + y; };
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));
  const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
  const uint32_t s1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
  const uint32_t s2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
  const uint32_t s3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  const int row = lane_id() >> 4;
  uint32_t add = 0;
  add = row >= 1 ? op(add, s0) : add;
  add = row >= 2 ? op(add, s1) : add;
  add = row >= 3 ? op(add, s2) : add;
  total = op(op(s0, s1), op(s2, s3));
  return op(v, add);
}

// Suffix max (over this lane and the lanes above it), values >= 0: DPP
// row_shl 1, 2, 4, 8, then the row heads of the rows above.
VRPMS_DEV uint32_t dpp_rscan_max(uint32_t v, uint32_t& total) {
  auto mx = [](uint32_t x, uint32_t y) { return x > y ? x : y; };
  v = mx(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, true));
  v = mx(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x102, 0xF, 0xF, true));
  v = mx(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, true));
  v = mx(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x108, 0xF, 0xF, true));
  const uint32_t h1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t h2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t h3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  const uint32_t h0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const int row = lane_id() >> 4;
  uint32_t add = 0;
  add = row <= 2 ? mx(add, h3) : add;
  add = row <= 1 ? mx(add, h2) : add;
  add = row <= 0 ? mx(add, h1) : add;
  total = mx(mx(h0, h1), mx(h2, h3));
  return mx(v, add);
}

struct SegTabs {
  uint32_t *PE, *PD, *LG, *dur, *dsp, *pmx, *smx, *sp;  // LG[q] = leg of the token at q
  uint16_t *tok, *SC, *SP, *RB, *FNE, *LNE1;
  uint16_t* RS;  // RS[r] = the first position of route r
  // heterogeneous fleets: per route its load (need) and the largest capacity
  // that splits it the same (allow); NB[d][r] = the first route >= r that
  // would split differently on vehicle r + delta(d) (R: none), delta =
  // -kSegShift..-1, 1..kSegShift; SEGR[r] = the segment of route r; cend[v] =
  // the last vehicle of v's run of equal capacities (0xffff: the run reaches
  // K - 1)
  uint32_t *need, *allow;
  uint16_t *NB, *SEGR, *cend;
};

#ifdef VRPMS_SEG_PROF
// per-chain counters (A/B builds only: tools/seg_prof.py): pricing ticks,
// rebuild ticks, steps, accepts, cross-wavefront exchange ticks, setup ticks,
// kernel ticks, rebuilds, then the rebuild's parts: positions, segments,
// routes, sparse table, then the pricing's (each closed by a wait for every
// outstanding load, so only roughly the kernel's own schedule): draw and
// junction tokens, round 1, round 2, round 3, composition, full
// re-evaluation (wall_clock64, 100 MHz)
constexpr int kSegProf = 22;  // + cut iterations (wave max, lane sum), search steps (wave max), dead lanes
__device__ unsigned long long g_seg_prof[kSegProf * 8192];
#endif

// HET: per-vehicle capacities.  OCC: wavefronts per SIMD the register budget
// allows -- 1 (the compiler's choice, ~270 registers) or 2 (capped at 256,
// a little spill): a launch with more wavefronts than SIMDs takes OCC = 2,
// whose second wavefront hides the first's dependent latency (X-1000, 1024
// chains x W = 2: 33-38 k steps/s per chain against 17-22 k at OCC = 1)
template <typename MatT, bool HET, int OCC>
__global__ __launch_bounds__(64 * kSegMaxWaves, OCC) void sa_seg_kernel(SegArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#ifdef VRPMS_SEG_PROF
  const unsigned long long pk0 = wall_clock64();
#endif
  // instance: demand / capacities / start times in LDS (matrix in L2), then
  // the depot legs leg[c] = D(0, c) = D(c, 0) (symmetric matrix)
  const StagedInst<MatT, 1> I = stage_inst<MatT, 1>(a.si, smem);
  const uint32_t N = (uint32_t)a.si.N;
  const MatT* M0 = static_cast<const MatT*>(a.si.mat);
  uint32_t* leg = reinterpret_cast<uint32_t*>(smem + inst_lds_bytes(a.si));
  for (uint32_t c = threadIdx.x; c < N; c += blockDim.x) leg[c] = (uint32_t)M0[c];
  __syncthreads();
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  // W = 1: cpw chains per workgroup, one wavefront each.  W > 1: one chain
  // per workgroup; its W wavefronts price 64 W M moves per step (move index
  // lane + 64 (cw + W mi)), the (key, index) minimum meets in LDS, and
  // wavefront 0 applies an accepted move and rebuilds the tables.
  const int W = a.W;
  const int cw = W > 1 ? wave : 0;
  const int slot = W > 1 ? 0 : wave;
  const int chain = W > 1 ? (int)blockIdx.x : (int)blockIdx.x * a.cpw + wave;
  if (chain >= a.chains) return;  // (W = 1) no block-wide barrier after this point
  const int n = a.n, K = a.si.K, RM = a.rm, LV = a.lv, SEGS = a.segs;
  const uint32_t cap = (uint32_t)I.sp.cap[0];
  // route r runs on vehicle r (the last vehicle's capacity past the fleet:
  // routes there serve no one, the fleet count rejects them)
  auto capv = [&](int v) __attribute__((always_inline)) -> uint32_t {
    return HET ? (uint32_t)I.sp.cap[v < 0 ? 0 : (v < K ? v : K - 1)] : cap;
  };
  const int32_t* dem = I.sp.dem;
  const uint32_t Nm1 = N - 1;
  SegTabs T;
  {
    const uint32_t np2 = ((uint32_t)n + 2u + 1u) & ~1u;
    uint32_t* u = reinterpret_cast<uint32_t*>(smem + inst_lds_bytes(a.si) + ((N * 4u + 15u) & ~15u) +
                                              (uint32_t)slot * a.chain_bytes);
    T.PE = u;
    T.PD = u + np2;
    T.LG = u + 2 * np2;
    T.dur = u + 3 * np2;
    T.dsp = T.dur + (RM + 1);
    T.pmx = T.dsp + (RM + 1);
    T.smx = T.pmx + (RM + 1);
    T.sp = T.smx + (RM + 1);
    uint16_t* h = reinterpret_cast<uint16_t*>(T.sp + (LV - 1) * RM);
    T.tok = h;
    T.SC = h + np2;
    T.SP = T.SC + np2;
    T.RB = T.SP + (SEGS + 2);
    T.FNE = T.RB + (SEGS + 2);
    T.LNE1 = T.FNE + (SEGS + 2);
    T.RS = T.LNE1 + (SEGS + 2);
    T.need = T.allow = nullptr;
    T.NB = T.SEGR = T.cend = nullptr;
    if (HET) {
      T.need = T.sp + (LV - 1) * RM;
      T.allow = T.need + (RM + 1);
      h = reinterpret_cast<uint16_t*>(T.allow + (RM + 1));
      T.tok = h;
      T.SC = h + np2;
      T.SP = T.SC + np2;
      T.RB = T.SP + (SEGS + 2);
      T.FNE = T.RB + (SEGS + 2);
      T.LNE1 = T.FNE + (SEGS + 2);
      T.RS = T.LNE1 + (SEGS + 2);
      T.NB = T.RS + (RM + 1);
      T.SEGR = T.NB + 2 * kSegShift * (RM + 1);
      T.cend = T.SEGR + (RM + 1);
      // cend[v] = the first u >= v whose successor's capacity differs: a
      // suffix maximum of 0xffff - u over those u, 64 vehicles at a time
      uint32_t carry = 0;
      for (int top = ((K - 1) / 64) * 64; top >= 0; top -= 64) {
        const int v = top + lane;
        const uint32_t x =
            (v < K - 1 && I.sp.cap[v + 1] != I.sp.cap[v]) ? 0xffffu - (uint32_t)v : 0u;
        uint32_t tm;
        const uint32_t m = max(dpp_rscan_max(x, tm), carry);
        if (v < K) T.cend[v] = (uint16_t)(m ? 0xffffu - m : 0xffffu);
        carry = max(carry, tm);
      }
    }
  }
  // vehicles v0..v1 share one capacity (v1 < v0: none)
  auto one_class = [&](int v0, int v1) __attribute__((always_inline)) -> bool {
    return v1 < v0 || (int)T.cend[v0 < K ? v0 : K - 1] >= v1;
  };
  // the NB row of shift d (0 < |d| <= kSegShift)
  auto nb_row = [&](int d) __attribute__((always_inline)) -> const uint16_t* {
    return T.NB + (d < 0 ? d + kSegShift : d + kSegShift - 1) * (RM + 1);
  };
  // routes r0..r1-1 split the same on vehicles r + d, |d| <= kSegShift (d = 0: yes)
  auto keeps = [&](int r0, int r1, int d) __attribute__((always_inline)) -> bool {
    if (d == 0 || r0 >= r1) return true;
    if (d < -kSegShift || d > kSegShift) return false;
    return (int)nb_row(d)[r0] >= r1;
  };
  SegXSlot* xs = reinterpret_cast<SegXSlot*>(smem + inst_lds_bytes(a.si) + ((N * 4u + 15u) & ~15u) +
                                             (uint32_t)slot * a.chain_bytes + a.chain_bytes -
                                             kSegXBytes);
  int32_t* xr = reinterpret_cast<int32_t*>(xs + 2 * kSegMaxWaves);  // S, R, Tt, seg_ok, ck lo/hi
  auto d0 = [&](uint32_t x, uint32_t y) __attribute__((always_inline)) -> uint32_t {
    if ((x | y) == 0u) return 0u;  // two depots: an empty route lasts 0
    if (x == 0u) return leg[y];
    if (y == 0u) return leg[x];
    return (uint32_t)M0[__umul24(x, N) + y];
  };
  int S = 0, R = 0, Tt = 0;
  bool seg_ok = false;  // the tables hold the tour (else: full re-evaluation of every move)
  auto SPX = [&](int k) __attribute__((always_inline)) -> int {
    return k < 0 ? -1 : (k >= S ? n : (int)T.SP[k]);
  };
  auto SPv = [&](int l) __attribute__((always_inline)) { return l ? T.sp + (l - 1) * RM : T.dur; };
  auto tourA = [&](int q) __attribute__((always_inline)) { return (uint32_t)T.tok[q]; };

  // ---- tables from the tokens in T.tok and the edges in T.PE[q + 1] -------
  // Positions qa..qb hold new tokens / raw edges; the prefix sums before qa
  // are current, and after qb every PE entry is off by the same amount
  // (pe_old = PE[qb + 1] before the edges qa..qb were rewritten): a move
  // permutes the tokens of its span in place, so the demand and separator
  // prefixes after it are unchanged and the edge prefix shifts by the
  // change of its junction edges.  The first build passes 0, n.
#ifdef VRPMS_SEG_PROF
  unsigned long long pf[kSegProf] = {};
  unsigned long long pmark = 0;
#define SEG_PT(k)                            \
  do {                                       \
    __builtin_amdgcn_s_waitcnt(0);           \
    const unsigned long long nw = wall_clock64(); \
    pf[k] += nw - pmark;                     \
    pmark = nw;                              \
  } while (0)
#else
#define SEG_PT(k) \
  do {            \
  } while (0)
#endif
  int reb_a = 0, reb_b = n;
  bool rb_valid = false;  // T.RB holds a previous split (the heterogeneous pass starts from it)
  bool tab_ok = false;    // the segment / route tables describe the tour before this rebuild
  uint32_t pe_old = 0;
  auto rebuild = [&]() __attribute__((always_inline)) {
    wave_sync();
#ifdef VRPMS_SEG_PROF
    pmark = wall_clock64();
#endif
    // positions: PE (edges) and PD (demands) prefix sums in one 64-bit DPP
    // scan, the separator count SC in a 32-bit one, separator positions SP
    const int qa = reb_a, qb = reb_b;
    uint64_t carry = ((uint64_t)T.PD[qa] << 32) | T.PE[qa];
    uint32_t scarry = qa ? (uint32_t)T.SC[qa] : 0u;
    if (qa == 0) carry = 0;
#pragma unroll 1
    for (int base = qa; base <= qb; base += 64) {
      const int q = base + lane;
      const bool in = q < n && q <= qb;
      const uint32_t c = in ? (uint32_t)T.tok[q] : 1u;
      uint64_t v = q <= qb ? ((uint64_t)(in && c ? (uint32_t)dem[c] : 0u) << 32) | T.PE[q + 1] : 0ull;
      const uint64_t tot = wave_scan_add_u64(v);
      uint32_t stot;
      const uint32_t sv = dpp_scan<false>(in && c == 0u ? 1u : 0u, stot);
      if (q <= qb) {
        T.PE[q + 1] = (uint32_t)(carry + v);
        T.PD[q + 1] = (uint32_t)((carry + v) >> 32);
      }
      if (in) {
        T.LG[q] = c ? leg[c] : 0u;
        T.SC[q + 1] = (uint16_t)(scarry + sv);
        if (c == 0u && scarry + sv <= (uint32_t)SEGS) T.SP[scarry + sv - 1] = (uint16_t)q;
      }
      carry += tot;
      scarry += stot;
    }
    if (qb < n) {  // the edge prefix after the span moves by its junctions' change
      const uint32_t dpe = (uint32_t)carry - pe_old;
      if (dpe != 0u)
#pragma unroll 4
        for (int q = qb + 1 + lane; q <= n; q += 64) T.PE[q + 1] += dpe;
    } else {
      S = (int)scarry;
    }
    if (lane == 0) {
      T.PE[0] = 0u;
      T.PD[0] = 0u;
      T.SC[0] = 0;
    }
    wave_sync();
    SEG_PT(8);
    seg_ok = S <= SEGS;
    if (!seg_ok) {
      tab_ok = false;
      return;
    }
    // segments, one lane each: how many routes the greedy split makes of it
    // (binary-searched capacity cuts), the first route RB, the nearest
    // non-empty segments at or before (LNE1, +1) / at or after (FNE).  A
    // heterogeneous fleet splits a segment on the vehicles from RB on, which
    // depend on the segments before it: the pass repeats from the previous
    // RB until no first route moves (a segment's count is then taken on its
    // own vehicles), or else one lane walks the segments in order.
    auto seg_routes = [&](int g, int vb) __attribute__((always_inline)) -> uint32_t {
      const int s0 = SPX(g - 1) + 1, s1 = SPX(g) - 1;
      uint32_t cnt = 1;
      int x = s0, v = vb;
      while (x <= s1 && T.PD[s1 + 1] - T.PD[x] > capv(v)) {  // cut: last q fitting from x
        const uint32_t thr = T.PD[x] + capv(v);
        int l = x, h = s1;  // first q in [x, s1] with PD[q + 1] > thr (exists)
        while (l < h) {
          const int md = (l + h) >> 1;
          if (T.PD[md + 1] > thr) h = md; else l = md + 1;
        }
        ++cnt;
        ++v;
        x = l;
      }
      return cnt;
    };
    // Incremental split (one capacity; round 6).  A move permutes the tokens
    // of positions qa..qb and nothing else, so every segment outside
    // SC[qa] .. SC[qb + 1] keeps its tokens, its demand-prefix differences
    // and its edges: its cuts, its route count and its routes' durations.
    // Only those segments are split again (one lane each); the routes after
    // them move by the change of route count (dur / RS shifted, RB bumped).
    // The prefix scans below (FNE, LNE1, dsp, pmx, smx, sparse table) still
    // run over everything: they search nothing.  Falls back to the full pass
    // when the span touches 64 segments or more, or the tables were not valid.
    int g_lo = 0, g_hi = S;  // the segments whose routes are (re)written below
    bool inc = false;
    bool empties_kept = false;  // (incremental) no segment became empty or non-empty
    if (!HET && tab_ok && !(qa == 0 && qb >= n)) {
      const int ga = (int)T.SC[qa];
      const int gb = qb < n ? min((int)T.SC[qb + 1], S) : S;
      const int r0 = T.RB[ga], r1o = T.RB[gb + 1], Rold = R;
      if (gb - ga < 64 && Rold - r1o <= 4 * 64) {
        const int g = ga + lane;
        const uint32_t cnt = g <= gb ? seg_routes(g, 0) : 0u;
        uint32_t tc;
        const uint32_t incl = dpp_scan<false>(cnt, tc);
        const int dR = (int)tc - (r1o - r0);
        if (Rold + dR <= RM) {
          inc = true;
          if (dR != 0) {  // routes r1o .. Rold - 1 move to r1o + dR ..
            uint32_t vd[4], vr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = r1o + lane + 64 * i;
              vd[i] = r < Rold ? T.dur[r] : 0u;
              vr[i] = r < Rold ? (uint32_t)T.RS[r] : 0u;
            }
            wave_sync();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = r1o + lane + 64 * i;
              if (r < Rold) {
                T.dur[r + dR] = vd[i];
                T.RS[r + dR] = (uint16_t)vr[i];
              }
            }
            for (int x = gb + 1 + lane; x <= S + 1; x += 64) T.RB[x] = (uint16_t)((int)T.RB[x] + dR);
          }
          if (g <= gb) T.RB[g] = (uint16_t)(r0 + (int)(incl - cnt));
          R = Rold + dR;
          g_lo = ga;
          g_hi = gb;
          // LNE1 / FNE (the nearest non-empty segments) change only when one
          // of the re-split segments became empty or non-empty: LNE1[g] == g
          // + 1 says segment g was non-empty before the move
          const bool flip = g <= gb && (T.LNE1[g] == (uint16_t)(g + 1)) !=
                                           (SPX(g) - 1 >= SPX(g - 1) + 1);
          empties_kept = __ballot(flip) == 0ull;
          // LNE1 (the last non-empty segment at or before g, + 1): a prefix
          // maximum over the segments, as the full pass forms it
          uint32_t lcarry = 0;
#pragma unroll 1
          for (int base = 0; !empties_kept && base <= S; base += 64) {
            const int gg = base + lane;
            const bool ne = gg <= S && SPX(gg) - 1 >= SPX(gg - 1) + 1;
            uint32_t tl;
            const uint32_t lne = dpp_scan<true>(ne ? (uint32_t)gg + 1u : 0u, tl);
            if (gg <= S) T.LNE1[gg] = (uint16_t)max(lcarry, lne);
            lcarry = max(lcarry, tl);
          }
          wave_sync();
        }
      }
    }
    uint32_t rcarry = 0;
    bool moved = true;
#pragma unroll 1
    for (int it = 0; !inc && moved && it < (HET ? 6 : 1); ++it) {
      rcarry = 0;
      uint32_t lcarry = 0;
      moved = false;
#pragma unroll 1
      for (int base = 0; base <= S; base += 64) {
        const int g = base + lane;
        uint32_t cnt = 0, ne = 0, guess = 0;
        if (g <= S) {
          const int s0 = SPX(g - 1) + 1, s1 = SPX(g) - 1;
          ne = s1 >= s0 ? 1u : 0u;
          guess = HET ? (!rb_valid && it == 0 ? (uint32_t)g : (uint32_t)T.RB[g]) : 0u;
          cnt = seg_routes(g, (int)guess);
        }
        uint32_t tc, tl;
        const uint32_t inc = dpp_scan<false>(cnt, tc);
        const uint32_t lne = dpp_scan<true>(ne ? (uint32_t)g + 1u : 0u, tl);
        const uint32_t rb = rcarry + inc - cnt;
        if (HET && __ballot(g <= S && rb != guess) != 0ull) moved = true;
        if (g <= S) {
          T.RB[g] = (uint16_t)rb;
          T.LNE1[g] = (uint16_t)max(lcarry, lne);
        }
        rcarry += tc;
        lcarry = max(lcarry, tl);
      }
      wave_sync();
    }
    if (HET && moved) {  // not settled: one lane, segment by segment
      if (lane == 0) {
        uint32_t v = 0;
        for (int g = 0; g <= S; ++g) {
          T.RB[g] = (uint16_t)v;
          v += seg_routes(g, (int)v);
        }
      }
      wave_sync();
      rcarry = (uint32_t)T.RB[S] + seg_routes(S, (int)T.RB[S]);
    }
    if (!inc) R = (int)rcarry;
    seg_ok = R <= RM;
    if (!seg_ok) {
      tab_ok = false;
      return;
    }
    uint32_t fcarry = 0;  // FNE[g] = S + 1 - (suffix max of S + 1 - g over non-empty g)
#pragma unroll 1
    for (int top = (S / 64) * 64; !empties_kept && top >= 0; top -= 64) {
      const int g = top + lane;
      uint32_t f = 0;
      if (g <= S) {
        const int s0 = SPX(g - 1) + 1, s1 = SPX(g) - 1;
        f = s1 >= s0 ? (uint32_t)(S + 1 - g) : 0u;
      }
      uint32_t tf;
      f = max(dpp_rscan_max(f, tf), fcarry);
      if (g <= S) T.FNE[g] = (uint16_t)(S + 1 - (int)f);
      fcarry = max(fcarry, tf);
    }
    if (lane == 0) T.RB[S + 1] = (uint16_t)R;
    wave_sync();
    SEG_PT(9);
    // route durations (heterogeneous: loads and allowances), one lane per
    // segment (incremental: the re-split segments only)
#pragma unroll 1
    for (int g = g_lo + lane; g <= g_hi; g += 64) {
      const int s0 = SPX(g - 1) + 1, s1 = SPX(g) - 1;
      int r = T.RB[g], x = s0;
      T.RS[r] = (uint16_t)s0;
      while (x <= s1 && T.PD[s1 + 1] - T.PD[x] > capv(r)) {
        const uint32_t thr = T.PD[x] + capv(r);
        int l = x, h = s1;
        while (l < h) {
          const int md = (l + h) >> 1;
          if (T.PD[md + 1] > thr) h = md; else l = md + 1;
        }
        if (HET) {  // cut before A[l]: this vehicle takes up to load + dem(A[l]) - 1
          T.need[r] = T.PD[l] - T.PD[x];
          T.allow[r] = T.PD[l + 1] - T.PD[x] - 1u;
          T.SEGR[r] = (uint16_t)g;
        }
        // route: depot -> A[x..l-1] -> depot
        T.dur[r++] = leg[T.tok[x]] + T.PE[l] - T.PE[x + 1] + leg[T.tok[l - 1]];
        x = l;
        T.RS[r] = (uint16_t)l;
      }
      // the last (or only) route: A[x..s1], closed by the separator (or the end)
      if (HET) {
        T.need[r] = x <= s1 ? T.PD[s1 + 1] - T.PD[x] : 0u;
        T.allow[r] = 0xffffffffu;
        T.SEGR[r] = (uint16_t)g;
      }
      T.dur[r] = x <= s1 ? leg[T.tok[x]] + T.PE[s1 + 2] - T.PE[x + 1] : T.PE[s1 + 2] - T.PE[x];
    }
    wave_sync();
    if (HET) {  // NB[d]: the next route that would split differently 1..kSegShift vehicles on / back
      // one pass over the routes (top down): each lane reads its route's
      // load and allowance once and scans the 2 kSegShift shifts from
      // registers (a suffix maximum of 0xffff - r over the routes that fail)
      uint32_t carry[2 * kSegShift];
#pragma unroll
      for (int d = 0; d < 2 * kSegShift; ++d) carry[d] = 0u;
#pragma unroll 1
      for (int top = (R / 64) * 64; top >= 0; top -= 64) {
        const int r = top + lane;
        const bool in = r < R;
        const uint32_t need = in ? T.need[r] : 0u, allow = in ? T.allow[r] : 0u;
#pragma unroll
        for (int d = 0; d < 2 * kSegShift; ++d) {
          const int dl = d < kSegShift ? d - kSegShift : d - kSegShift + 1;
          uint32_t v = 0;
          if (in) {
            const uint32_t c = capv(r + dl);
            v = (r + dl < 0 || need > c || c > allow) ? 0xffffu - (uint32_t)r : 0u;
          }
          uint32_t tm;
          const uint32_t m = max(dpp_rscan_max(v, tm), carry[d]);
          if (r <= R) T.NB[d * (RM + 1) + r] = (uint16_t)(m ? 0xffffu - m : (uint32_t)R);
          carry[d] = max(carry[d], tm);
        }
      }
      wave_sync();
    }
    // per-route prefix sums / maxima (dsp / pmx [r] over routes < r), suffix
    // maxima (smx [r] over routes >= r), sparse table of maxima
    uint32_t cds = 0, cmx = 0;
#pragma unroll 1
    for (int base = 0; base < R; base += 64) {
      const int r = base + lane;
      const uint32_t d = r < R ? T.dur[r] : 0u;
      uint32_t ts, tm;
      const uint32_t ids = dpp_scan<false>(d, ts), imx = dpp_scan<true>(d, tm);
      if (r < R) {
        T.dsp[r + 1] = cds + ids;
        T.pmx[r + 1] = max(cmx, imx);
      }
      cds += ts;
      cmx = max(cmx, tm);
    }
    uint32_t smx = 0;
#pragma unroll 1
    for (int top = (R / 64) * 64; top >= 0; top -= 64) {
      const int r = top + lane;
      uint32_t tm;
      const uint32_t sm = max(dpp_rscan_max(r < R ? T.dur[r] : 0u, tm), smx);
      if (r <= R) T.smx[r] = sm;
      smx = max(smx, tm);
    }
    if (lane == 0) {
      T.dsp[0] = 0u;
      T.pmx[0] = 0u;
    }
    wave_sync();
    SEG_PT(10);
#pragma unroll 1
    for (int l = 1; l < LV; ++l) {
      const int w = 1 << (l - 1);
      const uint32_t* src = SPv(l - 1);
      uint32_t* dst = SPv(l);
      for (int r = lane; r + 2 * w <= R; r += 64) dst[r] = max(src[r], src[r + w]);
      wave_sync();
    }
    SEG_PT(11);
    rb_valid = true;
    tab_ok = true;
    const int l1 = T.LNE1[S];
    Tt = l1 ? S - (l1 - 1) : S;
  };
  auto rmaxq = [&](int r0, int r1) __attribute__((always_inline)) -> uint32_t {  // routes r0..r1
    if (r0 > r1) return 0u;
    const int l = 31 - __builtin_clz((uint32_t)(r1 - r0 + 1));
    const uint32_t* t = SPv(l);
    return max(t[r0], t[r1 - (1 << l) + 1]);
  };

  // ---- the current tour: tokens and edges into LDS ----------------------------
  if (cw == 0) {
    const uint16_t* gcur = a.cur + (int64_t)chain * n;
    for (int q = lane; q <= n; q += 64) {
      const uint32_t c = q < n ? min((uint32_t)gcur[q], Nm1) : 0u;
      const uint32_t p = q >= 1 ? min((uint32_t)gcur[q - 1], Nm1) : 0u;
      if (q < n) T.tok[q] = (uint16_t)c;
      T.PE[q + 1] = d0(p, c);
    }
  }
  uint16_t* gbest = a.best + (int64_t)chain * n;
  uint64_t bk = a.best_key[chain];
  uint64_t ck = 0;
  bool need_build = true, first = true;
  float invT = a.inv_t0;
#pragma unroll 1
  for (int st = 0;; ++st) {
    if (need_build) {
#ifdef VRPMS_SEG_PROF
      const unsigned long long pb0 = wall_clock64();
#endif
      if (cw == 0) {
        rebuild();
        if (first) {  // the start tour's key: from the tables when it serves everyone
          if (seg_ok && R - Tt <= K) ck = cvrp_key(0, T.dsp[R], T.smx[0], I.sp.objective);
          else ck = eval_tour<true>(I.D, I.sp, tourA, n).key;
        }
        if (W > 1 && lane == 0) {
          xr[0] = S;
          xr[1] = R;
          xr[2] = Tt;
          xr[3] = seg_ok ? 1 : 0;
          xr[4] = (int32_t)(uint32_t)ck;
          xr[5] = (int32_t)(uint32_t)(ck >> 32);
        }
      }
      if (W > 1) {  // wavefront 0's tables and scalars
        __syncthreads();
        S = xr[0];
        R = xr[1];
        Tt = xr[2];
        seg_ok = xr[3] != 0;
        ck = ((uint64_t)(uint32_t)xr[5] << 32) | (uint32_t)xr[4];
      }
      first = false;
      need_build = false;
#ifdef VRPMS_SEG_PROF
      pf[1] += wall_clock64() - pb0;
      pf[7] += 1;
      if (st == 0) pf[5] = wall_clock64() - pk0;
#endif
      if (ck < bk) {
        bk = ck;
        if (cw == 0)
          for (int q = lane; q < n; q += 64) gbest[q] = T.tok[q];
      }
    }
    if (st >= a.steps || n < 2) break;
#ifdef VRPMS_SEG_PROF
    const unsigned long long pt0 = wall_clock64();
#endif
    const uint64_t step = a.step0 + (uint64_t)st;
    // an unserved customer cannot be accepted from a tour serving everyone
    // when 2^28 * invT puts the acceptance threshold at 0 (sa_route_kernel)
    const bool shortcut = (ck >> 56) == 0 && invT >= 0x1p-20f;
    uint64_t bkey = ~0ull;
    uint32_t bidx = 0xffffffffu, bw = 0;
#ifdef VRPMS_SEG_PROF
    int p_cut = 0, p_bs = 0, p_dead = 0;
#endif
    Move bmv{0, 0, 0};
    uint32_t bj0 = 0, bj1 = 0, bj2 = 0, bj3 = 0;
#pragma unroll 1
    for (int mi = 0; mi < a.M; ++mi) {
      const uint32_t idx = (uint32_t)(lane + 64 * (cw + W * mi));
#ifdef VRPMS_SEG_PROF
      pmark = wall_clock64();
#endif
      const u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)chain, idx,
                             a.seed_lo, a.seed_hi);
      const Move m = decode_move_window(r.x, r.y, r.z, n, a.window, a.window_types);
      const MoveMap mmap = move_map(m);
      auto B = [&](int p) __attribute__((always_inline)) -> uint32_t {  // moved tour, 0 outside
        return (uint32_t)p < (uint32_t)n ? tourA(map_src(mmap, p)) : 0u;
      };
      const int lo = min(m.i, m.j), hi = max(m.i, m.j);
      // the junction edges of the moved tour at positions lo, lo + 1, hi, hi + 1
      const uint32_t b0 = B(lo - 1), b1 = B(lo), b2 = B(lo + 1), b3 = B(hi - 1), b4 = B(hi),
                     b5 = B(hi + 1);
      const uint32_t jx0 = d0(b0, b1), jx1 = d0(b1, b2), jx2 = d0(b3, b4), jx3 = d0(b4, b5);
      uint64_t k = ~0ull;
      bool full = !seg_ok;
      if (seg_ok) {
        // The table reads a move needs are issued in three dependent rounds
        // (separator counts at the pieces' ends; separator positions and
        // route indices; prefix sums / legs at the runs' ends and route
        // table entries), then the pieces are composed in registers.  Only a
        // run that overflows the open route (a binary-searched capacity cut)
        // or a reversed multi-route segment reads the tables again.
        const bool opt = m.typ == kMove2Opt, swp = m.typ == kMoveSwap, fwd = m.i < m.j;
        // The moved span as pieces of the current tour (moved_index,
        // tour.hpp) in three slots -- 2-opt [A[i..j] reversed] | swap [A[j]]
        // [A[i+1..j-1]] [A[i]] | relocate i<j [A[i+1..j]] [A[i]] | relocate
        // i>j [A[i]] [A[j..i-1]] -- then the rest of the last changed segment
        // A[hi+1 .. en] and its closing separator.  Every lane runs the same
        // predicated steps per slot, so the wave's control flow stays
        // uniform: the part before the piece's first separator (in the moved
        // order) joins the open route, the separator closes it, whole
        // segments between its separators come from the route tables, the
        // part after its last separator opens the next route.
        int X[3], Y[3];
        uint32_t JV[3];
        X[0] = opt ? m.i : swp ? m.j : fwd ? m.i + 1 : m.i;
        Y[0] = opt ? m.j : swp ? m.j : fwd ? m.j : m.i;
        JV[0] = jx0;
        X[1] = opt ? 1 : swp ? m.i + 1 : fwd ? m.i : m.j;
        Y[1] = opt ? 0 : swp ? m.j - 1 : fwd ? m.i : m.i - 1;
        JV[1] = fwd && !swp ? jx2 : jx1;
        X[2] = swp ? m.i : 1;
        Y[2] = swp ? m.i : 0;
        JV[2] = jx2;
        SEG_PT(12);
        // round 1: separator counts
        const int s0 = T.SC[lo], sH = T.SC[hi + 1];
        const int lneS = T.LNE1[S];
        const uint32_t dspR = T.dsp[R];
        int SA[3], SB[3];
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool live = X[s] <= Y[s];
          SA[s] = live ? (int)T.SC[X[s]] : 0;
          SB[s] = live ? (int)T.SC[Y[s] + 1] : 0;
        }
        SEG_PT(13);
        // round 2: separator positions, route indices
        const int stp = SPX(s0 - 1) + 1, en = SPX(sH);
        const int ra = T.RB[s0], rz = T.RB[sH + 1];  // sH = the last changed segment
        const int ra1 = T.RB[s0 + 1];                // routes ra .. ra1 - 1 hold segment s0
        int SMIN[3], SMAX[3], R0[3], R1[3], GF[3], RG0[3], RG1[3];
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool hs = SA[s] != SB[s], rev = opt && s == 0;
          SMIN[s] = hs ? (int)T.SP[SA[s]] : 0;
          SMAX[s] = hs ? (int)T.SP[SB[s] - 1] : 0;
          // segments g0 = SA + 1 .. g1 = SB - 1 lie between the piece's
          // separators (SC[SP[k]] = k)
          const bool mid = SB[s] - SA[s] >= 2;
          R0[s] = mid ? (int)T.RB[SA[s] + 1] : 0;
          R1[s] = mid ? (int)T.RB[SB[s]] : 0;
          // (forward) the segment after the piece's last separator: its routes
          RG0[s] = hs && !rev ? (int)T.RB[SB[s]] : 0;
          RG1[s] = hs && !rev ? (int)T.RB[SB[s] + 1] : 0;
          GF[s] = mid ? (rev ? (int)T.FNE[SA[s] + 1] : (int)T.LNE1[SB[s] - 1] - 1) : 0;
        }
        SEG_PT(14);
        // round 3: the runs' prefix sums and legs, the route tables
        struct RunP {
          int x, y;
          uint32_t pdx, pdy, pex, pey, lgx, lgy;
        };
        auto pre = [&](int x, int y) __attribute__((always_inline)) -> RunP {
          RunP p{x, y, 0u, 0u, 0u, 0u, 0u, 0u};
          if (x <= y) {
            p.pdx = T.PD[x];
            p.pdy = T.PD[y + 1];
            p.pex = T.PE[x + 1];
            p.pey = T.PE[y + 1];
            p.lgx = T.LG[x];
            p.lgy = T.LG[y];
          }
          return p;
        };
        const RunP p_start = pre(stp, lo - 1);
        const RunP p_tail = pre(hi + 1, (en < n ? en : n) - 1);
        RunP PA[3], PDn[3];
        uint32_t ISUM[3], IMAX[3];
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool live = X[s] <= Y[s], hs = SA[s] != SB[s], rev = opt && s == 0;
          const int x = X[s], y = Y[s], smin = SMIN[s], smax = SMAX[s];
          PA[s] = pre(!hs ? x : rev ? smax + 1 : x, !hs ? (live ? y : x - 1) : rev ? y : smin - 1);
          PDn[s] = pre(hs ? (rev ? x : smax + 1) : 1, hs ? (rev ? smin - 1 : y) : 0);
          ISUM[s] = 0u;
          IMAX[s] = 0u;
          if (R1[s] > R0[s]) {
            ISUM[s] = T.dsp[R1[s]] - T.dsp[R0[s]];
            IMAX[s] = rmaxq(R0[s], R1[s] - 1);
          }
        }
        const uint32_t dspa = T.dsp[ra], dspz = T.dsp[rz], pmxa = T.pmx[ra], smxz = T.smx[rz];
        // Cut budget (one capacity, the tail after the last changed segment
        // keeps its customers, the unserved shortcut on): the moved tour has
        // S + 1 + cuts routes (a cut = a route closed by a customer that did
        // not fit) and Tt trailing separators, so it serves everyone iff its
        // cuts <= K - 1 - S + Tt.  Segments outside s0..sH keep their splits
        // (their cuts: (ra - s0) + (R - rz) - (S - sH)); once the composed
        // segments' cuts exceed what is left the move's key is the largest
        // (exactly what the fleet count below would give), so an overflowing
        // run stops there instead of binary-searching its cuts.
        const bool tail_kept = en < n && lneS - 1 > sH;
        const int bud = (!HET && shortcut && tail_kept)
                            ? (K - 1 - S + Tt) - ((ra - s0) + (R - rz) - (S - sH))
                            : 0x7fffffff;

        SEG_PT(15);
        // the open route and what the composition has closed
        uint32_t c_dur = 0, c_load = 0, c_pl = 0, c_sum = 0, c_max = 0;  // c_pl: leg of its last customer
        bool c_has = false;
        int c_cnt = 0;
        uint32_t isum = 0, imax = 0;
        int icnt = 0, seps = 0, cutc = 0;
        bool cust = false;
        // dead: the cuts exceeded the budget.  An int, not a bool: with two
        // bools, SimplifyCFG merged run()'s "c_has = true; return" and "dead =
        // true; return" into one store through a phi of their addresses, which
        // kept both in scratch memory (a scratch load on every run() call's
        // critical path); stores of different types are never merged
        int dead = 0;
        int vo = ra;  // (heterogeneous) the open route's vehicle
        auto close = [&]() __attribute__((always_inline)) {
          const uint32_t d = c_dur + c_pl;
          c_sum += d;
          c_max = max(c_max, d);
          ++c_cnt;
          ++vo;
          c_dur = c_load = c_pl = 0u;
          c_has = false;
        };
        // customers A[x..y] joined to the open route in the moved order (rev:
        // A[y] first), cut where the greedy split's next customer does not
        // fit; jv = the junction edge into the first one when the open route
        // holds a customer
        auto run = [&](const RunP& p, bool rev, uint32_t jv) __attribute__((always_inline)) {
          int x = p.x, y = p.y;
          if (x > y || dead) return;
          seps = 0;
          cust = true;
          if (p.pdy - p.pdx <= capv(vo) - c_load) {  // fits: from the round-3 values
            c_dur += (c_has ? jv : (rev ? p.lgy : p.lgx)) + p.pey - p.pex;
            c_load += p.pdy - p.pdx;
            c_pl = rev ? p.lgx : p.lgy;
            c_has = true;
            return;
          }
          // the prefix demands at the run's ends ride along: PD[x] / PD[y + 1]
          // are known from round 3 and, after a cut, from the appended part
          uint32_t pdx = p.pdx, pdy = p.pdy;
          while (true) {
            const uint32_t room = capv(vo) - c_load;
            const bool fits = pdy - pdx <= room;
            int pa = x, pb = y;
            if (!fits) {
              if (cutc >= bud) {  // one cut more than the fleet allows: no search
                dead = 1;
#ifdef VRPMS_SEG_PROF
                ++p_dead;
#endif
                return;
              }
              ++cutc;
#ifdef VRPMS_SEG_PROF
              ++p_cut;
#endif
              // first q in [x - 1, y + 1] with PD[q + 1] > thr, on the monotone
              // PD (one customer: it does not fit, q = x)
              const int thr = rev ? (int)(pdy - room) - 1 : (int)(pdx + room);
              int l = x, h = x;
              if (x < y) {
                l = x - 1;
                h = y + 1;
              }
              while (l < h) {
                const int md = (l + h) >> 1;
                if ((int)T.PD[md + 1] > thr) h = md; else l = md + 1;
#ifdef VRPMS_SEG_PROF
                ++p_bs;
#endif
              }
              if (rev) pa = l + 1; else pb = l - 1;
            }
            uint32_t pda = pdx, pdb = pdy;  // PD[pa], PD[pb + 1]
            if (pa <= pb) {
              if (!fits) {
                pda = rev ? T.PD[pa] : pdx;
                pdb = rev ? pdy : T.PD[pb + 1];
              }
              c_dur += (c_has ? jv : T.LG[rev ? pb : pa]) + T.PE[pb + 1] - T.PE[pa + 1];
              c_load += pdb - pda;
              c_pl = T.LG[rev ? pa : pb];
              c_has = true;
            }
            if (fits) break;
            close();
            // (nothing appended: x / y stay, and so do their prefix demands)
            if (rev) {
              y = pa - 1;
              if (pa <= pb) pdy = pda;  // PD[y + 1] = PD[pa]
            } else {
              x = pb + 1;
              if (pa <= pb) pdx = pdb;  // PD[x] = PD[pb + 1]
            }
          }
        };
        // A fresh vehicle at the start of segment g (routes g_r0 .. g_r1 - 1)
        // taking its customers up to y in the current order, on the current
        // vehicles: the current tour's split.  Its routes before the one
        // holding y are closed from the tables, that route's part up to y is
        // the open route -- no capacity cut is searched.  (Segments of one
        // route go through run(): their prefix never cuts.)
        auto aligned = [&](const RunP& p, int g_r0, int g_r1) __attribute__((always_inline)) {
          if (p.x > p.y || dead) return;
          seps = 0;
          cust = true;
          int l = g_r0, h = g_r1 - 1;  // the last route starting at or before y
          while (l < h) {
            const int md = (l + h + 1) >> 1;
            if ((int)T.RS[md] <= p.y) l = md; else h = md - 1;
          }
          if (l > g_r0) {
            c_sum += T.dsp[l] - T.dsp[g_r0];
            c_max = max(c_max, rmaxq(g_r0, l - 1));
            c_cnt += l - g_r0;
            vo += l - g_r0;
            cutc += l - g_r0;  // each route after a segment's first is a cut
          }
          const int xs = T.RS[l];
          c_dur = T.LG[xs] + p.pey - T.PE[xs + 1];
          c_load = p.pdy - T.PD[xs];
          c_pl = p.lgy;
          c_has = true;
        };
        // (heterogeneous) routes r..rend-1 of the current tour, the first on
        // vehicle vo: every route keeps its split on vehicle r + delta (delta =
        // vo - r) up to the first that does not (NB), whose segment is walked
        // on its new vehicles, delta then moving by its change of route count;
        // tabled routes add to (xs, xm, xc), walked ones close into the open
        // route's totals.  false: a shift beyond the tables (re-evaluate)
        auto shifted = [&](int r, int rend, uint32_t& xs, uint32_t& xm, int& xc)
                           __attribute__((always_inline)) -> bool {
          while (r < rend) {
            const int d = vo - r;
            if (d < -kSegShift || d > kSegShift) return false;
            const int l = d ? min((int)nb_row(d)[r], rend) : rend;
            const int gl = l < rend ? (int)T.SEGR[l] : 0;
            const int rs = l < rend ? (int)T.RB[gl] : rend;
            if (rs > r) {
              xs += T.dsp[rs] - T.dsp[r];
              xm = max(xm, rmaxq(r, rs - 1));
              xc += rs - r;
              vo += rs - r;
            }
            if (l >= rend) break;
            run(pre(SPX(gl - 1) + 1, SPX(gl) - 1), false, 0u);
            close();
            r = T.RB[gl + 1];
          }
          return true;
        };
        // the start of the first changed segment, up to lo: the current split
        // (the heterogeneous variant keeps round 3's run(): with the table
        // path its composition measured ~2 us slower per step, and
        // tools/het_rate.py 9.6 k -> 9.8 k steps/s without it)
        if (!HET && ra1 - ra > 1) aligned(p_start, ra, ra1);
        else run(p_start, false, 0u);
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool hs = SA[s] != SB[s], rev = opt && s == 0;
          // (A) up to the first separator in the moved order
          run(PA[s], rev, JV[s]);
          if (hs) {
            // (B) the separator closes the open route
            close();
            ++seps;
            // (C) whole segments between the piece's separators
            if (SB[s] - SA[s] >= 2) {
              const int g0 = SA[s] + 1, g1 = SB[s] - 1;
              const int r0 = R0[s], r1 = R1[s];
              // a reversal splits a segment of several routes differently;
              // (heterogeneous) forward they keep their splits when every
              // route does on the vehicles it moves to, reversed (which hands
              // them to the vehicles in reverse) when one capacity serves them
              // before and after
              bool tabled = !rev || r1 - r0 == g1 - g0 + 1, split = false;
              if (HET && tabled) {
                if (rev)
                  tabled = one_class(r0, r1 - 1) && one_class(vo, vo + r1 - r0 - 1) &&
                           capv(vo) == capv(r0);
                else if (!keeps(r0, r1, vo - r0))
                  split = true;  // forward: tables up to each route that fails, its segment walked
              }
              if (!tabled) {  // walk them
                for (int t = 0; t <= g1 - g0; ++t) {
                  const int g = rev ? g1 - t : g0 + t;
                  run(pre(SPX(g - 1) + 1, SPX(g) - 1), rev, 0u);
                  close();
                  ++seps;
                }
              } else {
                if (split) {
                  const int seps0 = seps;
                  const bool cust0 = cust;
                  if (!shifted(r0, r1, isum, imax, icnt)) full = true;
                  seps = seps0;
                  cust = cust0;
                } else {
                  isum += ISUM[s];
                  imax = max(imax, IMAX[s]);
                  icnt += r1 - r0;
                  vo += r1 - r0;
                }
                // the last customer in the moved order and the separators after it
                const int gf = GF[s];
                const bool has = rev ? gf <= g1 : gf >= g0;
                if (has) {
                  seps = rev ? gf - g0 + 1 : g1 + 1 - gf;
                  cust = true;
                } else {
                  seps += g1 - g0 + 1;
                }
              }
            }
          }
          // (D) the part after the last separator opens the next route: read
          // forward, the current split of that segment's start (on the same
          // vehicles)
          if (!HET && hs && !rev && RG1[s] - RG0[s] > 1) aligned(PDn[s], RG0[s], RG1[s]);
          else run(PDn[s], rev, 0u);
        }
        // the rest of the last changed segment, closed by its separator (or
        // the tour's end)
        run(p_tail, false, jx3);
        close();
        if (en < n) ++seps;
        // the unchanged tail: routes rz.. of the current tour.  A
        // heterogeneous fleet hands them to vehicles shifted by delta: routes
        // that keep their splits there come from the tables, the segment of
        // the first that does not is walked on its new vehicles, and delta
        // moves by that segment's change of route count
        uint32_t tsum = dspR - dspz, tmax = smxz;
        int tcnt = R - rz;
        if (HET) {
          tsum = tmax = 0u;
          tcnt = 0;
          const int seps0 = seps;
          const bool cust0 = cust;
          if (!shifted(rz, R, tsum, tmax, tcnt)) full = true;
          seps = seps0;
          cust = cust0;
        }
        const int Rb = ra + c_cnt + icnt + tcnt;
        int Tb = Tt;
        if (!tail_kept && cust) Tb = seps + (en < n ? n - 1 - en : 0);
        if (full) {
          // (heterogeneous) the tail moved by more than kSegShift vehicles
        } else if (dead) {
          k = ~0ull;  // over the cut budget: serves fewer (shortcut on)
        } else if (Rb - Tb <= K) {
          const uint32_t dsum = dspa + c_sum + isum + tsum;
          const uint32_t dmax = max(max(pmxa, tmax), max(imax, c_max));
          k = cvrp_key(0, dsum, dmax, I.sp.objective);
        } else if (shortcut) {
          k = ~0ull;
        } else {
          full = true;
        }
      }
      SEG_PT(16);
      if (full) {
        auto moved = [&](int q) { return tourA(map_src(mmap, q)); };
        k = eval_tour<true>(I.D, I.sp, moved, n).key;
      }
      SEG_PT(17);
      if (k < bkey) {  // ties keep the earlier (smaller) move index
        bkey = k;
        bidx = idx;
        bw = r.w;
        bmv = m;
        bj0 = jx0;
        bj1 = jx1;
        bj2 = jx2;
        bj3 = jx3;
      }
    }
    // the chain's (key, move index) minimum: over the lanes, then (W > 1)
    // over the wavefronts through LDS
    int wl;
    uint64_t k = wave_argmin_lane(bkey, wl);
    const uint32_t imin = wave_min_u32_uniform(bkey == k ? bidx : 0xffffffffu);
    const int bl = (int)(imin & 63u);
    uint32_t uw = (uint32_t)wave_bcast((int)bw, bl);
    Move mb;
    mb.typ = (uint32_t)wave_bcast((int)bmv.typ, bl);
    mb.i = wave_bcast(bmv.i, bl);
    mb.j = wave_bcast(bmv.j, bl);
    uint32_t w0 = (uint32_t)wave_bcast((int)bj0, bl), w1 = (uint32_t)wave_bcast((int)bj1, bl);
    uint32_t w2 = (uint32_t)wave_bcast((int)bj2, bl), w3 = (uint32_t)wave_bcast((int)bj3, bl);
#ifdef VRPMS_SEG_PROF
    const unsigned long long px0 = wall_clock64();
    pf[0] += px0 - pt0;
    {
      int mc = p_cut, sc = p_cut, mb = p_bs, sd = p_dead;
      for (int off = 32; off > 0; off >>= 1) {
        mc = max(mc, __shfl_xor(mc, off, 64));
        sc += __shfl_xor(sc, off, 64);
        mb = max(mb, __shfl_xor(mb, off, 64));
        sd += __shfl_xor(sd, off, 64);
      }
      pf[18] += (unsigned long long)mc;
      pf[19] += (unsigned long long)sc;
      pf[20] += (unsigned long long)mb;
      pf[21] += (unsigned long long)sd;
    }
#endif
    if (W > 1) {
      SegXSlot* xb = xs + (st & 1) * kSegMaxWaves;
      if (lane == 0) xb[cw] = SegXSlot{k, imin, uw, mb.typ, mb.i, mb.j, {w0, w1, w2, w3}, 0u};
      __syncthreads();
      SegXSlot b = xb[0];
      for (int v = 1; v < W; ++v) {
        const SegXSlot o = xb[v];
        if (o.key < b.key || (o.key == b.key && o.idx < b.idx)) b = o;
      }
      k = b.key;
      uw = b.w;
      mb.typ = b.typ;
      mb.i = b.i;
      mb.j = b.j;
      w0 = b.jx[0];
      w1 = b.jx[1];
      w2 = b.jx[2];
      w3 = b.jx[3];
    }
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      accept = (uw >> 8) < accept_threshold(dp, invT);
    }
#ifdef VRPMS_SEG_PROF
    pf[4] += wall_clock64() - px0;
    pf[2] += 1;
    pf[3] += accept ? 1 : 0;
#endif
    if (accept) {
      const int blo = min(mb.i, mb.j), bhi = max(mb.i, mb.j);
      // a move among separators only (e.g. two separators swapped) leaves the
      // tour as it is: no rebuild
      const bool same = (mb.typ == kMoveSwap && T.tok[blo] == T.tok[bhi]) ||
                        (mb.typ != kMoveSwap && T.SC[bhi + 1] - T.SC[blo] == bhi - blo + 1);
      ck = k;
      if (!same) {
        if (W > 1) __syncthreads();  // every wavefront is done reading the tables
        if (cw == 0) {
          const MoveMap mmb = move_map(mb);
          // the new tour's tokens (positions blo..bhi) and edges (into
          // positions blo..bhi + 1): a kept adjacency's edge is a difference
          // of PE (forward, or reversed on the symmetric matrix; PE is
          // complete even when the segment tables are not), the four
          // junctions are the winner's gathers
          const int hq = min(bhi + 1, n);
          reb_a = blo;
          reb_b = hq;
          pe_old = T.PE[hq + 1];
          uint32_t v_tok[kSegRegs], v_e[kSegRegs];
#pragma unroll
          for (int i = 0; i < kSegRegs; ++i) {
            if (blo + 64 * i > hq) break;
            const int q = blo + lane + 64 * i;
            v_tok[i] = 0u;
            v_e[i] = 0u;
            if (q > hq) continue;
            const int sq = map_src(mmb, q), sp = map_src(mmb, q - 1);
            if (q < n) v_tok[i] = T.tok[sq];
            if (q == blo) v_e[i] = w0;
            else if (q == blo + 1) v_e[i] = w1;
            else if (q == bhi) v_e[i] = w2;
            else if (q == bhi + 1) v_e[i] = w3;
            else if (sp + 1 == sq) v_e[i] = T.PE[sq + 1] - T.PE[sq];
            else v_e[i] = T.PE[sp + 1] - T.PE[sp];  // reversed: the edge between A[sq] and A[sp]
          }
          wave_sync();
#pragma unroll
          for (int i = 0; i < kSegRegs; ++i) {
            if (blo + 64 * i > hq) break;
            const int q = blo + lane + 64 * i;
            if (q > hq) continue;
            if (q < n) T.tok[q] = (uint16_t)v_tok[i];
            T.PE[q + 1] = v_e[i];
          }
        }
        need_build = true;
      } else if (ck < bk) {
        bk = ck;
        if (cw == 0)
          for (int q = lane; q < n; q += 64) gbest[q] = T.tok[q];
      }
    }
    invT = invT * a.inv_alpha;
  }
  if (cw != 0) return;
  uint16_t* gout = a.cur + (int64_t)chain * n;
  for (int q = lane; q < n; q += 64) gout[q] = T.tok[q];
  if (lane == 0) {
    a.cur_key[chain] = ck;
    a.best_key[chain] = bk;
#ifdef VRPMS_SEG_PROF
    pf[6] = wall_clock64() - pk0;
    if (chain < 8192)
      for (int i = 0; i < kSegProf; ++i) g_seg_prof[kSegProf * chain + i] += pf[i];
#endif
  }
}

// Host side: can the segment kernel run this SA call, and with what layout?
// Returns VRPMS_OK after launching, or 1 when it does not apply.
int launch_sa_seg(const vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur,
                  uint64_t* d_cur_key, uint16_t* d_best, uint64_t* d_best_key, int n,
                  uint32_t wtypes, int moves, hipStream_t s) {
  const Instance& in = ctx->inst;
  // every demand fits the smallest vehicle; per-vehicle capacities take the
  // heterogeneous variant
  if (in.problem != VRPMS_CVRP || in.H != 1 || !in.symmetric || in.max_dem > in.min_cap ||
      in.K > 65535 || n < 2 || n >= 64 * kSegRegs || n > 65535 || moves % 64 != 0 ||
      moves / 64 > kSegMaxMoves)
    return 1;
  // the prefix demands PD are u32 and the capacity cuts compare them (and
  // PD + a capacity) as int32: the total demand plus a capacity must stay
  // below 2^31, else the full re-evaluation kernels price the moves
  if ((int64_t)(in.N - 1) * (int64_t)in.max_dem + (int64_t)in.max_cap >= (int64_t)1 << 31) return 1;
  const bool het = !in.uniform_cap;
  SearchInst si = search_inst(ctx);
  si.mat_lds = 0;  // the matrix stays in L2: a move gathers <= 4 entries
  // separators: a tour of the N - 1 customers and n - (N - 1) separators
  const int segs = std::max(8, ((std::max(0, n - (in.N - 1)) + 2 + 7) & ~7));
  const int rm = std::max(2 * in.K + 2, segs + 2) + 8;
  if (rm > 65535) return 1;  // route indices are u16 in the tables
  const int lv = seg_levels(rm);
  const uint32_t cb = seg_chain_bytes(n, segs, rm, lv, het, in.K);
  const size_t base = inst_lds_bytes_host(si) + (((size_t)in.N * 4u + 15u) & ~(size_t)15u);
  // wavefronts per chain: W > 1 prices the step's moves on W SIMDs at once
  // (same moves, same winner, so the same trajectories as W = 1), while the
  // chains' wavefronts stay resident (two per SIMD with the OCC = 2 variant)
  // (round 5: at 1024 chains x 128 moves W = 1 wins while most moves are
  // accepted -- 30.3 k vs 23.2 k steps/s per chain from a hot start,
  // tools/seg_waves.py -- but loses over an annealing run, where pricing
  // dominates: 192 k vs 337 k steps per chain in 10 s, 84,475 vs 83,018,
  // tools/td_quality_scan.py --x1000; so W = 2 stays up to two wavefronts
  // per SIMD.  Staging the accept's span through LDS instead of the
  // registers below halved that annealing run -- 187 k vs 333 k steps per
  // chain, 84,421 vs 83,167 -- and was reverted.)
  int W = std::min(moves / 64, kSegMaxWaves);
  while (W > 1 && (int64_t)p->chains * W > 8 * (int64_t)ctx->num_cus) W >>= 1;
  if (ctx->opt_seg_waves > 0) W = std::min(ctx->opt_seg_waves, kSegMaxWaves);  // A/B
  while (W > 1 && (moves / 64) % W != 0) --W;
  int cpw = 4;
  // fewer chains than 4 per CU: spread them, one wavefront per workgroup
  if (p->chains < 4 * ctx->num_cus) cpw = p->chains < 2 * ctx->num_cus ? 1 : 2;
  if (W > 1) cpw = 1;
  while (cpw > 1 && base + (size_t)cpw * cb > ctx->max_lds) cpw >>= 1;
  const size_t lds = base + (size_t)cpw * cb;
  if (lds > ctx->max_lds) return 1;
  SegArgs a{si, p->chains, n, p->steps, p->window, wtypes, p->inv_t0, p->inv_alpha,
            (uint32_t)p->seed, (uint32_t)(p->seed >> 32), p->step0, d_cur, d_cur_key, d_best,
            d_best_key, moves / 64 / W, cpw, segs, rm, lv, cb, W};
  auto go = [&](auto kern) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<dim3((p->chains + cpw - 1) / cpw), dim3(64 * cpw * W), lds, s>>>(a);
  };
  // more wavefronts than SIMDs: the two-per-SIMD register budget
  const bool occ2 = (int64_t)p->chains * W > 4 * (int64_t)ctx->num_cus;
  if (het) {
    if (in.use16) occ2 ? go(sa_seg_kernel<uint16_t, true, 2>) : go(sa_seg_kernel<uint16_t, true, 1>);
    else occ2 ? go(sa_seg_kernel<int32_t, true, 2>) : go(sa_seg_kernel<int32_t, true, 1>);
  } else {
    if (in.use16) occ2 ? go(sa_seg_kernel<uint16_t, false, 2>) : go(sa_seg_kernel<uint16_t, false, 1>);
    else occ2 ? go(sa_seg_kernel<int32_t, false, 2>) : go(sa_seg_kernel<int32_t, false, 1>);
  }
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

}  // namespace vrpms

#ifdef VRPMS_SEG_PROF
extern "C" int vrpms_debug_seg_prof(unsigned long long* out, int count, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vrpms::g_seg_prof), sizeof(unsigned long long) * count) !=
      hipSuccess)
    return -2;
  if (reset) {
    static unsigned long long zero[vrpms::kSegProf * 8192];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(vrpms::g_seg_prof), zero, sizeof(zero));
  }
  return 0;
}
#undef SEG_PT
#endif
