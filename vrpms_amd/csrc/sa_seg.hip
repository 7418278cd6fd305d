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

constexpr int kSegRegs = 20;      // positions per lane in registers on a rebuild: n < 64 * 20
constexpr int kSegMaxMoves = 8;   // moves per lane per step (64 M per step)

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
};

// per-chain LDS: u32 [PE n+2 | PD n+2 | dur, dsp, pmx, smx rm+1 each | sparse
// (lv-1) x rm], then u16 [tok n+2 | SC n+2 | SP, RB, FNE, LNE1 segs+2 each]
__host__ __device__ inline uint32_t seg_chain_bytes(int n, int segs, int rm, int lv) {
  const uint32_t np2 = ((uint32_t)n + 2u + 1u) & ~1u;
  const uint32_t u32s = 2u * np2 + 4u * (uint32_t)(rm + 1) + (uint32_t)(lv - 1) * (uint32_t)rm;
  const uint32_t u16s = 2u * np2 + 4u * (uint32_t)(segs + 2);
  return (4u * u32s + 2u * u16s + 15u) & ~15u;
}

__host__ __device__ inline int seg_levels(int rm) {
  int lv = 1;
  while ((2 << (lv - 1)) <= rm) ++lv;
  return lv;
}

// Inclusive scans over the 64 lanes (shuffles): add, max, and min from the top lane down.
VRPMS_DEV uint32_t seg_scan_add(uint32_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, off, 64);
    if (lane >= off) v += o;
  }
  return v;
}
VRPMS_DEV int seg_scan_max(int v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(v, off, 64);
    if (lane >= off) v = max(v, o);
  }
  return v;
}
VRPMS_DEV int seg_rscan_min(int v) {  // min over lanes >= this one
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_down(v, off, 64);
    if (lane + off < 64) v = min(v, o);
  }
  return v;
}
VRPMS_DEV uint32_t seg_rscan_max(uint32_t v) {  // max over lanes >= this one
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = (uint32_t)__shfl_down((int)v, off, 64);
    if (lane + off < 64) v = max(v, o);
  }
  return v;
}

struct SegTabs {
  uint32_t *PE, *PD, *dur, *dsp, *pmx, *smx, *sp;
  uint16_t *tok, *SC, *SP, *RB, *FNE, *LNE1;
};

// The open route of a pricing walk and the routes it has closed.
struct SegAcc {
  uint32_t dur, load, prev;
  uint32_t rsum, rmax;
  int rcnt;
};

template <typename MatT>
__global__ __launch_bounds__(256) void sa_seg_kernel(SegArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // instance: demand / capacities / start times in LDS (matrix in L2), then
  // the depot legs leg[c] = D(0, c) = D(c, 0) (symmetric matrix)
  const StagedInst<MatT, 1> I = stage_inst<MatT, 1>(a.si, smem);
  const uint32_t N = (uint32_t)a.si.N;
  const MatT* M0 = static_cast<const MatT*>(a.si.mat);
  uint32_t* leg = reinterpret_cast<uint32_t*>(smem + inst_lds_bytes(a.si));
  for (uint32_t c = threadIdx.x; c < N; c += blockDim.x) leg[c] = (uint32_t)M0[c];
  __syncthreads();
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int chain = (int)blockIdx.x * a.cpw + wave;
  if (chain >= a.chains) return;  // no block-wide barrier after this point
  const int n = a.n, K = a.si.K, RM = a.rm, LV = a.lv, SEGS = a.segs;
  const uint32_t cap = (uint32_t)I.sp.cap[0];
  const int32_t* dem = I.sp.dem;
  const uint32_t Nm1 = N - 1;
  SegTabs T;
  {
    const uint32_t np2 = ((uint32_t)n + 2u + 1u) & ~1u;
    uint32_t* u = reinterpret_cast<uint32_t*>(smem + inst_lds_bytes(a.si) + ((N * 4u + 15u) & ~15u) +
                                              (uint32_t)wave * a.chain_bytes);
    T.PE = u;
    T.PD = u + np2;
    T.dur = u + 2 * np2;
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
  }
  auto d0 = [&](uint32_t x, uint32_t y) __attribute__((always_inline)) -> uint32_t {  // edge x -> y, 0 between two depots
    if ((x | y) == 0u) return 0u;
    if (x == 0u) return leg[y];
    if (y == 0u) return leg[x];
    return (uint32_t)M0[__umul24(x, N) + y];
  };
  auto SPX = [&](int k, int S) __attribute__((always_inline)) -> int { return k < 0 ? -1 : (k >= S ? n : (int)T.SP[k]); };
  auto SPv = [&](int l) __attribute__((always_inline)) { return l ? T.sp + (l - 1) * RM : T.dur; };

  // ---- tables of the current tour from its tokens and edges (registers:
  // position q = lane + 64 i; v_e[i] = edge into q, q <= n) -----------------
  int S = 0, R = 0, Tt = 0;
  bool seg_ok = true;  // the tables hold the tour (else: full re-evaluation of every move)
  uint32_t v_tok[kSegRegs], v_e[kSegRegs];  // the tour being (re)built, position lane + 64 i
  auto rebuild = [&]() __attribute__((always_inline)) {
    // positions: PE / PD prefix sums in one 64-bit DPP scan, SC in another
    uint64_t carry = 0, scarry = 0;
    wave_sync();
#pragma unroll
    for (int i = 0; i < kSegRegs; ++i) {
      if (64 * i > n) continue;  // wave-uniform; no break, so the loop unrolls
      const int q = lane + 64 * i;
      const bool in = q < n;
      const uint32_t c = in ? v_tok[i] : 1u;
      uint64_t v = q <= n ? ((uint64_t)(in && c ? (uint32_t)dem[c] : 0u) << 32) | v_e[i] : 0ull;
      uint64_t sv = (in && c == 0u) ? 1ull : 0ull;
      const uint64_t tot = wave_scan_add_u64(v);
      const uint64_t stot = wave_scan_add_u64(sv);
      if (q <= n) {
        T.PE[q + 1] = (uint32_t)(carry + v);
        T.PD[q + 1] = (uint32_t)((carry + v) >> 32);
      }
      if (in) {
        T.tok[q] = (uint16_t)c;
        T.SC[q + 1] = (uint16_t)(scarry + sv);
        if (c == 0u && scarry + sv <= (uint64_t)SEGS) T.SP[scarry + sv - 1] = (uint16_t)q;
      }
      carry += tot;
      scarry += stot;
    }
    if (lane == 0) {
      T.PE[0] = 0u;
      T.PD[0] = 0u;
      T.SC[0] = 0;
    }
    S = (int)scarry;
    wave_sync();
    if (S > SEGS) {
      seg_ok = false;
      return;
    }
    // segments: routes of each (one lane per segment), first route RB, the
    // nearest non-empty segments FNE / LNE1
    uint32_t rcarry = 0;
    int lcarry = 0;
    for (int base = 0; base <= S; base += 64) {
      const int g = base + lane;
      uint32_t cnt = 0;
      int ne = 0;
      if (g <= S) {
        const int s0 = SPX(g - 1, S) + 1, s1 = SPX(g, S) - 1;
        ne = s1 >= s0 ? 1 : 0;
        const uint32_t load = ne ? T.PD[s1 + 1] - T.PD[s0] : 0u;
        if (load <= cap) {
          cnt = 1;
        } else {  // greedy cuts, binary-searched on PD
          uint32_t ld = 0;
          int x = s0;
          cnt = 1;
          while (x <= s1) {
            const uint32_t room = cap - ld;
            if (T.PD[s1 + 1] - T.PD[x] <= room) break;
            int lo = x - 1, hi = s1;
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (T.PD[mid + 1] - T.PD[x] <= room) lo = mid; else hi = mid - 1;
            }
            ++cnt;
            ld = 0;
            x = lo + 1;
          }
        }
      }
      const uint32_t inc = seg_scan_add(cnt);
      const int lne = seg_scan_max(ne ? g + 1 : 0);
      if (g <= S) {
        T.RB[g] = (uint16_t)(rcarry + inc - cnt);
        T.LNE1[g] = (uint16_t)max(lcarry, lne);
      }
      rcarry += (uint32_t)__shfl((int)inc, 63, 64);
      lcarry = max(lcarry, __shfl(lne, 63, 64));
    }
    R = (int)rcarry;
    if (R > RM) {
      seg_ok = false;
      return;
    }
    int fcarry = S + 1;
    for (int top = ((S) / 64) * 64; top >= 0; top -= 64) {
      const int g = top + lane;
      int f = S + 1;
      if (g <= S) {
        const int s0 = SPX(g - 1, S) + 1, s1 = SPX(g, S) - 1;
        f = s1 >= s0 ? g : S + 1;
      }
      f = min(seg_rscan_min(f), fcarry);
      if (g <= S) T.FNE[g] = (uint16_t)f;
      fcarry = min(fcarry, __shfl(f, 0, 64));
    }
    if (lane == 0) T.RB[S + 1] = (uint16_t)R;
    wave_sync();
    // route durations: one lane per segment
    for (int g = lane; g <= S; g += 64) {
      const int s0 = SPX(g - 1, S) + 1, s1 = SPX(g, S) - 1;
      int r = T.RB[g];
      const uint32_t load = s1 >= s0 ? T.PD[s1 + 1] - T.PD[s0] : 0u;
      if (load <= cap) {
        T.dur[r] = T.PE[s1 + 2] - T.PE[s0];
      } else {
        uint32_t ld = 0, du = 0, prev = 0;
        int x = s0;
        while (x <= s1) {
          const uint32_t room = cap - ld;
          const uint32_t F = T.tok[x];
          const uint32_t ein = prev ? 0u : leg[F];  // a segment's routes start at the depot
          if (T.PD[s1 + 1] - T.PD[x] <= room) {
            du += ein + T.PE[s1 + 1] - T.PE[x + 1];
            prev = T.tok[s1];
            break;
          }
          int lo = x - 1, hi = s1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (T.PD[mid + 1] - T.PD[x] <= room) lo = mid; else hi = mid - 1;
          }
          du += ein + T.PE[lo + 1] - T.PE[x + 1];
          T.dur[r++] = du + leg[T.tok[lo]];
          du = ld = 0;
          prev = 0;
          x = lo + 1;
        }
        T.dur[r] = du + (prev ? leg[prev] : 0u);
      }
    }
    wave_sync();
    // per-route prefix sums / maxima, suffix maxima, sparse table
    uint32_t cds = 0, cmx = 0;
    for (int base = 0; base <= R; base += 64) {
      const int r = base + lane;
      const uint32_t d = r < R ? T.dur[r] : 0u;
      const uint32_t ids = seg_scan_add(d);
      const uint32_t imx = (uint32_t)seg_scan_max((int)d);  // durations < 2^31
      const uint32_t ex_mx = (uint32_t)__shfl_up((int)imx, 1, 64);
      if (r <= R) {
        T.dsp[r] = cds + ids - d;
        T.pmx[r] = max(cmx, lane ? ex_mx : 0u);
      }
      cds += (uint32_t)__shfl((int)ids, 63, 64);
      cmx = max(cmx, (uint32_t)__shfl((int)imx, 63, 64));
    }
    uint32_t smx = 0;
    for (int top = (R / 64) * 64; top >= 0; top -= 64) {
      const int r = top + lane;
      const uint32_t d = r < R ? T.dur[r] : 0u;
      const uint32_t s = max(seg_rscan_max(d), smx);
      if (r <= R) T.smx[r] = s;
      smx = max(smx, (uint32_t)__shfl((int)s, 0, 64));
    }
    wave_sync();
    for (int l = 1; l < LV; ++l) {
      const int w = 1 << (l - 1);
      const uint32_t* src = SPv(l - 1);
      uint32_t* dst = SPv(l);
      for (int r = lane; r + 2 * w <= R; r += 64) dst[r] = max(src[r], src[r + w]);
      wave_sync();
    }
    const int l1 = T.LNE1[S];
    Tt = l1 ? S - (l1 - 1) : S;
    seg_ok = true;
  };
  auto rmaxq = [&](int r0, int r1) __attribute__((always_inline)) -> uint32_t {  // max dur over routes r0..r1
    if (r0 > r1) return 0u;
    const int l = 31 - __builtin_clz((uint32_t)(r1 - r0 + 1));
    const uint32_t* t = SPv(l);
    return max(t[r0], t[r1 - (1 << l) + 1]);
  };

  // ---- the current tour ------------------------------------------------------
  {
    const uint16_t* gcur = a.cur + (int64_t)chain * n;
#pragma unroll
    for (int i = 0; i < kSegRegs; ++i) {
      const int q = lane + 64 * i;
      v_tok[i] = q < n ? min((uint32_t)gcur[q], Nm1) : 0u;
      const uint32_t p = q >= 1 && q - 1 < n ? min((uint32_t)gcur[q - 1], Nm1) : 0u;
      v_e[i] = q <= n ? d0(p, v_tok[i]) : 0u;
    }
    rebuild();
  }
  auto tourA = [&](int q) { return (uint32_t)T.tok[q]; };
  uint64_t ck;
  if (seg_ok && R - Tt <= K) {
    ck = cvrp_key(0, T.dsp[R], T.smx[0], I.sp.objective);
  } else {
    ck = eval_tour<true>(I.D, I.sp, tourA, n).key;
  }
  uint16_t* gbest = a.best + (int64_t)chain * n;
  uint64_t bk = a.best_key[chain];
  if (ck < bk) {
    bk = ck;
    for (int q = lane; q < n; q += 64) gbest[q] = T.tok[q];
  }

  float invT = a.inv_t0;
  for (int st = 0; st < a.steps && n >= 2; ++st) {
    const uint64_t step = a.step0 + (uint64_t)st;
    // an unserved customer cannot be accepted from a tour serving everyone
    // when 2^28 * invT puts the acceptance threshold at 0 (sa_route_kernel)
    const bool shortcut = (ck >> 56) == 0 && invT >= 0x1p-20f;
    uint64_t bkey = ~0ull;
    uint32_t bidx = 0xffffffffu, bw = 0;
    Move bmv{0, 0, 0};
    uint32_t bj[4] = {0, 0, 0, 0};
    for (int mm_ = 0; mm_ < a.M; ++mm_) {
      const uint32_t idx = (uint32_t)(lane + 64 * mm_);
      const u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)chain, idx,
                             a.seed_lo, a.seed_hi);
      const Move m = decode_move_window(r.x, r.y, r.z, n, a.window, a.window_types);
      const MoveMap mmap = move_map(m);
      auto B = [&](int p) -> uint32_t {  // token of the moved tour (0 outside the tour)
        return (uint32_t)p < (uint32_t)n ? tourA(map_src(mmap, p)) : 0u;
      };
      const int lo = min(m.i, m.j), hi = max(m.i, m.j);
      // junction edges of the moved tour at positions lo, lo + 1, hi, hi + 1
      const uint32_t b0 = B(lo - 1), b1 = B(lo), b2 = B(lo + 1), b3 = B(hi - 1), b4 = B(hi),
                     b5 = B(hi + 1);
      const uint32_t jx0 = d0(b0, b1), jx1 = d0(b1, b2), jx2 = d0(b3, b4), jx3 = d0(b4, b5);
      uint64_t k;
      if (seg_ok) {
        SegAcc c{0u, 0u, 0u, 0u, 0u, 0};
        uint32_t isum = 0, imax = 0;
        int icnt = 0, seps = 0;
        bool cust = false;
        auto close = [&]() __attribute__((always_inline)) {
          const uint32_t d = c.dur + (c.prev ? leg[c.prev] : 0u);
          c.rsum += d;
          c.rmax = max(c.rmax, d);
          ++c.rcnt;
          c.dur = c.load = c.prev = 0u;
        };
        // customers A[x..y] joined in the moved order (rev: A[y] first); jv =
        // the junction edge into the first one when the open route has a customer
        auto run = [&](int x, int y, bool rev, uint32_t jv) __attribute__((always_inline)) {
          if (x > y) return;
          seps = 0;
          cust = true;
          while (x <= y) {
            const uint32_t room = cap - c.load;
            const uint32_t F = rev ? T.tok[y] : T.tok[x];
            const uint32_t ein = c.prev ? jv : leg[F];
            if (T.PD[y + 1] - T.PD[x] <= room) {
              c.dur += ein + T.PE[y + 1] - T.PE[x + 1];
              c.load += T.PD[y + 1] - T.PD[x];
              c.prev = rev ? T.tok[x] : T.tok[y];
              return;
            }
            if (!rev) {
              int l = x - 1, h = y;  // last q with PD[q + 1] - PD[x] <= room
              while (l < h) {
                const int md = (l + h + 1) >> 1;
                if (T.PD[md + 1] - T.PD[x] <= room) l = md; else h = md - 1;
              }
              if (l >= x) {
                c.dur += ein + T.PE[l + 1] - T.PE[x + 1];
                c.load += T.PD[l + 1] - T.PD[x];
                c.prev = T.tok[l];
              }
              close();
              x = l + 1;
            } else {
              int l = x, h = y + 1;  // first z with PD[y + 1] - PD[z] <= room
              while (l < h) {
                const int md = (l + h) >> 1;
                if (T.PD[y + 1] - T.PD[md] <= room) h = md; else l = md + 1;
              }
              if (l <= y) {
                c.dur += ein + T.PE[y + 1] - T.PE[l + 1];
                c.load += T.PD[y + 1] - T.PD[l];
                c.prev = T.tok[l];
              }
              close();
              y = l - 1;
            }
          }
        };
        auto sep = [&]() __attribute__((always_inline)) {
          close();
          ++seps;
        };
        // A[x..y] in the moved order; jv = the junction edge into it
        auto piece = [&](int x, int y, bool rev, uint32_t jv) __attribute__((always_inline)) {
          if (x > y) return;
          const int sa = T.SC[x], sb = T.SC[y + 1];
          if (sa == sb) {
            run(x, y, rev, jv);
            return;
          }
          const int smin = T.SP[sa], smax = T.SP[sb - 1];
          if (rev) run(smax + 1, y, true, jv);
          else run(x, smin - 1, false, jv);
          sep();
          if (smin < smax) {  // whole segments of the current tour between the separators
            const int g0 = T.SC[smin] + 1, g1 = T.SC[smax];
            const int r0 = T.RB[g0], r1 = T.RB[g1 + 1];
            if (rev && r1 - r0 != g1 - g0 + 1) {
              // a segment of several routes splits differently reversed
              for (int g = g1; g >= g0; --g) {
                run(SPX(g - 1, S) + 1, SPX(g, S) - 1, true, 0u);
                sep();
              }
            } else {
              isum += T.dsp[r1] - T.dsp[r0];
              imax = max(imax, rmaxq(r0, r1 - 1));
              icnt += r1 - r0;
              if (rev) {
                const int gf = T.FNE[g0];
                if (gf <= g1) {
                  seps = gf - g0 + 1;
                  cust = true;
                } else {
                  seps += g1 - g0 + 1;
                }
              } else {
                const int gl = (int)T.LNE1[g1] - 1;
                if (gl >= g0) {
                  seps = g1 + 1 - gl;
                  cust = true;
                } else {
                  seps += g1 - g0 + 1;
                }
              }
            }
          }
          if (rev) run(x, smin - 1, true, 0u);
          else run(smax + 1, y, false, 0u);
        };
        const int s0 = T.SC[lo];
        const int stp = SPX(s0 - 1, S) + 1;
        const int en = SPX(T.SC[hi + 1], S);
        run(stp, lo - 1, false, 0u);
        // the moved span as pieces of the current tour (moved_index, tour.hpp),
        // then the rest of the last changed segment: four slots, one code path
        int px[4], py[4];
        uint32_t pj[4];  // junction edge into the slot (moved positions lo, lo + 1 / hi, hi, hi + 1)
        bool pr[4];
        {
          const bool opt = m.typ == kMove2Opt, swp = m.typ == kMoveSwap, fwd = m.i < m.j;
          // slot 0: 2-opt A[i..j] reversed | swap A[j] | relocate A[i+1..j] or A[i]
          px[0] = opt ? m.i : swp ? m.j : fwd ? m.i + 1 : m.i;
          py[0] = opt ? m.j : swp ? m.j : fwd ? m.j : m.i;
          pr[0] = opt;
          pj[0] = jx0;
          // slot 1: swap A[i+1..j-1] | relocate A[i] or A[j..i-1]
          px[1] = opt ? 1 : swp ? m.i + 1 : fwd ? m.i : m.j;
          py[1] = opt ? 0 : swp ? m.j - 1 : fwd ? m.i : m.i - 1;
          pr[1] = false;
          pj[1] = fwd && !swp ? jx2 : jx1;
          // slot 2: swap A[i]
          px[2] = swp ? m.i : 1;
          py[2] = swp ? m.i : 0;
          pr[2] = false;
          pj[2] = jx2;
          // slot 3: the rest of the last changed segment, to its separator
          px[3] = hi + 1;
          py[3] = en < n ? en : n - 1;
          pr[3] = false;
          pj[3] = jx3;
        }
#pragma unroll
        for (int sl = 0; sl < 4; ++sl) piece(px[sl], py[sl], pr[sl], pj[sl]);
        if (en >= n) close();  // the tour's end closes the last route
        const int glast = en < n ? (int)T.SC[en] : S;
        const int ra = T.RB[s0], rz = T.RB[glast + 1];
        const int RBn = R - (rz - ra) + c.rcnt + icnt;
        int Tb = Tt;
        const bool tail_kept = en < n && (int)T.LNE1[S] - 1 > glast;
        if (!tail_kept && cust) Tb = seps + (en < n ? n - 1 - en : 0);
        if (RBn - Tb <= K) {
          const uint32_t dsum = T.dsp[ra] + c.rsum + isum + T.dsp[R] - T.dsp[rz];
          const uint32_t dmax = max(max(T.pmx[ra], T.smx[rz]), max(imax, c.rmax));
          k = cvrp_key(0, dsum, dmax, I.sp.objective);
        } else if (shortcut) {
          k = ~0ull;
        } else {
          auto moved = [&](int q) { return tourA(map_src(mmap, q)); };
          k = eval_tour<true>(I.D, I.sp, moved, n).key;
        }
      } else {
        auto moved = [&](int q) { return tourA(map_src(mmap, q)); };
        k = eval_tour<true>(I.D, I.sp, moved, n).key;
      }
      if (k < bkey) {  // ties keep the earlier (smaller) move index
        bkey = k;
        bidx = idx;
        bw = r.w;
        bmv = m;
        bj[0] = jx0;
        bj[1] = jx1;
        bj[2] = jx2;
        bj[3] = jx3;
      }
    }
    // the chain's (key, move index) minimum
    int wl;
    const uint64_t kmin = wave_argmin_lane(bkey, wl);
    const uint32_t imin = wave_min_u32_uniform(bkey == kmin ? bidx : 0xffffffffu);
    const int bl = (int)(imin & 63u);
    const uint64_t k = kmin;
    const uint32_t uw = (uint32_t)wave_bcast((int)bw, bl);
    bool accept = k <= ck;
    if (!accept) {
      const uint64_t d = (k >> 28) - (ck >> 28);
      const uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      accept = (uw >> 8) < accept_threshold(dp, invT);
    }
    if (accept) {
      Move mb;
      mb.typ = (uint32_t)wave_bcast((int)bmv.typ, bl);
      mb.i = wave_bcast(bmv.i, bl);
      mb.j = wave_bcast(bmv.j, bl);
      const MoveMap mmb = move_map(mb);
      const int blo = min(mb.i, mb.j), bhi = max(mb.i, mb.j);
      uint32_t wj[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) wj[x] = (uint32_t)wave_bcast((int)bj[x], bl);
      // the new tour's tokens and edges: a kept adjacency's edge is a
      // difference of PE (forward, or reversed on the symmetric matrix), the
      // four junctions come from the winner's gathers
#pragma unroll
      for (int i = 0; i < kSegRegs; ++i) {
        const int q = lane + 64 * i;
        v_tok[i] = 0u;
        v_e[i] = 0u;
        if (q > n) continue;
        const int sq = map_src(mmb, q), sp = map_src(mmb, q - 1);
        if (q < n) v_tok[i] = T.tok[sq];
        if (q == blo) v_e[i] = wj[0];
        else if (q == blo + 1) v_e[i] = wj[1];
        else if (q == bhi) v_e[i] = wj[2];
        else if (q == bhi + 1) v_e[i] = wj[3];
        else if (sp + 1 == sq) v_e[i] = T.PE[sq + 1] - T.PE[sq];
        else v_e[i] = T.PE[sp + 1] - T.PE[sp];  // reversed: the edge between A[sq] and A[sp]
      }
      if (!seg_ok) {
        // tables not held (too many separators / routes): edges from L2
#pragma unroll
        for (int i = 0; i < kSegRegs; ++i) {
          const int q = lane + 64 * i;
          if (q > n) continue;
          const uint32_t p = q >= 1 ? tourA(map_src(mmb, q - 1)) : 0u;
          v_e[i] = d0(p, v_tok[i]);
        }
      }
      rebuild();
      ck = k;
      if (ck < bk) {
        bk = ck;
        for (int q = lane; q < n; q += 64) gbest[q] = T.tok[q];
      }
    }
    invT = invT * a.inv_alpha;
  }
  uint16_t* gout = a.cur + (int64_t)chain * n;
  for (int q = lane; q < n; q += 64) gout[q] = T.tok[q];
  if (lane == 0) {
    a.cur_key[chain] = ck;
    a.best_key[chain] = bk;
  }
}

// Host side: can the segment kernel run this SA call, and with what layout?
// Returns VRPMS_OK after launching, or 1 when it does not apply.
int launch_sa_seg(const vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur,
                  uint64_t* d_cur_key, uint16_t* d_best, uint64_t* d_best_key, int n,
                  uint32_t wtypes, int moves, hipStream_t s) {
  const Instance& in = ctx->inst;
  if (in.problem != VRPMS_CVRP || in.H != 1 || !in.symmetric || !in.uniform_cap ||
      in.max_dem > in.cap0 || n < 2 || n >= 64 * kSegRegs || n > 65535 || moves % 64 != 0 ||
      moves / 64 > kSegMaxMoves)
    return 1;
  SearchInst si = search_inst(ctx);
  si.mat_lds = 0;  // the matrix stays in L2: a move gathers <= 4 entries
  // separators: a tour of the N - 1 customers and n - (N - 1) separators
  const int segs = std::max(8, ((std::max(0, n - (in.N - 1)) + 2 + 7) & ~7));
  const int rm = std::max(2 * in.K + 2, segs + 2) + 8;
  const int lv = seg_levels(rm);
  const uint32_t cb = seg_chain_bytes(n, segs, rm, lv);
  const size_t base = inst_lds_bytes_host(si) + (((size_t)in.N * 4u + 15u) & ~(size_t)15u);
  int cpw = 4;
  // fewer chains than 4 per CU: spread them, one wavefront per workgroup
  if (p->chains < 4 * ctx->num_cus) cpw = p->chains < 2 * ctx->num_cus ? 1 : 2;
  while (cpw > 1 && base + (size_t)cpw * cb > ctx->max_lds) cpw >>= 1;
  const size_t lds = base + (size_t)cpw * cb;
  if (lds > ctx->max_lds) return 1;
  SegArgs a{si, p->chains, n, p->steps, p->window, wtypes, p->inv_t0, p->inv_alpha,
            (uint32_t)p->seed, (uint32_t)(p->seed >> 32), p->step0, d_cur, d_cur_key, d_best,
            d_best_key, moves / 64, cpw, segs, rm, lv, cb};
  auto go = [&](auto kern) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<dim3((p->chains + cpw - 1) / cpw), dim3(64 * cpw), lds, s>>>(a);
  };
  if (in.use16) go(sa_seg_kernel<uint16_t>);
  else go(sa_seg_kernel<int32_t>);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

}  // namespace vrpms
