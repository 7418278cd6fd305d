// Single-tour evaluation (frozen in oracle/spec.py)
// shared by the generic scoring kernel and every search kernel, so a tour
// scored inside SA/GA/ACO/BF is bit-identical to vrpms_eval's score of it.
#pragma once
#include "common.hpp"

namespace vrpms {

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

// Duration matrix view (LDS or global), [H][N][N].
template <typename MatT, int HM>
struct MatView {
  const MatT* M;
  uint32_t N, NN;
  int H;
  VRPMS_DEV int operator()(int t, uint32_t a, uint32_t b) const {
    // a, N < 2^24: the full-rate 24-bit multiply gives the same 32-bit product
    return (int)M[hour_of<HM>(t, H) * NN + __umul24(a, N) + b];
  }
};

struct SplitParams {
  const int32_t* dem;
  const int32_t* cap;
  const int32_t* start;
  int K;
  int objective;
};

struct TourCost {
  uint64_t key;
  int32_t sum, max, unv;
};

// A4 (TSP) / A5-A7 (CVRP greedy split, A10 separator tokens 0); `tour(i)`
// returns customer i (values >= N are clamped to N-1 so a corrupt tour can
// never fault).
template <bool CVRP, typename Mat, typename Tour>
VRPMS_DEV TourCost eval_tour(const Mat& D, const SplitParams& sp, const Tour& tour, int n) {
  const uint32_t Nm1 = D.N - 1;
  if constexpr (!CVRP) {
    const int t0 = sp.start[0];
    int t = t0;
    uint32_t prev = 0;
    for (int i = 0; i < n; ++i) {
      const uint32_t cc = min((uint32_t)tour(i), Nm1);
      t += D(t, prev, cc);
      prev = cc;
    }
    t += D(t, prev, 0);
    const int d = t - t0;
    return {pack_key(0, (uint32_t)d, 0), d, d, 0};
  } else {
    const int K = sp.K;
    int k = 0, load = 0, t = sp.start[0], capk = sp.cap[0];
    uint32_t prev = 0, unv = 0, dsum = 0, dmax = 0;
    for (int i = 0; i < n; ++i) {
      const uint32_t cc = min((uint32_t)tour(i), Nm1);
      if (cc == 0) {  // A10 separator: close route k (if any), open vehicle k + 1
        if (k < K) {
          if (prev) {
            t += D(t, prev, 0);
            const uint32_t rd = (uint32_t)(t - sp.start[k]);
            dsum += rd;
            dmax = max(dmax, rd);
          }
          ++k;
          if (k < K) {
            load = 0;
            t = sp.start[k];
            prev = 0;
            capk = sp.cap[k];
          }
        }
        continue;
      }
      const int dc = sp.dem[cc];
      if (k < K && load + dc > capk) {
        do {
          if (prev) {
            t += D(t, prev, 0);
            const uint32_t rd = (uint32_t)(t - sp.start[k]);
            dsum += rd;
            dmax = max(dmax, rd);
          }
          ++k;
          if (k < K) {
            load = 0;
            t = sp.start[k];
            prev = 0;
            capk = sp.cap[k];
          }
        } while (k < K && load + dc > capk);
      }
      if (k < K) {
        t += D(t, prev, cc);
        load += dc;
        prev = cc;
      } else {
        ++unv;
      }
    }
    if (k < K && prev) {
      t += D(t, prev, 0);
      const uint32_t rd = (uint32_t)(t - sp.start[k]);
      dsum += rd;
      dmax = max(dmax, rd);
    }
    return {cvrp_key(unv, dsum, dmax, sp.objective), (int32_t)dsum, (int32_t)dmax, (int32_t)unv};
  }
}

// ---------------------------------------------------------------------------
// Neighbourhood moves on a giant tour (oracle/spec.py decode_move / moved_index)
// ---------------------------------------------------------------------------
enum : uint32_t { kMoveSwap = 0, kMove2Opt = 1, kMoveRelocate = 2 };

struct Move {
  uint32_t typ;
  int i, j;
};

VRPMS_DEV Move decode_move(uint32_t r0, uint32_t r1, uint32_t r2, int n) {
  Move m;
  m.typ = r0 % 3u;
  m.i = (int)(r1 % (uint32_t)n);
  int j = (int)(r2 % (uint32_t)(n - 1));
  if (j >= m.i) ++j;
  m.j = j;
  if (m.typ != kMoveRelocate && m.i > m.j) {
    const int x = m.i;
    m.i = m.j;
    m.j = x;
  }
  return m;
}

// A13 (oracle/spec.py decode_move1): one word split by successive fixed-point
// multiplications -- type = hi(3x), i = hi(n lo(3x)), j' = hi((n-1) lo(n lo(3x)))
// -- six multiplies instead of three divisions by run-time moduli
VRPMS_DEV Move decode_move1(uint32_t x, int n) {
  Move m;
  const uint32_t f1 = x * 3u;
  m.typ = __umulhi(x, 3u);
  m.i = (int)__umulhi(f1, (uint32_t)n);
  const uint32_t f2 = f1 * (uint32_t)n;
  int j = (int)__umulhi(f2, (uint32_t)(n - 1));
  if (j >= m.i) ++j;
  m.j = j;
  if (m.typ != kMoveRelocate && m.i > m.j) {
    const int t = m.i;
    m.i = m.j;
    m.j = t;
  }
  return m;
}

// A11 (oracle/spec.py decode_move_window): the second position within
// `window` of the first; window <= 0 or 2 window + 1 >= n: decode_move.
// A12: only for the move types whose bit is set in `types` (7 = all).
VRPMS_DEV Move decode_move_window(uint32_t r0, uint32_t r1, uint32_t r2, int n, int window,
                                  uint32_t types) {
  if (window <= 0 || 2 * window + 1 >= n || !((types >> (r0 % 3u)) & 1u))
    return decode_move(r0, r1, r2, n);
  Move m;
  m.typ = r0 % 3u;
  m.i = (int)(r1 % (uint32_t)n);
  const int o = (int)(r2 % (uint32_t)(2 * window));
  const int d = o < window ? o - window : o - window + 1;
  int j = m.i + d;
  if (j < 0 || j >= n) j = m.i - d;
  m.j = j;
  if (m.typ != kMoveRelocate && m.i > m.j) {
    const int x = m.i;
    m.i = m.j;
    m.j = x;
  }
  return m;
}

// Position in the ORIGINAL tour read at position q of the moved tour.
VRPMS_DEV int moved_index(int q, const Move& m) {
  const int i = m.i, j = m.j;
  if (m.typ == kMoveSwap) return q == i ? j : (q == j ? i : q);
  if (m.typ == kMove2Opt) return (q >= i && q <= j) ? i + j - q : q;
  if (i < j) {
    if (q < i || q > j) return q;
    return q == j ? i : q + 1;
  }
  if (q < j || q > i) return q;
  return q == j ? i : q - 1;
}

// moved_index as a select chain with no divergent branches: one window of
// positions read at a + s*q (2-opt reversal, relocate shift) plus up to two
// pinned positions (swap ends, relocate target).  src(q) == moved_index(q, m)
// for every q; positions outside [0, n) map to themselves.
struct MoveMap {
  int lo, len, a, s, p1, v1, p2, v2;
};

VRPMS_DEV MoveMap move_map(const Move& m) {
  const int i = m.i, j = m.j;
  if (m.typ == kMoveSwap) return {0, 0, 0, 1, i, j, j, i};
  if (m.typ == kMove2Opt) return {i, j - i + 1, i + j, -1, -1, 0, -1, 0};
  if (i < j) return {i, j - i, 1, 1, j, i, -1, 0};
  return {j + 1, i - j, -1, 1, j, i, -1, 0};
}

VRPMS_DEV MoveMap identity_map() { return {0, 0, 0, 1, -1, 0, -1, 0}; }

VRPMS_DEV int map_src(const MoveMap& mm, int q) {
  int r = (uint32_t)(q - mm.lo) < (uint32_t)mm.len ? mm.a + mm.s * q : q;
  r = q == mm.p1 ? mm.v1 : r;
  return q == mm.p2 ? mm.v2 : r;
}

// Exact duration change of the static closed tour 0 -> T[0..n-1] -> 0 under
// move m (integer, so duration + delta == a full re-evaluation).  Swap and
// relocate touch at most 8 edges; 2-opt touches 4 on a symmetric matrix and
// additionally re-prices the reversed segment otherwise.  `d(a, b)` is D[a][b].
template <typename Dist, typename Tour>
VRPMS_DEV int tsp_move_delta(const Dist& d, const Tour& T, int n, const Move& m, bool symmetric) {
  auto at = [&](int q) -> uint32_t { return (q < 0 || q >= n) ? 0u : (uint32_t)T(q); };
  const int i = m.i, j = m.j;
  if (m.typ == kMoveSwap) {  // i < j
    const uint32_t a = at(i - 1), pi = at(i), pj = at(j), b = at(j + 1);
    if (j == i + 1) return d(a, pj) + d(pj, pi) + d(pi, b) - d(a, pi) - d(pi, pj) - d(pj, b);
    const uint32_t x = at(i + 1), y = at(j - 1);
    return d(a, pj) + d(pj, x) + d(y, pi) + d(pi, b) - d(a, pi) - d(pi, x) - d(y, pj) - d(pj, b);
  }
  if (m.typ == kMove2Opt) {  // reverse T[i..j], i < j
    const uint32_t a = at(i - 1), pi = at(i), pj = at(j), b = at(j + 1);
    int delta = d(a, pj) + d(pi, b) - d(a, pi) - d(pj, b);
    if (!symmetric)
      for (int q = i; q < j; ++q) delta += d(at(q + 1), at(q)) - d(at(q), at(q + 1));
    return delta;
  }
  if (i < j) {  // relocate T[i] to position j (later)
    const uint32_t a = at(i - 1), pi = at(i), x = at(i + 1), pj = at(j), b = at(j + 1);
    return d(a, x) + d(pj, pi) + d(pi, b) - d(a, pi) - d(pi, x) - d(pj, b);
  }
  // relocate T[i] to position j (earlier)
  const uint32_t a = at(j - 1), pj = at(j), y = at(i - 1), pi = at(i), b = at(i + 1);
  return d(a, pi) + d(pi, pj) + d(y, b) - d(a, pj) - d(y, pi) - d(pi, b);
}

// tsp_move_delta for a symmetric matrix without divergent branches: every
// move type is "add four edges, remove four edges" over the six tour
// positions i-1 .. j+1 (unused slots add and remove the same edge, which
// cancels exactly), so a wave whose lanes drew different move types issues
// 6 tour reads + 8 matrix gathers once instead of running every type's
// branch under its own exec mask.  Same integer result as tsp_move_delta.
template <typename Dist, typename Tour>
VRPMS_DEV int tsp_move_delta_sym(const Dist& d, const Tour& T, int n, const Move& m) {
  auto at = [&](int q) -> uint32_t { return (uint32_t)q < (uint32_t)n ? (uint32_t)T(q) : 0u; };
  const int i = m.i, j = m.j;
  const uint32_t im1 = at(i - 1), pi = at(i), ip1 = at(i + 1);
  const uint32_t jm1 = at(j - 1), pj = at(j), jp1 = at(j + 1);
  const bool swp = m.typ == kMoveSwap, opt = m.typ == kMove2Opt, rel = m.typ == kMoveRelocate;
  const bool adj = swp && j == i + 1, lo = rel && i < j, hi = rel && i > j;
  // plus edges (a_k, b_k), minus edges (c_k, e_k), k = 0..3
  // swap     : +(im1,pj) +(pj,ip1) +(jm1,pi) +(pi,jp1)  -(im1,pi) -(pi,ip1) -(jm1,pj) -(pj,jp1)
  // swap adj : +(im1,pj) +(pj,pi)  +(pi,jp1) pad        -(im1,pi) -(pi,pj)  -(pj,jp1) pad
  // 2-opt    : +(im1,pj) +(pi,jp1) pad       pad        -(im1,pi) -(pj,jp1) pad       pad
  // reloc i<j: +(im1,ip1) +(pj,pi) +(pi,jp1) pad        -(im1,pi) -(pi,ip1) -(pj,jp1) pad
  // reloc i>j: +(jm1,pi) +(pi,pj)  +(im1,ip1) pad       -(jm1,pj) -(im1,pi) -(pi,ip1) pad
  const uint32_t a0 = hi ? jm1 : im1, b0 = lo ? ip1 : (hi ? pi : pj);
  const uint32_t c0 = hi ? jm1 : im1, e0 = hi ? pj : pi;
  const uint32_t a1 = opt ? pi : (lo ? pj : (hi ? pi : pj));
  const uint32_t b1 = opt ? jp1 : (lo ? pi : (hi ? pj : (adj ? pi : ip1)));
  const uint32_t c1 = opt ? pj : (hi ? im1 : pi);
  const uint32_t e1 = opt ? jp1 : (hi ? pi : (adj ? pj : ip1));
  const uint32_t a2 = opt ? pi : (hi ? im1 : (swp && !adj ? jm1 : pi));
  const uint32_t b2 = opt ? pi : (hi ? ip1 : (swp && !adj ? pi : jp1));
  const uint32_t c2 = opt ? pi : (hi ? pi : (swp && !adj ? jm1 : pj));
  const uint32_t e2 = opt ? pi : (hi ? ip1 : (swp && !adj ? pj : jp1));
  const bool full = swp && !adj;
  const uint32_t a3 = pi, b3 = full ? jp1 : pi;
  const uint32_t c3 = full ? pj : pi, e3 = full ? jp1 : pi;
  return d(a0, b0) + d(a1, b1) + d(a2, b2) + d(a3, b3) - d(c0, e0) - d(c1, e1) - d(c2, e2) - d(c3, e3);
}

// tsp_move_delta_sym with the removed edges read from the current tour's edge
// cache: Ec(q) = d(T[q-1], T[q]) for q = 0..n (the depot at both ends).  Every
// removed edge is a tour edge at position i, i+1, j or j+1, so only the added
// edges are matrix gathers; the pads of the gather form are masked out on
// both sides.  Same integer result as tsp_move_delta.
// PADDED: T(-1) and T(n) read the depot (0) themselves.
template <bool PADDED = false, typename Dist, typename Tour, typename EdgeAt>
VRPMS_DEV int tsp_move_delta_sym_cached(const Dist& d, const Tour& T, const EdgeAt& Ec, int n,
                                        const Move& m) {
  auto at = [&](int q) -> uint32_t {
    if constexpr (PADDED) return (uint32_t)T(q);
    else return (uint32_t)q < (uint32_t)n ? (uint32_t)T(q) : 0u;
  };
  const int i = m.i, j = m.j;
  const uint32_t im1 = at(i - 1), pi = at(i), ip1 = at(i + 1);
  const uint32_t jm1 = at(j - 1), pj = at(j), jp1 = at(j + 1);
  const bool swp = m.typ == kMoveSwap, opt = m.typ == kMove2Opt, rel = m.typ == kMoveRelocate;
  const bool adj = swp && j == i + 1, lo = rel && i < j, hi = rel && i > j;
  const bool full = swp && !adj;
  // added edges as in tsp_move_delta_sym (slots 2 / 3 are pads for 2-opt / all but a full swap)
  const uint32_t a0 = hi ? jm1 : im1, b0 = lo ? ip1 : (hi ? pi : pj);
  const uint32_t a1 = opt ? pi : (lo ? pj : (hi ? pi : pj));
  const uint32_t b1 = opt ? jp1 : (lo ? pi : (hi ? pj : (adj ? pi : ip1)));
  const uint32_t a2 = hi ? im1 : (swp && !adj ? jm1 : pi);
  const uint32_t b2 = hi ? ip1 : (swp && !adj ? pi : jp1);
  const int g0 = d(a0, b0), g1 = d(a1, b1), g2 = d(a2, b2), g3 = d(pi, jp1);
  const int plus = g0 + g1 + (opt ? 0 : g2) + (full ? g3 : 0);
  // removed edges: swap i, i+1, j, j+1 (adjacent: i, i+1, j+1); 2-opt i, j+1;
  // relocate i<j: i, i+1, j+1; relocate i>j: j, i, i+1
  const int ei = Ec(i), ei1 = Ec(i + 1), ej = Ec(j), ej1 = Ec(j + 1);
  const int minus = ei + (opt ? 0 : ei1) + (full || hi ? ej : 0) + (swp || opt || lo ? ej1 : 0);
  return plus - minus;
}

// ---------------------------------------------------------------------------
// Deterministic SA acceptance threshold: floor(2^24 * exp(-dp * invT)) using
// only IEEE fp32 multiply/add/sub (built with -ffp-contract=off) and exact
// power-of-two scaling, so oracle/spec.py reproduces it bit for bit.
// ---------------------------------------------------------------------------
VRPMS_DEV uint32_t accept_threshold(uint32_t dp, float invT) {
  if (dp == 0) return 1u << 24;
  const float x = (float)dp * invT;           // >= 0
  const float y = x * 0x1.715476p+0f;            // x * log2(e)
  if (!(y < 24.0f)) return 0u;                // 2^-24 * 2^24 < 1
  const float kf = floorf(y);
  const float f = y - kf;                     // [0, 1)
  // 2^-f = exp(-f ln2), degree-6 Taylor polynomial in g = f * ln2 (|err| < 2e-6)
  const float g = f * 0x1.62e43p-1f;
  float p = 0x1.6c16c2p-10f;                   // 1/720
  p = p * g;
  p = 0x1.111112p-7f - p;                     // 1/120
  p = p * g;
  p = 0x1.555556p-5f - p;                      // 1/24
  p = p * g;
  p = 0x1.555556p-3f - p;                       // 1/6
  p = p * g;
  p = 0.5f - p;
  p = p * g;
  p = 1.0f - p;
  p = p * g;
  p = 1.0f - p;                               // ~ e^-g
  const int k = (int)kf;                      // 0..23
  const float scaled = p * (float)(1u << (24 - k));  // exact power-of-two scaling
  return (uint32_t)scaled;                    // truncation
}

// u < accept_threshold(dp, invT) for a wave-uniform draw u < 2^24, with an
// exact early answer before the polynomial: the polynomial p never exceeds
// 1.0f (1 - a non-negative product), so the threshold is at most 2^(24 - k),
// k = floor(dp invT log2 e), and a draw at or above that bound is rejected
// without evaluating it (at a cold temperature, almost every uphill move).
VRPMS_DEV bool accept_test(uint32_t dp, float invT, uint32_t u) {
  if (dp == 0) return u < (1u << 24);
  const float x = (float)dp * invT;
  const float y = x * 0x1.715476p+0f;
  if (!(y < 24.0f)) return false;
  const int k = __builtin_amdgcn_readfirstlane((int)floorf(y));
  if (u >= (1u << (24 - k))) return false;
  return u < accept_threshold(dp, invT);
}

}  // namespace vrpms
