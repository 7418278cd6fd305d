// Branch-free greedy split over the prefix-ret
// packed matrix, shared by the headline scoring kernel (eval_cvrp_words) and
// the CVRP SA chain kernel (sa_packed_kernel) so both produce the same key
// for the same tour, bit for bit, as oracle/spec.py eval_cvrp.
//
// Layout (capi.hip pack_prefix_kernel + bias_hi_kernel), uniform fleet:
//   E[a][b].lo = dem(b) << S + dur(a,b) + ret(b) - ret(a)       (mod 2^32)
//   E[a][b].hi = (out(b) + ret(b) | dem(b) << S) - lim,  lim = (cap + 1) << S
// A route's accumulator is acc = (load << S | cur + ret(last)) - lim, so a
// customer fits iff acc + lo is negative (sign bit), and the finished
// route's duration is acc & smask.
//   rd'  = (acc & smask) | 1 << KS      finished route, vehicle count above KS
//   dsum += f ? 0 : rd';  dmax = max(dmax, f ? 0 : rd')
//   acc  = f ? t : (dsum >= K << KS ? DEAD : hi)
// A10 separator tokens (0) need no special case: column 0 of E holds
// lo = 0x7fffffff (never fits: the route closes) and hi = -lim (an empty
// route), so a separator closes the route and opens the next vehicle.
// The vehicle counter lives in dsum's high bits, starting at 2^B - K so that
// exhausting the fleet sets bit 31; the accumulator is then parked at DEAD,
// which never fits again and adds no duration, so every later customer adds
// exactly one count: unvisited = count - K + 1.  No per-lane flags and no
// divergent branches.
#pragma once
#include "common.hpp"
#include "ctx.hpp"
#include "tour.hpp"

namespace vrpms {

struct FastSplit {
  const uint64_t* pack;     // biased prefix-ret matrix [N][N] (Instance::pack64w)
  int N, K, objective;
  uint32_t lim, smask;
  uint32_t ks, klim, dead;  // 1 << ks counts vehicles; klim = initial dsum; dead = biased DEAD
  bool carry;               // every customer demand >= 1: the fit test is acc + lo's carry
};

// Host: constants of the branch-free split for tours of n customers, or
// false when the instance is outside its exactness conditions (the caller
// then uses the generic split).  Defined in eval.hip.
bool fast_split_params(const vrpms_ctx* ctx, int n, FastSplit* out);

struct SplitAcc {
  uint32_t acc, dsum, dmax;

  VRPMS_DEV void init(const FastSplit& f) {
    acc = 0u - f.lim;
    dsum = f.klim;
    dmax = 0;
  }

  // One customer: `e` is the packed entry of (previous customer, customer).
  // Every select is a bitwise v_bfi on an arithmetic-shift mask; the sign
  // mask comes from the bitfield-extract intrinsic, which LLVM does not
  // re-form into a compare + select the way it does for (int)x >> 31.
  VRPMS_DEV void step(uint64_t e, uint32_t smask, uint32_t kinc, uint32_t deadacc) {
    auto bsel = [](uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); };
    auto sgn = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_sbfe((int)x, 31u, 1u); };
    const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);  // hi is pre-biased too
    const uint32_t t = acc + lo;
    const uint32_t fm = sgn(t);                                 // all ones: fits
    const uint32_t rdm = bsel(fm, 0u, (acc & smask) | kinc);    // finished route, +1 vehicle
    dsum += rdm;
    dmax = max(dmax, rdm);
    const uint32_t am = sgn(dsum);                              // all ones: fleet exhausted
    acc = bsel(fm, t, bsel(am, deadacc, hi));
  }

  // step() without the fleet-exhaustion test (a customer that does not fit
  // always opens a new route).  Exact until the K-th route closes, which
  // sets dsum's sign bit for good (the counter only grows, 2^B > n): a walk
  // that ends with dsum >= 0 equals the step() walk; one that does not is
  // re-walked with step() by the caller.
  VRPMS_DEV void step_fast(uint64_t e, uint32_t smask, uint32_t kinc) {
    auto bsel = [](uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); };
    auto sgn = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_sbfe((int)x, 31u, 1u); };
    const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
    const uint32_t t = acc + lo;
    const uint32_t fm = sgn(t);
    const uint32_t rdm = bsel(fm, 0u, (acc & smask) | kinc);
    dsum += rdm;
    dmax = max(dmax, rdm);
    acc = bsel(fm, t, hi);
  }
  VRPMS_DEV bool hit_fleet_limit() const { return (int32_t)dsum < 0; }

  VRPMS_DEV TourCost finish(const FastSplit& f, int n) const {
    const uint32_t kinc = 1u << f.ks;
    const bool dead = (int32_t)dsum < 0;
    const uint32_t count = (dsum >> f.ks) - (f.klim >> f.ks);  // vehicles closed (+ dead steps)
    uint32_t s = dsum & (kinc - 1u), m = dmax >= kinc ? dmax - kinc : 0u;
    uint32_t unv = 0;
    if (dead) {
      unv = count - (uint32_t)f.K + 1u;
    } else if (n > 0) {
      const uint32_t rd = acc & f.smask;  // close the last route
      s += rd;
      m = max(m, rd);
    }
    return {cvrp_key(unv, s, m, f.objective), (int32_t)s, (int32_t)m, (int32_t)unv};
  }
};

// The exact split of one tour with the fleet limit and A10 separators
// (token 0: close the route, open the next vehicle), walked token by token:
// the slow path for a lane whose fast walk met the fleet limit.  `tok(q)`
// is tour token q, `gat(a, b)` the biased packed entry E[a][b].  Once the
// K-th route has closed, customers are counted unvisited and separators are
// ignored.  Same result as step() + finish() on separator-free tours.
template <class Tok, class Gat>
VRPMS_DEV TourCost exact_split(const FastSplit& f, int n, Tok tok, Gat gat) {
  const uint32_t kinc = 1u << f.ks, fresh = 0u - f.lim;
  uint32_t acc = fresh, dsum = f.klim, dmax = 0, unv = 0, prev = 0;
  bool dead = false;
  for (int q = 0; q < n; ++q) {
    const uint32_t c = tok(q);
    if (dead) {
      unv += c != 0u;
      continue;
    }
    uint32_t next = fresh;  // a separator opens an empty route
    if (c != 0u) {
      const uint64_t e = gat(prev, c);
      const uint32_t t = acc + (uint32_t)e;
      if ((int32_t)t < 0) {  // fits
        acc = t;
        prev = c;
        continue;
      }
      next = (uint32_t)(e >> 32);  // opens a route holding c
    }
    const uint32_t rdm = (acc & f.smask) | kinc;  // close route k
    dsum += rdm;
    dmax = max(dmax, rdm);
    if ((int32_t)dsum < 0) {  // that was the K-th vehicle
      dead = true;
      unv += c != 0u;
      continue;
    }
    acc = next;
    prev = c;
  }
  uint32_t s = dsum & (kinc - 1u), m = dmax >= kinc ? dmax - kinc : 0u;
  if (!dead) {
    const uint32_t rd = acc & f.smask;  // close the last route (0 when empty)
    s += rd;
    m = max(m, rd);
  }
  return {cvrp_key(unv, s, m, f.objective), (int32_t)s, (int32_t)m, (int32_t)unv};
}

}  // namespace vrpms
