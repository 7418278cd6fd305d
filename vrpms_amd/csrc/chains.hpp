// The per-customer machinery of the LDS-packed scoring kernels, shared by
// eval_cvrp_words2 / eval_cvrp_rows2 / eval_cvrp_rows4 (eval_words.hip) and
// the fused GA island kernel (ga_fused.hip): the branch-free split step over
// the biased prefix-ret matrix E (split.hpp) and the gather addressing by
// v_perm_b32 + v_dot2_u32_u16 on four-customer tour words.
#pragma once
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "split.hpp"

namespace vrpms {

// VALU per ds_read slot in the interleaved schedule (A/B builds override)
#ifndef VRPMS_IL_VALU
#define VRPMS_IL_VALU 10
#endif

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const uint64_t lds_u64;
typedef __attribute__((address_space(3))) unsigned char lds_uc;

// v_perm selectors: bytes (x, 0, y, 0) of the 8-byte value {hi_word, lo_word}
constexpr uint32_t kSel01 = 0x0c010c00u;  // (c0, c1) of one word
constexpr uint32_t kSel12 = 0x0c020c01u;
constexpr uint32_t kSel23 = 0x0c030c02u;
constexpr uint32_t kSel30 = 0x0c040c03u;  // (c3 of lo_word = previous, c0 of hi_word = current)

// One customer of the branch-free split (split.hpp SplitAcc::step), with the
// route-closure value formed by v_and_or_b32 on a VGPR-resident smask.
// (A v_ashrrev/v_bfi form with VGPR lane masks was measured 1-9 % slower:
// inline asm makes LLVM pad every use with s_nop.)
VRPMS_DEV void split_step(SplitAcc& s, uint64_t e, uint32_t vsmask, uint32_t kinc,
                          uint32_t deadacc) {
  const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
  const uint32_t t = s.acc + lo;
  const bool fits = (int32_t)t < 0;
  const uint32_t rdm = fits ? 0u : ((s.acc & vsmask) | kinc);
  s.dsum += rdm;
  s.dmax = max(s.dmax, rdm);
  const bool exhausted = (int32_t)s.dsum < 0;
  s.acc = fits ? t : (exhausted ? deadacc : hi);
}

// The same step without the fleet-exhaustion test: a customer that does not
// fit always opens a new route, and dsum's vehicle counter keeps counting.
// Identical to split_step until the K-th route closes, which sets dsum's
// sign bit (the counter starts at 2^B - K) -- and that bit stays set, since
// the counter only grows and 2^B > n keeps it below 2^32.  So a chain whose
// dsum is non-negative at the end never met the exhaustion branch and its
// result is exact; the rare chain that did is re-walked with split_step
// (redo_exact).  Random CVRP-100 giant tours never exhaust the bench's
// fleet (0 of 200k), and this drops a compare + select per customer.
VRPMS_DEV void split_step_fast(SplitAcc& s, uint64_t e, uint32_t vsmask, uint32_t kinc) {
  const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
  const uint32_t t = s.acc + lo;
  const bool fits = (int32_t)t < 0;
  const uint32_t rdm = fits ? 0u : ((s.acc & vsmask) | kinc);
  s.dsum += rdm;
  s.dmax = max(s.dmax, rdm);
  s.acc = fits ? t : hi;
}

// split_step_fast with the fit test read from the add's carry (no compare):
// acc = (load - cap - 1) << S + low lies in [2^31, 2^32) and lo = dem << S +
// (low' - low) mod 2^32, so when dem >= 1 the second term is a positive
// number below 2^31 and acc + lo overflows 32 bits exactly when load + dem >
// cap -- the same test as the sign of t (fast_split_params bounds
// (cap + max_dem + 3) << S by 2^31).  A zero demand can make lo wrap (an edge
// term below 0) and carry on a fit: FastSplit::carry is set only when every
// customer demand is >= 1.  A separator (column 0, lo = 2^31 - 1) always
// carries.
VRPMS_DEV void split_step_carry(SplitAcc& s, uint64_t e, uint32_t vsmask, uint32_t kinc) {
  const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
  uint32_t t;
  const bool over = __builtin_add_overflow(s.acc, lo, &t);
  const uint32_t rdm = over ? ((s.acc & vsmask) | kinc) : 0u;
  s.dsum += rdm;
  s.dmax = max(s.dmax, rdm);
  s.acc = over ? hi : t;
}

// Copy the packed matrix E into LDS (16-byte vectors + an 8-byte tail).
VRPMS_DEV void stage_table(const uint64_t* pack, int N, unsigned char* smem) {
  const uint32_t ebytes = (uint32_t)N * N * 8;
  const v4u* src = reinterpret_cast<const v4u*>(pack);
  v4u* dst = reinterpret_cast<v4u*>(smem);
  for (uint32_t i = threadIdx.x; i < ebytes / 16; i += blockDim.x) dst[i] = src[i];
  if ((ebytes & 8u) && threadIdx.x == 0)
    reinterpret_cast<uint64_t*>(smem)[ebytes / 8 - 1] = pack[ebytes / 8 - 1];
  __syncthreads();
}

// ILP independent split chains of one lane, fed four customers (one word)
// at a time (CY: the carry form of the step, FastSplit::carry).
template <int ILP, bool CY = false>
struct WordChains {
  SplitAcc sa[ILP];
  uint32_t wprev[ILP];  // previous word (its byte 3 is the depot before the first word)
  uint32_t vsmask, kinc, deadacc, ebase;
  us2 w8;

  VRPMS_DEV void setup(const FastSplit& f, unsigned char* smem) {
    ebase = (uint32_t)(uintptr_t)(lds_uc*)smem;
    w8 = {(unsigned short)(8 * f.N), (unsigned short)8};
    kinc = 1u << f.ks;
    deadacc = f.dead;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vsmask) : "s"(f.smask));
  }
  VRPMS_DEV void reset(const FastSplit& f) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      sa[i].init(f);
      wprev[i] = 0;
    }
  }
  // E entry of the customer pair v_perm laid out as u16 halves; the table's
  // LDS base rides in the dot's accumulator, so the read needs no add.
  VRPMS_DEV uint64_t gat(uint32_t pair) const {
    const uint32_t addr = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, pair), w8, ebase, false);
    return *(lds_u64*)(uintptr_t)addr;
  }
  // the four gathers of word wd (wp = the word before it)
  VRPMS_DEV void issue(uint64_t (&g)[ILP][4], const uint32_t (&wd)[ILP],
                       const uint32_t (&wp)[ILP]) const {
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      g[i][0] = gat(__builtin_amdgcn_perm(wd[i], wp[i], kSel30));
      g[i][1] = gat(__builtin_amdgcn_perm(wd[i], wd[i], kSel01));
      g[i][2] = gat(__builtin_amdgcn_perm(wd[i], wd[i], kSel12));
      g[i][3] = gat(__builtin_amdgcn_perm(wd[i], wd[i], kSel23));
    }
  }
  VRPMS_DEV void steps(const uint64_t (&g)[ILP][4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        if constexpr (CY) split_step_carry(sa[i], g[i][q], vsmask, kinc);
        else split_step_fast(sa[i], g[i][q], vsmask, kinc);
      }
  }
  // The exact split of one tour (fleet limit, A10 separators), word by word
  // (word(w) returns tour word w): the slow path for a chain whose fast walk
  // met the fleet limit.
  template <class WordAt>
  VRPMS_DEV TourCost redo_exact(const FastSplit& f, int n, WordAt word) const {
    return exact_split(
        f, n, [&](int q) { return (word(q >> 2) >> (8 * (q & 3))) & 0xffu; },
        [&](uint32_t a, uint32_t b) { return gat(a | (b << 16)); });
  }
  // next word's address math (perm + dot2) interleaved into this word's
  // split chain, each ds_read well after its dot2
  VRPMS_DEV static void interleave() {
#if VRPMS_IL_VALU > 0
#pragma unroll
    for (int q = 0; q < 4 * ILP; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x2, VRPMS_IL_VALU, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#endif
  }
  // a partial last word of rem (1..3) customers
  VRPMS_DEV void partial(const uint32_t (&x)[ILP], int rem) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      const uint32_t sel[3] = {kSel30, kSel01, kSel12};
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q < rem)
          split_step(sa[i], gat(__builtin_amdgcn_perm(x[i], q ? x[i] : wprev[i], sel[q])), vsmask,
                     kinc, deadacc);
      wprev[i] = x[i];
    }
  }
};

VRPMS_DEV void store_cost(const TourCost& tc, int64_t c, uint64_t* keys, int32_t* sums,
                          int32_t* maxs, int32_t* unv) {
  keys[c] = tc.key;
  if (sums) sums[c] = tc.sum;
  if (maxs) maxs[c] = tc.max;
  if (unv) unv[c] = tc.unv;
}

}  // namespace vrpms
