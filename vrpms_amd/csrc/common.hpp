// Shared device helpers for the vrpms gfx950 library.
//
// Everything here is integer arithmetic except the SA acceptance test, which
// uses the deterministic exp2 below (IEEE basic ops only, built with
// -ffp-contract=off) so that the CPU oracle reproduces it bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VRPMS_DEV __device__ __forceinline__

namespace vrpms {

constexpr int kWave = 64;                 // CDNA wavefront width (never 32)

// Native 16-byte vector (HIP's uint4 is a union-wrapped struct that can
// defeat scalar replacement and push register arrays to scratch).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kKeyClamp = (1u << 28) - 1;
constexpr uint32_t kUnvClamp = 255;

// unv<<56 | min(P,2^28-1)<<28 | min(S,2^28-1).
VRPMS_DEV uint64_t pack_key(uint32_t unv, uint32_t primary, uint32_t secondary) {
  unv = unv < kUnvClamp ? unv : kUnvClamp;
  primary = primary < kKeyClamp ? primary : kKeyClamp;
  secondary = secondary < kKeyClamp ? secondary : kKeyClamp;
  return ((uint64_t)unv << 56) | ((uint64_t)primary << 28) | (uint64_t)secondary;
}

// A8 with the objective selector: 0 = sum first, 1 = max first.
VRPMS_DEV uint64_t cvrp_key(uint32_t unv, uint32_t dsum, uint32_t dmax, int objective) {
  return objective ? pack_key(unv, dmax, dsum) : pack_key(unv, dsum, dmax);
}

// Philox4x32-10 (Salmon et al. SC'11), Random123 constants.
struct u32x4 { uint32_t x, y, z, w; };

VRPMS_DEV u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                       uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    // one 32x32->64 multiply per product (v_mad_u64_u32) instead of a
    // v_mul_lo_u32 + v_mul_hi_u32 pair: same bits, half the multiplies
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return {c0, c1, c2, c3};
}

// Wave64 min over uint64 via cross-lane shuffles (xor butterfly, 6 steps).
VRPMS_DEV uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, kWave);
    v = o < v ? o : v;
  }
  return v;
}

// Lexicographic (key, idx) min across the wave.
VRPMS_DEV void wave_argmin(uint64_t& key, uint64_t& idx) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t ok = __shfl_xor(key, off, kWave);
    const uint64_t oi = __shfl_xor(idx, off, kWave);
    const bool take = ok < key || (ok == key && oi < idx);
    key = take ? ok : key;
    idx = take ? oi : idx;
  }
}

// Wave64 min over uint32 with every lane active, returned wave-uniform (SGPR):
// three DPP steps reduce each 16-lane row in VALU (xor 1, xor 2 inside quads,
// then the half-row and row mirrors), and four v_readlane + s_min combine the
// rows -- no LDS round trip, unlike a 6-step ds_bpermute butterfly.
VRPMS_DEV uint32_t wave_min_u32_uniform(uint32_t v) {
  auto step = [](uint32_t x, int ctrl) -> uint32_t {
    uint32_t o = 0;
    switch (ctrl) {  // the DPP control must be an immediate
      case 0: o = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false); break;   // quad [1,0,3,2]
      case 1: o = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false); break;   // quad [2,3,0,1]
      case 2: o = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false); break;  // row_half_mirror
      default: o = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false); break; // row_mirror
    }
    return min(x, o);
  };
  v = step(v, 0);
  v = step(v, 1);
  v = step(v, 2);
  v = step(v, 3);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return min(min(r0, r1), min(r2, r3));
}

// Wave64 OR over uint32 with every lane active, returned wave-uniform: the
// same DPP row reduction as wave_min_u32_uniform, rows combined in SGPRs.
VRPMS_DEV uint32_t wave_or_u32_uniform(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) | (uint32_t)__builtin_amdgcn_readlane((int)v, 16) |
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Lexicographic (key, lane) argmin with every lane active, both wave-uniform:
// the same DPP row reduction on the 64-bit key (two dword moves per step),
// the row minima combined in SGPRs, then the lowest lane holding the minimum
// from a ballot.  Same result as wave_argmin(key, lane) without ds_bpermute.
VRPMS_DEV uint64_t wave_argmin_lane(uint64_t key, int& who) {
  uint64_t v = key;
  auto take = [&](uint32_t olo, uint32_t ohi) {
    const uint64_t o = ((uint64_t)ohi << 32) | olo;
    v = o < v ? o : v;
  };
#define VRPMS_DPP_MIN64(ctrl)                                                        \
  take((uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, ctrl, 0xF, 0xF, false), \
       (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), ctrl, 0xF, 0xF, false))
  VRPMS_DPP_MIN64(0xB1);   // quad [1,0,3,2]
  VRPMS_DPP_MIN64(0x4E);   // quad [2,3,0,1]
  VRPMS_DPP_MIN64(0x141);  // row_half_mirror
  VRPMS_DPP_MIN64(0x140);  // row_mirror
#undef VRPMS_DPP_MIN64
  uint64_t m = ~0ull;
#pragma unroll
  for (int row = 0; row < 4; ++row) {
    const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 16 * row) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 16 * row);
    m = r < m ? r : m;
  }
  who = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(key == m));
  return m;
}

// x % d, exact, without the ~130-instruction integer division routine (most
// of it scalar, which a CU's many wavefronts then queue on): for 2^20 <= d <
// 2^62 the quotient is below 2^44, so one IEEE f64 division estimates it
// within +-1 (relative error ~3 * 2^-53), and the remainder is corrected in
// 64-bit integers.  Checked against % on 2e8 random / edge pairs (x near
// 2^64, d near 2^20 and 2^56, x near multiples of d) with the same IEEE
// arithmetic on the host.
VRPMS_DEV uint64_t umod64(uint64_t x, uint64_t d) {
  if (d < (1ull << 20) || d >= (1ull << 62)) return x % d;
  const uint64_t q = (uint64_t)((double)x / (double)d);
  int64_t r = (int64_t)(x - q * d);
  r = r < 0 ? r + (int64_t)d : r;
  r = r < 0 ? r + (int64_t)d : r;
  r = (uint64_t)r >= d ? r - (int64_t)d : r;
  r = (uint64_t)r >= d ? r - (int64_t)d : r;
  return (uint64_t)r;
}

VRPMS_DEV uint64_t readlane_u64(uint64_t v, int src) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
}

// Inclusive wave64 prefix sum of a uint64 with every lane active, in VALU:
// Hillis-Steele inside each 16-lane row by DPP row_shr 1, 2, 4, 8 (lanes
// shifted in from outside the row read 0), then the row totals (lanes 15, 31,
// 47 by v_readlane) added to the rows above them.  Returns the wave total,
// wave-uniform.  Same sums as a 6-step __shfl_up scan, no LDS round trips.
VRPMS_DEV uint64_t wave_scan_add_u64(uint64_t& v) {
#define VRPMS_ROW_SHR(k)                                                                          \
  {                                                                                             \
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x110 + k, 0xF, \
                                                              0xF, true);                       \
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32),       \
                                                              0x110 + k, 0xF, 0xF, true);       \
    v += ((uint64_t)hi << 32) | lo;                                                             \
  }
  VRPMS_ROW_SHR(1)
  VRPMS_ROW_SHR(2)
  VRPMS_ROW_SHR(4)
  VRPMS_ROW_SHR(8)
#undef VRPMS_ROW_SHR
  const uint64_t s0 = readlane_u64(v, 15), s1 = readlane_u64(v, 31);
  const uint64_t s2 = readlane_u64(v, 47), s3 = readlane_u64(v, 63);
  const int row = (int)(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) >> 4);
  v += (row >= 1 ? s0 : 0ull) + (row >= 2 ? s1 : 0ull) + (row >= 3 ? s2 : 0ull);
  return s0 + s1 + s2 + s3;
}

// Order this wavefront's LDS (and global) accesses before / after this point
// across its lanes (a wave's own memory operations need no workgroup barrier).
VRPMS_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// x of lane `src` (a wave-uniform index) broadcast through v_readlane.
VRPMS_DEV int wave_bcast(int x, int src) { return __builtin_amdgcn_readlane(x, src); }

}  // namespace vrpms
