// Headline scoring kernels, second generation: eval_cvrp_words2 (word-
// interleaved tours) and eval_cvrp_rows2 (the API's row-major uint8 tours).
//
// Contract: uniform-fleet CVRP with the
// biased prefix-ret matrix E (u64 [N][N], split.hpp) resident in LDS, one
// lane per candidate, bit-exact keys.  What changes is the instruction
// budget per customer (the kernels are LDS-gather / VALU issue bound,
// DESIGN.md §4):
//
//   * gather address in 2 VALU: v_perm_b32 lays the customer pair (a, b) out
//     as two u16 halves, v_dot2_u32_u16 against (8N, 8) gives the byte
//     offset a*8N + 8b directly -- the cross-word pair (last of the previous
//     word, first of this one) costs the same because v_perm takes two words
//     (was: byte extract, 24-bit multiply, shift, add);
//   * route closure in 2 VALU: v_and_or_b32 builds (acc & smask) | kinc with
//     smask held in a VGPR (gfx9 VOP3 reads one SGPR), then one cndmask;
//   * two candidates per lane (ILP = 2): two independent split chains hide
//     each other's gather latency, one 1024-lane workgroup per CU;
//   * the next word's address math is interleaved into the current word's
//     split chain (sched_group_barrier), so ds_reads issue well before use.
//
// eval_cvrp_rows2 reads the row-major layout directly: a 1024 * ILP-row tile
// is staged through LDS CW words at a time (coalesced 4*CW-byte row
// segments, register prefetch of the next chunk), and each lane then walks
// its ILP rows out of LDS with conflict-free ds_read_b32 (odd row stride
// CW + 1).  (Reading the rows in place -- one-dword or 16-byte loads per
// lane, no staging -- was measured at 10.3 and 12.5-16.0 G evals/s: each
// wave load touches ~50 128-B lines and the address path, not the LDS,
// bounds it; tools/rows_ab.py)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "common.hpp"
#include "ctx.hpp"
#include "split.hpp"
#include "chains.hpp"
#include "words.hpp"

namespace vrpms {

template <int R, int ILP, int LA, bool CY>
__global__ __launch_bounds__(1024) void eval_cvrp_words2(WordsArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  stage_table(a.f.pack, a.f.N, smem);
  WordChains<ILP, CY> ch;
  ch.setup(a.f, smem);
  const int64_t C = a.C;
  const int n = a.n, nw = (n + 3) >> 2, nfull = n >> 2;
  constexpr int SPAN = 1024 * ILP;  // candidates per workgroup pass
  const int64_t stride = (int64_t)gridDim.x * SPAN;
  const int nblk = nfull / R;  // blocks of R full words: the fast loop

  for (int64_t c0 = blockIdx.x * (int64_t)SPAN; c0 < C; c0 += stride) {
    // a lane's i-th candidate is c0 + tid + 1024 i (re-pointed at its first
    // one when past the end: computed, never stored).  Word w of every
    // candidate of this pass lives at row(w) = words + w*C + c0 (uniform,
    // SGPR) plus the lane's 32-bit offset.
    uint32_t lane[ILP];
    bool live[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      live[i] = c0 + threadIdx.x + 1024 * i < C;
      lane[i] = live[i] ? threadIdx.x + 1024u * i : threadIdx.x;
    }
    if (!live[0]) continue;
    const uint32_t* row = a.words + c0 * a.cstride;
    const int64_t wstride = a.wstride;
    // the lane's byte offset from the uniform row pointer: a buffer load
    // with the row in an SGPR descriptor (advanced by SALU) and a constant
    // 32-bit VGPR offset, so a load costs no address VALU
    uint32_t loff[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) loff[i] = lane[i] * a.cstride * 4u;
    auto ld = [&](const uint32_t* r, int i) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint32_t*>(r), (short)0, 0x7fffffff, 0x00020000);
      return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, loff[i], 0, 0);
    };
    uint32_t ring[ILP][R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) ring[i][u] = u < nw ? ld(row, i) : 0u;
      row += wstride;
    }
    ch.reset(a.f);
    // software pipeline: the gathers of word w + LA are issued before the
    // split steps of word w consume theirs
    uint64_t e[ILP][4], e1[ILP][4];
    if (nblk > 0) {
      uint32_t w0[ILP], w1[ILP];
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        w0[i] = ring[i][0];
        w1[i] = ring[i][1];
      }
      ch.issue(e, w0, ch.wprev);
      if constexpr (LA == 2) ch.issue(e1, w1, w0);
    }
    // one word: refill its ring slot, issue the gathers of word w + LA, step
    auto word = [&](int u, bool refill, bool has_next) {
      uint32_t wd[ILP], wn[ILP], wp[ILP];
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        wd[i] = ring[i][u];
        if (refill) ring[i][u] = ld(row, i);  // word w + R
      }
      if (refill) row += wstride;
      uint64_t f[ILP][4];
      if (has_next) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
          wn[i] = ring[i][(u + LA) % R];
          wp[i] = LA == 1 ? wd[i] : ring[i][(u + 1) % R];
        }
        ch.issue(f, wn, wp);
      }
      ch.interleave();
      ch.steps(e);
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        ch.wprev[i] = wd[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if constexpr (LA == 2) {
            e[i][q] = e1[i][q];
            if (has_next) e1[i][q] = f[i][q];
          } else if (has_next) {
            e[i][q] = f[i][q];
          }
        }
      }
    };
    for (int b = 0; b + 1 < nblk; ++b) {
#pragma unroll
      for (int u = 0; u < R; ++u) word(u, true, true);
    }
    if (nblk > 0) {
#pragma unroll
      for (int u = 0; u < R; ++u) word(u, false, u + LA < R);  // last block: no refills
    }
    // ragged tail (n not a multiple of 4R): word by word, the last one partial
    for (int w = nblk * R; w < nw; ++w) {
      const int rem = min(4, n - 4 * w);  // uniform
      const uint32_t* rw = a.words + c0 * a.cstride + (int64_t)w * wstride;
      uint32_t x[ILP];
#pragma unroll
      for (int i = 0; i < ILP; ++i) x[i] = ld(rw, i);
      if (rem == 4) {
        ch.issue(e, x, ch.wprev);
        ch.steps(e);
#pragma unroll
        for (int i = 0; i < ILP; ++i) ch.wprev[i] = x[i];
      } else {
        ch.partial(x, rem);
      }
    }
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      const int64_t c = c0 + threadIdx.x + 1024 * i;
      if (!live[i]) continue;
      // a walk that met the fleet limit is re-walked exactly
      const TourCost tc = (int32_t)ch.sa[i].dsum < 0
          ? ch.redo_exact(a.f, n, [&](int w) {
              return a.words[(int64_t)w * wstride + c * (int64_t)a.cstride];
            })
          : ch.sa[i].finish(a.f, n);
      store_cost(tc, c, a.keys, a.sums, a.maxs, a.unv);
    }
  }
}

// Row-major tours: tiles of 1024 * ILP rows, 64 * ILP rows per wave (rows l
// + 64 i of the wave's slice on lane l), staged through a wave-private LDS
// slice CW words per row at a time.  Wave-private staging needs no
// workgroup barrier: the 16 waves drift apart, so one wave's chunk
// transition (prefetch wait, LDS store, pipeline refill) overlaps the
// others' gathers.  (ILP, CW) trades chunk count against candidates per
// lane within the LDS left beside the packed matrix: (2, 8) = 2048-row tiles
// of 8-word chunks, (1, 16) = 1024-row tiles of 16-word chunks.
template <int CW, int ILP>
__global__ __launch_bounds__(1024) void eval_cvrp_rows2(RowsArgs a) {
  constexpr int RS = CW + 1;        // LDS row stride in dwords: odd, so b32 reads are conflict-free
  constexpr int WR = 64 * ILP;      // rows per wave
  constexpr int TR = 1024 * ILP;    // rows per tile
  constexpr int LPT = ILP * CW;     // staging dwords per lane per chunk
  constexpr int RPJ = 64 / CW;      // wave-slice rows per staging step
  static_assert(64 % CW == 0, "CW must divide 64");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int N = a.f.N;
  stage_table(a.f.pack, N, smem);
  const uint32_t e16 = ((uint32_t)N * N * 8 + 15u) & ~15u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63u;
  uint32_t* T = reinterpret_cast<uint32_t*>(smem + e16) + wave * WR * RS;
  WordChains<ILP> ch;
  ch.setup(a.f, smem);
  const int64_t C = a.C;
  const int n = a.n, nw = (n + 3) >> 2, nfull = n >> 2;
  const int nchunks = (nw + CW - 1) / CW;
  const int fullch = nfull / CW;  // chunks made of full words only
  const uint32_t ldw = (uint32_t)a.ld >> 2;
  // staging map: dword l + 64 j of a chunk is word l % CW of slice row
  // l / CW + j * RPJ; CW consecutive lanes read one 4*CW-byte row segment.
  // Addresses are a uniform (SGPR) base per j plus one 32-bit lane offset.
  const uint32_t r0 = l / CW, wl = l % CW;
  const int64_t tstride = (int64_t)gridDim.x * TR;
  uint32_t pf[LPT];
  // Chunk k of the wave's slice starting at row t, through a buffer
  // resource bounded at row C: rows past C (ragged last tile) read as 0 with
  // no fault and no branch; words past the tour are never used.
  const uint32_t lane_off = (r0 * ldw + wl) * 4;
  auto load_chunk = [&](int64_t t, int k) {
    // (wave-uniform values only: readfirstlane keeps the descriptor in SGPRs)
    const int64_t rows = t < C ? C - t : 0;
    const int nrec = __builtin_amdgcn_readfirstlane(rows < WR ? (int)rows * a.ld : WR * a.ld);
    const int64_t tb = t < C ? t : 0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(a.perms) + tb * (int64_t)a.ld, (short)0, nrec, 0x00020000);
#pragma unroll
    for (int j = 0; j < LPT; ++j)
      pf[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
          rs, lane_off + (uint32_t)(k * CW * 4 + j * RPJ * a.ld), 0, 0);
  };
  const uint32_t toff = (uint32_t)(uintptr_t)(lds_uc*)T + l * RS * 4;
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  // word j of the lane's row i of the staged chunk (conflict-free ds_read_b32)
  auto tw = [&](int i, int j) {
    return *(lds_u32*)(uintptr_t)(toff + (uint32_t)(i * 64 * RS * 4 + 4 * j));
  };
  // pf holds chunk k of the current tile: store it into the wave's slice
  // and prefetch what follows (the next chunk, or the next tile's first).
  // One wave owns the slice, and LDS keeps a wave's order, so its reads of
  // the previous chunk precede these stores and the stores precede the
  // reads after them; wave_barrier only pins the compiler's order.
  int64_t t0 = blockIdx.x * (int64_t)TR;
  if (t0 < C && nchunks > 0) load_chunk(t0 + wave * WR, 0);  // n == 0: no tour words at all
  for (; t0 < C; t0 += tstride) {
    ch.reset(a.f);
    for (int k = 0; k < nchunks; ++k) {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < LPT; ++j) T[(r0 + j * RPJ) * RS + wl] = pf[j];
      __builtin_amdgcn_wave_barrier();
      // in flight during the steps below
      if (k + 1 < nchunks) load_chunk(t0 + wave * WR, k + 1);
      else if (t0 + tstride < C) load_chunk(t0 + tstride + wave * WR, 0);
      if (k < fullch) {
        // software pipeline: the gathers of word j + 1 are issued before
        // the split steps of word j consume theirs
        uint64_t e[ILP][4];
        uint32_t cur[ILP];
#pragma unroll
        for (int i = 0; i < ILP; ++i) cur[i] = tw(i, 0);
        ch.issue(e, cur, ch.wprev);
#pragma unroll
        for (int j = 0; j < CW; ++j) {
          uint64_t f[ILP][4];
          uint32_t nx[ILP];
          if (j + 1 < CW) {
#pragma unroll
            for (int i = 0; i < ILP; ++i) nx[i] = tw(i, j + 1);
            ch.issue(f, nx, cur);
          }
          ch.steps(e);
#pragma unroll
          for (int i = 0; i < ILP; ++i) {
            ch.wprev[i] = cur[i];
            if (j + 1 < CW) {
              cur[i] = nx[i];
#pragma unroll
              for (int q = 0; q < 4; ++q) e[i][q] = f[i][q];
            }
          }
        }
      } else {
        // last chunk: full words, then the partial one (uniform guards)
#pragma unroll
        for (int j = 0; j < CW; ++j) {
          const int w = k * CW + j;
          uint32_t cur[ILP];
#pragma unroll
          for (int i = 0; i < ILP; ++i) cur[i] = w < nw ? tw(i, j) : 0u;
          if (w < nfull) {
            uint64_t g[ILP][4];
            ch.issue(g, cur, ch.wprev);
            ch.steps(g);
#pragma unroll
            for (int i = 0; i < ILP; ++i) ch.wprev[i] = cur[i];
          } else if (w < nw) {
            ch.partial(cur, n - 4 * w);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      const int64_t c = t0 + wave * WR + l + 64 * i;
      if (c >= C) continue;
      // a walk that met the fleet limit is re-walked exactly
      const TourCost tc = (int32_t)ch.sa[i].dsum < 0
          ? ch.redo_exact(a.f, n, [&](int w) {
              return *reinterpret_cast<const uint32_t*>(a.perms + c * (int64_t)a.ld + 4 * w);
            })
          : ch.sa[i].finish(a.f, n);
      store_cost(tc, c, a.keys, a.sums, a.maxs, a.unv);
    }
  }
}

int launch_words2(const vrpms_ctx* ctx, const WordsArgs& w, int R, hipStream_t s) {
  const Instance& in = ctx->inst;
  const size_t lds = ((size_t)in.N * in.N * 8 + 15) & ~(size_t)15;
  // Auto: two chains per lane (one 1024-lane workgroup per CU), two words of
  // gathers in flight when the matrix is small enough for two workgroups'
  // copies (N <= 101), else one.  Measured on CVRP-100 with the fast split
  // (tools/words_ab.py): ILP2/LA2 36.7, ILP2/LA1 36.2-36.7, ILP1/LA2 35.1,
  // ILP1/LA1 34.0-35.5 G evals/s.  (Before the fast split, at ~2.5 more
  // VALU per customer, ILP1/LA2 with two workgroups per CU led: 32.5 vs 31.6.)
  const bool two_wg = 2 * lds <= ctx->max_lds;
  const int ilp = ctx->opt_words_ilp ? ctx->opt_words_ilp : 2;  // 1: A/B builds only
  const int la = ctx->opt_words_lookahead ? ctx->opt_words_lookahead : (two_wg ? 2 : 1);
  // ILP >= 2 needs > 64 VGPRs: one 1024-lane workgroup per CU; ILP1 fits two
  const int per_cu = ilp >= 2 ? 1 : (two_wg ? 2 : 1);
  const int64_t blocks = (w.C + 1024 * ilp - 1) / (1024 * ilp);
  const int grid = (int)std::min<int64_t>(blocks, (int64_t)ctx->num_cus * per_cu);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, 1024, lds, s>>>(w);
  };
  // every customer demand >= 1: the fit test rides in the add's carry
  const bool cy = w.f.carry && ctx->opt_split_mode != 3;
  auto pick2 = [&](auto ilp_c, auto la_c, auto cy_c) {
    constexpr int I = decltype(ilp_c)::value, L = decltype(la_c)::value;
    constexpr bool C = decltype(cy_c)::value;
    switch (R) {
      case 4: go(eval_cvrp_words2<4, I, L, C>); break;
      case 5: go(eval_cvrp_words2<5, I, L, C>); break;
      case 6: go(eval_cvrp_words2<6, I, L, C>); break;
      case 7: go(eval_cvrp_words2<7, I, L, C>); break;
      default: go(eval_cvrp_words2<8, I, L, C>); break;
    }
  };
  auto pick = [&](auto ilp_c, auto la_c) {
    if (cy) pick2(ilp_c, la_c, std::true_type{});
    else pick2(ilp_c, la_c, std::false_type{});
  };
  using one = std::integral_constant<int, 1>;
  using two = std::integral_constant<int, 2>;
  const bool la2 = la == 2;
#ifdef VRPMS_AB
  // one candidate per lane: measured slower, built only for A/B runs
  // (VRPMS_OPT_WORDS_ILP = 1 is refused by the shipped library)
  if (ilp == 1) {
    la2 ? pick(one{}, two{}) : pick(one{}, one{});
    VRPMS_HIP(hipGetLastError());
    return VRPMS_OK;
  }
#endif
  la2 ? pick(two{}, two{}) : pick(two{}, one{});
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

int words2_ring(int n) {
  const int nw = (n + 3) / 4;
  int R = 8, waste = 1 << 30;
  for (int r = 8; r >= 4; --r) {
    const int wst = (nw + r - 1) / r * r - nw;
    if (wst < waste) { waste = wst; R = r; }
  }
  return R;
}

// LDS bytes of an eval_cvrp_rows2<CW, ILP> launch on this instance
static size_t rows2_lds(const FastSplit& f, int cw, int ilp) {
  return (((size_t)f.N * f.N * 8 + 15) & ~(size_t)15) + (size_t)1024 * ilp * (cw + 1) * 4;
}

// (CW, ILP) of eval_cvrp_rows2 for this instance: the configuration with the
// fewest chunk transitions per tour that fits the LDS, one candidate per
// lane on ties.  Measured on CVRP-100, 16 Mi tours (tools/rows_ab.py,
// profiles/round2_rows_ab.log): (16, 1) 32.1, (8, 1) 30.4, (8, 2) 23.0,
// (4, 2) 16.6 G evals/s -- fewer chunk restarts beat a second chain per
// lane, which also doubles the staging registers.  VRPMS_OPT_ROWS_CONFIG
// forces one.
static bool rows2_config(const vrpms_ctx* ctx, const FastSplit& f, int n, int* cw, int* ilp) {
  static const int kCfg[][2] = {{8, 2}, {16, 1}, {4, 2}, {8, 1}, {4, 1}};
  const int force = ctx->opt_rows_config;
  if (force > 0) {
    if (force > 5) return false;
    *cw = kCfg[force - 1][0];
    *ilp = kCfg[force - 1][1];
    return rows2_lds(f, *cw, *ilp) <= ctx->max_lds;
  }
  const int nw = (n + 3) / 4;
  int best = -1, best_chunks = 1 << 30;
  for (int c = 0; c < 5; ++c) {
    if (rows2_lds(f, kCfg[c][0], kCfg[c][1]) > ctx->max_lds) continue;
    const int chunks = (nw + kCfg[c][0] - 1) / kCfg[c][0];
    if (chunks < best_chunks || (chunks == best_chunks && kCfg[c][1] < kCfg[best][1])) {
      best = c;
      best_chunks = chunks;
    }
  }
  if (best < 0) return false;
  *cw = kCfg[best][0];
  *ilp = kCfg[best][1];
  return true;
}

int rows2_chunk_words(const vrpms_ctx* ctx, const FastSplit& f, int n) {
  int cw = 0, ilp = 0;
  return rows2_config(ctx, f, n, &cw, &ilp) ? cw : 0;
}

int launch_rows2(const vrpms_ctx* ctx, const RowsArgs& r, hipStream_t s) {
  int cw = 0, ilp = 0;
  if (!rows2_config(ctx, r.f, r.n, &cw, &ilp) || (r.ld & 3) != 0 || ((uintptr_t)r.perms & 3u) != 0)
    return fail(VRPMS_EINVAL, "launch_rows2: tile does not fit LDS or rows unaligned");
  const size_t lds = rows2_lds(r.f, cw, ilp);
  const int64_t tiles = (r.C + 1024 * ilp - 1) / (1024 * ilp);
  const int grid = (int)std::min<int64_t>(tiles, (int64_t)ctx->num_cus);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, 1024, lds, s>>>(r);
  };
  if (cw == 8 && ilp == 2) go(eval_cvrp_rows2<8, 2>);
  else if (cw == 16) go(eval_cvrp_rows2<16, 1>);
  else if (cw == 4 && ilp == 2) go(eval_cvrp_rows2<4, 2>);
  else if (cw == 8) go(eval_cvrp_rows2<8, 1>);
  else go(eval_cvrp_rows2<4, 1>);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

}  // namespace vrpms
