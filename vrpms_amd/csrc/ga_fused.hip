// Fused GA island kernel: one 1024-lane workgroup per island runs whole
// generations without leaving the CU (the reference's GA slot,
// api/vrp/ga/index.py:48-53, knobs api/parameters.py:18-23).
//
// Same trajectory as the three-kernel path of vrpms_ga_generation
// (ga_breed_kernel -> eval_cvrp_words2 -> ga_select_kernel, oracle/search.py
// ga_generation): binary tournaments, OX1, Philox-gated mutation, (mu +
// lambda) survivors by (key, index).  What changes is where the data lives:
//
//   * the packed prefix-ret matrix E, the island's parents AND children
//     (2P uint8 rows) and every key sit in LDS for the whole call;
//   * survivors are never copied: slot i of the population points at one
//     of the 2P rows (prow), and the next children are written into the P
//     rows no survivor holds (crow: the selection hands over the rows of the
//     pairs it drops);
//   * children are scored in place by the headline kernel's split step
//     (chains.hpp: v_perm + v_dot2 gather addressing, branch-free split,
//     exact re-walk of the rare lanes that meet the fleet limit);
//   * a mutation is folded into the child's OX1 writes (each gene goes to
//     the position the move sends its OX1 position to), and the genes taken
//     from A are marked with a per-child stamp instead of a cleared bitmap:
//     per child one pass over A's span and one over B, no barrier pass.
//
// The launch count per call drops from 3 per generation to 1, and no tour
// crosses HBM between generations.
#include <hip/hip_runtime.h>

#ifdef VRPMS_GA_PROF
// phase cycle counters per island (A/B builds only: tools/ga_prof.py)
// [island][0..3]: phase cycles; [4096 * 4 + island]: children re-walked
// exactly (met the fleet limit); [4096 * 5 + island]: cycles of the
// selection up to merge_select's run-sort barrier
namespace vrpms {
__device__ unsigned long long g_ga_prof[6 * 4096];
}
#define VRPMS_MS_MARK()                                                                \
  do {                                                                                 \
    if (threadIdx.x == 0) g_ga_prof[5 * 4096 + blockIdx.x] += wall_clock64();         \
  } while (0)
#endif

#include <algorithm>
#include <type_traits>

#include "chains.hpp"
#include "common.hpp"
#include "ctx.hpp"
#include "sort.hpp"
#include "split.hpp"
#include "tour.hpp"

namespace vrpms {

// children bred together per wavefront (each on its own stamp array)
#ifndef VRPMS_GA_NC
#define VRPMS_GA_NC 2
#endif

#ifdef VRPMS_GA_PROF
#define GA_T(k)                                                                        \
  do {                                                                                 \
    __syncthreads();                                                                   \
    if (threadIdx.x == 0) {                                                            \
      const unsigned long long now = wall_clock64();                                   \
      g_ga_prof[4 * blockIdx.x + (k)] += now - t_last;                                 \
      t_last = now;                                                                    \
    }                                                                                  \
  } while (0)
#else
#define GA_T(k) \
  do {          \
  } while (0)
#endif

struct GaFusedArgs {
  FastSplit f;
  int islands, pop, n, gens, M;
  uint32_t pmut, seed_lo, seed_hi;
  uint64_t gen0;
  uint32_t rs;  // LDS bytes per tour row (multiple of 4, rs / 4 odd)
  uint32_t off_rows, off_pk, off_ck, off_prow, off_crow, off_sk, off_si, off_used, off_sink;
  uint32_t off_rk, off_ri;  // child runs of merge_select
  uint16_t* pop_tours;  // [islands][pop][n] in/out
  uint64_t* pop_keys;   // [islands][pop] in/out
};

struct GaFusedLayout {
  size_t bytes;
  GaFusedArgs a;
};

static size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS carve of the fused kernel for (N, n, P); bytes > max_lds: does not fit.
static GaFusedLayout ga_fused_layout(int N, int n, int P) {
  GaFusedLayout L{};
  uint32_t rs = ((uint32_t)n + 3u) & ~3u;
  if (((rs / 4) & 1u) == 0) rs += 4;  // odd dword stride: rows spread over the banks
  int M = 1;
  while (M < 2 * P) M <<= 1;
  size_t off = al16((size_t)N * N * 8);
  GaFusedArgs& a = L.a;
  a.rs = rs;
  a.M = M;
  a.off_rows = (uint32_t)off;   off = al16(off + (size_t)2 * P * rs);
  a.off_pk = (uint32_t)off;     off = al16(off + (size_t)P * 8);
  a.off_ck = (uint32_t)off;     off = al16(off + (size_t)P * 8);
  a.off_prow = (uint32_t)off;   off = al16(off + (size_t)P * 2);
  a.off_crow = (uint32_t)off;   off = al16(off + (size_t)P * 4);  // two u16 arrays (double buffer)
  a.off_sk = (uint32_t)off;     off = al16(off + (size_t)M * 8);
  a.off_si = (uint32_t)off;     off = al16(off + (size_t)M * 4);
  a.off_used = (uint32_t)off;   off = al16(off + (size_t)16 * VRPMS_GA_NC * N);  // u8 stamp arrays
  a.off_sink = (uint32_t)off;   off = al16(off + 64);  // one sink dword per wave
  const size_t runs = (size_t)64 * ((P + 63) / 64);  // child runs of merge_select
  a.off_rk = (uint32_t)off;     off = al16(off + runs * 8);
  a.off_ri = (uint32_t)off;     off = al16(off + runs * 4);
  L.bytes = off;
  return L;
}

// Tournament of two between members x and y (x = r0 % pop, y = r1 % pop):
// the lower (key, index) wins (as ga_breed_kernel).
VRPMS_DEV int tourney2_xy(const uint64_t* keys, int x, int y) {
  const uint64_t kx = keys[x], ky = keys[y];
  return (ky < kx || (ky == kx && y < x)) ? y : x;
}

// H: 64-position slots per lane, ceil(n / 64)
// CY: every customer demand >= 1, so the scoring walk's fit test is the
// add's carry (split_step_carry, one VALU fewer per customer)
template <int H, bool CY>
__global__ __launch_bounds__(1024) void ga_fused_kernel(GaFusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int P = a.pop, n = a.n, island = blockIdx.x;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t rs = a.rs;
  uint8_t* rows = smem + a.off_rows;
  uint64_t* pk = reinterpret_cast<uint64_t*>(smem + a.off_pk);
  uint64_t* ck = reinterpret_cast<uint64_t*>(smem + a.off_ck);
  uint16_t* prow = reinterpret_cast<uint16_t*>(smem + a.off_prow);
  // crow[i]: the LDS row child i is bred into; the selection writes the
  // next generation's (the rows of the pairs it drops) into crow_next
  uint16_t* crow = reinterpret_cast<uint16_t*>(smem + a.off_crow);
  uint16_t* crow_next = crow + P;
  uint64_t* sk = reinterpret_cast<uint64_t*>(smem + a.off_sk);
  uint32_t* si = reinterpret_cast<uint32_t*>(smem + a.off_si);
  // mk[g] == the current child's stamp: gene g is in the child's A[lo..hi].
  // u8 stamps: an array spans N / 4 dwords, so a wave's 64 lookups at random
  // genes fall in at most 64 distinct dwords -- distinct banks or one
  // address, no bank conflicts; the arrays are cleared before the stamps wrap
  uint8_t* mk = smem + a.off_used + wave * (uint32_t)a.f.N;
  // the breed's sink: a dword per lane in sk (dead until the selection) when
  // it is large enough, so the sink stores of a half-wave hit 32 distinct
  // banks; else one shared dword per wave
  uint8_t* sink = a.M * 8 >= 16 * 256 ? reinterpret_cast<uint8_t*>(sk) + wave * 256 + lane * 4
                                      : smem + a.off_sink + 4 * wave;
  uint16_t* gpop = a.pop_tours + (int64_t)island * P * n;
  uint64_t* gkeys = a.pop_keys + (int64_t)island * P;

  // rows zeroed (tour tails stay 0 for the word reads), parents loaded
  for (uint32_t i = threadIdx.x; i < (uint32_t)P * rs / 2; i += blockDim.x)
    reinterpret_cast<uint32_t*>(rows)[i] = 0u;
  stage_table(a.f.pack, a.f.N, smem);  // ends with a barrier
  // a wavefront per row (no 64-bit division per element)
  for (int i = wave; i < P; i += (int)(blockDim.x >> 6))
    for (int q = lane; q < n; q += 64) rows[(uint32_t)i * rs + q] = (uint8_t)gpop[(int64_t)i * n + q];
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    prow[i] = (uint16_t)i;
    crow[i] = (uint16_t)(P + i);
    pk[i] = gkeys[i];
  }
  auto clear_stamps = [&]() {
    for (int i = threadIdx.x; i < 4 * VRPMS_GA_NC * a.f.N; i += blockDim.x)  // 16 NC N bytes
      reinterpret_cast<uint32_t*>(smem + a.off_used)[i] = 0u;
  };
  clear_stamps();
  __syncthreads();
  // survivors leave every generation ascending by (key, slot); the parents
  // handed in usually are too (the previous call's output), and then the
  // selection merges instead of sorting
  bool sorted_parents;
  {
    int bad = 0;
    for (int i = 1 + threadIdx.x; i < P; i += blockDim.x) bad |= pk[i - 1] > pk[i] ? 1 : 0;
    sorted_parents = __syncthreads_or(bad) == 0;
  }
  const int cpw = (P + 15) / 16;  // children per wavefront per generation
  int gclr = 0;                   // generation of the last stamp clear
  // The Philox draws of GB generations are taken in one pass: lane L holds
  // child w + 16 (L % cg) of generation g0 + L / cg (cg = cpw rounded up to a
  // power of two), so a wave's 64 lanes draw for 64 / cg generations at once
  // instead of drawing 16 useful children per pass.  What a draw decides
  // about the population (the tournaments) is still read each generation.
  const int cg = cpw <= 1 ? 1 : 1 << (32 - __builtin_clz((uint32_t)(cpw - 1)));
  const int GB = 64 / cg;
  int b_x0 = 0, b_y0 = 0, b_x1 = 0, b_y1 = 0;  // tournament members (A: x0, y0; B: x1, y1)
  int v_lo = 0, v_hi = 0, v_mut = 0;
  int v_mv = 0;  // the mutation: type | i << 2 | j << 10 (n <= 255)

  WordChains<1, CY> ch;
  ch.setup(a.f, smem);
  const int nfull = n >> 2;
#ifndef VRPMS_GA_SCORE_MINLPW
#define VRPMS_GA_SCORE_MINLPW 64
#endif
  // scoring lanes per wavefront (A/B knob VRPMS_GA_SCORE_MINLPW): 64, so
  // the first P / 64 wavefronts score -- spreading the children over more
  // wavefronts (16 or 32 lanes each) measured slower, the walk being
  // instruction-issue bound (tools/ga_prof.py)
  const int lpw = min(64, max(VRPMS_GA_SCORE_MINLPW, (P + 15) / 16));
#ifdef VRPMS_GA_PROF
  unsigned long long t_last = wall_clock64();
#endif
  for (int g = 0; g < a.gens; ++g) {
    const uint64_t gen = a.gen0 + (uint64_t)g;
    if ((g - gclr + 1) * cpw > 255) {  // this generation's stamps would pass 255
      __syncthreads();
      clear_stamps();
      __syncthreads();
      gclr = g;
    }
    // ---- breed: one child per wavefront at a time --------------------------
    // Lane k of wave w draws everything random about child w + 16k in
    // parallel (two Philox blocks, both tournaments, the OX1 cut points, the
    // mutation): 64 children per wave in one pass instead of 64 serial ones;
    // the blocks for GB generations at a time (above).
    if (g % GB == 0) {
      const int o = lane / cg, child = wave + 16 * (lane % cg);
      if (child < P && g + o < a.gens) {
        const uint64_t gg = gen + (uint64_t)o;
        const uint32_t cid = (uint32_t)(island * P + child);
        const u32x4 r = philox((uint32_t)gg, (uint32_t)(gg >> 32), cid, 0u, a.seed_lo, a.seed_hi);
        const u32x4 r2 = philox((uint32_t)gg, (uint32_t)(gg >> 32), cid, 1u, a.seed_lo, a.seed_hi);
        b_x0 = (int)(r.x % (uint32_t)P);
        b_y0 = (int)(r.y % (uint32_t)P);
        b_x1 = (int)(r.z % (uint32_t)P);
        b_y1 = (int)(r.w % (uint32_t)P);
        v_mut = 0;
        if (n >= 2) {
          int lo = (int)(r2.x % (uint32_t)n), hi = (int)(r2.y % (uint32_t)n);
          v_lo = lo < hi ? lo : hi;
          v_hi = lo < hi ? hi : lo;
          v_mut = r2.z < a.pmut ? 1 : 0;
          if (v_mut) {
            const Move m = decode_move(r2.w, r.x ^ r2.x, r.y ^ r2.y, n);
            v_mv = (int)(m.typ | ((uint32_t)m.i << 2) | ((uint32_t)m.j << 10));
          }
        }
      }
    }
    const int lb = (g % GB) * cg;  // this generation's lanes: lb .. lb + cg - 1
    // per child two broadcast words instead of five: the parents' LDS rows
    // (11 bits each) and the child's row with the OX1 cut points (n <= 255)
    // and the mutation flag (bit 27)
    int v_ab = 0, v_olh = 0;
    {
      const int k = lane - lb, child = wave + 16 * k;
      if (k >= 0 && k < cg && child < P) {
        v_olh = (int)((uint32_t)crow[child] | ((uint32_t)v_lo << 11) | ((uint32_t)v_hi << 19) |
                      ((uint32_t)v_mut << 27));
        v_ab = (int)((uint32_t)prow[tourney2_xy(pk, b_x0, b_y0)] |
                     ((uint32_t)prow[tourney2_xy(pk, b_x1, b_y1)] << 11));
      }
    }
    // Two children of the wave at a time (each with its own stamp array).
    // Lane L owns positions L + 64h (h < H) of the child: it reads parent
    // A's gene there and B's gene at OX1 fill index L + 64h (B from position
    // hi + 1 on, wrapping), both children's reads issued together; then the
    // span genes are written and stamped, B's genes looked up (a wave's LDS
    // operations run in order: no wait between the stamps and the lookups)
    // and compacted by ballot prefix counts.  Fixed H slots, no loops; a
    // mutation is applied afterwards, in place, to the children that mutate.
    // (Issuing the next pair's reads before the current pair's writes
    // measured slower: the breed is issue-bound, not read-latency bound.)
    // lanes holding a position of chunk h (lane + 64 h < n), as a wave mask
    uint64_t vmask[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int rem = n - 64 * h;
      vmask[h] = rem >= 64 ? ~0ull : (rem <= 0 ? 0ull : (1ull << rem) - 1ull);
    }
    auto breed = [&](auto nc_tag, int k) __attribute__((always_inline)) {
      constexpr int NC = decltype(nc_tag)::value;
      uint8_t* out[NC];
      uint8_t* m[NC];
      int lo[NC], hi[NC], filled[NC];
      uint32_t mut[NC];
      uint32_t stamp[NC], ga[NC][H], gb[NC][H];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t ab = (uint32_t)wave_bcast(v_ab, lb + k + c);
        const uint32_t olh = (uint32_t)wave_bcast(v_olh, lb + k + c);
        mut[c] = (olh >> 27) & 1u;
        const uint8_t* A = rows + (ab & 0x7FFu) * rs;
        const uint8_t* B = rows + (ab >> 11) * rs;
        out[c] = rows + (olh & 0x7FFu) * rs;
        m[c] = mk + (uint32_t)((k + c) % VRPMS_GA_NC) * 16u * (uint32_t)a.f.N;
        lo[c] = (int)((olh >> 11) & 0xFFu);
        hi[c] = (int)((olh >> 19) & 0xFFu);
        stamp[c] = 1u + (uint32_t)((g - gclr) * cpw + k + c);
        filled[c] = 0;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          // lanes past the tour read its last position (unused)
          const int q = min(lane + 64 * h, n - 1);
          // (hi + 1 + q) mod n with hi, q < n: the smaller of x and x - n
          // as unsigned (x - n wraps above x exactly when x < n)
          const uint32_t sx = (uint32_t)(hi[c] + 1 + q);
          const uint32_t src = min(sx, sx - (uint32_t)n);
          ga[c][h] = (uint32_t)A[q];
          gb[c][h] = (uint32_t)B[src];
        }
      }
      // every read issued here, before the first write (no sinking into the
      // exec-masked span writes, where each would wait on its own)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int h = 0; h < H; ++h) asm volatile("" : "+v"(ga[c][h]), "+v"(gb[c][h]));
      // OX1: out[lo..hi] = A[lo..hi], those genes stamped; the rest, from
      // position hi+1 (wrapping), are B's genes from B[hi+1] onwards
      // (wrapping) whose stamp is not this child's
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const int q = lane + 64 * h;
          // lanes outside the span store into their sink byte instead of
          // branching around the stores (no exec-mask bookkeeping; -0.1 us
          // per generation against exec-masked stores)
          const bool in = q >= lo[c] && q <= hi[c];
          *(in ? out[c] + q : sink) = (uint8_t)ga[c][h];
          *(in ? m[c] + ga[c][h] : sink) = (uint8_t)stamp[c];
        }
      wave_sync();
      uint32_t st[NC][H];
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int h = 0; h < H; ++h) st[c][h] = m[c][gb[c][h]];  // every lane: no branch
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int h = 0; h < H; ++h) asm volatile("" : "+v"(st[c][h]));
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const bool keep = (lane + 64 * h < n) & (st[c][h] != (stamp[c] & 0xFFu));
          // the compare's own lane mask (v_cmp to an SGPR pair) instead of
          // __ballot(keep), which materialises keep in a VGPR and compares again
          const uint64_t ball =
              __builtin_amdgcn_uicmp(st[c][h], stamp[c] & 0xFFu, 33 /* ICMP_NE */) & vmask[h];
          const int slot = filled[c] + (int)__builtin_amdgcn_mbcnt_hi(
                                           (uint32_t)(ball >> 32),
                                           __builtin_amdgcn_mbcnt_lo((uint32_t)ball, 0u));
          const uint32_t dx = (uint32_t)(hi[c] + 1 + slot);  // mod n, as above
          const uint32_t dst = min(dx, dx - (uint32_t)n);
          // (a kept gene's slot is always < n - (hi - lo + 1): exactly that
          // many of B's genes lie outside A's span, and dst stays in [0, n))
          *(keep ? out[c] + dst : sink) = (uint8_t)gb[c][h];
          filled[c] += __popcll(ball);
        }
      // the mutation, in place: new[q] = old[moved_index(q)] over the window
      // the move touches (the wave's reads finish before its writes)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (mut[c] != 0) {
          const uint32_t w = (uint32_t)wave_bcast(v_mv, lb + k + c);
          const Move mv{w & 3u, (int)((w >> 2) & 0xFFu), (int)(w >> 10)};
          const MoveMap fm = move_map(mv);
          const int w0 = min(mv.i, mv.j), w1 = max(mv.i, mv.j);
          wave_sync();
          uint32_t x[H];
#pragma unroll
          for (int h = 0; h < H; ++h) {
            const int q = min(w0 + lane + 64 * h, w1);
            x[h] = out[c][map_src(fm, q)];
          }
          wave_sync();
#pragma unroll
          for (int h = 0; h < H; ++h)
            if (w0 + lane + 64 * h <= w1) out[c][w0 + lane + 64 * h] = (uint8_t)x[h];
        }
    };
    if (n < 2) {
      for (int k = 0; wave + 16 * k < P; ++k) {
        const uint8_t* A = rows + ((uint32_t)wave_bcast(v_ab, lb + k) & 0x7FFu) * rs;
        uint8_t* out = rows + ((uint32_t)wave_bcast(v_olh, lb + k) & 0x7FFu) * rs;
        for (int q = lane; q < n; q += 64) out[q] = A[q];
      }
    } else {
      int k = 0;
#if VRPMS_GA_NC == 4
      for (; wave + 16 * (k + 3) < P; k += 4) breed(std::integral_constant<int, 4>{}, k);
#endif
      for (; wave + 16 * (k + 1) < P; k += 2) breed(std::integral_constant<int, 2>{}, k);
      if (wave + 16 * k < P) breed(std::integral_constant<int, 1>{}, k);
    }
    __syncthreads();
    GA_T(0);
    // ---- score the P children in place ---------------------------------------
    // the tour words are read a chunk of eight ahead (one wait per chunk,
    // not per word), each word's gathers one word ahead of its split steps
    for (int t = wave * lpw + lane; lane < lpw && t < P; t += 16 * lpw) {
      const uint32_t* rw = reinterpret_cast<const uint32_t*>(rows + (uint32_t)crow[t] * rs);
      ch.reset(a.f);
      constexpr int CW = 8;
      const int last = max(nfull - 1, 0);
      uint32_t cur[CW];
#pragma unroll
      for (int i = 0; i < CW; ++i) cur[i] = rw[min(i, last)];
      uint64_t e[1][4];
      if (nfull > 0) {
        const uint32_t w0[1] = {cur[0]};
        ch.issue(e, w0, ch.wprev);
      }
      // whole chunks whose eight words all have a next word: straight-line
      // code, so each wait is for exactly the gathers it needs
      const int full_chunks = nfull > 0 ? (nfull - 1) / CW : 0;
      int w = 0;
      for (; w < full_chunks * CW; w += CW) {
        uint32_t nxt[CW];
#pragma unroll
        for (int i = 0; i < CW; ++i) nxt[i] = rw[min(w + CW + i, last)];
#pragma unroll
        for (int i = 0; i < CW; ++i) {
          uint64_t nx[1][4];
          const uint32_t wn[1] = {i + 1 < CW ? cur[i + 1] : nxt[0]};
          const uint32_t wc[1] = {cur[i]};
          ch.issue(nx, wn, wc);
          // the next word's four gathers leave before this word's steps (the
          // scheduler would otherwise trail each one a step behind its use)
          __builtin_amdgcn_sched_barrier(0);
          ch.steps(e);
          ch.wprev[0] = cur[i];
#pragma unroll
          for (int x = 0; x < 4; ++x) e[0][x] = nx[0][x];
        }
#pragma unroll
        for (int i = 0; i < CW; ++i) cur[i] = nxt[i];
      }
      // the last 1..8 words
#pragma unroll
      for (int i = 0; i < CW; ++i) {
        if (w + i >= nfull) break;
        uint64_t nx[1][4];
        const bool more = w + i + 1 < nfull;
        const uint32_t wn[1] = {i + 1 < CW ? cur[i + 1] : 0u};
        const uint32_t wc[1] = {cur[i]};
        if (more) ch.issue(nx, wn, wc);
        ch.steps(e);
        ch.wprev[0] = cur[i];
        if (more)
#pragma unroll
          for (int x = 0; x < 4; ++x) e[0][x] = nx[0][x];
      }
      if (n & 3) {
        const uint32_t x[1] = {rw[nfull]};
        ch.partial(x, n & 3);
      }
#ifdef VRPMS_GA_PROF
      if ((int32_t)ch.sa[0].dsum < 0) atomicAdd(&g_ga_prof[4 * 4096 + blockIdx.x], 1ull);
#endif
      ck[t] = (int32_t)ch.sa[0].dsum < 0  // met the fleet limit: exact re-walk
                  ? ch.redo_exact(a.f, n, [&](int w) { return rw[w]; }).key
                  : ch.sa[0].finish(a.f, n).key;
    }
    __syncthreads();
    GA_T(1);
    // ---- (mu + lambda) survivors by (key, index) -----------------------------
    // si receives the survivors' LDS rows (merge_select maps them); with
    // 4P <= 1024 they are written straight over pk / prow
    const bool inplace = sorted_parents && 4 * P <= (int)blockDim.x;
    if (inplace) {
#ifdef VRPMS_GA_PROF
      if (threadIdx.x == 0) g_ga_prof[5 * 4096 + blockIdx.x] -= t_last;
#endif
      merge_select_inplace(pk, prow, ck, crow, crow_next, P,
                           reinterpret_cast<uint64_t*>(smem + a.off_rk),
                           reinterpret_cast<uint32_t*>(smem + a.off_ri), reinterpret_cast<uint32_t*>(sk));
    } else if (sorted_parents) {
#ifdef VRPMS_GA_PROF
      if (threadIdx.x == 0) g_ga_prof[5 * 4096 + blockIdx.x] -= t_last;
#endif
      merge_select(pk, ck, P, reinterpret_cast<uint64_t*>(smem + a.off_rk),
                   reinterpret_cast<uint32_t*>(smem + a.off_ri), sk, si, prow, crow, crow_next);
    } else {
      for (int i = threadIdx.x; i < a.M; i += blockDim.x) {
        sk[i] = i < P ? pk[i] : (i < 2 * P ? ck[i - P] : ~0ull);
        si[i] = (uint32_t)i;
      }
      __syncthreads();
      if (a.M >= 64 && a.M <= 1024) block_sort_pairs_waves(sk, si, a.M);
      else block_sort_pairs(sk, si, a.M);
      sorted_parents = true;
      uint16_t nrow[2] = {0, 0};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + 1024 * k;
        if (i < P) nrow[k] = si[i] < (uint32_t)P ? prow[si[i]] : crow[si[i] - P];
      }
      for (int i = P + threadIdx.x; i < 2 * P; i += blockDim.x)  // the dropped pairs' rows
        crow_next[i - P] = si[i] < (uint32_t)P ? prow[si[i]] : crow[si[i] - P];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + 1024 * k;
        if (i < P) si[i] = nrow[k];
      }
      __syncthreads();
    }
    GA_T(2);
    if (!inplace) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        prow[i] = (uint16_t)si[i];
        pk[i] = sk[i];
      }
      __syncthreads();
    }
    {  // the rows the selection dropped take the next children
      uint16_t* t = crow;
      crow = crow_next;
      crow_next = t;
    }
    GA_T(3);
  }
  for (int i = wave; i < P; i += (int)(blockDim.x >> 6)) {
    const uint32_t src = (uint32_t)prow[i] * rs;
    for (int q = lane; q < n; q += 64) gpop[(int64_t)i * n + q] = rows[src + q];
  }
  for (int i = threadIdx.x; i < P; i += blockDim.x) gkeys[i] = pk[i];
}

// Launch the fused kernel when the island fits the LDS beside the packed
// matrix; returns 1 if launched, 0 if the caller must use the three-kernel
// path, < 0 on error.
int launch_ga_fused(const vrpms_ctx* ctx, const vrpms_ga_params* p, uint16_t* d_pop,
                    uint64_t* d_keys, int n, hipStream_t s) {
  if (ctx->opt_ga_fused == 2) return 0;
  FastSplit f;
  if (n > 255 || p->pop > 1024 || !fast_split_params(ctx, n, &f)) return 0;
  GaFusedLayout L = ga_fused_layout(f.N, n, p->pop);
  if (L.bytes > ctx->max_lds) return 0;
  GaFusedArgs a = L.a;
  a.f = f;
  a.islands = p->islands;
  a.pop = p->pop;
  a.n = n;
  a.gens = p->generations;
  a.pmut = p->pmut;
  a.seed_lo = (uint32_t)p->seed;
  a.seed_hi = (uint32_t)(p->seed >> 32);
  a.gen0 = p->gen0;
  a.pop_tours = d_pop;
  a.pop_keys = d_keys;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.bytes);
    kern<<<p->islands, 1024, L.bytes, s>>>(a);
  };
  const int H = (n + 63) / 64;
  const bool cy = f.carry && ctx->opt_split_mode != 3;
  auto pick = [&](auto cy_tag) {
    constexpr bool C = decltype(cy_tag)::value;
    if (H <= 1) go(ga_fused_kernel<1, C>);
    else if (H == 2) go(ga_fused_kernel<2, C>);
    else if (H == 3) go(ga_fused_kernel<3, C>);
    else go(ga_fused_kernel<4, C>);
  };
  if (cy) pick(std::true_type{});
  else pick(std::false_type{});
  VRPMS_HIP(hipGetLastError());
  return 1;
}

}  // namespace vrpms

#ifdef VRPMS_GA_PROF
extern "C" int vrpms_debug_ga_prof(unsigned long long* out, int count, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vrpms::g_ga_prof), sizeof(unsigned long long) * count) !=
      hipSuccess)
    return -2;
  if (reset) {
    static unsigned long long zero[6 * 4096];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(vrpms::g_ga_prof), zero, sizeof(zero));
  }
  return 0;
}
#endif
