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
//     rows no survivor holds (crow, rebuilt by a ballot compaction);
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

#include <algorithm>
#include <type_traits>

#include "chains.hpp"
#include "common.hpp"
#include "ctx.hpp"
#include "sort.hpp"
#include "split.hpp"
#include "tour.hpp"

namespace vrpms {

#ifdef VRPMS_GA_PROF
// phase cycle counters per island (A/B builds only: tools/ga_prof.py)
__device__ unsigned long long g_ga_prof[4 * 4096];
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
  uint32_t off_rows, off_pk, off_ck, off_prow, off_crow, off_sk, off_si, off_used, off_bits;
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
  a.off_crow = (uint32_t)off;   off = al16(off + (size_t)P * 2);
  a.off_sk = (uint32_t)off;     off = al16(off + (size_t)M * 8);
  a.off_si = (uint32_t)off;     off = al16(off + (size_t)M * 4);
  a.off_used = (uint32_t)off;   off = al16(off + (size_t)32 * N);  // 2 u8 stamp arrays per wave
  a.off_bits = (uint32_t)off;   off = al16(off + ((size_t)2 * P / 32 + 1) * 4);
  const size_t runs = (size_t)64 * ((P + 63) / 64);
  a.off_rk = (uint32_t)off;     off = al16(off + runs * 8);
  a.off_ri = (uint32_t)off;     off = al16(off + runs * 4);
  L.bytes = off;
  return L;
}

// Tournament of two: the lower (key, index) wins (as ga_breed_kernel).
VRPMS_DEV int tourney2(const uint64_t* keys, int pop, uint32_t r0, uint32_t r1) {
  const int x = (int)(r0 % (uint32_t)pop), y = (int)(r1 % (uint32_t)pop);
  const uint64_t kx = keys[x], ky = keys[y];
  return (ky < kx || (ky == kx && y < x)) ? y : x;
}

__global__ __launch_bounds__(1024) void ga_fused_kernel(GaFusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int P = a.pop, n = a.n, island = blockIdx.x;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t rs = a.rs;
  uint8_t* rows = smem + a.off_rows;
  uint64_t* pk = reinterpret_cast<uint64_t*>(smem + a.off_pk);
  uint64_t* ck = reinterpret_cast<uint64_t*>(smem + a.off_ck);
  uint16_t* prow = reinterpret_cast<uint16_t*>(smem + a.off_prow);
  uint16_t* crow = reinterpret_cast<uint16_t*>(smem + a.off_crow);
  uint64_t* sk = reinterpret_cast<uint64_t*>(smem + a.off_sk);
  uint32_t* si = reinterpret_cast<uint32_t*>(smem + a.off_si);
  // mk[g] == the current child's stamp: gene g is in the child's A[lo..hi].
  // u8 stamps: an array spans N / 4 dwords, so a wave's 64 lookups at random
  // genes fall in at most 64 distinct dwords -- distinct banks or one
  // address, no bank conflicts; the arrays are cleared before the stamps wrap
  uint8_t* mk = smem + a.off_used + wave * (uint32_t)a.f.N;
  uint32_t* bits = reinterpret_cast<uint32_t*>(smem + a.off_bits);
  uint16_t* gpop = a.pop_tours + (int64_t)island * P * n;
  uint64_t* gkeys = a.pop_keys + (int64_t)island * P;

  // rows zeroed (tour tails stay 0 for the word reads), parents loaded
  for (uint32_t i = threadIdx.x; i < (uint32_t)P * rs / 2; i += blockDim.x)
    reinterpret_cast<uint32_t*>(rows)[i] = 0u;
  stage_table(a.f.pack, a.f.N, smem);  // ends with a barrier
  for (int64_t e = threadIdx.x; e < (int64_t)P * n; e += blockDim.x) {
    const int i = (int)(e / n), q = (int)(e % n);
    rows[(uint32_t)i * rs + q] = (uint8_t)gpop[e];
  }
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    prow[i] = (uint16_t)i;
    crow[i] = (uint16_t)(P + i);
    pk[i] = gkeys[i];
  }
  auto clear_stamps = [&]() {
    for (int i = threadIdx.x; i < 8 * a.f.N; i += blockDim.x)  // 32 N bytes
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

  WordChains<1> ch;
  ch.setup(a.f, smem);
  const int nfull = n >> 2;
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
    // Lane k of wave w first draws everything random about child w + 16k in
    // parallel (two Philox blocks, both tournaments, the OX1 cut points, the
    // mutation): 64 children per wave in one pass instead of 64 serial ones.
    int v_pa = 0, v_pb = 0, v_lo = 0, v_hi = 0, v_mut = 0, v_mtyp = 0, v_mi = 0, v_mj = 0;
    int v_out = 0;
    {
      const int child = wave + 16 * lane;
      if (child < P) {
        v_out = crow[child];
        const uint32_t cid = (uint32_t)(island * P + child);
        const u32x4 r = philox((uint32_t)gen, (uint32_t)(gen >> 32), cid, 0u, a.seed_lo, a.seed_hi);
        const u32x4 r2 =
            philox((uint32_t)gen, (uint32_t)(gen >> 32), cid, 1u, a.seed_lo, a.seed_hi);
        v_pa = prow[tourney2(pk, P, r.x, r.y)];
        v_pb = prow[tourney2(pk, P, r.z, r.w)];
        if (n >= 2) {
          int lo = (int)(r2.x % (uint32_t)n), hi = (int)(r2.y % (uint32_t)n);
          v_lo = lo < hi ? lo : hi;
          v_hi = lo < hi ? hi : lo;
          v_mut = r2.z < a.pmut ? 1 : 0;
          if (v_mut) {
            const Move m = decode_move(r2.w, r.x ^ r2.x, r.y ^ r2.y, n);
            v_mtyp = (int)m.typ;
            v_mi = m.i;
            v_mj = m.j;
          }
        }
      }
    }
    // Two children of the wave at a time (each with its own stamp array),
    // their A spans, B reads and stamp lookups issued together: the LDS
    // round trips of one child hide behind the other's.
    auto breed = [&](auto nc_tag, int k) __attribute__((always_inline)) {
      constexpr int NC = decltype(nc_tag)::value;
      const uint8_t* A[NC];
      const uint8_t* B[NC];
      uint8_t* out[NC];
      uint8_t* m[NC];
      int lo[NC], hi[NC], mi[NC], mj[NC], rest[NC], filled[NC];
      bool mut[NC];
      uint32_t mtyp[NC], stamp[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        A[c] = rows + (uint32_t)wave_bcast(v_pa, k + c) * rs;
        B[c] = rows + (uint32_t)wave_bcast(v_pb, k + c) * rs;
        out[c] = rows + (uint32_t)wave_bcast(v_out, k + c) * rs;
        m[c] = mk + (uint32_t)((k + c) & 1) * 16u * (uint32_t)a.f.N;
        lo[c] = wave_bcast(v_lo, k + c);
        hi[c] = wave_bcast(v_hi, k + c);
        // the child's mutation (wave-uniform) folded into its writes: the
        // gene OX1 puts at position p goes to the position the move maps p
        // to (the inverse of moved_index), so no copy-and-gather pass follows
        mut[c] = wave_bcast(v_mut, k + c) != 0;
        mtyp[c] = (uint32_t)wave_bcast(v_mtyp, k + c);
        mi[c] = wave_bcast(v_mi, k + c);
        mj[c] = wave_bcast(v_mj, k + c);
        stamp[c] = 1u + (uint32_t)((g - gclr) * cpw + k + c);
        rest[c] = n - (hi[c] - lo[c] + 1);
        filled[c] = 0;
      }
      auto dst_of = [&](int c, int p) __attribute__((always_inline)) -> int {
        if (!mut[c]) return p;
        const int i = mi[c], j = mj[c];
        if (mtyp[c] == kMoveSwap) return p == i ? j : (p == j ? i : p);
        if (mtyp[c] == kMove2Opt) return (p >= i && p <= j) ? i + j - p : p;
        if (i < j) return p == i ? j : ((p > i && p <= j) ? p - 1 : p);
        return p == i ? j : ((p >= j && p < i) ? p + 1 : p);
      };
      // OX1: out[lo..hi] = A[lo..hi]; the rest, from position hi+1
      // (wrapping), are B's genes from B[hi+1] onwards (wrapping) not yet
      // used -- a gene is used when its stamp is this child's (no bitmap to
      // clear)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        for (int q = lo[c] + lane; q <= hi[c]; q += 64) {
          const uint32_t gq = A[c][q];
          out[c][dst_of(c, q)] = (uint8_t)gq;
          m[c][gq] = (uint8_t)stamp[c];
        }
      wave_sync();
      for (int base = 0; base < n; base += 128) {
        uint32_t gq[NC][2];
        bool keep[NC][2];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int q = base + 64 * h + lane;
            int src = hi[c] + 1 + q;
            src = src >= n ? src - n : src;
            gq[c][h] = q < n ? (uint32_t)B[c][src] : 0u;
          }
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            keep[c][h] = base + 64 * h + lane < n && m[c][gq[c][h]] != stamp[c];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint64_t ball = __ballot(keep[c][h]);
            const int slot = filled[c] + __popcll(ball & ((1ull << lane) - 1ull));
            if (keep[c][h] && slot < rest[c]) {
              int dst = hi[c] + 1 + slot;
              dst = dst >= n ? dst - n : dst;
              out[c][dst_of(c, dst)] = (uint8_t)gq[c][h];
            }
            filled[c] += __popcll(ball);
          }
      }
    };
    if (n < 2) {
      for (int k = 0; wave + 16 * k < P; ++k) {
        const uint8_t* A = rows + (uint32_t)wave_bcast(v_pa, k) * rs;
        uint8_t* out = rows + (uint32_t)wave_bcast(v_out, k) * rs;
        for (int q = lane; q < n; q += 64) out[q] = A[q];
      }
    } else {
      int k = 0;
      for (; wave + 16 * (k + 1) < P; k += 2) breed(std::integral_constant<int, 2>{}, k);
      if (wave + 16 * k < P) breed(std::integral_constant<int, 1>{}, k);
    }
    __syncthreads();
    GA_T(0);
    // ---- score the P children in place ---------------------------------------
    for (int t = threadIdx.x; t < P; t += blockDim.x) {
      const uint32_t* rw = reinterpret_cast<const uint32_t*>(rows + (uint32_t)crow[t] * rs);
      ch.reset(a.f);
      uint64_t e[1][4];
      if (nfull > 0) {
        const uint32_t w0[1] = {rw[0]};
        ch.issue(e, w0, ch.wprev);
      }
      for (int w = 0; w < nfull; ++w) {
        const uint32_t cur[1] = {rw[w]};
        uint64_t nx[1][4];
        const bool more = w + 1 < nfull;
        if (more) {
          const uint32_t wn[1] = {rw[w + 1]};
          ch.issue(nx, wn, cur);
        }
        ch.steps(e);
        ch.wprev[0] = cur[0];
        if (more)
#pragma unroll
          for (int x = 0; x < 4; ++x) e[0][x] = nx[0][x];
      }
      if (n & 3) {
        const uint32_t x[1] = {rw[nfull]};
        ch.partial(x, n & 3);
      }
      ck[t] = (int32_t)ch.sa[0].dsum < 0  // met the fleet limit: exact re-walk
                  ? ch.redo_exact(a.f, n, [&](int w) { return rw[w]; }).key
                  : ch.sa[0].finish(a.f, n).key;
    }
    __syncthreads();
    GA_T(1);
    // ---- (mu + lambda) survivors by (key, index) -----------------------------
    if (sorted_parents) {
      merge_select(pk, ck, P, reinterpret_cast<uint64_t*>(smem + a.off_rk),
                   reinterpret_cast<uint32_t*>(smem + a.off_ri), sk, si);
    } else {
      for (int i = threadIdx.x; i < a.M; i += blockDim.x) {
        sk[i] = i < P ? pk[i] : (i < 2 * P ? ck[i - P] : ~0ull);
        si[i] = (uint32_t)i;
      }
      __syncthreads();
      if (a.M >= 64 && a.M <= 1024) block_sort_pairs_waves(sk, si, a.M);
      else block_sort_pairs(sk, si, a.M);
      sorted_parents = true;
    }
    GA_T(2);
    uint16_t nrow[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = threadIdx.x + 1024 * k;
      if (i < P) nrow[k] = si[i] < (uint32_t)P ? prow[si[i]] : crow[si[i] - P];
    }
    for (uint32_t w = threadIdx.x; w <= (uint32_t)(2 * P) / 32; w += blockDim.x) bits[w] = 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = threadIdx.x + 1024 * k;
      if (i < P) {
        prow[i] = nrow[k];
        pk[i] = sk[i];
        atomicOr(&bits[nrow[k] >> 5], 1u << (nrow[k] & 31u));
      }
    }
    __syncthreads();
    // the P rows no survivor holds, in row order, take the next children
    if (wave == 0) {
      const int nwords = (2 * P + 31) / 32;  // <= 64 (P <= 1024)
      uint32_t fr = 0;
      if (lane < nwords) {
        fr = ~bits[lane];
        const int tail = 2 * P - 32 * lane;
        if (tail < 32) fr &= (1u << tail) - 1u;
      }
      const int cnt = __popc(fr);
      int incl = cnt;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off, 64);
        if (lane >= off) incl += o;
      }
      int slot = incl - cnt;
      while (fr) {
        const int b = __ffs((int)fr) - 1;
        crow[slot++] = (uint16_t)(32 * lane + b);
        fr &= fr - 1u;
      }
    }
    __syncthreads();
    GA_T(3);
  }
  for (int64_t e = threadIdx.x; e < (int64_t)P * n; e += blockDim.x) {
    const int i = (int)(e / n), q = (int)(e % n);
    gpop[e] = rows[(uint32_t)prow[i] * rs + q];
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
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(ga_fused_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.bytes);
  ga_fused_kernel<<<p->islands, 1024, L.bytes, s>>>(a);
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
    static unsigned long long zero[4 * 4096];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(vrpms::g_ga_prof), zero, sizeof(zero));
  }
  return 0;
}
#endif
