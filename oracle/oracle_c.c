/* oracle_c.c -- C restatement of oracle/spec.py.  TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (large-batch parity against the HIP library) and by
 * bench.py's cpu_baseline leg ("kind": "port": the reference ships no CPU
 * solver, SURVEY.md §0.1, so this restatement of the frozen Appendix-A spec
 * is the CPU path timed beside the GPU).  Never linked into libvrpms.
 *
 * Semantics follow oracle/spec.py line by line:
 *   eval_tsp   <- spec.eval_tsp   (A4; anchors api/parameters.py:41-43, src/solver.py:24)
 *   eval_cvrp  <- spec.eval_cvrp  (A5-A7 + A10 separators; anchors api/parameters.py:11-12,
 *                                  src/solver.py:24,27)
 *   pack_key   <- spec.pack_key   (A8)
 * Arithmetic is int64 here (the spec uses unbounded ints); the A9 guard
 * keeps every value inside int32 for the device.
 */
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define CLAMP28 ((1ULL << 28) - 1)

static uint64_t pack_key(int64_t unv, int64_t p, int64_t s) {
  uint64_t u = unv > 255 ? 255 : (uint64_t)unv;
  uint64_t pp = (uint64_t)p > CLAMP28 ? CLAMP28 : (uint64_t)p;
  uint64_t ss = (uint64_t)s > CLAMP28 ? CLAMP28 : (uint64_t)s;
  return (u << 56) | (pp << 28) | ss;
}

static inline int64_t edge(const int32_t* D, int H, int N, int64_t t, int a, int b) {
  int64_t h = (t / 60) % H;
  return D[(h * N + a) * (int64_t)N + b];
}

static inline int perm_at(const uint8_t* p8, const uint16_t* p16, int64_t c, int64_t ld, int i) {
  return p8 ? (int)p8[c * ld + i] : (int)p16[c * ld + i];
}

static void eval_tsp(const int32_t* D, int H, int N, int64_t start, const uint8_t* p8,
                     const uint16_t* p16, int64_t c, int64_t ld, int n, int64_t* dur) {
  int64_t t = start;
  int prev = 0;
  for (int i = 0; i < n; ++i) {
    int x = perm_at(p8, p16, c, ld, i);
    t += edge(D, H, N, t, prev, x);
    prev = x;
  }
  t += edge(D, H, N, t, prev, 0);
  *dur = t - start;
}

static void eval_cvrp(const int32_t* D, int H, int N, const int32_t* dem, const int32_t* cap,
                      const int32_t* st, int K, const uint8_t* p8, const uint16_t* p16, int64_t c,
                      int64_t ld, int n, int64_t* dsum, int64_t* dmax, int64_t* unv) {
  int k = 0, prev = 0;
  int64_t load = 0, t = K ? st[0] : 0, s = 0, m = 0, u = 0;
  for (int i = 0; i < n; ++i) {
    int x = perm_at(p8, p16, c, ld, i);
    if (x == 0) { /* A10 separator: close the route, open the next vehicle */
      if (k < K) {
        if (prev != 0) {
          int64_t te = t + edge(D, H, N, t, prev, 0);
          int64_t rd = te - st[k];
          s += rd;
          if (rd > m) m = rd;
        }
        ++k;
        if (k < K) {
          load = 0;
          t = st[k];
          prev = 0;
        }
      }
      continue;
    }
    while (k < K && load + dem[x] > cap[k]) {
      if (prev != 0) {
        int64_t te = t + edge(D, H, N, t, prev, 0);
        int64_t rd = te - st[k];
        s += rd;
        if (rd > m) m = rd;
      }
      ++k;
      if (k < K) {
        load = 0;
        t = st[k];
        prev = 0;
      }
    }
    if (k >= K) {
      ++u;
      continue;
    }
    t += edge(D, H, N, t, prev, x);
    load += dem[x];
    prev = x;
  }
  if (k < K && prev != 0) {
    int64_t te = t + edge(D, H, N, t, prev, 0);
    int64_t rd = te - st[k];
    s += rd;
    if (rd > m) m = rd;
  }
  *dsum = s;
  *dmax = m;
  *unv = u;
}

/* Batched evaluation, OpenMP over candidates.  problem 0 = TSP, 1 = CVRP. */
int oracle_eval_batch(int problem, const int32_t* D, int H, int N, const int32_t* dem,
                      const int32_t* cap, const int32_t* st, int K, int objective,
                      const uint8_t* p8, const uint16_t* p16, int64_t C, int n, int64_t ld,
                      uint64_t* keys, int32_t* sums, int32_t* maxs, int32_t* unvs, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
  for (int64_t c = 0; c < C; ++c) {
    int64_t s, m, u;
    if (problem == 0) {
      eval_tsp(D, H, N, st[0], p8, p16, c, ld, n, &s);
      m = s;
      u = 0;
      keys[c] = pack_key(0, s, 0);
    } else {
      eval_cvrp(D, H, N, dem, cap, st, K, p8, p16, c, ld, n, &s, &m, &u);
      keys[c] = objective ? pack_key(u, m, s) : pack_key(u, s, m);
    }
    if (sums) sums[c] = (int32_t)s;
    if (maxs) maxs[c] = (int32_t)m;
    if (unvs) unvs[c] = (int32_t)u;
  }
  return 0;
}

/* ------------------------------------------------------------------------
 * SA restatement (oracle/search.py sa_run, SURVEY.md §8a' sa_chain_step):
 * per chain and step, `moves` (64 W) Philox-sampled moves are scored, the best
 * (key, lane) is accepted if no worse or if (u >> 8) < threshold(dp, invT).
 * Used as the CPU solver at equal wall time (bench.py "quality") and as a
 * large-size parity check of the GPU SA.  Build with -ffp-contract=off.
 * ---------------------------------------------------------------------- */
typedef struct {
  uint32_t x, y, z, w;
} u32x4;

static u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                    uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
  }
  u32x4 o = {c0, c1, c2, c3};
  return o;
}

typedef struct {
  int typ, i, j;
} move_t;

static move_t decode_move(uint32_t r0, uint32_t r1, uint32_t r2, int n) {
  move_t m;
  m.typ = (int)(r0 % 3u);
  m.i = (int)(r1 % (uint32_t)n);
  m.j = (int)(r2 % (uint32_t)(n - 1));
  if (m.j >= m.i) ++m.j;
  if (m.typ != 2 && m.i > m.j) {
    int t = m.i;
    m.i = m.j;
    m.j = t;
  }
  return m;
}

/* A13 (oracle/spec.py decode_move1): one word split by successive
 * fixed-point multiplications (type, then i, then j') */
static move_t decode_move1(uint32_t x, int n) {
  move_t m;
  uint64_t p = 3ull * x;
  m.typ = (int)(p >> 32);
  p = (uint64_t)(uint32_t)n * (uint32_t)p;
  m.i = (int)(p >> 32);
  p = (uint64_t)(uint32_t)(n - 1) * (uint32_t)p;
  m.j = (int)(p >> 32);
  if (m.j >= m.i) ++m.j;
  if (m.typ != 2 && m.i > m.j) {
    int t = m.i;
    m.i = m.j;
    m.j = t;
  }
  return m;
}

/* A11 (oracle/spec.py decode_move_window): j within `window` of i, for the
 * move types in `types` (A12; 0 = all) */
static move_t decode_move_window(uint32_t r0, uint32_t r1, uint32_t r2, int n, int window,
                                 uint32_t types) {
  if (!types) types = 7u;
  if (window <= 0 || 2 * window + 1 >= n || !((types >> (r0 % 3u)) & 1u))
    return decode_move(r0, r1, r2, n);
  move_t m;
  m.typ = (int)(r0 % 3u);
  m.i = (int)(r1 % (uint32_t)n);
  const int o = (int)(r2 % (uint32_t)(2 * window));
  const int d = o < window ? o - window : o - window + 1;
  m.j = m.i + d;
  if (m.j < 0 || m.j >= n) m.j = m.i - d;
  if (m.typ != 2 && m.i > m.j) {
    int t = m.i;
    m.i = m.j;
    m.j = t;
  }
  return m;
}

static inline int moved_index(int q, const move_t* m) {
  int i = m->i, j = m->j;
  if (m->typ == 0) return q == i ? j : (q == j ? i : q);
  if (m->typ == 1) return (q >= i && q <= j) ? i + j - q : q;
  if (i < j) {
    if (q < i || q > j) return q;
    return q == j ? i : q + 1;
  }
  if (q < j || q > i) return q;
  return q == j ? i : q - 1;
}

typedef struct {
  int problem, H, N, K, objective;
  const int32_t *D, *dem, *cap, *st;
} inst_t;

/* key of tour T read through move m (m == NULL: identity) */
static uint64_t tour_key(const inst_t* I, const uint16_t* T, int n, const move_t* m) {
  if (I->problem == 0) {
    int64_t t = I->st[0];
    int prev = 0;
    for (int q = 0; q < n; ++q) {
      int x = T[m ? moved_index(q, m) : q];
      t += edge(I->D, I->H, I->N, t, prev, x);
      prev = x;
    }
    t += edge(I->D, I->H, I->N, t, prev, 0);
    return pack_key(0, t - I->st[0], 0);
  }
  int k = 0, prev = 0, K = I->K;
  int64_t load = 0, t = K ? I->st[0] : 0, s = 0, mx = 0, u = 0;
  for (int q = 0; q < n; ++q) {
    int x = T[m ? moved_index(q, m) : q];
    if (x == 0) { /* A10 separator */
      if (k < K) {
        if (prev != 0) {
          int64_t rd = t + edge(I->D, I->H, I->N, t, prev, 0) - I->st[k];
          s += rd;
          if (rd > mx) mx = rd;
        }
        ++k;
        if (k < K) {
          load = 0;
          t = I->st[k];
          prev = 0;
        }
      }
      continue;
    }
    while (k < K && load + I->dem[x] > I->cap[k]) {
      if (prev != 0) {
        int64_t rd = t + edge(I->D, I->H, I->N, t, prev, 0) - I->st[k];
        s += rd;
        if (rd > mx) mx = rd;
      }
      ++k;
      if (k < K) {
        load = 0;
        t = I->st[k];
        prev = 0;
      }
    }
    if (k >= K) {
      ++u;
      continue;
    }
    t += edge(I->D, I->H, I->N, t, prev, x);
    load += I->dem[x];
    prev = x;
  }
  if (k < K && prev != 0) {
    int64_t rd = t + edge(I->D, I->H, I->N, t, prev, 0) - I->st[k];
    s += rd;
    if (rd > mx) mx = rd;
  }
  return I->objective ? pack_key(u, mx, s) : pack_key(u, s, mx);
}

static uint32_t accept_threshold(uint32_t dp, float invT) {
  if (dp == 0) return 1u << 24;
  float x = (float)dp * invT;
  float y = x * 0x1.715476p+0f;
  if (!(y < 24.0f)) return 0u;
  float kf = floorf(y);
  float f = y - kf;
  float g = f * 0x1.62e43p-1f;
  float p = 0x1.6c16c2p-10f;
  p = p * g;
  p = 0x1.111112p-7f - p;
  p = p * g;
  p = 0x1.555556p-5f - p;
  p = p * g;
  p = 0x1.555556p-3f - p;
  p = p * g;
  p = 0.5f - p;
  p = p * g;
  p = 1.0f - p;
  p = p * g;
  p = 1.0f - p;
  int k = (int)kf;
  float scaled = p * (float)(1u << (24 - k));
  return (uint32_t)scaled;
}

int oracle_sa_run(int problem, const int32_t* D, int H, int N, const int32_t* dem,
                  const int32_t* cap, const int32_t* st, int K, int objective, uint16_t* cur,
                  uint64_t* cur_key, uint16_t* best, uint64_t* best_key, int chains, int n,
                  int steps, float inv_t0, float inv_alpha, uint64_t seed, uint64_t step0,
                  int window, uint32_t window_types, int threads, int moves) {
  inst_t I = {problem, H, N, K, objective, D, dem, cap, st};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int c = 0; c < chains; ++c) {
    uint16_t* A = cur + (int64_t)c * n;
    uint16_t* Bst = best + (int64_t)c * n;
    uint16_t tmp[65536];
    uint64_t ck = tour_key(&I, A, n, NULL), bk = best_key[c];
    if (ck < bk) {
      bk = ck;
      memcpy(Bst, A, (size_t)n * 2);
    }
    float invT = inv_t0;
    for (int s = 0; s < steps && n >= 2; ++s) {
      uint64_t step = step0 + (uint64_t)s;
      uint64_t kbest = ~0ull;
      int lbest = 0;
      move_t mbest = {0, 0, 0};
      uint32_t wbest = 0;
      for (int lane = 0; lane < moves; ++lane) {
        u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)c, (uint32_t)lane, k0,
                         k1);
        move_t m = decode_move_window(r.x, r.y, r.z, n, window, window_types);
        uint64_t kk = tour_key(&I, A, n, &m);
        if (kk < kbest) {
          kbest = kk;
          lbest = lane;
          mbest = m;
          wbest = r.w;
        }
      }
      (void)lbest;
      int acc = kbest <= ck;
      if (!acc) {
        uint64_t d = (kbest >> 28) - (ck >> 28);
        uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
        acc = (wbest >> 8) < accept_threshold(dp, invT);
      }
      if (acc) {
        for (int q = 0; q < n; ++q) tmp[q] = A[moved_index(q, &mbest)];
        memcpy(A, tmp, (size_t)n * 2);
        ck = kbest;
        if (ck < bk) {
          bk = ck;
          memcpy(Bst, A, (size_t)n * 2);
        }
      }
      invT = invT * inv_alpha;
    }
    cur_key[c] = ck;
    best_key[c] = bk;
  }
  return 0;
}

/* Throughput-mode restatement (oracle/search.py tsp_batch_sa, the C-ABI's
 * vrpms_tsp_batch_sa): R static TSP requests, int32 [R][N][N]; per request 4
 * chains from Philox Fisher-Yates starts (counters (~0, ~0, 4r + w, i)), SA
 * steps drawing from one Philox block per lane per four steps (A13:
 * counters (s >> 2, 0, 4r + w, lane), word s & 3 decoded by decode_move1)
 * and one per chain for the acceptance draws (counters (s >> 2, 1, 4r + w,
 * 0), word s & 3), every candidate priced by a full
 * re-evaluation (the device prices by O(1) deltas, so equality checks them);
 * the answer is the best (key, chain).  Out: tours [R][N-1], keys [R]. */
int oracle_tsp_batch_sa(const int32_t* mats, int R, int N, int steps, float inv_t0,
                        float inv_alpha, uint64_t seed, uint16_t* out_tours, uint64_t* out_keys,
                        int threads) {
  const int n = N - 1;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  int32_t zero = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int r = 0; r < R; ++r) {
    inst_t I = {0, 1, N, 1, 0, mats + (int64_t)r * N * N, NULL, NULL, &zero};
    uint16_t A[256], B[256], Bst[256], best_t[256];
    uint64_t best_k = ~0ull;
    for (int w = 0; w < 4; ++w) {
      const uint32_t cid = (uint32_t)(4 * r + w);
      for (int q = 0; q < n; ++q) A[q] = (uint16_t)(q + 1);
      for (int i = n - 1; i >= 1; --i) {
        u32x4 x = philox(0xffffffffu, 0xffffffffu, cid, (uint32_t)i, k0, k1);
        int j = (int)(x.x % (uint32_t)(i + 1));
        uint16_t t = A[i];
        A[i] = A[j];
        A[j] = t;
      }
      uint64_t ck = tour_key(&I, A, n, NULL), bk = ck;
      memcpy(Bst, A, (size_t)n * 2);
      float invT = inv_t0;
      for (int s = 0; s < steps && n >= 2; ++s) {
        uint64_t kbest = ~0ull;
        move_t mbest = {0, 0, 0};
        const u32x4 ra = philox((uint32_t)(s >> 2), 1u, cid, 0u, k0, k1);  /* the chain's draws */
        const uint32_t a4[4] = {ra.x, ra.y, ra.z, ra.w};
        const uint32_t wbest = a4[s & 3];
        for (int lane = 0; lane < 64; ++lane) {
          u32x4 rr = philox((uint32_t)(s >> 2), 0u, cid, (uint32_t)lane, k0, k1);
          const uint32_t w4[4] = {rr.x, rr.y, rr.z, rr.w};
          move_t m = decode_move1(w4[s & 3], n);
          uint64_t kk = tour_key(&I, A, n, &m);
          if (kk < kbest) {
            kbest = kk;
            mbest = m;
          }
        }
        int acc = kbest <= ck;
        if (!acc) {
          uint64_t d = (kbest >> 28) - (ck >> 28);
          uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
          acc = (wbest >> 8) < accept_threshold(dp, invT);
        }
        if (acc) {
          for (int q = 0; q < n; ++q) B[q] = A[moved_index(q, &mbest)];
          memcpy(A, B, (size_t)n * 2);
          ck = kbest;
          if (ck < bk) {
            bk = ck;
            memcpy(Bst, A, (size_t)n * 2);
          }
        }
        invT = invT * inv_alpha;
      }
      if (bk < best_k) {
        best_k = bk;
        memcpy(best_t, Bst, (size_t)n * 2);
      }
    }
    memcpy(out_tours + (int64_t)r * n, best_t, (size_t)n * 2);
    out_keys[r] = best_k;
  }
  return 0;
}

/* Brute force restatement (oracle/search.py bf, vrpms_bf_run): the minimum
 * (key, rank) over lexicographic ranks [r0, r1) of the permutations of
 * 1..n (n <= 20), OpenMP over contiguous rank blocks.  out[0] = key,
 * out[1] = rank (UINT64_MAX, UINT64_MAX when the range is empty). */
static void unrank_perm(uint64_t r, int n, uint16_t* p) {
  uint64_t f[21];
  f[0] = 1;
  for (int i = 1; i <= 20; ++i) f[i] = f[i - 1] * (uint64_t)i;
  int avail[20];
  for (int i = 0; i < n; ++i) avail[i] = i + 1;
  int m = n;
  for (int i = 0; i < n; ++i) {
    uint64_t d = r / f[n - 1 - i];
    r %= f[n - 1 - i];
    p[i] = (uint16_t)avail[d];
    for (int x = (int)d; x < m - 1; ++x) avail[x] = avail[x + 1];
    --m;
  }
}

static void next_perm16(uint16_t* p, int n) {
  int i = n - 2;
  while (i >= 0 && p[i] >= p[i + 1]) --i;
  if (i < 0) return;
  int j = n - 1;
  while (p[j] <= p[i]) --j;
  uint16_t t = p[i];
  p[i] = p[j];
  p[j] = t;
  for (int a = i + 1, b = n - 1; a < b; ++a, --b) {
    t = p[a];
    p[a] = p[b];
    p[b] = t;
  }
}

int oracle_bf(int problem, const int32_t* D, int H, int N, const int32_t* dem, const int32_t* cap,
              const int32_t* st, int K, int objective, int n, uint64_t r0, uint64_t r1,
              uint64_t* out, int threads) {
  inst_t I = {problem, H, N, K, objective, D, dem, cap, st};
  uint64_t bk = ~0ull, br = ~0ull;
  if (n < 1 || n > 20 || r1 <= r0) {
    out[0] = bk;
    out[1] = br;
    return 0;
  }
  const int64_t blocks = 4096;
  const uint64_t span = r1 - r0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
  {
    uint64_t lk = ~0ull, lr = ~0ull;
    uint16_t p[20];
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < blocks; ++b) {
      const uint64_t ub = (uint64_t)b, q = span / (uint64_t)blocks, rem = span % (uint64_t)blocks;
      const uint64_t lo = r0 + q * ub + (ub < rem ? ub : rem);
      const uint64_t hi = lo + q + (ub < rem ? 1u : 0u);
      if (lo >= hi) continue;
      unrank_perm(lo, n, p);
      for (uint64_t rk = lo; rk < hi; ++rk) {
        const uint64_t k = tour_key(&I, p, n, NULL);
        if (k < lk || (k == lk && rk < lr)) {
          lk = k;
          lr = rk;
        }
        next_perm16(p, n);
      }
    }
#ifdef _OPENMP
#pragma omp critical
#endif
    if (lk < bk || (lk == bk && lr < br)) {
      bk = lk;
      br = lr;
    }
  }
  out[0] = bk;
  out[1] = br;
  return 0;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------------
 * oracle_sa_run_resync: the same SA as oracle_sa_run (same streams, same
 * moves, same keys, so the same trajectories bit for bit), with each
 * candidate priced by walking only the part of the moved tour whose split
 * can differ -- the CPU baseline of the quality leg, so that the host side
 * is not handicapped by full re-walks while the GPU prices route-locally.
 *
 * On a uniform fleet (one capacity, one start time) the greedy split's
 * future from a position depends on the state (load, t, prev) only, not on
 * which vehicle is driving.  Tokens before lo = min(i, j) are unchanged, so
 * the walk starts from the current tour's state after lo - 1.  Where the
 * moved tour reads a contiguous run of the current tour (src(q) = q + off),
 * a walk state equal to the current state at src(q) stays equal to the end
 * of the run: the walk jumps there, adding the routes the current tour
 * closes in between (prefix sums of route durations, a sparse table for
 * their maximum).  A fleet of different vehicles (per-vehicle capacities or
 * start times, api/parameters.py:11-12) re-synchronises only on the same
 * vehicle too (w.k == k[src(q)]): the future then runs on the same vehicles
 * from the same state.  A walk that would reach the K-th vehicle, a current
 * tour that exhausts the fleet and TSP fall back to the full walk
 * (tour_key), so every key equals tour_key's.
 * ---------------------------------------------------------------------- */
typedef struct {
  int64_t load, t, s, mx;
  int prev, k;
} walk_t;

typedef struct {
  int n, K, levels;
  int64_t *load, *t; /* after-state of position q */
  int *prev, *k;     /* k = routes closed after q */
  int* lastcust;     /* last position <= q holding a customer (-1: none) */
  int* pos_cl;       /* position of the token that made closure r */
  int kpos;          /* position of the closure that used the K-th vehicle (n: none) */
  int64_t *cd;       /* duration of closure r (0: empty route) */
  int64_t *cs;       /* cs[r] = sum of cd[0..r-1] */
  int64_t *sp;       /* sparse table [levels][K + 1] of cd maxima */
  int alive;         /* the current tour leaves no customer unvisited */
} split_t;

static int64_t sp_max(const split_t* S, int a, int b) { /* max cd[a..b], 0 when empty */
  if (b < a) return 0;
  int l = 31 - __builtin_clz((unsigned)(b - a + 1));
  const int64_t* row = S->sp + (int64_t)l * (S->K + 1);
  int64_t x = row[a], y = row[b - (1 << l) + 1];
  return x > y ? x : y;
}

static inline void close_route(const inst_t* I, walk_t* w) {
  if (w->prev != 0) {
    int64_t rd = w->t + edge(I->D, I->H, I->N, w->t, w->prev, 0) - I->st[w->k];
    w->s += rd;
    if (rd > w->mx) w->mx = rd;
  }
  ++w->k;
  if (w->k < I->K) {
    w->load = 0;
    w->t = I->st[w->k];
    w->prev = 0;
  }
}

/* one token of the greedy split (tour_key's loop body); returns 0 when a
 * customer finds the fleet exhausted (the caller then prices the move in
 * full).  Once k >= K the state is stale and only separators may follow. */
static inline int walk_token(const inst_t* I, walk_t* w, int x) {
  if (x == 0) {
    if (w->k < I->K) close_route(I, w);
    return 1;
  }
  while (w->k < I->K && w->load + I->dem[x] > I->cap[w->k]) close_route(I, w);
  if (w->k >= I->K) return 0;
  w->t += edge(I->D, I->H, I->N, w->t, w->prev, x);
  w->load += I->dem[x];
  w->prev = x;
  return 1;
}

static uint64_t walk_finish(const inst_t* I, walk_t* w) {
  if (w->k < I->K && w->prev != 0) {
    int64_t rd = w->t + edge(I->D, I->H, I->N, w->t, w->prev, 0) - I->st[w->k];
    w->s += rd;
    if (rd > w->mx) w->mx = rd;
  }
  return I->objective ? pack_key(0, w->mx, w->s) : pack_key(0, w->s, w->mx);
}

static void split_build(const inst_t* I, const uint16_t* T, split_t* S) {
  walk_t w = {0, I->K ? I->st[0] : 0, 0, 0, 0, 0};
  int last = -1;
  S->alive = 1;
  S->kpos = S->n;
  for (int q = 0; q < S->n; ++q) {
    int k0 = w.k;
    int64_t s0 = w.s;
    if (!walk_token(I, &w, T[q])) {
      S->alive = 0;
      return;
    }
    /* closures k0..w.k-1: the first one carries the route's duration, later
     * ones (oversize demand) are empty routes */
    for (int r = k0; r < w.k; ++r) {
      S->cd[r] = r == k0 ? w.s - s0 : 0;
      S->pos_cl[r] = q;
    }
    if (k0 < I->K && w.k >= I->K) S->kpos = q;
    if (T[q] != 0) last = q;
    S->lastcust[q] = last;
    S->load[q] = w.load;
    S->t[q] = w.t;
    S->prev[q] = w.prev;
    S->k[q] = w.k;
  }
  const int ncl = w.k;
  S->cs[0] = 0;
  for (int r = 0; r < ncl; ++r) S->cs[r + 1] = S->cs[r] + S->cd[r];
  for (int r = 0; r < ncl; ++r) S->sp[r] = S->cd[r];
  for (int l = 1; l < S->levels; ++l) {
    int64_t* row = S->sp + (int64_t)l * (S->K + 1);
    const int64_t* pr = row - (S->K + 1);
    for (int r = 0; r + (1 << l) <= ncl; ++r) {
      int64_t x = pr[r], y = pr[r + (1 << (l - 1))];
      row[r] = x > y ? x : y;
    }
  }
}

/* Jump the walk, whose state equals the current tour's after position a,
 * to position b (> a) of the current tour, adding the routes it closes in
 * between.  Returns the position reached (b, or the last one before the
 * current tour used its K-th vehicle), or -1 when the walk would leave a
 * customer unvisited there. */
static inline int walk_jump(const split_t* S, walk_t* w, int a, int b, int K) {
  if (S->k[b] >= K) b = S->kpos - 1; /* past kpos the current state is stale */
  if (b <= a) return a;
  const int r0 = S->k[a], r1 = S->k[b], room = K - w->k;
  int rl = r1; /* closures r0..rl-1 happen in the walk */
  if (r1 - r0 >= room) {
    /* the walk uses its K-th vehicle at closure r0 + room - 1: only
     * separators may follow it up to b */
    rl = r0 + room;
    if (S->lastcust[b] >= S->pos_cl[rl - 1]) return -1;
  }
  w->s += S->cs[rl] - S->cs[r0];
  int64_t m = sp_max(S, r0, rl - 1);
  if (m > w->mx) w->mx = m;
  w->k += rl - r0;
  w->load = S->load[b];
  w->t = S->t[b];
  w->prev = S->prev[b];
  return b;
}

/* `hopeless`: the current tour serves everyone and a key with unvisited
 * customers can never be accepted at this temperature (dp >= 2^28 gives a
 * zero threshold), so such a move is given the largest key instead of being
 * counted exactly -- it cannot win over a feasible move, and a winner that
 * is infeasible is rejected either way (as on the device). */
static uint64_t resync_key(const inst_t* I, const uint16_t* T, int n, const move_t* m,
                           const split_t* S, int hopeless, int uniform) {
  int i = m->i, j = m->j;
  int lo = i < j ? i : j;
  /* runs of the moved tour that read the current tour contiguously:
   * (start, end, offset), at most two */
  int rs[2], re[2], ro[2], nr = 0;
  if (m->typ == 0) {
    if (i + 1 <= j - 1) { rs[nr] = i + 1; re[nr] = j - 1; ro[nr++] = 0; }
    if (j + 1 <= n - 1) { rs[nr] = j + 1; re[nr] = n - 1; ro[nr++] = 0; }
  } else if (m->typ == 1) {
    if (j + 1 <= n - 1) { rs[nr] = j + 1; re[nr] = n - 1; ro[nr++] = 0; }
  } else if (i < j) {
    rs[nr] = i; re[nr] = j - 1; ro[nr++] = 1;
    if (j + 1 <= n - 1) { rs[nr] = j + 1; re[nr] = n - 1; ro[nr++] = 0; }
  } else {
    rs[nr] = j + 1; re[nr] = i; ro[nr++] = -1;
    if (i + 1 <= n - 1) { rs[nr] = i + 1; re[nr] = n - 1; ro[nr++] = 0; }
  }
  walk_t w;
  if (lo == 0 || S->k[lo - 1] >= I->K) {
    if (lo) return tour_key(I, T, n, m); /* (a current tour that ends in exhaustion) */
    w.load = 0; w.t = I->st[0]; w.prev = 0; w.k = 0; w.s = 0; w.mx = 0;
  } else {
    int a = lo - 1, r = S->k[a];
    w.load = S->load[a]; w.t = S->t[a]; w.prev = S->prev[a]; w.k = r;
    w.s = S->cs[r];
    w.mx = sp_max(S, 0, r - 1);
  }
  int run = 0;
  for (int q = lo; q < n; ++q) {
    if (!walk_token(I, &w, T[moved_index(q, m)]))
      return hopeless ? ~0ull : tour_key(I, T, n, m);
    while (run < nr && re[run] < q) ++run;
    if (run < nr && q >= rs[run] && q < re[run] && w.k < I->K) {
      const int c = q + ro[run];
      /* a fleet of different vehicles: the same state on the same vehicle */
      if (S->k[c] < I->K && w.load == S->load[c] && w.t == S->t[c] && w.prev == S->prev[c] &&
          (uniform || w.k == S->k[c])) {
        const int b = walk_jump(S, &w, c, re[run] + ro[run], I->K);
        if (b < 0) return hopeless ? ~0ull : tour_key(I, T, n, m);
        q = b - ro[run];
      }
    }
  }
  return walk_finish(I, &w);
}

/* ------------------------------------------------------------------------
 * Segment pricing (oracle/route_model.py SegTables / price_seg; the device's
 * sa_seg_kernel): uniform capacity, every demand fits an empty vehicle,
 * static symmetric matrix, any tour.  With unlimited vehicles the greedy
 * split is the concatenation over separator-delimited segments of each
 * segment's own split from an empty vehicle, and a route's duration is a
 * sum of consecutive edges of the tour (a separator standing for the depot):
 * prefix sums over the positions price every contiguous run of a moved tour
 * (forward, or reversed on a symmetric matrix) in O(1), a binary search on
 * the prefix demands finds a capacity cut, and the fleet limit is one count
 * (R routes, T separators after the last customer: served iff R - T <= K).
 * ---------------------------------------------------------------------------- */
typedef struct {
  int n, S, R, T, levels;
  int64_t *PE, *PD;             /* [n + 2], [n + 1] */
  int *SC, *SP, *PC, *NC, *RB;  /* [n + 1] each (RB: [S + 2]) */
  int64_t *dur, *dsp, *pmx, *smx, *sp; /* per route [n + 2]; sparse [levels][n + 2] */
} seg_t;

typedef struct {
  int64_t dur, load;
  int prev;
  int64_t rsum, rmax;
  int rcnt;
  int64_t* out; /* route durations (table build) or NULL */
  int cuts, bud, dead; /* capacity cuts so far, the most the fleet allows, over it */
} sacc_t;

static inline int64_t d0(const inst_t* I, int a, int b) {
  return (a == 0 && b == 0) ? 0 : (int64_t)I->D[(int64_t)a * I->N + b];
}
static inline int sspx(const seg_t* C, int k) { return k < 0 ? -1 : (k >= C->S ? C->n : C->SP[k]); }

static inline void s_close(const inst_t* I, sacc_t* a) {
  const int64_t d = a->dur + d0(I, a->prev, 0);
  if (a->out) a->out[a->rcnt] = d;
  a->rsum += d;
  if (d > a->rmax) a->rmax = d;
  ++a->rcnt;
  a->dur = a->load = 0;
  a->prev = 0;
}

/* customers A[a..b] (no separator) joined to the open route in the moved
 * order (rev: A[b] first), cut wherever the next customer does not fit */
static void s_run(const inst_t* I, const seg_t* C, const uint16_t* A, int a, int b, int rev,
                  sacc_t* c) {
  const int64_t *PE = C->PE, *PD = C->PD, cap = I->cap[0];
  while (a <= b && !c->dead) {
    const int64_t room = cap - c->load;
    if (PD[b + 1] - PD[a] <= room) {
      c->dur += d0(I, c->prev, rev ? A[b] : A[a]) + PE[b + 1] - PE[a + 1];
      c->load += PD[b + 1] - PD[a];
      c->prev = rev ? A[a] : A[b];
      return;
    }
    if (c->cuts >= c->bud) { /* one cut more than the fleet allows: no search */
      c->dead = 1;
      return;
    }
    ++c->cuts;
    if (!rev) {
      int lo = a - 1, hi = b; /* last q in [a - 1, b] with PD[q + 1] - PD[a] <= room */
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (PD[mid + 1] - PD[a] <= room) lo = mid; else hi = mid - 1;
      }
      if (lo >= a) {
        c->dur += d0(I, c->prev, A[a]) + PE[lo + 1] - PE[a + 1];
        c->load += PD[lo + 1] - PD[a];
        c->prev = A[lo];
      }
      s_close(I, c);
      a = lo + 1;
    } else {
      int lo = a, hi = b + 1; /* first x in [a, b + 1] with PD[b + 1] - PD[x] <= room */
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (PD[b + 1] - PD[mid] <= room) hi = mid; else lo = mid + 1;
      }
      if (lo <= b) {
        c->dur += d0(I, c->prev, A[b]) + PE[b + 1] - PE[lo + 1];
        c->load += PD[b + 1] - PD[lo];
        c->prev = A[lo];
      }
      s_close(I, c);
      b = lo - 1;
    }
  }
}

static void seg_build(const inst_t* I, const uint16_t* A, int n, seg_t* C) {
  C->n = n;
  C->PE[0] = C->PD[0] = 0;
  C->SC[0] = 0;
  int S = 0, last = -1;
  for (int p = 0; p <= n; ++p) {
    const int a = p ? A[p - 1] : 0, b = p < n ? A[p] : 0;
    C->PE[p + 1] = C->PE[p] + d0(I, a, b);
    if (p < n) {
      C->PD[p + 1] = C->PD[p] + (b ? I->dem[b] : 0);
      C->SC[p + 1] = C->SC[p] + (b == 0);
      if (b == 0) C->SP[S++] = p;
      if (b) last = p;
      C->PC[p] = last;
    }
  }
  C->S = S;
  C->NC[n] = n;
  for (int q = n - 1; q >= 0; --q) C->NC[q] = A[q] ? q : C->NC[q + 1];
  sacc_t c = {0, 0, 0, 0, 0, 0, C->dur, 0, 0x7fffffff, 0};
  for (int g = 0; g <= S; ++g) {
    C->RB[g] = c.rcnt;
    s_run(I, C, A, sspx(C, g - 1) + 1, sspx(C, g) - 1, 0, &c);
    s_close(I, &c);
  }
  const int R = c.rcnt;
  C->R = R;
  C->RB[S + 1] = R;
  C->T = n ? n - 1 - C->PC[n - 1] : 0;
  C->dsp[0] = C->pmx[0] = 0;
  for (int r = 0; r < R; ++r) {
    C->dsp[r + 1] = C->dsp[r] + C->dur[r];
    C->pmx[r + 1] = C->pmx[r] > C->dur[r] ? C->pmx[r] : C->dur[r];
  }
  C->smx[R] = 0;
  for (int r = R - 1; r >= 0; --r) C->smx[r] = C->smx[r + 1] > C->dur[r] ? C->smx[r + 1] : C->dur[r];
  for (int r = 0; r < R; ++r) C->sp[r] = C->dur[r];
  for (int l = 1; l < C->levels; ++l) {
    int64_t* row = C->sp + (int64_t)l * (n + 2);
    const int64_t* pr = row - (n + 2);
    for (int r = 0; r + (1 << l) <= R; ++r) {
      const int64_t x = pr[r], y = pr[r + (1 << (l - 1))];
      row[r] = x > y ? x : y;
    }
  }
}

static int64_t seg_rmax(const seg_t* C, int a, int b) { /* max dur[a..b] */
  if (b < a) return 0;
  const int l = 31 - __builtin_clz((unsigned)(b - a + 1));
  const int64_t* row = C->sp + (int64_t)l * (C->n + 2);
  const int64_t x = row[a], y = row[b - (1 << l) + 1];
  return x > y ? x : y;
}

typedef struct {
  sacc_t c;
  int64_t isum, imax;
  int icnt, seps, cust;
} sreg_t;

static inline void g_sep(const inst_t* I, sreg_t* g) {
  s_close(I, &g->c);
  ++g->seps;
}
static inline void g_run(const inst_t* I, const seg_t* C, const uint16_t* A, int a, int b, int rev,
                         sreg_t* g) {
  if (a > b) return;
  s_run(I, C, A, a, b, rev, &g->c);
  g->seps = 0;
  g->cust = 1;
}

static void g_piece(const inst_t* I, const seg_t* C, const uint16_t* A, int a, int b, int rev,
                    sreg_t* g) {
  if (a > b) return;
  const int* SC = C->SC;
  if (SC[b + 1] == SC[a]) {
    g_run(I, C, A, a, b, rev, g);
    return;
  }
  const int smin = sspx(C, SC[a]), smax = sspx(C, SC[b + 1] - 1);
  if (rev) g_run(I, C, A, smax + 1, b, 1, g);
  else g_run(I, C, A, a, smin - 1, 0, g);
  g_sep(I, g);
  if (smin < smax) { /* whole segments of A between the piece's separators */
    const int g0 = SC[smin] + 1, g1 = SC[smax];
    const int r0 = C->RB[g0], r1 = C->RB[g1 + 1];
    if (rev && r1 - r0 != g1 - g0 + 1) { /* several routes: a reversal splits differently */
      for (int s = g1; s >= g0; --s) {
        g_run(I, C, A, sspx(C, s - 1) + 1, sspx(C, s) - 1, 1, g);
        g_sep(I, g);
      }
    } else {
      g->isum += C->dsp[r1] - C->dsp[r0];
      const int64_t m = seg_rmax(C, r0, r1 - 1);
      if (m > g->imax) g->imax = m;
      g->icnt += r1 - r0;
      if (rev) {
        const int c = C->NC[smin];
        if (c < smax) { g->seps = SC[c] - SC[smin]; g->cust = 1; }
        else g->seps += SC[smax] - SC[smin];
      } else {
        const int c = C->PC[smax];
        if (c > smin) { g->seps = SC[smax + 1] - SC[c + 1]; g->cust = 1; }
        else g->seps += SC[smax] - SC[smin];
      }
    }
  }
  if (rev) g_run(I, C, A, a, smin - 1, 1, g);
  else g_run(I, C, A, smax + 1, b, 0, g);
}

/* Key of A moved by m (route_model.price_seg); *unserved = 1 (key 0) when
 * the moved tour leaves a customer unvisited.  `hopeless` (such a move can
 * never be accepted): the moved tour has S + 1 + cuts routes and, when the
 * tail after the last changed segment keeps its customers, the current
 * tour's T trailing separators, so it serves everyone iff its cuts <=
 * K - 1 - S + T; segments outside the changed ones keep their cuts, and an
 * overflowing run past the rest of that budget stops there (unserved)
 * instead of searching its cuts -- the device's rule (sa_seg_kernel). */
static uint64_t seg_key(const inst_t* I, const uint16_t* A, const seg_t* C, const move_t* m,
                        int hopeless, int* unserved) {
  const int n = C->n, i = m->i, j = m->j;
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  const int* SC = C->SC;
  const int s0 = SC[lo], st = sspx(C, s0 - 1) + 1, en = sspx(C, SC[hi + 1]);
  const int glast = en < n ? SC[en] : C->S;
  const int ra = C->RB[s0], rz = C->RB[glast + 1];
  const int tail_kept = en < n && C->PC[n - 1] > en;
  sreg_t g;
  memset(&g, 0, sizeof(g));
  g.c.bud = hopeless && tail_kept
                ? (I->K - 1 - C->S + C->T) - ((ra - s0) + (C->R - rz) - (C->S - glast))
                : 0x7fffffff;
  g_run(I, C, A, st, lo - 1, 0, &g);
  if (m->typ == 1) {
    g_piece(I, C, A, i, j, 1, &g);
  } else if (m->typ == 0) {
    g_piece(I, C, A, j, j, 0, &g);
    g_piece(I, C, A, i + 1, j - 1, 0, &g);
    g_piece(I, C, A, i, i, 0, &g);
  } else if (i < j) {
    g_piece(I, C, A, i + 1, j, 0, &g);
    g_piece(I, C, A, i, i, 0, &g);
  } else {
    g_piece(I, C, A, i, i, 0, &g);
    g_piece(I, C, A, j, i - 1, 0, &g);
  }
  if (en < n) {
    g_piece(I, C, A, hi + 1, en, 0, &g);
  } else {
    g_run(I, C, A, hi + 1, n - 1, 0, &g);
    s_close(I, &g.c);
  }
  const int R = C->R - (rz - ra) + g.c.rcnt + g.icnt;
  int Tb = C->T;
  if (!tail_kept && g.cust) Tb = g.seps + (en < n ? n - 1 - en : 0);
  *unserved = g.c.dead || R - Tb > I->K;
  if (*unserved) return 0;
  const int64_t dsum = C->dsp[ra] + g.c.rsum + g.isum + C->dsp[C->R] - C->dsp[rz];
  int64_t dmax = C->pmx[ra] > C->smx[rz] ? C->pmx[ra] : C->smx[rz];
  if (g.imax > dmax) dmax = g.imax;
  if (g.c.rmax > dmax) dmax = g.c.rmax;
  return I->objective ? pack_key(0, dmax, dsum) : pack_key(0, dsum, dmax);
}

int oracle_sa_run_resync(int problem, const int32_t* D, int H, int N, const int32_t* dem,
                         const int32_t* cap, const int32_t* st, int K, int objective,
                         uint16_t* cur, uint64_t* cur_key, uint16_t* best, uint64_t* best_key,
                         int chains, int n, int steps, float inv_t0, float inv_alpha,
                         uint64_t seed, uint64_t step0, int window, uint32_t window_types,
                         int threads, int moves) {
  int uniform = problem == 1 && K > 0;
  for (int k = 1; uniform && k < K; ++k) uniform = cap[k] == cap[0] && st[k] == st[0];
  if (problem != 1 || K <= 0 || n < 2)
    return oracle_sa_run(problem, D, H, N, dem, cap, st, K, objective, cur, cur_key, best,
                         best_key, chains, n, steps, inv_t0, inv_alpha, seed, step0, window,
                         window_types, threads, moves);
  inst_t I = {problem, H, N, K, objective, D, dem, cap, st};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  int levels = 1;
  while ((1 << levels) <= K) ++levels;
  /* segment pricing: static symmetric matrix, every demand fits a vehicle */
  int sym = H == 1;
  for (int a = 0; sym && a < N; ++a)
    for (int b = a + 1; sym && b < N; ++b) sym = D[(int64_t)a * N + b] == D[(int64_t)b * N + a];
  for (int c = 1; sym && c < N; ++c) sym = dem[c] <= cap[0];
  sym = sym && uniform; /* segment pricing: one capacity (seg_key reads cap[0]) */
  int clevels = 1;
  while ((1 << clevels) <= n + 2) ++clevels;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
  {
    seg_t C;
    C.levels = clevels;
    C.PE = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 2));
    C.PD = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    C.SC = (int*)malloc(sizeof(int) * (size_t)(n + 1));
    C.SP = (int*)malloc(sizeof(int) * (size_t)(n + 1));
    C.PC = (int*)malloc(sizeof(int) * (size_t)(n + 1));
    C.NC = (int*)malloc(sizeof(int) * (size_t)(n + 1));
    C.RB = (int*)malloc(sizeof(int) * (size_t)(n + 2));
    C.dur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 2));
    C.dsp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 3));
    C.pmx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 3));
    C.smx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 3));
    C.sp = (int64_t*)malloc(sizeof(int64_t) * (size_t)clevels * (size_t)(n + 2));
    split_t S;
    S.n = n;
    S.K = K;
    S.levels = levels;
    S.load = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    S.t = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    S.prev = (int*)malloc(sizeof(int) * (size_t)n);
    S.k = (int*)malloc(sizeof(int) * (size_t)n);
    S.lastcust = (int*)malloc(sizeof(int) * (size_t)n);
    S.pos_cl = (int*)malloc(sizeof(int) * (size_t)(K + 1));
    S.cd = (int64_t*)malloc(sizeof(int64_t) * (size_t)(K + 1));
    S.cs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(K + 2));
    S.sp = (int64_t*)malloc(sizeof(int64_t) * (size_t)levels * (size_t)(K + 1));
    uint16_t* tmp = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)n);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int c = 0; c < chains; ++c) {
      uint16_t* A = cur + (int64_t)c * n;
      uint16_t* Bst = best + (int64_t)c * n;
      uint64_t ck = tour_key(&I, A, n, NULL), bk = best_key[c];
      if (ck < bk) {
        bk = ck;
        memcpy(Bst, A, (size_t)n * 2);
      }
      if (sym) seg_build(&I, A, n, &C);
      else split_build(&I, A, &S);
      float invT = inv_t0;
      for (int s = 0; s < steps; ++s) {
        uint64_t step = step0 + (uint64_t)s;
        uint64_t kbest = ~0ull;
        move_t mbest = {0, 0, 0};
        uint32_t wbest = 0;
        const int hopeless = (ck >> 56) == 0 && accept_threshold(1u << 28, invT) == 0;
        for (int lane = 0; lane < moves; ++lane) {
          u32x4 r = philox((uint32_t)step, (uint32_t)(step >> 32), (uint32_t)c, (uint32_t)lane,
                           k0, k1);
          move_t m = decode_move_window(r.x, r.y, r.z, n, window, window_types);
          uint64_t kk;
          if (sym) {
            int unserved = 0;
            kk = seg_key(&I, A, &C, &m, hopeless, &unserved);
            if (unserved) kk = hopeless ? ~0ull : tour_key(&I, A, n, &m);
          } else {
            kk = S.alive ? resync_key(&I, A, n, &m, &S, hopeless, uniform)
                         : tour_key(&I, A, n, &m);
          }
          if (kk < kbest) {
            kbest = kk;
            mbest = m;
            wbest = r.w;
          }
        }
        int acc = kbest <= ck;
        if (!acc) {
          uint64_t d = (kbest >> 28) - (ck >> 28);
          uint32_t dp = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
          acc = (wbest >> 8) < accept_threshold(dp, invT);
        }
        if (acc) {
          for (int q = 0; q < n; ++q) tmp[q] = A[moved_index(q, &mbest)];
          memcpy(A, tmp, (size_t)n * 2);
          ck = kbest;
          if (sym) seg_build(&I, A, n, &C);
          else split_build(&I, A, &S);
          if (ck < bk) {
            bk = ck;
            memcpy(Bst, A, (size_t)n * 2);
          }
        }
        invT = invT * inv_alpha;
      }
      cur_key[c] = ck;
      best_key[c] = bk;
    }
    free(S.load); free(S.t); free(S.prev); free(S.k); free(S.lastcust); free(S.pos_cl);
    free(S.cd); free(S.cs); free(S.sp); free(tmp);
    free(C.PE); free(C.PD); free(C.SC); free(C.SP); free(C.PC); free(C.NC); free(C.RB);
    free(C.dur); free(C.dsp); free(C.pmx); free(C.smx); free(C.sp);
  }
  return 0;
}
