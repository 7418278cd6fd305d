/* oracle_c.c -- C restatement of oracle/spec.py.  TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (large-batch parity against the HIP library) and by
 * bench.py's cpu_baseline leg ("kind": "port": the reference ships no CPU
 * solver, SURVEY.md §0.1, so this restatement of the frozen Appendix-A spec
 * is the CPU path timed beside the GPU).  Never linked into libvrpms.
 *
 * Semantics follow oracle/spec.py line by line:
 *   eval_tsp   <- spec.eval_tsp   (A4; anchors api/parameters.py:41-43, src/solver.py:24)
 *   eval_cvrp  <- spec.eval_cvrp  (A5-A7; anchors api/parameters.py:11-12, src/solver.py:27)
 *   pack_key   <- spec.pack_key   (A8)
 * Arithmetic is int64 here (the spec uses unbounded ints); the A9 guard
 * keeps every value inside int32 for the device.
 */
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

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
