/* sanitize_driver.c -- TEST INFRASTRUCTURE: drives every entry point of the
 * C restatement (oracle_c.c) on small random instances so that a build with
 * -fsanitize=address,undefined (tests/test_oracle_sanitize.py) checks its
 * index arithmetic: CVRP / TSP / hour-indexed evaluation, full-walk, resync
 * and segment-priced SA (separators, windows, several moves per step,
 * heterogeneous fleets), the batched TSP SA and brute force.  Exits 0 when
 * the resync / segment SA trajectories equal the full-walk ones. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_eval_batch(int problem, const int32_t* D, int H, int N, const int32_t* dem,
                      const int32_t* cap, const int32_t* st, int K, int objective, const uint8_t* p8,
                      const uint16_t* p16, int64_t C, int n, int64_t ld, uint64_t* keys, int32_t* sums,
                      int32_t* maxs, int32_t* unv, int threads);
int oracle_sa_run(int problem, const int32_t* D, int H, int N, const int32_t* dem,
                  const int32_t* cap, const int32_t* st, int K, int objective, uint16_t* cur,
                  uint64_t* cur_key, uint16_t* best, uint64_t* best_key, int chains, int n,
                  int steps, float inv_t0, float inv_alpha, uint64_t seed, uint64_t step0,
                  int window, uint32_t window_types, int threads, int moves);
int oracle_sa_run_resync(int problem, const int32_t* D, int H, int N, const int32_t* dem,
                         const int32_t* cap, const int32_t* st, int K, int objective,
                         uint16_t* cur, uint64_t* cur_key, uint16_t* best, uint64_t* best_key,
                         int chains, int n, int steps, float inv_t0, float inv_alpha,
                         uint64_t seed, uint64_t step0, int window, uint32_t window_types,
                         int threads, int moves);
int oracle_tsp_batch_sa(const int32_t* mats, int R, int N, int steps, float inv_t0,
                        float inv_alpha, uint64_t seed, uint16_t* out_tours, uint64_t* out_keys,
                        int threads);
int oracle_bf(int problem, const int32_t* D, int H, int N, const int32_t* dem, const int32_t* cap,
              const int32_t* st, int K, int objective, int n, uint64_t r0, uint64_t r1,
              uint64_t* out, int threads);

static uint32_t rng_state = 12345u;
static uint32_t rnd(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 17;
  rng_state ^= rng_state << 5;
  return rng_state;
}

/* random symmetric (or asymmetric) H x N x N matrix, zero diagonal */
static int32_t* matrix(int H, int N, int sym) {
  int32_t* D = (int32_t*)malloc(sizeof(int32_t) * (size_t)H * N * N);
  for (int h = 0; h < H; ++h)
    for (int a = 0; a < N; ++a)
      for (int b = 0; b < N; ++b) {
        int32_t* x = D + ((size_t)h * N + a) * N + b;
        if (a == b) *x = 0;
        else if (sym && b < a) *x = D[((size_t)h * N + b) * N + a];
        else *x = 3 + (int32_t)(rnd() % 300);
      }
  return D;
}

/* tours: a Fisher-Yates order of 1..n_c plus n_sep separators (0) */
static void tours(uint16_t* T, int chains, int n_c, int n_sep) {
  const int n = n_c + n_sep;
  for (int c = 0; c < chains; ++c) {
    uint16_t* t = T + (size_t)c * n;
    for (int q = 0; q < n; ++q) t[q] = q < n_c ? (uint16_t)(q + 1) : 0;
    for (int q = n - 1; q > 0; --q) {
      int j = (int)(rnd() % (uint32_t)(q + 1));
      uint16_t x = t[q];
      t[q] = t[j];
      t[j] = x;
    }
  }
}

static int sa_case(int n_c, int K, int H, int sym, int het, int window, uint32_t types,
                   int moves, int steps, float inv_t0) {
  const int N = n_c + 1, n_sep = K - 1, n = n_c + n_sep, chains = 3;
  int32_t* D = matrix(H, N, sym);
  int32_t* dem = (int32_t*)malloc(sizeof(int32_t) * N);
  int32_t *cap = (int32_t*)malloc(sizeof(int32_t) * K), *st = (int32_t*)malloc(sizeof(int32_t) * K);
  int64_t tot = 0;
  dem[0] = 0;
  for (int c = 1; c < N; ++c) tot += dem[c] = 1 + (int32_t)(rnd() % 10);
  for (int k = 0; k < K; ++k) {
    cap[k] = (int32_t)(tot * 11 / (10 * K)) + 10 + (het ? (int32_t)(rnd() % 7) : 0);
    st[k] = het ? (int32_t)(rnd() % 120) : 0;
  }
  uint16_t* P = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)chains * n);
  tours(P, chains, n_c, n_sep);
  uint16_t *c0 = malloc(2 * (size_t)chains * n), *b0 = malloc(2 * (size_t)chains * n);
  uint16_t *c1 = malloc(2 * (size_t)chains * n), *b1 = malloc(2 * (size_t)chains * n);
  uint64_t ck0[3], bk0[3], ck1[3], bk1[3];
  memcpy(c0, P, 2 * (size_t)chains * n);
  memcpy(b0, P, 2 * (size_t)chains * n);
  memcpy(c1, P, 2 * (size_t)chains * n);
  memcpy(b1, P, 2 * (size_t)chains * n);
  for (int c = 0; c < chains; ++c) bk0[c] = bk1[c] = ~0ull;
  oracle_sa_run(1, D, H, N, dem, cap, st, K, 0, c0, ck0, b0, bk0, chains, n, steps, inv_t0,
                1.0f / 0.99f, 7, 3, window, types, 1, moves);
  oracle_sa_run_resync(1, D, H, N, dem, cap, st, K, 0, c1, ck1, b1, bk1, chains, n, steps, inv_t0,
                       1.0f / 0.99f, 7, 3, window, types, 1, moves);
  int ok = memcmp(c0, c1, 2 * (size_t)chains * n) == 0 && memcmp(ck0, ck1, sizeof ck0) == 0 &&
           memcmp(bk0, bk1, sizeof bk0) == 0;
  /* evaluation of the final tours, u16 and u8 rows */
  uint64_t keys[3];
  int32_t sums[3], maxs[3], unv[3];
  oracle_eval_batch(1, D, H, N, dem, cap, st, K, 1, NULL, c0, chains, n, n, keys, sums, maxs, unv, 1);
  if (N <= 256) {
    uint8_t* p8 = (uint8_t*)malloc((size_t)chains * n);
    for (size_t i = 0; i < (size_t)chains * n; ++i) p8[i] = (uint8_t)c0[i];
    oracle_eval_batch(1, D, H, N, dem, cap, st, K, 0, p8, NULL, chains, n, n, keys, sums, maxs, unv, 1);
    free(p8);
  }
  free(D); free(dem); free(cap); free(st); free(P); free(c0); free(b0); free(c1); free(b1);
  return ok;
}

int main(void) {
  int fails = 0;
  /* segment pricing: static symmetric, one capacity (windowed, full range, several moves) */
  fails += !sa_case(60, 6, 1, 1, 0, 8, 2, 64, 120, 1.0f / 40.0f);
  fails += !sa_case(40, 5, 1, 1, 0, 0, 0, 128, 120, 1.0f / 40.0f);
  fails += !sa_case(90, 4, 1, 1, 0, 6, 0, 64, 80, 1e-7f);     /* hot: no shortcut */
  /* resync walks: hour-indexed, asymmetric; full walks: heterogeneous fleet */
  fails += !sa_case(30, 4, 24, 1, 0, 5, 0, 64, 60, 1.0f / 60.0f);
  fails += !sa_case(35, 4, 1, 0, 0, 6, 2, 64, 60, 1.0f / 60.0f);
  fails += !sa_case(25, 3, 1, 1, 1, 0, 0, 64, 60, 1.0f / 60.0f);
  /* TSP: batched SA and plain evaluation */
  {
    const int R = 4, N = 20;
    int32_t* M = (int32_t*)malloc(sizeof(int32_t) * (size_t)R * N * N);
    for (int r = 0; r < R; ++r) {
      int32_t* m = matrix(1, N, r & 1);
      memcpy(M + (size_t)r * N * N, m, sizeof(int32_t) * N * N);
      free(m);
    }
    uint16_t tours_out[4 * 19];
    uint64_t keys[4];
    oracle_tsp_batch_sa(M, R, N, 50, 1.0f / 50.0f, 1.0f / 0.99f, 5, tours_out, keys, 1);
    int32_t st0 = 0;
    oracle_eval_batch(0, M, 1, N, NULL, NULL, &st0, 1, 0, NULL, tours_out, R, 19, 19, keys, NULL,
                      NULL, NULL, 1);
    free(M);
  }
  /* brute force, CVRP and TSP, a window of ranks */
  {
    const int n = 8, N = 9, K = 3;
    int32_t* D = matrix(1, N, 1);
    int32_t dem[9] = {0, 3, 4, 2, 5, 1, 2, 3, 4}, cap[3] = {9, 9, 9}, st[3] = {0, 0, 0};
    uint64_t out[2];
    oracle_bf(1, D, 1, N, dem, cap, st, K, 0, n, 0, 40320, out, 1);
    oracle_bf(0, D, 1, N, NULL, NULL, st, 1, 0, n, 1000, 9000, out, 1);
    free(D);
  }
  if (fails) fprintf(stderr, "%d SA case(s) differ between the full and the resync / segment walks\n",
                     fails);
  printf("sanitize driver: %s\n", fails ? "MISMATCH" : "ok");
  return fails ? 1 : 0;
}
