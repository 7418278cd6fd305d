// Device-side population plumbing of the search runners and the island
// model: everything the Python runners used to do with
// torch ops now runs in these kernels, so the search path issues no torch
// compute.
//
//   random_tours_kernel   Philox Fisher-Yates start tours, one lane per row,
//                         the row in LDS (oracle/spec.py philox_tour)
//   topk_chunk_kernel     E smallest (key, index) of a 2048-entry chunk by a
//                         bitonic sort in LDS; chunks -> levels -> one list
//   gather / scatter      elite rows out of a pool, migrants into it
//   inject_sorted_kernel  GA islands: migrants take the last slots of each
//                         island, which is re-sorted by (key, index)
//   island pack / merge   the E elites as one message (keys + tours), and the
//                         E best of `world` gathered messages by (key, rank,
//                         position); vrpms_island_exchange moves the messages
//                         with one RCCL all-gather over xGMI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>

#include "common.hpp"
#include "ctx.hpp"
#include "sort.hpp"

namespace vrpms {

// ---------------------------------------------------------------------------
// Philox Fisher-Yates start tours: row r of `count` is the permutation of
// 1..n+S made by, for i = n+S-1 .. 1, swapping t[i] with t[w % (i + 1)]
// where w is word (i & 3) of philox((i >> 2, 0xfffffffe, r, stream), seed);
// tokens n+1..n+S are then written as 0 (A10 route separators).
// ---------------------------------------------------------------------------
struct RandArgs {
  int64_t count;
  int n, nsep, ld, out_bytes, in_lds;  // tokens = n + nsep; values > n leave as 0 (A10)
  uint32_t seed_lo, seed_hi, stream_id;
  void* out;
};

__global__ __launch_bounds__(64) void random_tours_kernel(RandArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int64_t row = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (row >= a.count) return;
  const int n = a.n + a.nsep, nc = a.n;
  // the lane's working row: its LDS slice, or the output row itself
  uint16_t* T = a.in_lds ? reinterpret_cast<uint16_t*>(smem) + threadIdx.x * (uint32_t)n : nullptr;
  uint8_t* o8 = static_cast<uint8_t*>(a.out) + row * a.ld;
  uint16_t* o16 = static_cast<uint16_t*>(a.out) + row * a.ld;
  auto rd = [&](int q) -> uint32_t {
    if (T) return T[q];
    return a.out_bytes == 1 ? o8[q] : o16[q];
  };
  auto wr = [&](int q, uint32_t v) {
    if (T) T[q] = (uint16_t)v;
    else if (a.out_bytes == 1) o8[q] = (uint8_t)v;
    else o16[q] = (uint16_t)v;
  };
  for (int q = 0; q < n; ++q) wr(q, (uint32_t)(q + 1));
  u32x4 w{0, 0, 0, 0};
  for (int i = n - 1; i >= 1; --i) {
    if ((i & 3) == 3 || i == n - 1)
      w = philox((uint32_t)(i >> 2), 0xfffffffeu, (uint32_t)row, a.stream_id, a.seed_lo, a.seed_hi);
    const uint32_t x = (i & 3) == 0 ? w.x : (i & 3) == 1 ? w.y : (i & 3) == 2 ? w.z : w.w;
    const int j = (int)(x % (uint32_t)(i + 1));
    const uint32_t ti = rd(i), tj = rd(j);
    wr(i, tj);
    wr(j, ti);
  }
  for (int q = 0; q < n; ++q) {
    uint32_t v = rd(q);
    v = v > (uint32_t)nc ? 0u : v;  // the nsep largest tokens are separators
    if (a.out_bytes == 1) o8[q] = (uint8_t)v;
    else o16[q] = (uint16_t)v;
  }
}

// Separator insertion (oracle/spec.py insert_separators): row r of `out`
// is row r of `in` (customers only, n of them) with a 0 wherever the greedy
// split would open the next route (at most n_sep, never before the first
// customer), the unused separators appended.  One lane per row.
__global__ void insert_separators_kernel(const uint16_t* __restrict__ in, int64_t count, int n,
                                         int nsep, const int32_t* __restrict__ dem,
                                         const int32_t* __restrict__ cap, int K,
                                         uint16_t* __restrict__ out) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= count) return;
  const uint16_t* t = in + r * n;
  uint16_t* o = out + r * (int64_t)(n + nsep);
  int load = 0, used = 0, w = 0;
  for (int q = 0; q < n; ++q) {
    const uint32_t c = t[q];
    const int d = dem[c];
    if (used < nsep && load > 0 && load + d > cap[min(used, K - 1)]) {
      o[w++] = 0;
      ++used;
      load = 0;
    }
    load += d;
    o[w++] = (uint16_t)c;
  }
  while (w < n + nsep) o[w++] = 0;
}

// First-fit start (oracle/spec.py pack_separators): the customers of row r
// of `in`, in order, each join the first of B = n_sep + 1 routes with room
// (route b holds cap[min(b, K-1)]; none: the last route); out = route 0, 0,
// route 1, 0, ..., each route in input order.  One wavefront per row: the
// 64 lanes test 64 routes per ballot; lane 0 books the load and, at the end,
// places the customers.  LDS per wave: load [B] i32, start [B] i32, bin [n] u16.
__global__ __launch_bounds__(256) void pack_separators_kernel(
    const uint16_t* __restrict__ in, int64_t count, int n, int nsep,
    const int32_t* __restrict__ dem, const int32_t* __restrict__ cap, int K,
    uint32_t wave_bytes, uint16_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = (int)(threadIdx.x & 63u);
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= count) return;  // no block-wide barrier below
  const int B = nsep + 1;
  int32_t* load = reinterpret_cast<int32_t*>(smem + wave * wave_bytes);
  int32_t* start = load + B;
  uint16_t* bin = reinterpret_cast<uint16_t*>(start + B);
  const uint16_t* t = in + r * n;
  uint16_t* o = out + r * (int64_t)(n + nsep);
  for (int b = lane; b < B; b += 64) load[b] = 0;
  wave_sync();
  for (int q = 0; q < n; ++q) {
    const int d = dem[t[q]];
    int first = B - 1;
    for (int base = 0; base < B; base += 64) {
      const int b = base + lane;
      const bool fits = b < B && load[b] + d <= cap[min(b, K - 1)];
      const uint64_t ball = __ballot(fits);
      if (ball) {
        first = base + (int)__builtin_ctzll(ball);
        break;
      }
    }
    if (lane == 0) {
      load[first] += d;
      bin[q] = (uint16_t)first;
    }
    wave_sync();
  }
  if (lane == 0) {
    // customers per route -> first position of each route (separators between)
    for (int b = 0; b < B; ++b) start[b] = 0;
    for (int q = 0; q < n; ++q) ++start[bin[q]];
    int pos = 0;
    for (int b = 0; b < B; ++b) {
      const int c = start[b];
      start[b] = pos;
      pos += c;
      if (b + 1 < B) o[pos++] = 0;
    }
    for (int q = 0; q < n; ++q) o[start[bin[q]]++] = t[q];
  }
}

constexpr int kTopChunk = 2048;

// Per chunk of kTopChunk entries: the E smallest (key', index) pairs, where
// key' = ~key when `invert` (so the LARGEST keys come first, ties still by
// ascending index) and index = idx_in[i] or the position i.  Pads: (~0, ~0).
struct TopArgs {
  const uint64_t* keys;
  const uint32_t* idx_in;  // nullable
  int64_t count;
  int E, invert;
  uint64_t* out_keys;      // [chunks][E] (key' order)
  uint32_t* out_idx;
};

__global__ __launch_bounds__(1024) void topk_chunk_kernel(TopArgs a) {
  __shared__ uint64_t sk[kTopChunk];
  __shared__ uint32_t si[kTopChunk];
  const int64_t base = (int64_t)blockIdx.x * kTopChunk;
  for (int i = threadIdx.x; i < kTopChunk; i += blockDim.x) {
    const int64_t g = base + i;
    if (g < a.count) {
      const uint64_t k = a.keys[g];
      sk[i] = a.invert ? ~k : k;
      si[i] = a.idx_in ? a.idx_in[g] : (uint32_t)g;
    } else {
      sk[i] = ~0ull;
      si[i] = 0xffffffffu;
    }
  }
  __syncthreads();
  block_sort_pairs(sk, si, kTopChunk);
  for (int e = threadIdx.x; e < a.E; e += blockDim.x) {
    a.out_keys[(int64_t)blockIdx.x * a.E + e] = sk[e];
    a.out_idx[(int64_t)blockIdx.x * a.E + e] = si[e];
  }
}

// rows idx[e] of the pool -> (tours_out[e], keys_out[e])
__global__ void gather_rows_kernel(const uint16_t* __restrict__ tours,
                                   const uint64_t* __restrict__ keys, int n,
                                   const uint32_t* __restrict__ idx, int E, uint16_t* tours_out,
                                   uint64_t* keys_out) {
  const int e = blockIdx.x;
  if (e >= E) return;
  const uint32_t r = idx[e];
  for (int q = threadIdx.x; q < n; q += blockDim.x) tours_out[(int64_t)e * n + q] = tours[(int64_t)r * n + q];
  if (threadIdx.x == 0) keys_out[e] = keys[r];
}

// migrant e -> row idx[e] of the pool
__global__ void scatter_rows_kernel(uint16_t* tours, uint64_t* keys, int n,
                                    const uint32_t* __restrict__ idx, int E,
                                    const uint16_t* __restrict__ in_tours,
                                    const uint64_t* __restrict__ in_keys) {
  const int e = blockIdx.x;
  if (e >= E) return;
  const uint32_t r = idx[e];
  for (int q = threadIdx.x; q < n; q += blockDim.x) tours[(int64_t)r * n + q] = in_tours[(int64_t)e * n + q];
  if (threadIdx.x == 0) keys[r] = in_keys[e];
}

// ACO colony bests: migrant e (< count) replaces row e when strictly better
__global__ void inject_better_kernel(uint16_t* tours, uint64_t* keys, int n, int E,
                                     const uint16_t* __restrict__ in_tours,
                                     const uint64_t* __restrict__ in_keys) {
  const int e = blockIdx.x;
  if (e >= E) return;
  if (!(in_keys[e] < keys[e])) return;  // block-uniform: every thread tests before the barrier
  for (int q = threadIdx.x; q < n; q += blockDim.x) tours[(int64_t)e * n + q] = in_tours[(int64_t)e * n + q];
  __syncthreads();                       // ... and keys[e] changes only after it
  if (threadIdx.x == 0) keys[e] = in_keys[e];
}

// GA islands (one block per island of P members, sorted by (key, index)):
// migrant e goes to island e % groups, slot P - 1 - e / groups; the island is
// then re-sorted by (key, index).  `tmp` holds the island's new rows while
// the old ones are still being read.
__global__ __launch_bounds__(1024) void inject_sorted_kernel(uint16_t* tours, uint64_t* keys, int n,
                                                             int groups, int P, int E,
                                                             const uint16_t* __restrict__ in_tours,
                                                             const uint64_t* __restrict__ in_keys,
                                                             uint16_t* tmp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int M = 1;
  while (M < P) M <<= 1;
  uint64_t* sk = reinterpret_cast<uint64_t*>(smem);
  uint32_t* si = reinterpret_cast<uint32_t*>(sk + M);
  uint32_t* src = si + M;  // slot -> source: < P old row, >= P migrant (index - P)
  const int g = blockIdx.x;
  uint64_t* K = keys + (int64_t)g * P;
  uint16_t* T = tours + (int64_t)g * P * n;
  uint16_t* W = tmp + (int64_t)g * P * n;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    sk[i] = i < P ? K[i] : ~0ull;
    si[i] = (uint32_t)i;
    if (i < P) src[i] = (uint32_t)i;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int e = g; e < E; e += groups) {
      const int slot = P - 1 - e / groups;
      if (slot < 0) break;
      sk[slot] = in_keys[e];
      src[slot] = (uint32_t)(P + e);
    }
  __syncthreads();
  block_sort_pairs(sk, si, M);
  for (int64_t x = threadIdx.x; x < (int64_t)P * n; x += blockDim.x) {
    const int i = (int)(x / n), q = (int)(x % n);
    const uint32_t s = src[si[i]];
    W[x] = s < (uint32_t)P ? T[(int64_t)s * n + q] : in_tours[(int64_t)(s - P) * n + q];
  }
  for (int i = threadIdx.x; i < P; i += blockDim.x) K[i] = sk[i];
  __syncthreads();
  for (int64_t x = threadIdx.x; x < (int64_t)P * n; x += blockDim.x) T[x] = W[x];
}

// island message: [E keys u64][E x n tours u16], padded to 16 bytes
static size_t msg_bytes(int E, int n) { return ((size_t)E * 8 + (size_t)E * n * 2 + 15) & ~(size_t)15; }

// gathered messages -> contiguous candidate keys [world * E]
__global__ void msg_keys_kernel(const unsigned char* msgs, size_t mbytes, int world, int E,
                                uint64_t* keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= world * E) return;
  const int r = i / E, e = i % E;
  keys[i] = reinterpret_cast<const uint64_t*>(msgs + (size_t)r * mbytes)[e];
}

// winners (gathered position p = r * E + e) -> (tours_out, keys_out)
__global__ void msg_gather_kernel(const unsigned char* msgs, size_t mbytes, int E, int n,
                                  const uint32_t* __restrict__ idx, uint16_t* tours_out,
                                  uint64_t* keys_out) {
  const int e = blockIdx.x;
  const uint32_t p = idx[e];
  const int r = (int)(p / (uint32_t)E), x = (int)(p % (uint32_t)E);
  const unsigned char* m = msgs + (size_t)r * mbytes;
  const uint16_t* t = reinterpret_cast<const uint16_t*>(m + (size_t)E * 8) + (size_t)x * n;
  for (int q = threadIdx.x; q < n; q += blockDim.x) tours_out[(int64_t)e * n + q] = t[q];
  if (threadIdx.x == 0) keys_out[e] = reinterpret_cast<const uint64_t*>(m)[x];
}

// Poll a non-blocking communicator until its pending operation (creation,
// or the enqueue of a collective) has completed or failed; ncclInProgress
// back means the deadline passed first.
static ncclResult_t wait_comm(ncclComm_t comm, std::chrono::steady_clock::time_point deadline) {
  ncclResult_t state = ncclInProgress;
  while (true) {
    const ncclResult_t r = ncclCommGetAsyncError(comm, &state);
    if (r != ncclSuccess) return r;
    if (state != ncclInProgress) return state;
    if (std::chrono::steady_clock::now() > deadline) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Tear down the context's communicator: a non-blocking one is finalized and
// polled to completion before it is destroyed (aborted if that fails or does
// not finish within the deadline).
static void release_comm(vrpms_ctx* ctx) {
  if (!ctx->comm) return;
  ncclComm_t comm = static_cast<ncclComm_t>(ctx->comm);
  ctx->comm = nullptr;
  ctx->comm_world = 1;
  ncclResult_t r = ncclCommFinalize(comm);
  if (r == ncclSuccess || r == ncclInProgress)
    r = wait_comm(comm, std::chrono::steady_clock::now() +
                            std::chrono::seconds(ctx->opt_island_timeout_s));
  if (r == ncclSuccess) (void)ncclCommDestroy(comm);
  else (void)ncclCommAbort(comm);
}

// The pool scratch is grown with a plain hipFree + hipMalloc: hipFree
// synchronises the device, so work still queued on the caller's stream that
// reads the old buffer (RCCL receive area, top-E levels) completes first.
// Every pool / island call enqueues on the one stream it is given and the
// context is used by one host thread at a time (include/vrpms.h threading
// rule); a stream-ordered allocator would need hipFreeAsync on that stream.
static int ensure_pool_scratch(vrpms_ctx* ctx, size_t bytes) {
  if (ctx->pool_scratch_bytes >= bytes) return VRPMS_OK;
  (void)hipFree(ctx->pool_scratch);
  ctx->pool_scratch = nullptr;
  ctx->pool_scratch_bytes = 0;
  if (hipMalloc(&ctx->pool_scratch, bytes) != hipSuccess)
    return fail(VRPMS_ENOMEM, "pool scratch allocation failed");
  ctx->pool_scratch_bytes = bytes;
  return VRPMS_OK;
}

// Scratch carve for the selection levels, after `reserve` bytes.
struct TopScratch {
  uint64_t* k[2];
  uint32_t* i[2];
};

static size_t top_bytes(int64_t count, int E) {
  const int64_t chunks = (count + kTopChunk - 1) / kTopChunk;
  return 2 * ((size_t)chunks * E * 12 + 256);
}

// E smallest (key', index) of keys[0..count) into (*k_out, *i_out) (device
// pointers into the scratch at `base`).  Levels: chunks of 2048 -> E each.
static int topk(const uint64_t* keys, int64_t count, int E, int invert, unsigned char* base,
                uint64_t** k_out, uint32_t** i_out, hipStream_t s) {
  const int64_t chunks0 = (count + kTopChunk - 1) / kTopChunk;
  const size_t half = (size_t)chunks0 * E * 12 + 256;
  uint64_t* kb[2] = {reinterpret_cast<uint64_t*>(base), reinterpret_cast<uint64_t*>(base + half)};
  uint32_t* ib[2] = {reinterpret_cast<uint32_t*>(base + (size_t)chunks0 * E * 8 + 128),
                     reinterpret_cast<uint32_t*>(base + half + (size_t)chunks0 * E * 8 + 128)};
  const uint64_t* in_k = keys;
  const uint32_t* in_i = nullptr;
  int64_t n = count;
  int flip = 0, inv = invert;
  while (true) {
    const int64_t chunks = (n + kTopChunk - 1) / kTopChunk;
    TopArgs t{in_k, in_i, n, E, inv, kb[flip], ib[flip]};
    topk_chunk_kernel<<<(unsigned)chunks, 1024, 0, s>>>(t);
    VRPMS_HIP(hipGetLastError());
    if (chunks == 1) break;
    in_k = kb[flip];
    in_i = ib[flip];
    n = chunks * E;
    inv = 0;  // later levels already hold key'
    flip ^= 1;
  }
  *k_out = kb[flip];
  *i_out = ib[flip];
  return VRPMS_OK;
}

static int check_pool(const vrpms_pool* p, const char* who) {
  if (!p || !p->tours || !p->keys || p->count <= 0 || p->n < 0)
    return fail(VRPMS_EINVAL, std::string(who) + ": bad pool");
  return VRPMS_OK;
}

static int do_elites(vrpms_ctx* ctx, const vrpms_pool* p, int E, uint16_t* t_out, uint64_t* k_out,
                     size_t reserve, hipStream_t s) {
  uint64_t* tk;
  uint32_t* ti;
  unsigned char* base = static_cast<unsigned char*>(ctx->pool_scratch) + reserve;
  int rc = topk(p->keys, p->count, E, 0, base, &tk, &ti, s);
  if (rc) return rc;
  gather_rows_kernel<<<E, 128, 0, s>>>(p->tours, p->keys, p->n, ti, E, t_out, k_out);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

static int do_inject(vrpms_ctx* ctx, const vrpms_pool* p, int mode, const uint16_t* t_in,
                     const uint64_t* k_in, int E, size_t reserve, hipStream_t s) {
  unsigned char* base = static_cast<unsigned char*>(ctx->pool_scratch) + reserve;
  if (mode == VRPMS_INJECT_WORST) {
    uint64_t* tk;
    uint32_t* ti;
    int rc = topk(p->keys, p->count, E, 1, base, &tk, &ti, s);
    if (rc) return rc;
    scatter_rows_kernel<<<E, 128, 0, s>>>(p->tours, p->keys, p->n, ti, E, t_in, k_in);
  } else if (mode == VRPMS_INJECT_BETTER) {
    const int m = std::min(E, p->count);
    inject_better_kernel<<<m, 128, 0, s>>>(p->tours, p->keys, p->n, m, t_in, k_in);
  } else {
    const int P = p->count / p->groups;
    int M = 1;
    while (M < P) M <<= 1;
    const size_t lds = (size_t)M * 12 + (size_t)P * 4;
    inject_sorted_kernel<<<p->groups, 1024, lds, s>>>(p->tours, p->keys, p->n, p->groups, P, E,
                                                      t_in, k_in, reinterpret_cast<uint16_t*>(base));
  }
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

static int check_mode(const vrpms_ctx* ctx, const vrpms_pool* p, int mode, int E, const char* who) {
  if (mode != VRPMS_INJECT_WORST && mode != VRPMS_INJECT_SORTED && mode != VRPMS_INJECT_BETTER)
    return fail(VRPMS_EINVAL, std::string(who) + ": unknown inject mode");
  if (mode == VRPMS_INJECT_WORST && E > p->count)
    return fail(VRPMS_EINVAL, std::string(who) + ": more migrants than rows");
  if (mode == VRPMS_INJECT_SORTED) {
    if (p->groups <= 0 || p->count % p->groups != 0)
      return fail(VRPMS_EINVAL, std::string(who) + ": groups must divide count");
    const int P = p->count / p->groups;
    int M = 1;
    while (M < P) M <<= 1;
    if ((size_t)M * 12 + (size_t)P * 4 > std::min<size_t>(ctx->max_lds, 65536))
      return fail(VRPMS_EINVAL, std::string(who) + ": island too large for the LDS sort");
  }
  return VRPMS_OK;
}

// bytes of pool scratch an inject needs beyond `reserve`
static size_t inject_bytes(const vrpms_pool* p, int mode, int E) {
  if (mode == VRPMS_INJECT_WORST) return top_bytes(p->count, E);
  if (mode == VRPMS_INJECT_SORTED) return (size_t)p->count * p->n * 2 + 256;
  return 0;
}

}  // namespace vrpms

using namespace vrpms;

extern "C" {

int vrpms_random_tours(vrpms_ctx* ctx, int64_t count, int32_t n, int32_t n_sep, int64_t ld,
                       int32_t tour_bytes, uint64_t seed, uint32_t stream_id, void* d_tours,
                       void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_random_tours: ctx is NULL");
  if (count < 0 || n < 0 || n_sep < 0 || ld < (int64_t)n + n_sep ||
      (tour_bytes != 1 && tour_bytes != 2))
    return fail(VRPMS_EINVAL,
                "vrpms_random_tours: need count >= 0, n, n_sep >= 0, n + n_sep <= ld, tour_bytes 1 or 2");
  if ((tour_bytes == 1 && n + n_sep > 255) || n + n_sep > 65535)
    return fail(VRPMS_EINVAL, "vrpms_random_tours: token ids do not fit the tour element");
  const int tokens = n + n_sep;
  if (count == 0 || tokens == 0) return VRPMS_OK;
  if (!d_tours) return fail(VRPMS_EINVAL, "vrpms_random_tours: d_tours is NULL");
  VRPMS_HIP(hipSetDevice(ctx->device));
  // each lane shuffles its row in LDS when 64 rows fit, else in place in HBM
  const size_t lds = (size_t)64 * tokens * 2;
  const bool in_lds = lds <= ctx->max_lds;
  RandArgs a{count, n, n_sep, (int)ld, tour_bytes, in_lds ? 1 : 0, (uint32_t)seed,
             (uint32_t)(seed >> 32), stream_id, d_tours};
  if (in_lds && lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(random_tours_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  random_tours_kernel<<<(unsigned)((count + 63) / 64), 64, in_lds ? lds : 0,
                        (hipStream_t)stream>>>(a);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

int vrpms_insert_separators(vrpms_ctx* ctx, const uint16_t* d_in, int64_t count, int32_t n,
                            int32_t n_sep, uint16_t* d_out, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_insert_separators: ctx is NULL");
  if (!ctx->has_instance || ctx->inst.problem != VRPMS_CVRP)
    return fail(VRPMS_ESTATE, "vrpms_insert_separators: needs a CVRP instance");
  if (count < 0 || n < 0 || n > ctx->inst.N - 1 || n_sep < 0)
    return fail(VRPMS_EINVAL, "vrpms_insert_separators: need count >= 0, 0 <= n <= N-1, n_sep >= 0");
  if (count == 0 || n + n_sep == 0) return VRPMS_OK;
  if (!d_in || !d_out) return fail(VRPMS_EINVAL, "vrpms_insert_separators: NULL buffer");
  VRPMS_HIP(hipSetDevice(ctx->device));
  const Instance& in = ctx->inst;
  insert_separators_kernel<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      d_in, count, n, n_sep, in.dem, in.cap, in.K, d_out);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

int vrpms_pack_separators(vrpms_ctx* ctx, const uint16_t* d_in, int64_t count, int32_t n,
                          int32_t n_sep, uint16_t* d_out, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_pack_separators: ctx is NULL");
  if (!ctx->has_instance || ctx->inst.problem != VRPMS_CVRP)
    return fail(VRPMS_ESTATE, "vrpms_pack_separators: needs a CVRP instance");
  if (count < 0 || n < 0 || n > ctx->inst.N - 1 || n_sep < 0 || n_sep > 4095)
    return fail(VRPMS_EINVAL, "vrpms_pack_separators: need count >= 0, 0 <= n <= N-1, 0 <= n_sep < 4096");
  if (count == 0 || n + n_sep == 0) return VRPMS_OK;
  if (!d_in || !d_out) return fail(VRPMS_EINVAL, "vrpms_pack_separators: NULL buffer");
  VRPMS_HIP(hipSetDevice(ctx->device));
  const Instance& in = ctx->inst;
  const uint32_t wave_bytes = ((uint32_t)(n_sep + 1) * 8u + (uint32_t)n * 2u + 15u) & ~15u;
  const size_t lds = (size_t)4 * wave_bytes;
  if (lds > ctx->max_lds) return fail(VRPMS_EINVAL, "vrpms_pack_separators: tours too long for LDS");
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pack_separators_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  pack_separators_kernel<<<(unsigned)((count + 3) / 4), 256, lds, (hipStream_t)stream>>>(
      d_in, count, n, n_sep, in.dem, in.cap, in.K, wave_bytes, d_out);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

int vrpms_pool_elites(vrpms_ctx* ctx, const vrpms_pool* pool, int32_t E, uint16_t* d_tours,
                      uint64_t* d_keys, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_pool_elites: ctx is NULL");
  if (int rc = check_pool(pool, "vrpms_pool_elites")) return rc;
  if (E <= 0 || E > pool->count || E > kTopChunk / 2 || !d_tours || !d_keys)
    return fail(VRPMS_EINVAL, "vrpms_pool_elites: need 0 < E <= min(count, 1024) and outputs");
  VRPMS_HIP(hipSetDevice(ctx->device));
  if (int rc = ensure_pool_scratch(ctx, top_bytes(pool->count, E))) return rc;
  return do_elites(ctx, pool, E, d_tours, d_keys, 0, (hipStream_t)stream);
}

int vrpms_pool_inject(vrpms_ctx* ctx, const vrpms_pool* pool, int32_t mode,
                      const uint16_t* d_tours, const uint64_t* d_keys, int32_t E, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_pool_inject: ctx is NULL");
  if (int rc = check_pool(pool, "vrpms_pool_inject")) return rc;
  if (E <= 0 || E > kTopChunk / 2 || !d_tours || !d_keys)
    return fail(VRPMS_EINVAL, "vrpms_pool_inject: need 0 < E <= 1024 and migrants");
  if (int rc = check_mode(ctx, pool, mode, E, "vrpms_pool_inject")) return rc;
  VRPMS_HIP(hipSetDevice(ctx->device));
  if (int rc = ensure_pool_scratch(ctx, inject_bytes(pool, mode, E))) return rc;
  return do_inject(ctx, pool, mode, d_tours, d_keys, E, 0, (hipStream_t)stream);
}

int64_t vrpms_island_msg_bytes(int32_t E, int32_t n) {
  if (E <= 0 || n < 0) return fail(VRPMS_EINVAL, "vrpms_island_msg_bytes: need E > 0, n >= 0");
  return (int64_t)msg_bytes(E, n);
}

int vrpms_island_pack(vrpms_ctx* ctx, const vrpms_pool* pool, int32_t E, void* d_msg,
                      void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_island_pack: ctx is NULL");
  if (int rc = check_pool(pool, "vrpms_island_pack")) return rc;
  if (E <= 0 || E > pool->count || E > kTopChunk / 2 || !d_msg)
    return fail(VRPMS_EINVAL, "vrpms_island_pack: need 0 < E <= min(count, 1024) and a message");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (int rc = ensure_pool_scratch(ctx, top_bytes(pool->count, E))) return rc;
  const size_t mb = msg_bytes(E, pool->n);
  unsigned char* m = static_cast<unsigned char*>(d_msg);
  VRPMS_HIP(hipMemsetAsync(m + (size_t)E * 8 + (size_t)E * pool->n * 2, 0,
                           mb - (size_t)E * 8 - (size_t)E * pool->n * 2, s));
  return do_elites(ctx, pool, E, reinterpret_cast<uint16_t*>(m + (size_t)E * 8),
                   reinterpret_cast<uint64_t*>(m), 0, s);
}

// the E best of `world` gathered messages by (key, rank, position)
static int merge_msgs(vrpms_ctx* ctx, const void* d_msgs, int world, int E, int n, uint16_t* t_out,
                      uint64_t* k_out, size_t reserve, hipStream_t s) {
  unsigned char* base = static_cast<unsigned char*>(ctx->pool_scratch) + reserve;
  uint64_t* cand = reinterpret_cast<uint64_t*>(base);
  const size_t cb = ((size_t)world * E * 8 + 255) & ~(size_t)255;
  const size_t mb = msg_bytes(E, n);
  msg_keys_kernel<<<(world * E + 255) / 256, 256, 0, s>>>(static_cast<const unsigned char*>(d_msgs),
                                                          mb, world, E, cand);
  VRPMS_HIP(hipGetLastError());
  uint64_t* tk;
  uint32_t* ti;
  int rc = topk(cand, (int64_t)world * E, E, 0, base + cb, &tk, &ti, s);
  if (rc) return rc;
  msg_gather_kernel<<<E, 128, 0, s>>>(static_cast<const unsigned char*>(d_msgs), mb, E, n, ti,
                                      t_out, k_out);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

static size_t merge_bytes(int world, int E) {
  return (((size_t)world * E * 8 + 255) & ~(size_t)255) + top_bytes((int64_t)world * E, E);
}

int vrpms_island_merge(vrpms_ctx* ctx, const void* d_msgs, int32_t world, int32_t E, int32_t n,
                       uint16_t* d_tours, uint64_t* d_keys, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_island_merge: ctx is NULL");
  if (world <= 0 || E <= 0 || E > kTopChunk / 2 || n < 0 || !d_msgs || !d_tours || !d_keys)
    return fail(VRPMS_EINVAL, "vrpms_island_merge: bad arguments");
  VRPMS_HIP(hipSetDevice(ctx->device));
  if (int rc = ensure_pool_scratch(ctx, merge_bytes(world, E))) return rc;
  return merge_msgs(ctx, d_msgs, world, E, n, d_tours, d_keys, 0, (hipStream_t)stream);
}

int vrpms_island_unique_id(void* out) {
  if (!out) return fail(VRPMS_EINVAL, "vrpms_island_unique_id: out is NULL");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess)
    return fail(VRPMS_EHIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out, &id, sizeof(id));
  return VRPMS_OK;
}

int vrpms_island_init(vrpms_ctx* ctx, const void* unique_id, int32_t rank, int32_t world) {
  if (!ctx || !unique_id) return fail(VRPMS_EINVAL, "vrpms_island_init: NULL ctx/id");
  if (world <= 0 || rank < 0 || rank >= world)
    return fail(VRPMS_EINVAL, "vrpms_island_init: need 0 <= rank < world");
  VRPMS_HIP(hipSetDevice(ctx->device));
  if (ctx->comm) {
    release_comm(ctx);
  }
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  // non-blocking creation + deadline: a rank that never joins (it failed
  // before reaching this call) turns into VRPMS_ETIMEOUT on the others
  // instead of a process that hangs in ncclCommInitRank
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRankConfig(&comm, world, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress)
    return fail(VRPMS_EHIP, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  const auto deadline =
      std::chrono::steady_clock::now() + std::chrono::seconds(ctx->opt_island_timeout_s);
  r = wait_comm(comm, deadline);
  if (r != ncclSuccess) {
    if (comm) (void)ncclCommAbort(comm);
    if (r == ncclInProgress)
      return fail(VRPMS_ETIMEOUT, "vrpms_island_init: not every rank joined within " +
                                      std::to_string(ctx->opt_island_timeout_s) + " s");
    return fail(VRPMS_EHIP, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  }
  ctx->comm = comm;
  ctx->comm_rank = rank;
  ctx->comm_world = world;
  return VRPMS_OK;
}

int vrpms_island_world(vrpms_ctx* ctx) { return ctx && ctx->comm ? ctx->comm_world : 0; }

int vrpms_island_exchange(vrpms_ctx* ctx, const vrpms_pool* src, const vrpms_pool* dst,
                          int32_t mode, int32_t E, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_island_exchange: ctx is NULL");
  if (int rc = check_pool(src, "vrpms_island_exchange")) return rc;
  if (int rc = check_pool(dst, "vrpms_island_exchange")) return rc;
  if (src->n != dst->n) return fail(VRPMS_EINVAL, "vrpms_island_exchange: pools differ in n");
  if (E <= 0 || E > src->count || E > kTopChunk / 2)
    return fail(VRPMS_EINVAL, "vrpms_island_exchange: need 0 < E <= min(src count, 1024)");
  if (int rc = check_mode(ctx, dst, mode, E, "vrpms_island_exchange")) return rc;
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  const int world = ctx->comm ? ctx->comm_world : 1;
  const int n = src->n;
  const size_t mb = msg_bytes(E, n);
  // scratch: [send msg][world msgs][winners: tours, keys][work area]
  const size_t win_t = (((size_t)E * n * 2) + 255) & ~(size_t)255;
  const size_t win_k = ((size_t)E * 8 + 255) & ~(size_t)255;
  const size_t head = mb + (size_t)world * mb + win_t + win_k;
  const size_t work = std::max({top_bytes(src->count, E), merge_bytes(world, E),
                                inject_bytes(dst, mode, E)});
  if (int rc = ensure_pool_scratch(ctx, head + work)) return rc;
  unsigned char* sp = static_cast<unsigned char*>(ctx->pool_scratch);
  unsigned char* send = sp;
  unsigned char* recv = sp + mb;
  uint16_t* wt = reinterpret_cast<uint16_t*>(recv + (size_t)world * mb);
  uint64_t* wk = reinterpret_cast<uint64_t*>(reinterpret_cast<unsigned char*>(wt) + win_t);
  VRPMS_HIP(hipMemsetAsync(send, 0, mb, s));
  int rc = do_elites(ctx, src, E, reinterpret_cast<uint16_t*>(send + (size_t)E * 8),
                     reinterpret_cast<uint64_t*>(send), head, s);
  if (rc) return rc;
  if (ctx->comm) {
    // non-blocking communicator: the enqueue may report ncclInProgress
    ncclComm_t comm = static_cast<ncclComm_t>(ctx->comm);
    ncclResult_t r = ncclAllGather(send, recv, mb, ncclUint8, comm, s);
    if (r == ncclInProgress)
      r = wait_comm(comm, std::chrono::steady_clock::now() +
                              std::chrono::seconds(ctx->opt_island_timeout_s));
    if (r != ncclSuccess) {
      // a communicator left with an operation pending (or in error) is never
      // used again: abort it, so later exchanges fall back to the local copy
      // (world 1) and vrpms_island_world reports 0
      (void)ncclCommAbort(comm);
      ctx->comm = nullptr;
      ctx->comm_world = 1;
      return fail(r == ncclInProgress ? VRPMS_ETIMEOUT : VRPMS_EHIP,
                  std::string("ncclAllGather: ") + ncclGetErrorString(r));
    }
  } else {
    VRPMS_HIP(hipMemcpyAsync(recv, send, mb, hipMemcpyDeviceToDevice, s));
  }
  rc = merge_msgs(ctx, recv, world, E, n, wt, wk, head, s);
  if (rc) return rc;
  return do_inject(ctx, dst, mode, wt, wk, E, head, s);
}

}  // extern "C"

namespace vrpms {
// called by vrpms_ctx_destroy
void island_release(vrpms_ctx* ctx) {
  release_comm(ctx);
  (void)hipFree(ctx->pool_scratch);
  ctx->pool_scratch = nullptr;
  ctx->pool_scratch_bytes = 0;
}
}  // namespace vrpms
