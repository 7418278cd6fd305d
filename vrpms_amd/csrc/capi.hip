// C-ABI plumbing: errors, context lifetime, instance loading / validation and
// the derived on-chip layouts.  The compute entry points live
// in eval.hip (scoring) and the solver .hip files.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <string>
#include <vector>

#include "common.hpp"
#include "ctx.hpp"

namespace vrpms {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(VRPMS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// stats layout: 0 min_dur 1 max_dur 2 min_dem 3 max_dem 4 min_cap 5 max_cap
//               6 min_start 7 max_start 8 asymmetric (slice 0) 9 asymmetric (any slice)
__global__ void stats_init_kernel(int32_t* s) {
  if (threadIdx.x < 8) s[threadIdx.x] = (threadIdx.x & 1) ? INT_MIN : INT_MAX;
  if (threadIdx.x == 8 || threadIdx.x == 9) s[threadIdx.x] = 0;
}

// s[8] |= any D[a][b] != D[b][a] in hour slice 0 (selects the O(1) 2-opt
// delta); s[9] |= the same in any slice (sa_td_kernel's reverse rows).
__global__ void asym_kernel(const int32_t* __restrict__ D, int N, int H, int32_t* s) {
  const int64_t NN = (int64_t)N * N, total = NN * H;
  int asym0 = 0, asym = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = i / NN, e = i - h * NN, a = e / N, b = e - a * N;
    const bool x = D[i] != D[h * NN + b * N + a];
    asym |= x;
    asym0 |= x && h == 0;
  }
  if (__any(asym0) && (threadIdx.x & 63) == 0) atomicOr(s + 8, 1);
  if (__any(asym) && (threadIdx.x & 63) == 0) atomicOr(s + 9, 1);
}

// [H][N][N] -> [N][N][H] (H = 24): the 24 hourly durations of an edge in one
// 48-byte row, which sa_td_kernel caches per tour position.
__global__ void hour_minor_kernel(const uint16_t* __restrict__ in, int64_t NN, int H,
                                  uint16_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < NN * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i / H, h = i - e * H;
    out[i] = in[h * NN + e];
  }
}

__device__ __forceinline__ void block_minmax_commit(int vmin, int vmax, int32_t* smin,
                                                    int32_t* smax) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    vmin = min(vmin, __shfl_xor(vmin, off, kWave));
    vmax = max(vmax, __shfl_xor(vmax, off, kWave));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(smin, vmin);
    atomicMax(smax, vmax);
  }
}

__global__ void stats_kernel(const int32_t* __restrict__ dur, int64_t total,
                             const int32_t* __restrict__ dem, int N,
                             const int32_t* __restrict__ cap, const int32_t* __restrict__ start,
                             int K, int32_t* s) {
  int vmin = INT_MAX, vmax = INT_MIN;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int v = dur[i];
    vmin = min(vmin, v);
    vmax = max(vmax, v);
  }
  block_minmax_commit(vmin, vmax, s + 0, s + 1);
  if (blockIdx.x == 0) {
    int a = INT_MAX, b = INT_MIN, c = INT_MAX, d = INT_MIN, e = INT_MAX, f = INT_MIN;
    for (int i = threadIdx.x; i < N; i += blockDim.x)
      if (dem && i > 0) { a = min(a, dem[i]); b = max(b, dem[i]); }
    for (int i = threadIdx.x; i < K; i += blockDim.x) {
      if (cap) { c = min(c, cap[i]); d = max(d, cap[i]); }
      e = min(e, start[i]);
      f = max(f, start[i]);
    }
    block_minmax_commit(a, b, s + 2, s + 3);
    block_minmax_commit(c, d, s + 4, s + 5);
    block_minmax_commit(e, f, s + 6, s + 7);
  }
}

__global__ void to_u16_kernel(const int32_t* __restrict__ in, uint16_t* __restrict__ out,
                              int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint16_t)in[i];
}

// Packed static-CVRP layout: E[a][b] = dur(a,b) | (ret(b) | out(b) << w | dem(b) << 2w) << 32
// where ret(b) = D[b][0] and out(b) = D[0][b].  One 8-byte LDS gather per
// customer then yields the edge, the demand test and both depot legs a
// route closure needs (eval.hip, eval_cvrp_packed).
__global__ void pack64_kernel(const int32_t* __restrict__ D, const int32_t* __restrict__ dem,
                              int N, int w, uint64_t* __restrict__ out) {
  const int64_t total = (int64_t)N * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int a = (int)(i / N), b = (int)(i % N);
    uint32_t hi = 0;
    if (b > 0)
      hi = (uint32_t)D[(int64_t)b * N] | ((uint32_t)D[b] << w) | ((uint32_t)dem[b] << (2 * w));
    out[i] = (uint64_t)(uint32_t)D[(int64_t)a * N + b] | ((uint64_t)hi << 32);
  }
}

// Prefix-ret layout (uniform fleet).  A route's accumulator is
// acc = load << S | (cur + ret(prev)); appending b after a adds
// lo(a,b) = dem(b) << S + dur(a,b) + ret(b) - ret(a), which may be negative in
// its low part but keeps acc exact in 32-bit two's complement because the
// true running value stays in [0, 2^S).  ret(depot) is taken as 0.
__global__ void pack_prefix_kernel(const int32_t* __restrict__ D, const int32_t* __restrict__ dem,
                                   int N, int S, uint64_t* __restrict__ out) {
  const int64_t total = (int64_t)N * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int a = (int)(i / N), b = (int)(i % N);
    // column 0 (A10 separator): never fits, opens an empty route (hi = 0)
    uint32_t lo = 0x7fffffffu, hi = 0;
    if (b > 0) {
      const int64_t retb = D[(int64_t)b * N], reta = a > 0 ? D[(int64_t)a * N] : 0;
      const int64_t d = (int64_t)D[(int64_t)a * N + b] + retb - reta;
      lo = (uint32_t)(((int64_t)dem[b] << S) + d);
      hi = (uint32_t)(D[b] + retb) | ((uint32_t)dem[b] << S);
    }
    out[i] = (uint64_t)lo | ((uint64_t)hi << 32);
  }
}

// Same layout with the open-route word biased by -lim (mod 2^32), so the
// words kernel can keep its accumulator biased and test capacity by sign.
__global__ void bias_hi_kernel(const uint64_t* __restrict__ in, int64_t total, uint32_t lim,
                               uint64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = in[i];
    out[i] = (e & 0xffffffffull) | ((uint64_t)((uint32_t)(e >> 32) - lim) << 32);
  }
}

static int bits_for(int v) {
  int b = 1;
  while (b < 31 && (1 << b) <= v) ++b;
  return b;
}

static void free_instance(Instance& in) {
  (void)hipFree(in.mat32);
  (void)hipFree(in.mat16);
  (void)hipFree(in.mat16h);
  (void)hipFree(in.pack64);
  (void)hipFree(in.pack64p);
  (void)hipFree(in.pack64w);
  (void)hipFree(in.dem);
  (void)hipFree(in.cap);
  (void)hipFree(in.start);
  in = Instance();
}

}  // namespace vrpms

using namespace vrpms;

extern "C" {

int vrpms_version(void) { return (0 << 16) | 1; }

const char* vrpms_last_error(void) { return g_last_error.c_str(); }

int vrpms_ctx_create(int device, vrpms_ctx** out) {
  if (!out) return fail(VRPMS_EINVAL, "vrpms_ctx_create: out is NULL");
  *out = nullptr;
  int count = 0;
  VRPMS_HIP(hipGetDeviceCount(&count));
  if (device < 0 || device >= count)
    return fail(VRPMS_EINVAL, "vrpms_ctx_create: device " + std::to_string(device) +
                                  " out of range (" + std::to_string(count) + " devices)");
  VRPMS_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  VRPMS_HIP(hipGetDeviceProperties(&prop, device));
  vrpms_ctx* c = new (std::nothrow) vrpms_ctx();
  if (!c) return fail(VRPMS_ENOMEM, "vrpms_ctx_create: out of host memory");
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  c->max_lds = prop.sharedMemPerBlock;
  if (hipMalloc(&c->d_stats, 64) != hipSuccess || hipMalloc(&c->d_scratch, 64) != hipSuccess) {
    (void)hipFree(c->d_stats);
    delete c;
    return fail(VRPMS_ENOMEM, "vrpms_ctx_create: hipMalloc scratch failed");
  }
  *out = c;
  return VRPMS_OK;
}

int vrpms_ctx_destroy(vrpms_ctx* ctx) {
  if (!ctx) return VRPMS_OK;
  (void)hipSetDevice(ctx->device); (void)hipDeviceSynchronize();
  island_release(ctx);
  free_instance(ctx->inst);
  (void)hipFree(ctx->d_stats);
  (void)hipFree(ctx->d_scratch);
  (void)hipFree(ctx->search_scratch);
  delete ctx;
  return VRPMS_OK;
}

int vrpms_set_option(vrpms_ctx* ctx, int32_t option, int32_t value) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_set_option: ctx is NULL");
  if (option == VRPMS_OPT_SPLIT_MODE) {
    if (value != 0 && value != 2 && value != 3)
      return fail(VRPMS_EINVAL,
                  "vrpms_set_option: split mode must be 0 (auto), 2 (branchy) or 3 (no carry form)");
    ctx->opt_split_mode = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_STAGED_M) {
    if (value < 0 || value > 2)
      return fail(VRPMS_EINVAL, "vrpms_set_option: staged M must be 0 (auto), 1 or 2");
    ctx->opt_staged_m = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_WORDS_KERNEL) {
    if (value < 0 || value > 1)
      return fail(VRPMS_EINVAL, "vrpms_set_option: words kernel must be 0 (auto) or 1");
    ctx->opt_words_kernel = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_SA_ROUTE) {
    if (value != 0 && value != 2 && value != 3 && value != 4)
      return fail(VRPMS_EINVAL,
                  "vrpms_set_option: SA route must be 0 (auto), 2 (full walks), 3 (route walks) "
                  "or 4 (hour-row walks)");
    ctx->opt_sa_route = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_ROUTE_WG_PER_CU) {
    if (value < 0 || value > 2)
      return fail(VRPMS_EINVAL, "vrpms_set_option: route workgroups per CU must be 0 (auto), 1 or 2");
    ctx->opt_route_wg_per_cu = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_GA_FUSED) {
    if (value != 0 && value != 2)
      return fail(VRPMS_EINVAL, "vrpms_set_option: GA fused must be 0 (auto) or 2 (three kernels)");
    ctx->opt_ga_fused = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_ROWS_CONFIG) {
    if (value < 0 || value > 5)
      return fail(VRPMS_EINVAL, "vrpms_set_option: rows config must be 0 (auto) or 1..5");
    ctx->opt_rows_config = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_WORDS_LOOKAHEAD) {
    if (value < 0 || value > 2)
      return fail(VRPMS_EINVAL, "vrpms_set_option: words lookahead must be 0 (auto), 1 or 2");
    ctx->opt_words_lookahead = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_WORDS_ILP) {
#ifdef VRPMS_AB
    if (value < 0 || value > 2)
      return fail(VRPMS_EINVAL, "vrpms_set_option: words ILP must be 0 (auto), 1 or 2");
#else
    if (value != 0 && value != 2)
      return fail(VRPMS_EINVAL,
                  "vrpms_set_option: words ILP must be 0 (auto) or 2 (the one-candidate-per-lane "
                  "variant is built only with -DVRPMS_AB)");
#endif
    ctx->opt_words_ilp = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_SEG_WAVES) {
    if (value < 0 || value > 4)
      return fail(VRPMS_EINVAL, "vrpms_set_option: segment-kernel wavefronts must be 0 (auto) .. 4");
    ctx->opt_seg_waves = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_ACO_CONSTRUCT) {
    if (value != 0 && value != 2)
      return fail(VRPMS_EINVAL, "vrpms_set_option: ACO construct must be 0 (auto) or 2 (L2 path)");
    ctx->opt_aco_construct = value;
    return VRPMS_OK;
  }
  if (option == VRPMS_OPT_ISLAND_TIMEOUT_S) {
    if (value <= 0)
      return fail(VRPMS_EINVAL, "vrpms_set_option: island timeout must be > 0 seconds");
    ctx->opt_island_timeout_s = value;
    return VRPMS_OK;
  }
  return fail(VRPMS_EINVAL, "vrpms_set_option: unknown option " + std::to_string(option));
}

int vrpms_set_instance(vrpms_ctx* ctx, int32_t problem, const int32_t* d_dur, int32_t H,
                       int32_t N, const int32_t* d_demand, const int32_t* d_cap,
                       const int32_t* d_start, int32_t K, int32_t objective, void* stream) {
  if (!ctx) return fail(VRPMS_EINVAL, "vrpms_set_instance: ctx is NULL");
  if (problem != VRPMS_TSP && problem != VRPMS_CVRP)
    return fail(VRPMS_EINVAL, "vrpms_set_instance: unknown problem " + std::to_string(problem));
  if (!d_dur || !d_start) return fail(VRPMS_EINVAL, "vrpms_set_instance: d_dur/d_start NULL");
  if (N < 1 || N > 65535) return fail(VRPMS_EINVAL, "vrpms_set_instance: N must be in [1, 65535]");
  if (H < 1 || H > 1024) return fail(VRPMS_EINVAL, "vrpms_set_instance: H must be in [1, 1024]");
  if ((int64_t)H * N * N >= (1LL << 31))
    return fail(VRPMS_EINVAL, "vrpms_set_instance: H*N*N must stay below 2^31 elements");
  if (problem == VRPMS_CVRP && (!d_demand || !d_cap || K < 1 || K > 65535))
    return fail(VRPMS_EINVAL, "vrpms_set_instance: CVRP needs demand, capacities and 1<=K<=65535");
  if (problem == VRPMS_TSP && K != 1)
    return fail(VRPMS_EINVAL, "vrpms_set_instance: TSP takes exactly one start time (K=1)");
  if (objective != VRPMS_OBJ_SUM && objective != VRPMS_OBJ_MAX)
    return fail(VRPMS_EINVAL, "vrpms_set_instance: objective must be 0 (sum) or 1 (max)");
  VRPMS_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;

  free_instance(ctx->inst);
  ctx->has_instance = false;
  Instance& in = ctx->inst;
  in.problem = problem;
  in.H = H;
  in.N = N;
  in.K = K;
  in.objective = objective;
  const int64_t total = (int64_t)H * N * N;
  VRPMS_HIP(hipMalloc(&in.mat32, total * 4));
  VRPMS_HIP(hipMalloc(&in.dem, (size_t)N * 4));
  VRPMS_HIP(hipMalloc(&in.cap, (size_t)K * 4));
  VRPMS_HIP(hipMalloc(&in.start, (size_t)K * 4));
  VRPMS_HIP(hipMemcpyAsync(in.mat32, d_dur, total * 4, hipMemcpyDeviceToDevice, s));
  VRPMS_HIP(hipMemcpyAsync(in.start, d_start, (size_t)K * 4, hipMemcpyDeviceToDevice, s));
  if (problem == VRPMS_CVRP) {
    VRPMS_HIP(hipMemcpyAsync(in.dem, d_demand, (size_t)N * 4, hipMemcpyDeviceToDevice, s));
    VRPMS_HIP(hipMemcpyAsync(in.cap, d_cap, (size_t)K * 4, hipMemcpyDeviceToDevice, s));
  } else {
    VRPMS_HIP(hipMemsetAsync(in.dem, 0, (size_t)N * 4, s));
    VRPMS_HIP(hipMemsetAsync(in.cap, 0x7f, (size_t)K * 4, s));
  }

  // Validation (non-negative ints, A2) and the A9 int32 guard.
  stats_init_kernel<<<1, 64, 0, s>>>(ctx->d_stats);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, (int64_t)ctx->num_cus * 4);
  stats_kernel<<<grid, 256, 0, s>>>(in.mat32, total, problem == VRPMS_CVRP ? in.dem : nullptr, N,
                                    problem == VRPMS_CVRP ? in.cap : nullptr, in.start, K,
                                    ctx->d_stats);
  VRPMS_HIP(hipGetLastError());
  asym_kernel<<<grid, 256, 0, s>>>(in.mat32, N, H, ctx->d_stats);
  VRPMS_HIP(hipGetLastError());
  int32_t st[10];
  std::vector<int32_t> caps(K);
  VRPMS_HIP(hipMemcpyAsync(st, ctx->d_stats, sizeof(st), hipMemcpyDeviceToHost, s));
  VRPMS_HIP(hipMemcpyAsync(caps.data(), in.cap, (size_t)K * 4, hipMemcpyDeviceToHost, s));
  VRPMS_HIP(hipStreamSynchronize(s));
  if (st[0] < 0) return fail(VRPMS_EINVAL, "vrpms_set_instance: negative duration in matrix");
  if (problem == VRPMS_CVRP) {
    if (N > 1 && st[2] < 0) return fail(VRPMS_EINVAL, "vrpms_set_instance: negative demand");
    if (st[4] < 0) return fail(VRPMS_EINVAL, "vrpms_set_instance: negative capacity");
  }
  if (st[6] < 0) return fail(VRPMS_EINVAL, "vrpms_set_instance: negative start time");
  in.max_dur = st[1];
  in.max_dem = problem == VRPMS_CVRP && N > 1 ? st[3] : 0;
  in.min_dem = problem == VRPMS_CVRP && N > 1 ? st[2] : 0;
  in.min_cap = problem == VRPMS_CVRP ? st[4] : INT_MAX;
  in.max_cap = problem == VRPMS_CVRP ? st[5] : INT_MAX;
  in.max_start = st[7];
  in.min_start = st[6];
  in.symmetric = st[8] == 0;
  in.sym_all = st[9] == 0;
  in.cap0 = caps[0];
  in.uniform_cap = std::all_of(caps.begin(), caps.end(), [&](int32_t c) { return c == caps[0]; });
  const long double bound = (long double)in.max_start + (long double)(N + K + 1) * in.max_dur;
  if ((int64_t)in.max_cap + in.max_dem >= 2147483648LL && problem == VRPMS_CVRP)
    return fail(VRPMS_ERANGE, "vrpms_set_instance: capacity + demand overflows int32");
  if (bound >= 2147483648.0L)
    return fail(VRPMS_ERANGE, "vrpms_set_instance: start + (N+K+1)*max_duration overflows int32 "
                              "(A9 guard)");

  in.use16 = in.max_dur <= 65535;
  if (in.use16) {
    VRPMS_HIP(hipMalloc(&in.mat16, total * 2));
    to_u16_kernel<<<grid, 256, 0, s>>>(in.mat32, in.mat16, total);
    VRPMS_HIP(hipGetLastError());
    // hour-minor rows for the hour-indexed SA walks (bounded: 48 bytes per edge)
    if (H == 24 && total * 2 <= ((int64_t)1 << 30)) {
      VRPMS_HIP(hipMalloc(&in.mat16h, total * 2));
      hour_minor_kernel<<<grid, 256, 0, s>>>(in.mat16, (int64_t)N * N, H, in.mat16h);
      VRPMS_HIP(hipGetLastError());
    }
  }
  const size_t elem = in.use16 ? 2 : 4;
  in.tier = (size_t)total * elem <= 64 * 1024 ? kTierLds : kTierGlobal;
  if (problem == VRPMS_CVRP && H == 1 && N <= 128) {
    const int w = bits_for(in.max_dur);
    if (2 * w + bits_for(in.max_dem) <= 32) {
      in.pack_w = w;
      VRPMS_HIP(hipMalloc(&in.pack64, (size_t)N * N * 8));
      pack64_kernel<<<(N * N + 255) / 256, 256, 0, s>>>(in.mat32, in.dem, N, w, in.pack64);
      VRPMS_HIP(hipGetLastError());
      in.tier = kTierLdsPacked;
    }
    // prefix-ret layout: S bits hold any route's cur + ret(last) <= (N+1)*max_dur,
    // the bits above hold load + demand <= cap + max_dem.
    const int64_t route_bound = (int64_t)(N + 1) * in.max_dur;
    int S = 1;
    while (S < 31 && ((int64_t)1 << S) <= route_bound) ++S;
    const int64_t load_bound = (int64_t)in.cap0 + in.max_dem + 1;
    if (in.pack64 && in.uniform_cap && S < 32 && (load_bound << S) < ((int64_t)1 << 32)) {
      in.pref_S = S;
      in.pref_lim = (uint32_t)(((int64_t)in.cap0 + 1) << S);
      in.pref_smask = (uint32_t)(((int64_t)1 << S) - 1);
      VRPMS_HIP(hipMalloc(&in.pack64p, (size_t)N * N * 8));
      pack_prefix_kernel<<<(N * N + 255) / 256, 256, 0, s>>>(in.mat32, in.dem, N, S, in.pack64p);
      VRPMS_HIP(hipGetLastError());
      VRPMS_HIP(hipMalloc(&in.pack64w, (size_t)N * N * 8));
      bias_hi_kernel<<<(N * N + 255) / 256, 256, 0, s>>>(in.pack64p, (int64_t)N * N, in.pref_lim,
                                                         in.pack64w);
      VRPMS_HIP(hipGetLastError());
    }
  }
  VRPMS_HIP(hipStreamSynchronize(s));
  ctx->has_instance = true;
  return VRPMS_OK;
}

}  // extern "C"
