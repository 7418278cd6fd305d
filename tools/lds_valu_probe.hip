// Overlap probe: does VALU work issued beside random ds_read_b64 gathers
// hide under the LDS bank-conflict cycles, or add to them?  Each lane issues
// 4 random gathers per iteration over an N*N u64 table (the CVRP-100 packed
// matrix size, 1024-lane workgroups, 2 per CU as eval_cvrp_words2) and V
// extra dependent-chain VALU ops per gather that do not feed the addresses.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/lds_valu_probe tools/lds_valu_probe.hip
//   ./tools/lds_valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                             \
    }                                                                       \
  } while (0)

template <int V>
__global__ __launch_bounds__(1024) void probe(const uint64_t* __restrict__ table, uint32_t slots,
                                              int iters, uint64_t* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* T = reinterpret_cast<uint64_t*>(smem);
  for (uint32_t i = threadIdx.x; i < slots; i += blockDim.x) T[i] = table[i];
  __syncthreads();
  uint32_t s0 = (blockIdx.x * 1024u + threadIdx.x) * 2654435761u + 1u;
  uint32_t s1 = s0 * 747796405u + 2891336453u, s2 = s1 * 747796405u + 2891336453u,
           s3 = s2 * 747796405u + 2891336453u;
  uint32_t x0 = s0, x1 = s1, x2 = s2, x3 = s3;
  uint64_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    s0 = s0 * 1664525u + 1013904223u;
    s1 = s1 * 1664525u + 1013904223u;
    s2 = s2 * 1664525u + 1013904223u;
    s3 = s3 * 1664525u + 1013904223u;
    const uint64_t g0 = T[__umulhi(s0, slots)], g1 = T[__umulhi(s1, slots)],
                   g2 = T[__umulhi(s2, slots)], g3 = T[__umulhi(s3, slots)];
#pragma unroll
    for (int v = 0; v < V; ++v) {  // four independent chains, V ops each
      x0 = (x0 ^ (uint32_t)g0) + 0x9e3779b9u;
      x1 = (x1 ^ (uint32_t)g1) + 0x7f4a7c15u;
      x2 = (x2 ^ (uint32_t)g2) + 0x85ebca6bu;
      x3 = (x3 ^ (uint32_t)g3) + 0xc2b2ae35u;
      asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    acc ^= g0 ^ g1 ^ g2 ^ g3;
  }
  if ((acc ^ x0 ^ x1 ^ x2 ^ x3) == 0x123456789abcdefull) sink[0] = acc;
}

template <int V>
int run(const uint64_t* d_t, uint32_t slots, int blocks, uint64_t* d_sink) {
  const size_t lds = slots * 8;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe<V>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int iters = 4096;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  probe<V><<<blocks, 1024, lds>>>(d_t, slots, iters, d_sink);
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) probe<V><<<blocks, 1024, lds>>>(d_t, slots, iters, d_sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double gathers = 5.0 * blocks * 1024.0 * iters * 4;
  const double rate = gathers / (ms * 1e-3);
  // VALU per gather: V chain ops x 2 (xor + add) + ~3 address ops
  printf("{\"V\": %d, \"valu_per_gather\": %d, \"gathers_per_s\": %.4g, \"ms\": %.3f}\n", V,
         2 * V + 3, rate, ms / 5);
  return 0;
}

int main() {
  const uint32_t N = 101, slots = N * N;
  std::vector<uint64_t> h(slots);
  for (uint32_t i = 0; i < slots; ++i) h[i] = i * 0x9e3779b97f4a7c15ull;
  uint64_t *d_t, *d_sink;
  CK(hipMalloc(&d_t, slots * 8));
  CK(hipMalloc(&d_sink, 8));
  CK(hipMemcpy(d_t, h.data(), slots * 8, hipMemcpyHostToDevice));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int blocks = 2 * p.multiProcessorCount * 4;
  printf("{\"cus\": %d, \"clock_khz\": %d}\n", p.multiProcessorCount, p.clockRate);
  if (run<0>(d_t, slots, blocks, d_sink) || run<1>(d_t, slots, blocks, d_sink) ||
      run<2>(d_t, slots, blocks, d_sink) || run<3>(d_t, slots, blocks, d_sink) ||
      run<4>(d_t, slots, blocks, d_sink) || run<6>(d_t, slots, blocks, d_sink) ||
      run<8>(d_t, slots, blocks, d_sink))
    return 1;
  CK(hipFree(d_t));
  CK(hipFree(d_sink));
  return 0;
}
