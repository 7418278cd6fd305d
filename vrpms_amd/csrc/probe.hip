// Roofline probe: the measured random LDS-gather ceiling R_gather
// (roofline.achieved = evals/s x G / R_gather).
//
// Every lane issues ds_read_b64 gathers at uniformly random 8-byte slots of
// an LDS-resident table the size of the CVRP-100 packed matrix, with the
// eval kernel's occupancy (1024-lane workgroups, table-limited to 2 per CU).
// Four independent LCG address streams per lane keep >= 4 gathers in
// flight and ~3 VALU per gather, so the bank-conflicted LDS is the bound.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "ctx.hpp"

namespace vrpms {

__global__ __launch_bounds__(1024) void lds_gather_probe(const uint64_t* __restrict__ table,
                                                         uint32_t slots, int iters,
                                                         uint64_t* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* T = reinterpret_cast<uint64_t*>(smem);
  for (uint32_t i = threadIdx.x; i < slots; i += blockDim.x) T[i] = table[i];
  __syncthreads();
  uint32_t s0 = (blockIdx.x * 1024u + threadIdx.x) * 2654435761u + 1u;
  uint32_t s1 = s0 * 747796405u + 2891336453u, s2 = s1 * 747796405u + 2891336453u,
           s3 = s2 * 747796405u + 2891336453u;
  uint64_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    s0 = s0 * 1664525u + 1013904223u;
    s1 = s1 * 1664525u + 1013904223u;
    s2 = s2 * 1664525u + 1013904223u;
    s3 = s3 * 1664525u + 1013904223u;
    acc ^= T[__umulhi(s0, slots)] ^ T[__umulhi(s1, slots)] ^ T[__umulhi(s2, slots)] ^
           T[__umulhi(s3, slots)];
  }
  if (acc == 0x123456789abcdefull) sink[0] = acc;  // keeps the gathers live
}

// L2-gather ceiling for the staged kernels (cfg 3 / cfg 4): every lane
// issues random 2-byte loads into a uint16 table of `slots` entries (the
// 1.94 MB hour-indexed TD-200 matrix / the 2.0 MB X-1000 matrix stay L2
// resident per XCD).  Eight independent LCG streams per lane keep eight
// loads in flight; full occupancy (2048 lanes per CU).
__global__ __launch_bounds__(256) void l2_gather_probe(const uint16_t* __restrict__ table,
                                                       uint32_t slots, int iters,
                                                       uint64_t* __restrict__ sink) {
  uint32_t s[8];
  s[0] = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 1u;
#pragma unroll
  for (int i = 1; i < 8; ++i) s[i] = s[i - 1] * 747796405u + 2891336453u;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s[i] = s[i] * 1664525u + 1013904223u;
      acc += table[__umulhi(s[i], slots)];
    }
  }
  if (acc == 0x9abcdefu) sink[0] = acc;  // keeps the gathers live
}

}  // namespace vrpms

using namespace vrpms;

extern "C" int vrpms_probe_l2_gather(vrpms_ctx* ctx, const uint16_t* d_table, int32_t slots,
                                     int32_t iters, int32_t blocks, uint64_t* d_sink,
                                     void* stream) {
  if (!ctx || !d_table || !d_sink || slots <= 0 || iters <= 0 || blocks <= 0)
    return fail(VRPMS_EINVAL, "vrpms_probe_l2_gather: bad arguments");
  VRPMS_HIP(hipSetDevice(ctx->device));
  l2_gather_probe<<<blocks, 256, 0, (hipStream_t)stream>>>(d_table, (uint32_t)slots, iters,
                                                           d_sink);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}

extern "C" int vrpms_probe_lds_gather(vrpms_ctx* ctx, const uint64_t* d_table, int32_t slots,
                                      int32_t iters, int32_t blocks, uint64_t* d_sink,
                                      void* stream) {
  if (!ctx || !d_table || !d_sink || slots <= 0 || iters <= 0 || blocks <= 0)
    return fail(VRPMS_EINVAL, "vrpms_probe_lds_gather: bad arguments");
  if ((size_t)slots * 8 > ctx->max_lds)
    return fail(VRPMS_EINVAL, "vrpms_probe_lds_gather: table exceeds LDS");
  VRPMS_HIP(hipSetDevice(ctx->device));
  const size_t lds = (size_t)slots * 8;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lds_gather_probe),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  lds_gather_probe<<<blocks, 1024, lds, (hipStream_t)stream>>>(d_table, (uint32_t)slots, iters,
                                                               d_sink);
  VRPMS_HIP(hipGetLastError());
  return VRPMS_OK;
}
