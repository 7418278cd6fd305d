// ds_permute_b32 with a partial exec mask: what do lanes that nobody writes
// to receive?  (GA breed design probe; prints one line per case)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int* out) {
  const int lane = threadIdx.x;
  int v = 0x55;
  // only even lanes push (value 1000 + lane) to lane (lane + 2) % 64
  if ((lane & 1) == 0) v = __builtin_amdgcn_ds_permute(((lane + 2) & 63) * 4, 1000 + lane);
  out[lane] = v;
  // all lanes active: odd lanes push to nobody special (to themselves), even to lane+2
  int w = __builtin_amdgcn_ds_permute(((lane & 1) ? lane : ((lane + 2) & 63)) * 4, 2000 + lane);
  out[64 + lane] = w;
  // a ballot of "received" with a partial writer set
  int got = 0;
  if (lane < 8) got = __builtin_amdgcn_ds_permute((lane * 5) * 4, 1);
  int r = __builtin_amdgcn_ds_permute(0, 0);  // all lanes write to lane 0
  (void)r;
  out[128 + lane] = got;
}
int main() {
  int* d;
  hipMalloc(&d, 192 * 4);
  hipMemset(d, 0xff, 192 * 4);
  k<<<1, 64>>>(d);
  int h[192];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("partial exec (even lanes push to lane+2):");
  for (int i = 0; i < 16; ++i) printf(" %d", h[i]);
  printf("\nall active:");
  for (int i = 0; i < 16; ++i) printf(" %d", h[64 + i]);
  printf("\nlanes<8 push 1 to 5*lane:");
  for (int i = 0; i < 40; ++i) printf(" %d", h[128 + i]);
  printf("\n");
  return 0;
}
