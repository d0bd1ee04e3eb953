// Semantics check of __builtin_amdgcn_permlane32_swap on gfx950 (tools only): prints both outputs per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out) {
  const unsigned v = 100 + threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  out[threadIdx.x] = r[0];
  out[64 + threadIdx.x] = r[1];
}

int main() {
  unsigned* d;
  unsigned h[128];
  (void)hipMalloc(&d, sizeof(h));
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0 %u r1 %u\n", l, h[l], h[64 + l]);
  return 0;
}
