// Microbenchmark: ceiling of random 32-B row gathers from a table far larger than the Infinity Cache (gfx950).
// The affine solver's memory side at cfg4: every lane loads one uniformly random 32-B row (two 16-B loads), a wave
// keeps B rows per lane in flight, nothing else.  Cold caches (a 1 GiB buffer is rewritten before every launch).
// Reports rows/s, the row bytes/s (32 B per row: the affine kernel's algorithmic accounting) and the DRAM sector
// bytes/s (64 B per row).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/gather32 tools/micro/gather32.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// grid-stride over `nrows_total` gathers; each lane issues B independent row loads before consuming them
template <int B>
__global__ __launch_bounds__(256) void k_gather(const float4* __restrict__ tab, uint32_t nrows_tab, int64_t n,
                                                float* __restrict__ out) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (int64_t i = tid * B; i < n; i += stride * B) {
    float4 v[B][2];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint32_t row = hash32((uint32_t)(i + b) * 2654435761u) % nrows_tab;
      v[b][0] = tab[(int64_t)row * 2];
      v[b][1] = tab[(int64_t)row * 2 + 1];
    }
#pragma unroll
    for (int b = 0; b < B; ++b) acc += v[b][0].x + v[b][1].w;
  }
  if (acc == 1.2345f) out[0] = acc;
}

template <int B>
static void run(const float4* tab, uint32_t nrows, int64_t n, float* out, float* flush, size_t flush_n, int blocks) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemsetAsync(flush, rep, flush_n * sizeof(float)));
    CK(hipEventRecord(e0));
    k_gather<B><<<blocks, 256>>>(tab, nrows, n, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  printf("B=%d blocks=%d: %.3f ms  %.2f G rows/s  row bytes %.0f GB/s  64-B sectors %.0f GB/s\n", B, blocks, best,
         n / (best * 1e-3) / 1e9, n * 32.0 / (best * 1e-3) / 1e9, n * 64.0 / (best * 1e-3) / 1e9);
}

int main() {
  const uint32_t nrows = 86398977u;  // cfg4's pool: 86.4 M rows × 32 B = 2.76 GB
  const int64_t n = 262144LL * 64;   // the rows of 262,144 ranges × 64 candidates
  float4* tab;
  float *out, *flush;
  const size_t flush_n = (size_t)1 << 28;
  CK(hipMalloc(&tab, (size_t)nrows * 32));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&flush, flush_n * sizeof(float)));
  CK(hipMemset(tab, 0, (size_t)nrows * 32));
  for (int blocks : {2048, 8192}) {
    run<1>(tab, nrows, n, out, flush, flush_n, blocks);
    run<2>(tab, nrows, n, out, flush, flush_n, blocks);
    run<4>(tab, nrows, n, out, flush, flush_n, blocks);
    run<8>(tab, nrows, n, out, flush, flush_n, blocks);
  }
  CK(hipFree(tab));
  CK(hipFree(out));
  CK(hipFree(flush));
  return 0;
}
