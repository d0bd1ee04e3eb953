// Microbenchmark: ceiling of the similarity-search inner loop on gfx950.
// Per tile: one ds_read_b128 (A fragment) → v_mfma_f32_32x32x16_f16 → optional 16-way int max tree.
// 2 workgroups × 8 waves per CU (4 waves/SIMD), like k_sim_topk_f16.  Reports cycles per tile per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int imax16(const floatx16& a) {
  auto I = [&](int i) { return __float_as_int(a[i]); };
  auto mx = [](int x, int y) { return x > y ? x : y; };
  const int m0 = mx(mx(I(0), I(1)), I(2)), m1 = mx(mx(I(3), I(4)), I(5)), m2 = mx(mx(I(6), I(7)), I(8));
  const int m3 = mx(mx(I(9), I(10)), I(11)), m4 = mx(mx(I(12), I(13)), I(14));
  return mx(mx(mx(m0, m1), mx(m2, m3)), mx(m4, I(15)));
}

template <int MODE>
__global__ __launch_bounds__(512, 4) void k(const half8* __restrict__ src, int iters, int* out) {
  __shared__ half8 lds[2][256];
  const int tid = threadIdx.x, lane = tid & 63, col = lane & 31, h = lane >> 5;
  if (tid < 512) lds[tid >> 8][tid & 255] = src[tid];
  __syncthreads();
  const half8 b = src[lane];
  int acc = 0;
  for (int it = 0; it < iters; ++it) {
    const half8* l = &lds[h][col];
    if (MODE == 0) {  // MFMA only
      floatx16 c = {};
#pragma unroll
      for (int t = 0; t < 8; ++t) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(l[(t & 7) * 32 / 32 * 0 + t % 8 * 0], b, c, 0, 0, 0);
      acc += __float_as_int(c[0]) ^ __float_as_int(c[15]);
    } else if (MODE == 1) {  // serial: read, mfma, max
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const half8 a = l[t * 32 % 256];
        acc ^= imax16(__builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, floatx16{}, 0, 0, 0));
      }
    } else {  // two tiles in flight
      half8 a0 = l[0], a1 = l[32];
      floatx16 c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b, floatx16{}, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 8; t += 2) {
        if (t + 2 < 8) a0 = l[(t + 2) * 32 % 256];
        const floatx16 c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b, floatx16{}, 0, 0, 0);
        if (t + 3 < 8) a1 = l[(t + 3) * 32 % 256];
        acc ^= imax16(c0);
        if (t + 2 < 8) c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b, floatx16{}, 0, 0, 0);
        acc ^= imax16(c1);
      }
    }
  }
  if (acc == 0x12345) out[0] = acc;
}

int main() {
  half8* src; int* out;
  hipMalloc(&src, 512 * sizeof(half8)); hipMalloc(&out, 4);
  hipMemset(src, 0x3c, 512 * sizeof(half8));
  const int iters = 20000, blocks = 256 * 2;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    kern<<<blocks, 512>>>(src, iters, out);
    hipEventRecord(e0);
    kern<<<blocks, 512>>>(src, iters, out);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double tiles_per_simd = (double)blocks * 8 * iters * 8 / 1024.0;
    printf("%-28s %8.3f ms  %6.1f ns/tile/SIMD  (= %.1f cycles @2.1GHz)\n", name, ms, ms * 1e6 / tiles_per_simd,
           ms * 1e-3 / tiles_per_simd * 2.1e9);
  };
  run(k<0>, "mfma only (dependent acc)");
  run(k<1>, "serial read+mfma+max");
  run(k<2>, "two tiles in flight");
  return 0;
}
