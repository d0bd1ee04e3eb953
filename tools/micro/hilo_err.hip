// Micro-check of the similarity search's two fp16 score estimates against exact arithmetic (gfx950).
//   s16 = MFMA(d_hi, q_hi)                                   (the stream's pre-filter)
//   shl = MFMA(d_hi, q_lo) + MFMA(d_lo, q_hi) + s16, f32 acc   (the replay's refined score; x_lo = f16(x − x_hi))
// over unit-head 16-d vectors (random and near-duplicates of the queries, which maximise Σ|q_k d_k|).  Prints the
// largest |s16 − s| and |shl − s| against the f64 dot s and against the f32 sgemv-order score.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/hilo_err tools/micro/hilo_err.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void k(const half8* __restrict__ dhi, const half8* __restrict__ dlo, const half8* __restrict__ qhi,
                  const half8* __restrict__ qlo, int ntiles, float* __restrict__ s16, float* __restrict__ shl) {
  const int lane = threadIdx.x & 63, col = lane & 31, h = lane >> 5;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntiles) return;
  const half8 bh = qhi[col * 2 + h], bl = qlo[col * 2 + h];
  const int d = t * 32 + col;
  const half8 ah = dhi[d * 2 + h], al = dlo[d * 2 + h];
  const floatx16 a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, floatx16{}, 0, 0, 0);
  floatx16 a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, a0, 0, 0, 0);
  a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, a1, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    const int dd = t * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
    s16[(size_t)dd * 32 + col] = a0[r];
    shl[(size_t)dd * 32 + col] = a1[r];
  }
}

static float sgemv(const float* q, const float* d) {
  float l[8];
  for (int j = 0; j < 8; ++j) l[j] = std::fmaf(q[j + 8], d[j + 8], q[j] * d[j]);
  float r[4];
  for (int i = 0; i < 4; ++i) r[i] = l[i] + l[i + 4];
  return (r[0] + r[1]) + (r[2] + r[3]);
}

int main() {
  const int N = 32 * 8192;
  std::mt19937 g(1);
  std::normal_distribution<float> nrm(0.f, 1.f);
  auto unit_heads = [&](float* v) {
    for (int hh = 0; hh < 2; ++hh) {
      double s = 0;
      for (int j = 0; j < 8; ++j) s += (double)v[8 * hh + j] * v[8 * hh + j];
      const float n = (float)std::sqrt(s);
      for (int j = 0; j < 8; ++j) v[8 * hh + j] /= n;
    }
  };
  std::vector<float> Q(32 * 16), D((size_t)N * 16);
  for (auto& x : Q) x = nrm(g);
  for (int i = 0; i < 32; ++i) unit_heads(&Q[i * 16]);
  for (int i = 0; i < N; ++i) {
    float* v = &D[(size_t)i * 16];
    const bool dup = (i % 3) == 0;
    const float eps = (i % 7) * 1e-3f;
    for (int j = 0; j < 16; ++j) v[j] = dup ? Q[(i % 32) * 16 + j] + eps * nrm(g) : nrm(g);
    if ((i % 11) == 0)  // small magnitudes (fp16 subnormal lo parts)
      for (int j = 0; j < 16; ++j) v[j] *= (j % 2) ? 1e-4f : 1.f;
    unit_heads(v);
  }
  auto split = [](const std::vector<float>& x, std::vector<_Float16>& hi, std::vector<_Float16>& lo) {
    hi.resize(x.size());
    lo.resize(x.size());
    for (size_t i = 0; i < x.size(); ++i) {
      hi[i] = (_Float16)x[i];
      lo[i] = (_Float16)(x[i] - (float)hi[i]);
    }
  };
  std::vector<_Float16> qh, ql, dh, dl;
  split(Q, qh, ql);
  split(D, dh, dl);
  _Float16 *dqh, *dql, *ddh, *ddl;
  float *ds16, *dshl;
  hipMalloc(&dqh, qh.size() * 2);
  hipMalloc(&dql, ql.size() * 2);
  hipMalloc(&ddh, dh.size() * 2);
  hipMalloc(&ddl, dl.size() * 2);
  hipMalloc(&ds16, (size_t)N * 32 * 4);
  hipMalloc(&dshl, (size_t)N * 32 * 4);
  hipMemcpy(dqh, qh.data(), qh.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dql, ql.data(), ql.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(ddh, dh.data(), dh.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(ddl, dl.data(), dl.size() * 2, hipMemcpyHostToDevice);
  const int ntiles = N / 32;
  k<<<(ntiles + 3) / 4, 256>>>((const half8*)ddh, (const half8*)ddl, (const half8*)dqh, (const half8*)dql, ntiles,
                               ds16, dshl);
  std::vector<float> s16((size_t)N * 32), shl((size_t)N * 32);
  hipMemcpy(s16.data(), ds16, s16.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(shl.data(), dshl, shl.size() * 4, hipMemcpyDeviceToHost);
  double e16 = 0, ehl = 0, ehl_sg = 0, e16_sg = 0, esg = 0, smax = 0;
  for (int d = 0; d < N; ++d)
    for (int q = 0; q < 32; ++q) {
      double s = 0;
      for (int j = 0; j < 16; ++j) s += (double)Q[q * 16 + j] * D[(size_t)d * 16 + j];
      const float sg = sgemv(&Q[q * 16], &D[(size_t)d * 16]);
      const size_t i = (size_t)d * 32 + q;
      e16 = std::fmax(e16, std::fabs(s16[i] - s));
      ehl = std::fmax(ehl, std::fabs(shl[i] - s));
      e16_sg = std::fmax(e16_sg, std::fabs((double)s16[i] - sg));
      ehl_sg = std::fmax(ehl_sg, std::fabs((double)shl[i] - sg));
      esg = std::fmax(esg, std::fabs(sg - s));
      smax = std::fmax(smax, s);
    }
  std::printf("pairs %d  max score %.6f\n", N * 32, smax);
  std::printf("max |s16 - s64| %.4e   max |s16 - s32sgemv| %.4e\n", e16, e16_sg);
  std::printf("max |shl - s64| %.4e   max |shl - s32sgemv| %.4e   max |s32sgemv - s64| %.4e\n", ehl, ehl_sg, esg);
  return 0;
}
