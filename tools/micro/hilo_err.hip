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
#include <string>
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

__global__ void k_denorm(float* out) {
  // one MFMA whose only non-zero products are fp16 subnormals: 2^-24 · 1 and (3·2^-24) · 0.5
  const int lane = threadIdx.x & 63;
  half8 a{}, b{};
  if (lane == 0) { a[0] = (_Float16)5.9604645e-8f; a[1] = (_Float16)1.7881393e-7f; }
  if (lane == 0) { b[0] = (_Float16)1.0f; b[1] = (_Float16)0.5f; }
  const floatx16 r = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, floatx16{}, 0, 0, 0);
  if (lane == 0) out[0] = r[0];
}

// Adversarial unit-head vectors (argv[1] == "adv"): components exactly halfway between fp16 neighbours (the hi
// split rounds to even, the lo part is a whole half-ulp), components below 2^-14 (fp16-subnormal hi parts) and
// below 2^-3 (fp16-subnormal lo parts); heads scaled by powers of two only, so the constructions stay exact.
static void adversarial(float* v, std::mt19937& g) {
  std::uniform_int_distribution<int> mant(0, 1023), ex(-6, -1), kind(0, 3), sgn(0, 1);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  for (int hh = 0; hh < 2; ++hh) {
    const int kd = kind(g);
    for (int j = 0; j < 8; ++j) {
      float x;
      if (kd == 0 || (kd == 3 && j < 4)) {
        x = std::ldexp((float)(1024 + mant(g)) + 0.5f, ex(g) - 10);  // fp16 midpoint
      } else if (kd == 1) {
        x = (j % 2) ? std::ldexp(1.f + u(g), -15 - (j % 9)) : std::ldexp((float)(1024 + mant(g)) + 0.5f, -11);
      } else {
        x = std::ldexp(u(g), -4 - (j % 3));  // < 2^-3: fp16-subnormal lo parts
      }
      v[8 * hh + j] = sgn(g) ? -x : x;
    }
    for (;;) {  // norm ≤ 1 by exact halvings
      double s = 0;
      for (int j = 0; j < 8; ++j) s += (double)v[8 * hh + j] * v[8 * hh + j];
      if (s <= 1.0) break;
      for (int j = 0; j < 8; ++j) v[8 * hh + j] *= 0.5f;
    }
  }
}

int main(int argc, char** argv) {
  const bool adv = argc > 1 && std::string(argv[1]) == "adv";
  {
    float* dout;
    hipMalloc(&dout, 4);
    k_denorm<<<1, 64>>>(dout);
    float r = 0;
    hipMemcpy(&r, dout, 4, hipMemcpyDeviceToHost);
    std::printf("fp16-subnormal MFMA products: %.9g (expected %.9g: %s)\n", r, 5.9604645e-8 + 0.5 * 1.7881393e-7,
                r == (float)(5.9604645e-8 + 0.5 * 1.7881393e-7) ? "kept" : "FLUSHED");
  }
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
  for (int i = 0; i < 32; ++i) {
    if (adv) adversarial(&Q[i * 16], g); else unit_heads(&Q[i * 16]);
  }
  for (int i = 0; i < N; ++i) {
    float* v = &D[(size_t)i * 16];
    const bool dup = (i % 3) == 0;
    if (adv) {
      adversarial(v, g);
      if (dup)  // the query itself with one component moved to a neighbouring fp16 midpoint
        for (int j = 0; j < 16; ++j) v[j] = Q[(i % 32) * 16 + j] * ((j == i % 16) ? 0.99951171875f : 1.f);
      continue;
    }
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
