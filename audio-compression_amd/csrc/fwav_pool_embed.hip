// fwav_pool_embed.hip — domain pool (mean-pooled sliding tiles) and the 16-d two-head DCT embedding.
//
// Replaces (reference /root/reference/fractal.py):
//   build_domains_memmap     :285-334  pool[d, k] = mean(signal[d·step + k·bl : … + bl]), bl = tile // rs
//   build_domain_embeddings  :238-280  → multi_head_embedding :166-175 → tile_embedding :178-208 (tonal head)
//                                        + transient_embedding :154-164
//
// Pool.  Each mean is numpy's pairwise float32 sum / bl (bit-exact).  When bl % step == 0 (every config in
// BASELINE.json), pool[d, k] = S[d + k·(bl/step)] with S[j] the mean of the bl samples starting at j·step,
// so only ≈ n/step block means are computed instead of nd·rs (8× less work at tile 2048): k_block_means.
// Otherwise k_domain_pool computes every (d, k) directly.
//
// Embedding (per domain, one thread).  The reference runs scipy's pocketfft per row; here the orthonormal
// DCT-II rows the embedding keeps are constant matrices built on the host in float64 (fwav_embed_tables),
// with the linspace(1, 2, n) weights folded in, evaluated in f64:
//   tonal[j]     = f32( Σ_n C[j+1][n]·w[j+1]·x[n] ),  j < min(8, rs−1), zero-padded; ‖·‖ f32, /‖·‖ if > 1e-8
//   transient[k] = Σ_n C[k][n]·w[n]·f64(x[n] − x[n−1]),  k < min(8, rs); f64 norm; /‖·‖ if > 1e-8; → f32
// Parity is |Δ| ≤ 1e-6 against the reference goldens (SURVEY Appendix A rule 2).
// Invariant relied on elsewhere: each head has norm ≤ 1 (normalised, or zero).  The similarity search's fp16 error
// bound δ (fwav_topk.hip kF16Delta) assumes Σ|q_k d_k| ≤ ‖q‖‖d‖ ≤ 2; a change here that breaks it (e.g. honouring
// transient_weight) must change δ too.  Checked by tests (test_embedding_heads_at_most_unit_norm, full-size cfg3).
#include "fwav_common.h"
#include "../../include/fwav.h"

namespace fwav {

constexpr int kPoolThreads = 256;

template <int BL>
__device__ __forceinline__ float block_mean_fixed(const float* __restrict__ x) {
  auto f = [&](int i) { return x[i]; };
  return pw_sum_n<BL>(f) / (float)BL;
}

// S[j] = pairwise_mean(sig[j*step : j*step + bl]),  j < ns.
template <int BL>
__global__ void k_block_means(const float* __restrict__ sig, int64_t ns, int step, int bl, float* __restrict__ S) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ns) return;
  const float* x = sig + j * step;
  if constexpr (BL > 0) {
    S[j] = block_mean_fixed<BL>(x);
  } else {
    auto f = [&](int i) { return x[i]; };
    S[j] = pw_sum(f, bl) / (float)bl;
  }
}

// General pool: one thread per (d, k).
__global__ void k_domain_pool(const float* __restrict__ sig, int64_t nd, int rs, int step, int bl,
                              float* __restrict__ pool) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nd * rs) return;
  int64_t d = t / rs;
  int k = (int)(t - d * rs);
  const float* x = sig + d * step + (int64_t)k * bl;
  auto f = [&](int i) { return x[i]; };
  pool[t] = pw_sum(f, bl) / (float)bl;
}

// Embedding of one domain row x[0..rs) read as src[d*a + k*b]; optionally writes the pool row.
//   tab layout (f64): tonal rows [8][rs] then transient rows [8][rs]; zero rows past take / tk.
template <int RS>
__global__ void k_embed(const float* __restrict__ src, int64_t nd, int rs, int64_t a, int64_t b,
                        const double* __restrict__ tab, float* __restrict__ pool_out, float* __restrict__ emb,
                        _Float16* __restrict__ emb16) {
  int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= nd) return;
  const int n = RS > 0 ? RS : rs;
  const float* xs = src + d * a;
  const int take = n - 1 < 8 ? n - 1 : 8;
  const int tk = n < 8 ? n : 8;
  const double* tt = tab;
  const double* td = tab + 8 * n;
  float e[8];
  double t[8];
  if constexpr (RS > 0) {
    float x[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) x[i] = xs[i * b];
    if (pool_out) {
#pragma unroll
      for (int i = 0; i < RS; ++i) pool_out[d * RS + i] = x[i];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < RS; ++i) acc += tt[j * RS + i] * (double)x[i];
      e[j] = j < take ? (float)acc : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = 0.0;
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      const double dd = (double)(i == 0 ? x[0] - x[0] : x[i] - x[i - 1]);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] += td[j * RS + i] * dd;
    }
  } else {
    if (pool_out) {
      for (int i = 0; i < n; ++i) pool_out[d * n + i] = xs[i * b];
    }
    for (int j = 0; j < 8; ++j) {
      double acc = 0.0;
      for (int i = 0; i < n; ++i) acc += tt[j * n + i] * (double)xs[i * b];
      e[j] = j < take ? (float)acc : 0.0f;
    }
    for (int j = 0; j < 8; ++j) t[j] = 0.0;
    for (int i = 0; i < n; ++i) {
      float xi = xs[i * b];
      float xp = i == 0 ? xi : xs[(i - 1) * b];
      double dd = (double)(xi - xp);
      for (int j = 0; j < 8; ++j) t[j] += td[j * n + i] * dd;
    }
  }
  // tonal: f32 norm (short sdot: sequential), normalise if > 1e-8
  float s2 = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s2 = s2 + e[j] * e[j];
  float nrm = sqrtf(s2);
  if (nrm > 1e-8f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = e[j] / nrm;
  }
  // transient: f64 norm over the tk kept coefficients
  double s2d = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s2d += j < tk ? t[j] * t[j] : 0.0;
  double nd64 = sqrt(s2d);
  float tf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    double v = j < tk ? t[j] : 0.0;
    if (nd64 > 1e-8) v = v / nd64;
    tf[j] = (float)v;
  }
  // concatenation [tonal 8 | transient tk] then zero pad to 16 (multi_head_embedding :170-175)
  float out[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) out[j] = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = e[j];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (j < tk) out[8 + j] = tf[j];
  float4* o4 = reinterpret_cast<float4*>(emb + d * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) o4[j] = make_float4(out[4 * j], out[4 * j + 1], out[4 * j + 2], out[4 * j + 3]);
  if (emb16 != nullptr) {
    // fp16 copies for the similarity search, tiled [chunk of 256][half h][256][8] (fwav_topk.hip): the high part
    // x_hi = f16(x) (the stream's pre-filter), then, one table further on, the low part x_lo = f16(x − x_hi)
    // (the replay's refined score x_hi·y_hi + x_hi·y_lo + x_lo·y_hi)
    const int64_t c = d >> 8, j = d & 255;
    const int64_t n16 = ((nd + 255) >> 8) * 256 * 16;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      typedef _Float16 half8 __attribute__((ext_vector_type(8)));
      half8 vh, vl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        vh[e] = (_Float16)out[8 * hh + e];
        vl[e] = (_Float16)(out[8 * hh + e] - (float)vh[e]);
      }
      *reinterpret_cast<half8*>(emb16 + ((c * 2 + hh) * 256 + j) * 8) = vh;
      *reinterpret_cast<half8*>(emb16 + n16 + ((c * 2 + hh) * 256 + j) * 8) = vl;
    }
  }
}

template <int RS>
static void launch_embed(const float* src, int64_t nd, int rs, int64_t a, int64_t b, const double* tab,
                         float* pool_out, float* emb, _Float16* emb16, hipStream_t st) {
  k_embed<RS><<<cdiv(nd, kPoolThreads), kPoolThreads, 0, st>>>(src, nd, rs, a, b, tab, pool_out, emb, emb16);
}

}  // namespace fwav

using namespace fwav;

extern "C" {

size_t fwav_emb16_elems(int64_t nd) { return (size_t)(2 * ((nd + 255) / 256) * 256 * 16); }

// Host-side f64 tables for fwav_pool_embed: tab[16 * rs] (tonal 8 rows, transient 8 rows).
int fwav_embed_tables(int rs, double* tab) {
  FWAV_CHECK_ARG(rs >= 1 && rs <= kMaxPairwise && tab, FWAV_ERR_ARG, "fwav_embed_tables: bad args");
  const double pi = 3.14159265358979323846;
  const int n = rs;
  auto w = [&](int i) { return n == 1 ? 1.0 : 1.0 + (double)i / (double)(n - 1); };  // np.linspace(1, 2, n)
  auto c = [&](int k, int i) {
    double f = k == 0 ? std::sqrt(1.0 / n) : std::sqrt(2.0 / n);
    return f * std::cos(pi * k * (2.0 * i + 1.0) / (2.0 * n));
  };
  const int take = n - 1 < 8 ? n - 1 : 8;
  const int tk = n < 8 ? n : 8;
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < n; ++i) tab[j * n + i] = j < take ? c(j + 1, i) * w(j + 1) : 0.0;
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < n; ++i) tab[8 * n + j * n + i] = j < tk ? c(j, i) * w(i) : 0.0;
  return FWAV_OK;
}

size_t fwav_pool_workspace_size(int64_t n, int tile, int rs, int step) {
  const int bl = tile / rs;
  if (n < tile || bl % step != 0) return 0;
  const int64_t nd = (n - tile) / step + 1;
  const int64_t ns = (nd - 1) + (int64_t)(rs - 1) * (bl / step) + 1;
  return (size_t)ns * sizeof(float);
}

// Domain pool + embedding.  pool: f32[nd*rs], emb: f32[nd*16], tab: device copy of fwav_embed_tables(rs).
// emb16 (optional): fp16 high and low parts in the tiled layout the similarity search streams,
// f16[fwav_emb16_elems(nd)] = 2 tables of ceil(nd/256)*256*16; rows past nd are zeroed here.
int fwav_pool_embed(const float* sig, int64_t n, int tile, int rs, int step, const double* tab, float* pool,
                    float* emb, void* emb16, void* workspace, size_t ws_bytes, void* stream) {
  FWAV_CHECK_ARG(sig && pool && emb && tab && tile > 0 && rs > 0 && step > 0, FWAV_ERR_ARG,
                 "fwav_pool_embed: bad args");
  FWAV_CHECK_ARG(n >= tile, FWAV_ERR_SHAPE, "fwav_pool_embed: n < tile");
  const int bl = tile / rs;
  FWAV_CHECK_ARG(bl >= 1 && bl <= kMaxPairwise && rs <= kMaxPairwise, FWAV_ERR_SHAPE,
                 "fwav_pool_embed: block length out of range");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nd = (n - tile) / step + 1;
  const float* src;
  int64_t a, b;
  float* pool_out;
  if (bl % step == 0) {
    FWAV_CHECK_ARG(ws_bytes >= fwav_pool_workspace_size(n, tile, rs, step) && workspace, FWAV_ERR_WORKSPACE,
                   "fwav_pool_embed: workspace too small");
    const int64_t m = bl / step;
    const int64_t ns = (nd - 1) + (int64_t)(rs - 1) * m + 1;
    float* S = (float*)workspace;
    const int64_t g = cdiv(ns, kPoolThreads);
    if (bl == 256) k_block_means<256><<<g, kPoolThreads, 0, st>>>(sig, ns, step, bl, S);
    else if (bl == 128) k_block_means<128><<<g, kPoolThreads, 0, st>>>(sig, ns, step, bl, S);
    else k_block_means<0><<<g, kPoolThreads, 0, st>>>(sig, ns, step, bl, S);
    src = S; a = 1; b = m; pool_out = pool;
  } else {
    k_domain_pool<<<cdiv(nd * rs, kPoolThreads), kPoolThreads, 0, st>>>(sig, nd, rs, step, bl, pool);
    src = pool; a = rs; b = 1; pool_out = nullptr;
  }
  _Float16* e16 = (_Float16*)emb16;
  if (e16 != nullptr && (nd & 255) != 0) {
    // zero the padded tail of the last chunk (both halves of both tables)
    const int64_t c = nd >> 8, j0 = nd & 255;
    const int64_t n16 = ((nd + 255) >> 8) * 256 * 16;
    for (int tb = 0; tb < 2; ++tb)
      for (int hh = 0; hh < 2; ++hh)
        (void)hipMemsetAsync(e16 + tb * n16 + ((c * 2 + hh) * 256 + j0) * 8, 0,
                             (size_t)(256 - j0) * 8 * sizeof(_Float16), st);
  }
  switch (rs) {
    case 4: launch_embed<4>(src, nd, rs, a, b, tab, pool_out, emb, e16, st); break;
    case 8: launch_embed<8>(src, nd, rs, a, b, tab, pool_out, emb, e16, st); break;
    case 16: launch_embed<16>(src, nd, rs, a, b, tab, pool_out, emb, e16, st); break;
    default: launch_embed<0>(src, nd, rs, a, b, tab, pool_out, emb, e16, st); break;
  }
  FWAV_LAUNCH_CHECK("fwav_pool_embed");
  return FWAV_OK;
}

}  // extern "C"
