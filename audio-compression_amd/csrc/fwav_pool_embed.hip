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
// Embedding (per domain, one thread), bit-exact with the reference for range sizes 4, 8 and 16 (every config in
// BASELINE.json and the goldens):
//   tonal[j]     = f32( f32-DCT(x)[j+1] · w[j+1] ), j < min(8, rs−1), zero-padded to 8; ‖·‖ as np.linalg.norm of a
//                  1-D float32 vector evaluates it (OpenBLAS sdot: f32 products summed in f64, rounded to f32, f32
//                  sqrt); / ‖·‖ in f32 if ‖·‖ > f32(1e-8)                                    (fractal.py:178-208)
//   transient[k] = f64-DCT(f64(x[n] − x[n−1]) · w[n])[k], k < min(8, rs); ‖·‖ as ddot (n < 16: a sequential f64 fma
//                  chain) then sqrt; / ‖·‖ if > 1e-8; → f32                                  (fractal.py:154-164)
// with the DCTs scipy's own pocketfft operation sequence in each precision (fwav_dct.h) and w = np.linspace(1, 2, rs)
// as numpy computes it (i·(1/(rs−1)) + 1, last = 2).  Other range sizes take the f64 matrix DCT (within 1e-6,
// SURVEY Appendix A rule 2).  fwav_embed_tables packs the matrices and pocketfft's constants for both precisions.
#include "fwav_common.h"
#include "fwav_dct.h"
#include "../../include/fwav.h"

#include <utility>
#include <vector>

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
// fp16 copies of embedding row d for the similarity search, tiled [chunk of 256][half h][256][8] (fwav_topk.hip): the
// high part x_hi = f16(x) (the stream's pre-filter), then, one table further on, the low part x_lo = f16(x − x_hi)
// (the replay's refined score x_hi·y_hi + x_hi·y_lo + x_lo·y_hi).  Both conversions round to nearest even and keep
// fp16 subnormals (the hi/lo error bound, DESIGN §3.1, counts on them).
__device__ __forceinline__ void store_emb16(_Float16* __restrict__ emb16, int64_t nd, int64_t d, const float (&out)[16]) {
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
  float tf[8];
  if constexpr (RS == 4 || RS == 8 || RS == 16) {
    // exact path: scipy's pocketfft DCTs and numpy's / OpenBLAS's norm orders (see the file header)
    DctK<float, RS> kf;
    DctK<double, RS> kd;
    dct_load(kf, tab + 16 * RS);
    dct_load(kd, tab + 16 * RS + dct_block(RS));
    float x[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) x[i] = xs[i * b];
    if (pool_out) {
#pragma unroll
      for (int i = 0; i < RS; ++i) pool_out[d * RS + i] = x[i];
    }
    float c[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) c[i] = x[i];
    dct2_ortho<float, RS>(c, kf);
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = j < take ? (float)((double)c[j + 1 < RS ? j + 1 : 0] * kd.w[j + 1 < RS ? j + 1 : 0]) : 0.0f;
    double acc = 0.0;  // sdot: f32 products, f64 sum in index order, f32 result
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = acc + (double)(e[j] * e[j]);
    const float nrm = sqrtf((float)acc);
    if (nrm > 1e-8f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = e[j] / nrm;
    }
    double dv[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) dv[i] = (double)(i == 0 ? x[0] - x[0] : x[i] - x[i - 1]) * kd.w[i];
    dct2_ortho<double, RS>(dv, kd);
    double s2 = 0.0;  // ddot, n < 16: fma chain
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < tk) s2 = __builtin_fma(dv[j < RS ? j : 0], dv[j < RS ? j : 0], s2);
    const double nrmd = sqrt(s2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double v = j < tk ? dv[j < RS ? j : 0] : 0.0;
      if (nrmd > 1e-8) v = v / nrmd;
      tf[j] = (float)v;
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
    double acc = 0.0;  // tonal norm in sdot order
    for (int j = 0; j < 8; ++j) acc = acc + (double)(e[j] * e[j]);
    const float nrm = sqrtf((float)acc);
    if (nrm > 1e-8f) {
      for (int j = 0; j < 8; ++j) e[j] = e[j] / nrm;
    }
    double s2d = 0.0;  // transient: ddot fma chain over the tk kept coefficients
    for (int j = 0; j < 8; ++j)
      if (j < tk) s2d = __builtin_fma(t[j], t[j], s2d);
    const double nd64 = sqrt(s2d);
    for (int j = 0; j < 8; ++j) {
      double v = j < tk ? t[j] : 0.0;
      if (nd64 > 1e-8) v = v / nd64;
      tf[j] = (float)v;
    }
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
  if (emb16 != nullptr) store_emb16(emb16, nd, d, out);
}

// Domain-embedding rows → the fp16 tables of the search (store_emb16), for embeddings produced elsewhere.
__global__ __launch_bounds__(kPoolThreads) void k_emb16(const float* __restrict__ emb, int64_t nd,
                                                        _Float16* __restrict__ emb16) {
  const int64_t d = (int64_t)blockIdx.x * kPoolThreads + threadIdx.x;
  if (d >= nd) return;
  float out[16];
  const float4* p = reinterpret_cast<const float4*>(emb + d * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 v = p[j];
    out[4 * j] = v.x; out[4 * j + 1] = v.y; out[4 * j + 2] = v.z; out[4 * j + 3] = v.w;
  }
  store_emb16(emb16, nd, d, out);
}

template <int RS>
static void launch_embed(const float* src, int64_t nd, int rs, int64_t a, int64_t b, const double* tab,
                         float* pool_out, float* emb, _Float16* emb16, hipStream_t st) {
  k_embed<RS><<<cdiv(nd, kPoolThreads), kPoolThreads, 0, st>>>(src, nd, rs, a, b, tab, pool_out, emb, emb16);
}

// pocketfft's sincos_2pibyn<T>(n)[idx] (Thigh = double for float and double): a two-level table of octant-reduced
// cos/sin in double, entries multiplied in double — reproduced so that the twiddles are pocketfft's own values.
struct SinCos2PiByN {
  size_t n, shift, mask;
  std::vector<std::pair<double, double>> v1, v2;
  static std::pair<double, double> calc(size_t x, size_t n, double ang) {
    x <<= 3;
    if (x < 4 * n) {
      if (x < 2 * n) {
        if (x < n) return {std::cos(double(x) * ang), std::sin(double(x) * ang)};
        return {std::sin(double(2 * n - x) * ang), std::cos(double(2 * n - x) * ang)};
      }
      x -= 2 * n;
      if (x < n) return {-std::sin(double(x) * ang), std::cos(double(x) * ang)};
      return {-std::cos(double(2 * n - x) * ang), std::sin(double(2 * n - x) * ang)};
    }
    x = 8 * n - x;
    if (x < 2 * n) {
      if (x < n) return {std::cos(double(x) * ang), -std::sin(double(x) * ang)};
      return {std::sin(double(2 * n - x) * ang), -std::cos(double(2 * n - x) * ang)};
    }
    x -= 2 * n;
    if (x < n) return {-std::sin(double(x) * ang), -std::cos(double(x) * ang)};
    return {-std::cos(double(2 * n - x) * ang), -std::sin(double(2 * n - x) * ang)};
  }
  explicit SinCos2PiByN(size_t n_) : n(n_) {
    const long double pi = 3.141592653589793238462643383279502884197L;
    const double ang = (double)(0.25L * pi / (long double)n);
    const size_t nval = (n + 2) / 2;
    shift = 1;
    while (((size_t)1 << shift) * ((size_t)1 << shift) < nval) ++shift;
    mask = ((size_t)1 << shift) - 1;
    v1.resize(mask + 1);
    v1[0] = {1.0, 0.0};
    for (size_t i = 1; i < v1.size(); ++i) v1[i] = calc(i, n, ang);
    v2.resize((nval + mask) / (mask + 1));
    v2[0] = {1.0, 0.0};
    for (size_t i = 1; i < v2.size(); ++i) v2[i] = calc(i * (mask + 1), n, ang);
  }
  std::pair<double, double> operator[](size_t idx) const {
    if (2 * idx <= n) {
      const auto x1 = v1[idx & mask], x2 = v2[idx >> shift];
      return {x1.first * x2.first - x1.second * x2.second, x1.first * x2.second + x1.second * x2.first};
    }
    idx = n - idx;
    const auto x1 = v1[idx & mask], x2 = v2[idx >> shift];
    return {x1.first * x2.first - x1.second * x2.second, -(x1.first * x2.second + x1.second * x2.first)};
  }
};

// DctK<T, n> constants (T = double if dbl, else float, stored as doubles) exactly as pocketfft / numpy compute them:
// T_dcst23 twiddle[i] = T(sincos_2pibyn(4n)[i+1].r); the first rfftp factor's twiddles (comp_twiddle); fct =
// T(1/sqrt(long double(2n))); sqrt2 = T(1.414…L); w = np.linspace(1, 2, n) in double (arange · (1/(n−1)) + 1, last 2).
void dct_constants(int n, bool dbl, double* out) {
  auto r = [&](long double v) { return dbl ? (double)v : (double)(float)v; };
  for (int i = 0; i < 9; ++i) out[n + i] = 0.0;
  const SinCos2PiByN s4(4 * (size_t)n), s1((size_t)n);
  for (int i = 0; i < n; ++i) out[i] = r(s4[i + 1].first);
  if (n == 8) {  // radb2, l1 = 1, ido = 4
    out[n + 0] = r(s1[1].first);
    out[n + 1] = r(s1[1].second);
  } else if (n == 16) {  // radb4, l1 = 1, ido = 4
    for (int j = 1; j < 4; ++j) {
      out[n + (j - 1) * 3 + 0] = r(s1[j].first);
      out[n + (j - 1) * 3 + 1] = r(s1[j].second);
    }
  }
  const double step = 1.0 / (double)(n - 1);
  for (int i = 0; i < n; ++i) out[n + 9 + i] = i == n - 1 ? 2.0 : (double)i * step + 1.0;
  out[2 * n + 9] = r(1.0L / std::sqrt((long double)(2 * n)));
  out[2 * n + 10] = r(1.414213562373095048801688724209698L);
}

}  // namespace fwav

using namespace fwav;

extern "C" {

size_t fwav_emb16_elems(int64_t nd) { return (size_t)(2 * ((nd + 255) / 256) * 256 * 16); }

// Host-side f64 tables for fwav_pool_embed: tab[fwav_embed_tables_size(rs)] = the matrices (tonal 8 rows, transient 8
// rows of rs) and, for rs = 4, 8, 16, pocketfft's constants in float32 then float64 (DctK layout, dct_constants).
size_t fwav_embed_tables_size(int rs) {
  return (size_t)16 * rs + ((rs == 4 || rs == 8 || rs == 16) ? 2 * (size_t)dct_block(rs) : 0);
}

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
  if (rs == 4 || rs == 8 || rs == 16) {
    dct_constants(rs, false, tab + 16 * rs);
    dct_constants(rs, true, tab + 16 * rs + dct_block(rs));
  }
  return FWAV_OK;
}

// Test hook (host): scipy.fftpack.dct(x, norm='ortho') of n = 4, 8, 16 doubles (dbl = 1) or floats (dbl = 0, passed
// and returned as doubles) through fwav_dct.h — the code the embedding kernel runs, instantiated on the host.
int fwav_debug_dct2(int n, int dbl, const double* x, double* out) {
  FWAV_CHECK_ARG((n == 4 || n == 8 || n == 16) && x && out, FWAV_ERR_ARG, "fwav_debug_dct2: n must be 4, 8 or 16");
  double tab[2 * (2 * 16 + 11)];
  dct_constants(n, dbl != 0, tab);
  auto run = [&](auto tag, auto nn) {
    using T = decltype(tag);
    constexpr int N = decltype(nn)::value;
    DctK<T, N> k;
    dct_load(k, tab);
    T c[N];
    for (int i = 0; i < N; ++i) c[i] = (T)x[i];
    dct2_ortho<T, N>(c, k);
    for (int i = 0; i < N; ++i) out[i] = (double)c[i];
  };
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  using I16 = std::integral_constant<int, 16>;
  if (dbl) {
    if (n == 4) run(0.0, I4{}); else if (n == 8) run(0.0, I8{}); else run(0.0, I16{});
  } else {
    if (n == 4) run(0.0f, I4{}); else if (n == 8) run(0.0f, I8{}); else run(0.0f, I16{});
  }
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
// fp16 search tables (f16[fwav_emb16_elems(nd)]) of embedding rows emb f32[nd*16], as fwav_pool_embed writes them.
int fwav_emb16_from_emb(const float* emb, int64_t nd, void* emb16, void* stream) {
  FWAV_CHECK_ARG(emb && emb16 && nd > 0, FWAV_ERR_ARG, "fwav_emb16_from_emb: bad args");
  hipStream_t st = (hipStream_t)stream;
  _Float16* e16 = (_Float16*)emb16;
  if ((nd & 255) != 0) {
    const int64_t c = nd >> 8, j0 = nd & 255;
    const int64_t n16 = ((nd + 255) >> 8) * 256 * 16;
    for (int tb = 0; tb < 2; ++tb)
      for (int hh = 0; hh < 2; ++hh)
        (void)hipMemsetAsync(e16 + tb * n16 + ((c * 2 + hh) * 256 + j0) * 8, 0,
                             (size_t)(256 - j0) * 8 * sizeof(_Float16), st);
  }
  k_emb16<<<cdiv(nd, kPoolThreads), kPoolThreads, 0, st>>>(emb, nd, e16);
  FWAV_LAUNCH_CHECK("fwav_emb16_from_emb");
  return FWAV_OK;
}

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
