// fwav_common.h — shared device helpers for the MI355X (gfx950) fractal-WAV kernels.
//
// Arithmetic contract (pinned by oracle/fractal_oracle.py against the reference
// goldens): every reduction is numpy's pairwise_sum order with numpy's initial "0 +", every elementwise op is
// one separately rounded f32 op.  The library is compiled with -ffp-contract=off and correctly rounded f32
// divide/sqrt, so `a * b + c` below is two roundings, exactly as numpy evaluates it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstring>

namespace fwav {

// ----------------------------------------------------------------------------------------- status
// Thread-local last-error string returned by fwav_last_error(); no exceptions cross the C ABI.
void set_error(const char* fmt, ...);

#define FWAV_CHECK_ARG(cond, code, ...)        \
  do {                                         \
    if (!(cond)) {                             \
      ::fwav::set_error(__VA_ARGS__);          \
      return (code);                           \
    }                                          \
  } while (0)

#define FWAV_LAUNCH_CHECK(what)                                                         \
  do {                                                                                  \
    hipError_t e_ = hipGetLastError();                                                  \
    if (e_ != hipSuccess) {                                                             \
      ::fwav::set_error("%s: %s", (what), hipGetErrorString(e_));                       \
      return FWAV_ERR_HIP;                                                              \
    }                                                                                   \
  } while (0)

constexpr int kWave = 64;
constexpr int kXcds = 8;  // MI355X: workgroups are dealt round-robin over 8 XCDs, each with its own 4 MiB L2

// Bijective XCD-aware renumbering of workgroup b of nwg: the blocks that share an XCD (b ≡ x mod 8) get one
// contiguous run of logical indices, so neighbouring work items — which gather overlapping rows — share an L2
// (cdna_hip_programming.md §5.5 T1; placement is a speed choice only, never relied on for correctness).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nwg) {
  const int64_t x = b % kXcds, q = nwg / kXcds, r = nwg % kXcds;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / kXcds;
}

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ----------------------------------------------------------------------- numpy pairwise reductions
// pairwise_sum (numpy loops_utils.h.src) of f(off .. off+n-1):
//   n < 8: sequential from 0;  8 <= n <= 128: 8 strided accumulators + tree + sequential tail;
//   n > 128: split at n2 = n/2 - (n/2)%8 and add the halves.
// Generic over the element type T = decltype(f(i)): float, or a 2-wide float vector (two independent sums in
// one packed-f32 instruction stream; each lane of the vector is rounded exactly like the scalar sum).
template <class F>
__device__ __forceinline__ auto pw_leaf(const F& f, int off, int n) -> decltype(f(0)) {
  using T = decltype(f(0));
  if (n < 8) {
    T r = (T)0.0f;
    for (int i = 0; i < n; ++i) r = r + f(off + i);
    return r;
  }
  T r0 = f(off + 0), r1 = f(off + 1), r2 = f(off + 2), r3 = f(off + 3);
  T r4 = f(off + 4), r5 = f(off + 5), r6 = f(off + 6), r7 = f(off + 7);
  const int m = n - (n & 7);
  for (int i = 8; i < m; i += 8) {
    r0 = r0 + f(off + i + 0);
    r1 = r1 + f(off + i + 1);
    r2 = r2 + f(off + i + 2);
    r3 = r3 + f(off + i + 3);
    r4 = r4 + f(off + i + 4);
    r5 = r5 + f(off + i + 5);
    r6 = r6 + f(off + i + 6);
    r7 = r7 + f(off + i + 7);
  }
  T res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (int i = m; i < n; ++i) res = res + f(off + i);
  return res;
}

template <int D, class F>
__device__ __forceinline__ auto pw_rec(const F& f, int off, int n) -> decltype(f(0)) {
  if constexpr (D == 0) {
    return pw_leaf(f, off, n);
  } else {
    if (n <= 128) return pw_leaf(f, off, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_rec<D - 1>(f, off, n2) + pw_rec<D - 1>(f, off + n2, n - n2);
  }
}

// np.add.reduce over n <= kMaxPairwise elements: numpy starts the output at 0 (so -0 sums to +0).
constexpr int kMaxPairwise = 1024;
// Records of the search's tie list (fwav_sim_topk `ties`): the query, then its K-th place tie group (fwav_topk.hip
// record_tie), int32 each.
constexpr int kTieRec = 9;
template <class F>
__device__ __forceinline__ auto pw_sum(const F& f, int n) -> decltype(f(0)) {
  return 0.0f + pw_rec<3>(f, 0, n);
}

// Compile-time-length variant (fully unrolled, register-resident operands).
template <int N, class F>
__device__ __forceinline__ auto pw_sum_n(const F& f) -> decltype(f(0)) {
  return 0.0f + pw_rec<3>(f, 0, N);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// The reference's f32 similarity scores, emb_dom @ q (fractal.py:537), in the order its BLAS evaluates them: numpy's
// sgemv on the (n_domains, 16) table goes to OpenBLAS 0.3.29 sgemv_t (Haswell/Zen/SkylakeX kernels), which scores
// a column (domain) with one of three kernels (oracle/fractal_oracle.py sgemv_col_kind / sgemv_scores, pinned
// against numpy on every column for 1, 3, 5, 7 and 8 threads):
//   kind 0, the 4-column microkernel: 8 fma lanes l_j = fma(d[j+8], q[j+8], 0 + d[j]·q[j]), then 256 → 128 bits and
//           two horizontal adds: ((l0 + l4) + (l1 + l5)) + ((l2 + l6) + (l3 + l7));
//   kind 1, the 4x2 tail kernel (SSE): l_j = (((0 + p_j) + p_{j+4}) + p_{j+8}) + p_{j+12} of the rounded products
//           p_k = d[k]·q[k], then (l0 + l1) + (l2 + l3);
//   kind 2, the 4x1 tail kernel: l_j = (0 + p_j) + p_{j+8} (8 lanes), then ((l0 + l4) + (l1 + l5)) + ((l2 + l6) + …).
// Which kernel scores domain d depends on how gemv_thread.c splits the nd columns over OpenBLAS's T threads (T = 1
// while 16·nd < 460,800): widths ceil(rest / threads left), i.e. the first nd mod T chunks one column wider, and each
// chunk's last (width mod 4) columns go to the tail kernels (2 → 4x2, 1 → 4x1, 3 → 4x2 then 4x1).  D(k) and Q(k)
// return the k-th element of the domain row and of the query.
struct SgemvSplit {
  uint32_t q, r;  // chunk width q; the first r chunks are q + 1 wide
};
__host__ inline SgemvSplit make_sgemv_split(int64_t nd, int threads) {
  const int64_t T = (16 * nd < 460800 || threads < 1) ? 1 : threads;
  return SgemvSplit{(uint32_t)(nd / T), (uint32_t)(nd % T)};
}
__device__ __forceinline__ int sgemv_kind(uint32_t d, const SgemvSplit& sp) {
  const uint32_t big = sp.r * (sp.q + 1);
  uint32_t w, start;
  if (d < big) {
    w = sp.q + 1;
    start = d - d % w;
  } else {
    w = sp.q;
    start = d - (d - big) % w;
  }
  const uint32_t pos = d - start, t = w & 3u;
  if (pos < w - t) return 0;
  return ((t & 2u) && pos < w - t + 2) ? 1 : 2;
}
// First column of d's thread chunk; [d0, d1] is all kind 0 iff d1 is kind 0 and d0 ≥ sgemv_chunk_start(d1)
// (each chunk's kind-0 columns are a prefix of it).
__device__ __forceinline__ uint32_t sgemv_chunk_start(uint32_t d, const SgemvSplit& sp) {
  const uint32_t big = sp.r * (sp.q + 1);
  return d < big ? d - d % (sp.q + 1) : d - (d - big) % sp.q;
}
template <class D, class Q>
__device__ __forceinline__ float sgemv16(const D& d, const Q& q, int kind = 0) {
  if (kind == 0) {
    float l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = __builtin_fmaf(d(j + 8), q(j + 8), 0.0f + d(j) * q(j));
    return ((l[0] + l[4]) + (l[1] + l[5])) + ((l[2] + l[6]) + (l[3] + l[7]));
  }
  float p[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) p[k] = d(k) * q(k);
  if (kind == 1) {
    float l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) l[j] = (((0.0f + p[j]) + p[j + 4]) + p[j + 8]) + p[j + 12];
    return (l[0] + l[1]) + (l[2] + l[3]);
  }
  float l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) l[j] = (0.0f + p[j]) + p[j + 8];
  return ((l[0] + l[4]) + (l[1] + l[5])) + ((l[2] + l[6]) + (l[3] + l[7]));
}

// np.clip(x, -c, c) keeps NaN (comparisons false).
__device__ __forceinline__ float clip_sym(float x, float c) { return x < -c ? -c : (x > c ? c : x); }

// Order-preserving map of f32 to u32 (larger float → larger key; NaN above +inf).
__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

}  // namespace fwav

// C-ABI status codes (mirrored in include/fwav.h).
#ifndef FWAV_OK
#define FWAV_OK 0
#define FWAV_ERR_ARG (-1)
#define FWAV_ERR_SHAPE (-2)
#define FWAV_ERR_K (-3)
#define FWAV_ERR_HIP (-4)
#define FWAV_ERR_WORKSPACE (-5)
#endif
