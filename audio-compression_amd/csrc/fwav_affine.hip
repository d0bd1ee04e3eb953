// fwav_affine.hip — batched affine least squares with mirror + first-minimum select (bit-exact).
//
// Replaces (reference /root/reference/fractal.py):
//   _flush_gpu_batch   :852-870
//   _process_gpu_batch :757-850   for range b and slot j over [K candidates | K mirrored]:
//       r̄ = mean(R); r̃ = R − r̄; d̄ = mean(D); d̃ = D − d̄; s = Σd̃r̃ / (Σd̃d̃ + 1e-12); o = r̄ − s·d̄;
//       err = ‖(s·D + o) − R‖₂; err = +inf where cand < 0; j* = argmin(err) (first); emit
//       (cand_clamped[j*], clip(s, ±s_clip), o, j* ≥ K, err)            (quirks Q3, Q4)
//   The reference's corr/min_err (:807-808) are dead and not computed.
//
// One wave per range, lane c ↔ candidate c (c, c+64, …): the lane gathers its pool row once and
// evaluates both orientations from registers (mirror = reversed register index).  Reductions are numpy
// pairwise order over rs, every op a separately rounded f32 op (-ffp-contract=off): bit-exact with the
// reference (tests/test_gpu_parity.py).  The argmin is a 6-step xor-shuffle reduction with numpy's
// tie/NaN rules (first NaN wins, else smallest err, else lowest slot).
// Bytes per range: 4·rs (range) + 4·K (candidates) + 4·K·rs (gathered rows) + 17 (outputs).
#include "fwav_common.h"
#include "../../include/fwav.h"

// -DFWAV_AFF_* knobs build A/B variants of the debug library only (tools/ab_build.sh adds -DFWAV_DEBUG_API)
#if !defined(FWAV_DEBUG_API) && (defined(FWAV_AFF_ABL) || defined(FWAV_AFF_BATCH) || defined(FWAV_AFF_XCD))
#error "experiment switches build the debug library only (-DFWAV_DEBUG_API)"
#endif

namespace fwav {

constexpr int kAffWaves = 4;

struct Best {
  float err, s, o;
  int slot, dom;
};

__device__ __forceinline__ bool better(float e1, int s1, float e2, int s2) {
  const bool n1 = e1 != e1, n2 = e2 != e2;
  if (n1 || n2) return (n1 && n2) ? s1 < s2 : n1;
  return e1 < e2 || (e1 == e2 && s1 < s2);
}

template <int RS>
__device__ __forceinline__ void eval_orient(const float (&X)[RS], const float (&R)[RS], const float (&rc)[RS], float rm,
                                            float& s, float& o, float& err) {
  auto fx = [&](int i) { return X[i]; };
  const float dm = pw_sum_n<RS>(fx) / (float)RS;
  float dc[RS];
#pragma unroll
  for (int i = 0; i < RS; ++i) dc[i] = X[i] - dm;
  auto fn = [&](int i) { return dc[i] * rc[i]; };
  auto fd = [&](int i) { return dc[i] * dc[i]; };
  const float num = pw_sum_n<RS>(fn);
  const float den = pw_sum_n<RS>(fd) + 1e-12f;
  s = num / den;
  o = rm - s * dm;
  auto fe = [&](int i) {
    const float df = (s * X[i] + o) - R[i];
    return df * df;
  };
  err = sqrtf(pw_sum_n<RS>(fe));
}

template <int RS>
__global__ __launch_bounds__(64 * kAffWaves) void k_affine(const float* __restrict__ ranges, int64_t nr,
                                                           const int32_t* __restrict__ cand, int K,
                                                           const float* __restrict__ pool, float s_clip,
                                                           int32_t* __restrict__ out_idx, float* __restrict__ out_s,
                                                           float* __restrict__ out_o, uint8_t* __restrict__ out_sym,
                                                           float* __restrict__ out_err) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kAffWaves + (threadIdx.x >> 6);
  if (r >= nr) return;
  float R[RS], rc[RS];
#pragma unroll
  for (int i = 0; i < RS; ++i) R[i] = ranges[r * RS + i];
  auto fr = [&](int i) { return R[i]; };
  const float rm = pw_sum_n<RS>(fr) / (float)RS;
#pragma unroll
  for (int i = 0; i < RS; ++i) rc[i] = R[i] - rm;

  Best b{INFINITY, 0.f, 0.f, 0x7fffffff, 0};
  bool have = false;
  const int32_t* cr = cand + r * (int64_t)K;
  for (int c = lane; c < K; c += 64) {
    const int32_t ci = cr[c];
    const int32_t di = ci < 0 ? 0 : ci;
    float D[RS], M[RS];
    if constexpr (RS % 4 == 0) {
      const float4* p = reinterpret_cast<const float4*>(pool + (int64_t)di * RS);
#pragma unroll
      for (int j = 0; j < RS / 4; ++j) {
        float4 v = p[j];
        D[4 * j] = v.x; D[4 * j + 1] = v.y; D[4 * j + 2] = v.z; D[4 * j + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < RS; ++i) D[i] = pool[(int64_t)di * RS + i];
    }
#pragma unroll
    for (int i = 0; i < RS; ++i) M[i] = D[RS - 1 - i];
    float s0, o0, e0, s1, o1, e1;
    eval_orient<RS>(D, R, rc, rm, s0, o0, e0);
    eval_orient<RS>(M, R, rc, rm, s1, o1, e1);
    if (ci < 0) { e0 = INFINITY; e1 = INFINITY; }
    if (!have || better(e0, c, b.err, b.slot)) { b = Best{e0, s0, o0, c, di}; have = true; }
    if (better(e1, K + c, b.err, b.slot)) b = Best{e1, s1, o1, K + c, di};
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    Best o;
    o.err = __shfl_xor(b.err, m);
    o.s = __shfl_xor(b.s, m);
    o.o = __shfl_xor(b.o, m);
    o.slot = __shfl_xor(b.slot, m);
    o.dom = __shfl_xor(b.dom, m);
    if (better(o.err, o.slot, b.err, b.slot)) b = o;
  }
  if (lane == 0) {
    out_idx[r] = b.dom;
    out_s[r] = clip_sym(b.s, fabsf(s_clip));
    out_o[r] = b.o;
    out_sym[r] = (uint8_t)(b.slot >= K);
    out_err[r] = b.err;
  }
}

// Generic rs (runtime), rows read from global memory; same arithmetic.
__global__ __launch_bounds__(64 * kAffWaves) void k_affine_any(const float* __restrict__ ranges, int64_t nr, int rs,
                                                               const int32_t* __restrict__ cand, int K,
                                                               const float* __restrict__ pool, float s_clip,
                                                               int32_t* __restrict__ out_idx, float* __restrict__ out_s,
                                                               float* __restrict__ out_o, uint8_t* __restrict__ out_sym,
                                                               float* __restrict__ out_err) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kAffWaves + (threadIdx.x >> 6);
  if (r >= nr) return;
  const float* R = ranges + r * rs;
  auto fr = [&](int i) { return R[i]; };
  const float rm = pw_sum(fr, rs) / (float)rs;
  Best b{INFINITY, 0.f, 0.f, 0x7fffffff, 0};
  bool have = false;
  const int32_t* cr = cand + r * (int64_t)K;
  for (int c = lane; c < K; c += 64) {
    const int32_t ci = cr[c];
    const int32_t di = ci < 0 ? 0 : ci;
    const float* D = pool + (int64_t)di * rs;
    for (int orient = 0; orient < 2; ++orient) {
      auto X = [&](int i) { return orient ? D[rs - 1 - i] : D[i]; };
      const float dm = pw_sum(X, rs) / (float)rs;
      auto fn = [&](int i) { return (X(i) - dm) * (R[i] - rm); };
      auto fd = [&](int i) {
        const float t = X(i) - dm;
        return t * t;
      };
      const float num = pw_sum(fn, rs);
      const float den = pw_sum(fd, rs) + 1e-12f;
      const float s = num / den;
      const float o = rm - s * dm;
      auto fe = [&](int i) {
        const float df = (s * X(i) + o) - R[i];
        return df * df;
      };
      float e = sqrtf(pw_sum(fe, rs));
      if (ci < 0) e = INFINITY;
      const int slot = orient * K + c;
      if (!have || better(e, slot, b.err, b.slot)) { b = Best{e, s, o, slot, di}; have = true; }
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    Best o;
    o.err = __shfl_xor(b.err, m);
    o.s = __shfl_xor(b.s, m);
    o.o = __shfl_xor(b.o, m);
    o.slot = __shfl_xor(b.slot, m);
    o.dom = __shfl_xor(b.dom, m);
    if (better(o.err, o.slot, b.err, b.slot)) b = o;
  }
  if (lane == 0) {
    out_idx[r] = b.dom;
    out_s[r] = clip_sym(b.s, fabsf(s_clip));
    out_o[r] = b.o;
    out_sym[r] = (uint8_t)(b.slot >= K);
    out_err[r] = b.err;
  }
}


// ------------------------------------------------------------------ batched kernel (K <= 64, rs 4/8/16)
// Lane c ↔ candidate c; a wave handles kAffBatch consecutive ranges.  Per range the work is two dependent
// round trips (candidate row → pool rows) and ~250 VALU ops, so the wave issues all candidate loads of its
// batch, then all row gathers, then does the math: kAffBatch ranges' latencies overlap and no register is
// carried across a loop (a software-pipelined persistent loop made the compiler rotate registers and wait
// for every load at the loop head).  The range samples are wave-uniform (scalar loads).  Both orientations
// are evaluated together in packed f32 (v_pk_mul_f32 / v_pk_add_f32; each half is one correctly rounded f32
// op, so the numpy order and results are unchanged) — the VALU is the bound here, at 4 cycles per wave64
// op.  The argmin is two DPP wave reductions on (NaN-first error order, slot) followed by readlanes of the
// winner, instead of a 5-value shuffle tree.
template <int RS>
__device__ __forceinline__ void gather_row(const float* __restrict__ pool, int32_t ci, float (&D)[RS]) {
  const int64_t di = ci < 0 ? 0 : ci;
  if constexpr (RS % 4 == 0) {
    const float4* p = reinterpret_cast<const float4*>(pool + di * RS);
#pragma unroll
    for (int j = 0; j < RS / 4; ++j) {
      const float4 v = p[j];
      D[4 * j] = v.x; D[4 * j + 1] = v.y; D[4 * j + 2] = v.z; D[4 * j + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < RS; ++i) D[i] = pool[di * RS + i];
  }
}

extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);

template <int RS>
__device__ __forceinline__ void affine_one(const float (&R)[RS], int64_t r, int32_t ci, bool has,
                                           int K, const float (&D)[RS], float s_clip, int32_t* out_idx,
                                           float* out_s, float* out_o, uint8_t* out_sym, float* out_err) {
  const int lane = threadIdx.x & 63;
  float rc[RS];
  auto fr = [&](int i) { return R[i]; };
  const float rm = pw_sum_n<RS>(fr) / (float)RS;
#pragma unroll
  for (int i = 0; i < RS; ++i) rc[i] = R[i] - rm;

  // .x = candidate as stored, .y = mirrored
  f32x2 X[RS];
#pragma unroll
  for (int i = 0; i < RS; ++i) X[i] = f32x2{D[i], D[RS - 1 - i]};
  auto fx = [&](int i) { return X[i]; };
  const f32x2 dm = pw_sum_n<RS>(fx) / (float)RS;
  f32x2 dc[RS];
#pragma unroll
  for (int i = 0; i < RS; ++i) dc[i] = X[i] - dm;
  auto fd = [&](int i) { return dc[i] * dc[i]; };
  const f32x2 den = pw_sum_n<RS>(fd) + 1e-12f;
  auto fn = [&](int i) { return dc[i] * rc[i]; };
  const f32x2 num = pw_sum_n<RS>(fn);
  const f32x2 sv = num / den;
  const f32x2 ov = rm - sv * dm;
  auto fe = [&](int i) {
    const f32x2 df = (sv * X[i] + ov) - R[i];
    return df * df;
  };
  const f32x2 ss = pw_sum_n<RS>(fe);
  float e0 = sqrtf(ss.x), e1 = sqrtf(ss.y);
  if (ci < 0) { e0 = INFINITY; e1 = INFINITY; }
  // lane-local best of slot `lane` and slot K + lane (first minimum, NaN first), then the wave's
  const bool take1 = better(e1, K + lane, e0, lane);
  const float eb = take1 ? e1 : e0;
  const uint32_t slot = take1 ? (uint32_t)(K + lane) : (uint32_t)lane;
  const uint32_t ekey = has ? ((eb != eb) ? 0u : __float_as_uint(eb) + 1u) : 0xffffffffu;
  const uint32_t kmin = __ockl_wfred_min_u32(ekey);
  const uint32_t smin = __ockl_wfred_min_u32((has && ekey == kmin) ? slot : 0xffffffffu);
  const int wl = (int)(smin < (uint32_t)K ? smin : smin - (uint32_t)K);
  auto bcast = [&](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), wl)); };
  const float sb = bcast(take1 ? sv.y : sv.x);
  const float ob = bcast(take1 ? ov.y : ov.x);
  const float erb = bcast(eb);
  const int db = __builtin_amdgcn_readlane(ci < 0 ? 0 : ci, wl);
  if (lane == 0) {
    out_idx[r] = db;
    out_s[r] = clip_sym(sb, fabsf(s_clip));
    out_o[r] = ob;
    out_sym[r] = (uint8_t)(smin >= (uint32_t)K);
    out_err[r] = erb;
  }
}

#ifndef FWAV_AFF_BATCH
#define FWAV_AFF_BATCH 4
#endif
constexpr int kAffBatch = FWAV_AFF_BATCH;  // ranges per wave in k_affine_batch
#ifndef FWAV_AFF_ABL
#define FWAV_AFF_ABL 0
#endif
#ifndef FWAV_AFF_XCD
#define FWAV_AFF_XCD 1
#endif

template <int RS>
__global__ __launch_bounds__(64 * kAffWaves) void k_affine_batch(const float* __restrict__ ranges, int64_t nr,
                                                                 const int32_t* __restrict__ cand, int K,
                                                                 const float* __restrict__ pool, float s_clip,
                                                                 int32_t* __restrict__ out_idx,
                                                                 float* __restrict__ out_s, float* __restrict__ out_o,
                                                                 uint8_t* __restrict__ out_sym,
                                                                 float* __restrict__ out_err) {
  const int lane = threadIdx.x & 63;
  // consecutive ranges have largely the same candidates (query i is domain row i, and domains i and i+1 are windows
  // `step` samples apart), so consecutive blocks run on one XCD and find each other's rows in its L2
#if FWAV_AFF_XCD
  const int64_t blk = xcd_block(blockIdx.x, gridDim.x);
#else
  const int64_t blk = blockIdx.x;
#endif
  const int64_t wave = blk * kAffWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r0 = wave * kAffBatch;
  if (r0 >= nr) return;
  const bool has = lane < K;
  const int lane_c = has ? lane : K - 1;
  // all candidate loads, then all row gathers, then the math: kAffBatch ranges' round trips overlap
  int32_t c[kAffBatch];
#pragma unroll
  for (int j = 0; j < kAffBatch; ++j) {
    const int64_t r = r0 + j < nr ? r0 + j : nr - 1;
    c[j] = cand[r * K + lane_c];
  }
  float D[kAffBatch][RS];
#pragma unroll
  for (int j = 0; j < kAffBatch; ++j) gather_row<RS>(pool, c[j], D[j]);
#if FWAV_AFF_ABL
  // ablation build (tools/affine_probe.py): the same loads, no solve — the memory side's time alone
  float acc = 0.0f;
#pragma unroll
  for (int j = 0; j < kAffBatch; ++j)
#pragma unroll
    for (int i = 0; i < RS; ++i) acc += D[j][i];
  if (acc == 1.2345f) out_err[r0] = acc;
  return;
#endif
  // range rows: wave-uniform and read-only → constant address space → scalar loads
  const __attribute__((address_space(4))) float* rg = (const __attribute__((address_space(4))) float*)ranges;
#pragma unroll
  for (int j = 0; j < kAffBatch; ++j) {
    const int64_t r = r0 + j;
    if (r >= nr) break;
    float R[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) R[i] = rg[r * RS + i];
    affine_one<RS>(R, r, has ? c[j] : -1, has, K, D[j], s_clip, out_idx, out_s, out_o, out_sym, out_err);
  }
}

// ------------------------------------------------------------------ tie check (fwav_tie_check)
// The search lists every query whose top K + 1 scores hold exactly equal values (fwav_topk.hip tie_flags): for those
// the reference's candidate order — or, at the K-th place, its candidate set — is whatever numpy's argpartition and
// argsort leave equal keys in (fractal.py:537-541).  The search emits (score desc, index asc) instead; this kernel
// decides, per listed query, whether that can change the match (fractal.py:816-824: the first minimum over
// [K originals | K mirrors]).  Equal scores occupy one contiguous run of positions in both orders, so a reordering
// moves candidates only within their run: the first slot that attains the minimum error keeps its candidate unless
// another candidate of the same run attains it too (originals first; the mirrors only decide when no original
// does).  A tie at the K-th place lets numpy choose which members G of the K-th score's group fill the last places;
// that cannot change the match when every member of G — the search records the ones left out — fits strictly worse
// (both orientations) than the best candidate outside G, whose slot is then the minimum whatever the choice.  Queries
// that fail either test, and K-th place ties whose group the search could not collect (or all of them with
// exact_sets == 1: the candidate sets themselves are then the reference's; every listed query with exact_sets == 2:
// the whole candidate rows, order included, are then the reference's), go to `resolve` for the host (fwav.ties:
// exact score rows + numpy's own calls).  One wave per listed query, K ≤ 64 (lane c ↔ position c); for K > 64 every
// listed query is resolved.
__device__ __forceinline__ bool same_err(float a, float b) { return (a != a && b != b) || a == b; }

// Both orientations' errors of tile `di` against range R, exactly as fwav_affine computes them.
template <int RS>
__device__ __forceinline__ void pair_errors(const float* __restrict__ R, int rs, const float* __restrict__ pool,
                                            int32_t di, float& e0, float& e1) {
  if constexpr (RS > 0) {
    float Rr[RS], rc[RS], D[RS], M[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) Rr[i] = R[i];
    auto fr = [&](int i) { return Rr[i]; };
    const float rm = pw_sum_n<RS>(fr) / (float)RS;
#pragma unroll
    for (int i = 0; i < RS; ++i) rc[i] = Rr[i] - rm;
#pragma unroll
    for (int i = 0; i < RS; ++i) D[i] = pool[(int64_t)di * RS + i];
#pragma unroll
    for (int i = 0; i < RS; ++i) M[i] = D[RS - 1 - i];
    float s0, o0, s1, o1;
    eval_orient<RS>(D, Rr, rc, rm, s0, o0, e0);
    eval_orient<RS>(M, Rr, rc, rm, s1, o1, e1);
  } else {
    const int n = rs;
    auto fr = [&](int i) { return R[i]; };
    const float rm = pw_sum(fr, n) / (float)n;
    const float* D = pool + (int64_t)di * n;
    float ee[2];
    for (int orient = 0; orient < 2; ++orient) {
      auto X = [&](int i) { return orient ? D[n - 1 - i] : D[i]; };
      const float dm = pw_sum(X, n) / (float)n;
      auto fn = [&](int i) { return (X(i) - dm) * (R[i] - rm); };
      auto fd = [&](int i) {
        const float t = X(i) - dm;
        return t * t;
      };
      const float num = pw_sum(fn, n);
      const float den = pw_sum(fd, n) + 1e-12f;
      const float s = num / den;
      const float o = rm - s * dm;
      auto fe = [&](int i) {
        const float df = (s * X(i) + o) - R[i];
        return df * df;
      };
      ee[orient] = sqrtf(pw_sum(fe, n));
    }
    e0 = ee[0];
    e1 = ee[1];
  }
}

template <int RS>
__global__ __launch_bounds__(256) void k_tie_check(const float* __restrict__ ranges, int rs,
                                                   const int32_t* __restrict__ cand, int K,
                                                   const float* __restrict__ pool, const float* __restrict__ emb,
                                                   int64_t q_offset, SgemvSplit sp, const int32_t* __restrict__ ties,
                                                   int exact_sets, int32_t* __restrict__ resolve) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= ties[0]) return;
  const int32_t* rec = ties + 1 + (int64_t)kTieRec * w;
  const int32_t ent = rec[0];
  const int32_t row = ent >> 1;
  const bool boundary = (ent & 1) != 0;
  const int ng = boundary ? rec[1] : 0;  // tied domains left out of the K (−1: group not collected)
  bool dep = K > 64 || exact_sets >= 2 || (boundary && (exact_sets || ng < 0));
  if (!dep) {
    const int n = RS > 0 ? RS : rs;
    const bool has = lane < K;
    const int32_t ci = has ? cand[(int64_t)row * K + lane] : -1;
    const int32_t di = ci < 0 ? 0 : ci;
    // exact scores (the search's order) → runs of equal scores → run id per position
    const float* qp = emb + ((int64_t)row + q_offset) * 16;
    const float* dp = emb + (int64_t)di * 16;
    const float sc = sgemv16([&](int k) { return dp[k]; }, [&](int k) { return qp[k]; }, sgemv_kind((uint32_t)di, sp));
    const float prev = __shfl_up(sc, 1);
    const bool start = has && (lane == 0 || prev != sc);
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const int run = __popcll(__ballot(start) & le);
    const float* R = ranges + (int64_t)row * n;
    float e0, e1;
    pair_errors<RS>(R, rs, pool, di, e0, e1);
    if (ci < 0) { e0 = INFINITY; e1 = INFINITY; }
    // the minimum error (first-minimum / NaN-first order of the reference's argmin)
    auto arg_min = [&](bool on, float& be, int& bs) {
      be = on ? e0 : INFINITY;
      bs = on ? lane : 0x7fffffff;
      if (on && better(e1, K + lane, be, bs)) { be = e1; bs = K + lane; }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) {
        const float oe = __shfl_xor(be, m);
        const int os = __shfl_xor(bs, m);
        if (better(oe, os, be, bs)) { be = oe; bs = os; }
      }
    };
    float be;
    int bs;
    arg_min(has, be, bs);
    if (boundary) {
      // G = the K-th score's group: its members in the K and the ng left out (rec[2 ..]); each must fit strictly
      // worse than the best candidate outside G (a NaN error never does)
      const float S = __shfl(sc, K - 1);
      const bool in_g = has && sc == S;
      float bo;
      int so;
      arg_min(has && !in_g, bo, so);
      bool bad = in_g && !(e0 > bo && e1 > bo);
      if (lane < ng) {
        float x0, x1;
        pair_errors<RS>(R, rs, pool, rec[2 + lane], x0, x1);
        bad = bad || !(x0 > bo && x1 > bo);
      }
      dep = __ballot(bad) != 0ull;
    }
    if (!dep) {
      uint64_t att = __ballot(has && same_err(e0, be));
      if (att == 0ull) att = __ballot(has && same_err(e1, be));
      const int first = __builtin_ctzll(att);
      const int run0 = __shfl(run, first);
      dep = __popcll(att & __ballot(run == run0)) >= 2;
    }
  }
  if (dep && lane == 0) {
    const int pos = atomicAdd(resolve, 1);
    resolve[1 + pos] = row;
  }
}

// Diagnostic (bench roofline): the ceiling of the affine solver's memory side on this device — n uniformly random
// rows of `rs` floats (16-B aligned) gathered from a table of nrows, 4 rows in flight per lane, nothing computed
// (tools/micro/gather32.hip measured 44 G rows/s for 32-B rows of a 2.76 GB table: a request-rate limit).
__device__ __forceinline__ uint32_t gather_hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__global__ __launch_bounds__(256) void k_gather_rows(const float4* __restrict__ tab, uint32_t nrows, int q4, int64_t n,
                                                     float* __restrict__ out) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (int64_t i = tid * 4; i < n; i += stride * 4) {
    float4 v[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t row = gather_hash((uint32_t)(i + b) * 2654435761u) % nrows;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < q4) v[b][k] = tab[(int64_t)row * q4 + k];
    }
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < q4) acc += v[b][k].x;
  }
  if (acc == 1.2345f) out[0] = acc;
}


// Tie fix-up (fwav.ties.apply_rows): numpy-ranked candidate rows in, the affine re-solve's five outputs out, each
// in one launch instead of a gather/scatter per array.  One wave per row in; one thread per row out.
__global__ __launch_bounds__(64) void k_tie_rows_in(const int32_t* __restrict__ rows, const int32_t* __restrict__ new_cand,
                                                    int K, int32_t* __restrict__ cand, const float* __restrict__ ranges,
                                                    int rs, float* __restrict__ ranges_out) {
  const int64_t i = blockIdx.x;
  const int64_t r = rows[i];
  for (int t = threadIdx.x; t < K; t += 64) cand[r * K + t] = new_cand[i * K + t];
  for (int t = threadIdx.x; t < rs; t += 64) ranges_out[i * rs + t] = ranges[r * rs + t];
}

__global__ __launch_bounds__(256) void k_tie_rows_out(const int32_t* __restrict__ rows, int64_t n,
                                                      const int32_t* __restrict__ idx_in, const float* __restrict__ s_in,
                                                      const float* __restrict__ o_in, const uint8_t* __restrict__ sym_in,
                                                      const float* __restrict__ err_in, int32_t* __restrict__ idx,
                                                      float* __restrict__ s, float* __restrict__ o,
                                                      uint8_t* __restrict__ sym, float* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  idx[r] = idx_in[i];
  s[r] = s_in[i];
  o[r] = o_in[i];
  sym[r] = sym_in[i];
  err[r] = err_in[i];
}

}  // namespace fwav

using namespace fwav;

extern "C" {

int fwav_debug_gather_rows(const float* table, int64_t n_rows, int rs, int64_t n, float* sink, void* stream) {
  FWAV_CHECK_ARG(table && sink && n_rows > 0 && n_rows < 0xffffffffLL && n >= 0 && (rs == 4 || rs == 8 || rs == 16),
                 FWAV_ERR_ARG, "fwav_debug_gather_rows: bad args");
  if (n == 0) return FWAV_OK;
  k_gather_rows<<<8192, 256, 0, (hipStream_t)stream>>>((const float4*)table, (uint32_t)n_rows, rs / 4, n, sink);
  FWAV_LAUNCH_CHECK("fwav_debug_gather_rows");
  return FWAV_OK;
}

int fwav_tie_check(const float* ranges, int64_t n_ranges, int rs, const int32_t* cand, int K, const float* pool,
                   int64_t nd, const float* emb, int64_t q_offset, int blas_threads, const int32_t* ties,
                   int64_t max_ties, int exact_sets, int32_t* resolve, void* stream) {
  FWAV_CHECK_ARG(ranges && cand && pool && emb && ties && resolve && n_ranges >= 0 && rs >= 1 && K >= 1 && nd >= 1 &&
                     nd < (int64_t)0x7fffffff && max_ties >= 0 && blas_threads >= 1 && blas_threads <= 4096,
                 FWAV_ERR_ARG, "fwav_tie_check: bad args");
  FWAV_CHECK_ARG(rs <= kMaxPairwise, FWAV_ERR_SHAPE, "fwav_tie_check: rs > %d", kMaxPairwise);
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(resolve, 0, sizeof(int32_t), st);
  if (max_ties == 0) return FWAV_OK;
  const SgemvSplit sp = make_sgemv_split(nd, blas_threads);
  const int64_t grid = cdiv(max_ties, 4);
  switch (rs) {
    case 4: k_tie_check<4><<<grid, 256, 0, st>>>(ranges, rs, cand, K, pool, emb, q_offset, sp, ties, exact_sets, resolve); break;
    case 8: k_tie_check<8><<<grid, 256, 0, st>>>(ranges, rs, cand, K, pool, emb, q_offset, sp, ties, exact_sets, resolve); break;
    case 16: k_tie_check<16><<<grid, 256, 0, st>>>(ranges, rs, cand, K, pool, emb, q_offset, sp, ties, exact_sets, resolve); break;
    default: k_tie_check<0><<<grid, 256, 0, st>>>(ranges, rs, cand, K, pool, emb, q_offset, sp, ties, exact_sets, resolve);
  }
  FWAV_LAUNCH_CHECK("fwav_tie_check");
  return FWAV_OK;
}

int fwav_affine(const float* ranges, int64_t nr, int rs, const int32_t* cand, int K, const float* pool, int64_t nd,
                float s_clip, int32_t* out_idx, float* out_s, float* out_o, uint8_t* out_sym, float* out_err,
                void* stream) {
  FWAV_CHECK_ARG(ranges && cand && pool && out_idx && out_s && out_o && out_sym && out_err, FWAV_ERR_ARG,
                 "fwav_affine: null pointer");
  FWAV_CHECK_ARG(nr >= 0 && rs >= 1 && K >= 1 && nd >= 1, FWAV_ERR_SHAPE, "fwav_affine: bad shape");
  FWAV_CHECK_ARG(rs <= kMaxPairwise, FWAV_ERR_SHAPE, "fwav_affine: rs > %d", kMaxPairwise);
  if (nr == 0) return FWAV_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t grid = cdiv(nr, kAffWaves);
  const int thr = 64 * kAffWaves;
  if (K <= 64 && (rs == 4 || rs == 8 || rs == 16)) {
    switch (rs) {
#define FWAV_AFF_PIPE(RSV)                                                                                   \
  case RSV:                                                                                                  \
    k_affine_batch<RSV><<<cdiv(nr, kAffWaves * kAffBatch), thr, 0, st>>>(ranges, nr, cand, K, pool, s_clip,  \
                                                                         out_idx, out_s, out_o, out_sym, out_err); \
    break;
      FWAV_AFF_PIPE(4)
      FWAV_AFF_PIPE(8)
      FWAV_AFF_PIPE(16)
#undef FWAV_AFF_PIPE
    }
    FWAV_LAUNCH_CHECK("fwav_affine");
    return FWAV_OK;
  }
  switch (rs) {
    case 4: k_affine<4><<<grid, thr, 0, st>>>(ranges, nr, cand, K, pool, s_clip, out_idx, out_s, out_o, out_sym, out_err); break;
    case 8: k_affine<8><<<grid, thr, 0, st>>>(ranges, nr, cand, K, pool, s_clip, out_idx, out_s, out_o, out_sym, out_err); break;
    case 16: k_affine<16><<<grid, thr, 0, st>>>(ranges, nr, cand, K, pool, s_clip, out_idx, out_s, out_o, out_sym, out_err); break;
    default:
      k_affine_any<<<grid, thr, 0, st>>>(ranges, nr, rs, cand, K, pool, s_clip, out_idx, out_s, out_o, out_sym, out_err);
  }
  FWAV_LAUNCH_CHECK("fwav_affine");
  return FWAV_OK;
}

int fwav_tie_rows_in(const int32_t* rows, int64_t n, const int32_t* new_cand, int K, int32_t* cand,
                     const float* ranges, int rs, float* ranges_out, void* stream) {
  FWAV_CHECK_ARG(n == 0 || (rows && new_cand && cand && ranges && ranges_out), FWAV_ERR_ARG,
                 "fwav_tie_rows_in: null pointer");
  FWAV_CHECK_ARG(n >= 0 && K >= 1 && rs >= 1, FWAV_ERR_SHAPE, "fwav_tie_rows_in: bad shape");
  if (n == 0) return FWAV_OK;
  k_tie_rows_in<<<n, 64, 0, (hipStream_t)stream>>>(rows, new_cand, K, cand, ranges, rs, ranges_out);
  FWAV_LAUNCH_CHECK("fwav_tie_rows_in");
  return FWAV_OK;
}

int fwav_tie_rows_out(const int32_t* rows, int64_t n, const int32_t* idx_in, const float* s_in, const float* o_in,
                      const uint8_t* sym_in, const float* err_in, int32_t* out_idx, float* out_s, float* out_o,
                      uint8_t* out_sym, float* out_err, void* stream) {
  FWAV_CHECK_ARG(n == 0 || (rows && idx_in && s_in && o_in && sym_in && err_in && out_idx && out_s && out_o && out_sym &&
                            out_err), FWAV_ERR_ARG, "fwav_tie_rows_out: null pointer");
  FWAV_CHECK_ARG(n >= 0, FWAV_ERR_SHAPE, "fwav_tie_rows_out: bad shape");
  if (n == 0) return FWAV_OK;
  k_tie_rows_out<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(rows, n, idx_in, s_in, o_in, sym_in, err_in, out_idx,
                                                               out_s, out_o, out_sym, out_err);
  FWAV_LAUNCH_CHECK("fwav_tie_rows_out");
  return FWAV_OK;
}

}  // extern "C"
