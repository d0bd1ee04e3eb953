// fwav_signal.hip — voiced detection, range formation and the energy prune, on device.
//
// Replaces (reference /root/reference/fractal.py):
//   voiced_detection            :880-909   frame energy → 5-tap smoothing → hysteresis → per-sample mask
//   compress_audio range setup  :1079-1112 signal·mask, reflect pad to a multiple of rs, reshape
//   cpu_worker energy prune     :601-603   mean(r²) < 0.75·thr  → no candidates (all −1)
//
// The hysteresis loop (:902-907) is sequential in the reference; here a frame's state is the decision of
// the last frame that was > hi (voiced) or < lo (unvoiced), found with a max-scan over positions:
//   k_voiced_decide (per frame, + per-block last decisive position) → k_voiced_carry (one block, exclusive
//   prefix max over blocks) → k_frame_state (in-block max-scan + carry) → k_form_ranges (per sample).
#include "fwav_common.h"
#include "../../include/fwav.h"

namespace fwav {

__device__ __forceinline__ int64_t reflect_idx(int64_t p, int64_t n) {
  // np.pad(mode='reflect') index for p >= 0 on the right side (period 2(n-1)).
  if (p < n) return p;
  if (n == 1) return 0;
  const int64_t period = 2 * (n - 1);
  int64_t q = p % period;
  return q < n ? q : period - q;
}

constexpr int kFramesPerBlock = 1024;
constexpr int kSignalThreads = 256;

// Smoothed energy of frame i: np.convolve(e, ones(w, f32)/w, 'same') (fractal.py:893-895) as numpy evaluates it
// (measured against np.convolve on wide-range random energies; oracle smooth5):
//   nf ≥ w: window [i − w/2, i − w/2 + w) ∩ [0, nf).  A full window is numpy's small_correlate: f32 products added in
//           f32 in e order.  A partial window (the first w/2 and last w − w/2 − 1 frames) is the dtype dot (OpenBLAS
//           sdot): f32 products accumulated in f64 in e order, then rounded.
//   nf < w: numpy swaps the operands (the kernel correlated with reversed e); frame i covers the e indices j with
//           0 ≤ t − j ≤ w − 1, t = i + (nf − 1)/2, taken in reversed order: f32 when all nf overlap, else the f64 dot.
__device__ __forceinline__ float smooth_at(const float* e, int64_t nf, int64_t i, int w, float k) {
  int64_t lo, hi;  // inclusive e index range
  bool rev;
  if (nf >= w) {
    lo = i - w / 2;
    hi = lo + w - 1;
    rev = false;
  } else {
    hi = i + (nf - 1) / 2;
    lo = hi - (w - 1);
    rev = true;
  }
  const bool full = rev ? (lo <= 0 && hi >= nf - 1) : (lo >= 0 && hi <= nf - 1);
  lo = lo < 0 ? 0 : lo;
  hi = hi > nf - 1 ? nf - 1 : hi;
  const int64_t cnt = hi - lo + 1;
  if (full) {
    float s = 0.0f;
    for (int64_t t = 0; t < cnt; ++t) s = s + e[rev ? hi - t : lo + t] * k;
    return s;
  }
  double d = 0.0;
  for (int64_t t = 0; t < cnt; ++t) d += (double)(e[rev ? hi - t : lo + t] * k);
  return (float)d;
}

__global__ void k_frame_energy(const float* __restrict__ sig, int64_t n, int frame, int64_t nf,
                               float* __restrict__ energy) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nf) return;
  const int64_t base = i * frame;
  auto sq = [&](int j) {
    float x = sig[reflect_idx(base + j, n)];
    return x * x;
  };
  energy[i] = pw_sum(sq, frame) / (float)frame;
}

// dec[i] ∈ {1 voiced, 0 unvoiced, -1 keep};  blast[b] = last decisive frame position in block b or -1.
__global__ void k_voiced_decide(const float* __restrict__ energy, int64_t nf, int w, float k, float hi,
                                float lo, int8_t* __restrict__ dec, int64_t* __restrict__ blast) {
  __shared__ int64_t red[kSignalThreads / kWave];
  const int64_t b0 = (int64_t)blockIdx.x * kFramesPerBlock;
  int64_t last = -1;
  for (int t = threadIdx.x; t < kFramesPerBlock; t += blockDim.x) {
    int64_t i = b0 + t;
    if (i >= nf) break;
    float es = smooth_at(energy, nf, i, w, k);
    int8_t d = es > hi ? 1 : (es < lo ? 0 : -1);
    dec[i] = d;
    if (d >= 0) last = i > last ? i : last;
  }
  for (int o = 32; o > 0; o >>= 1) {
    int64_t v = __shfl_xor(last, o);
    last = v > last ? v : last;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = last;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t m = -1;
    for (int j = 0; j < (int)(blockDim.x / kWave); ++j) m = red[j] > m ? red[j] : m;
    blast[blockIdx.x] = m;
  }
}

// carry[b] = max(blast[0..b-1]) (exclusive), one block.
__global__ void k_voiced_carry(const int64_t* __restrict__ blast, int64_t nb, int64_t* __restrict__ carry) {
  __shared__ int64_t wsum[1024 / kWave];
  __shared__ int64_t running;
  if (threadIdx.x == 0) running = -1;
  __syncthreads();
  for (int64_t c = 0; c < nb; c += blockDim.x) {
    int64_t i = c + threadIdx.x;
    int64_t v = i < nb ? blast[i] : -1;
    // inclusive max-scan within the wave
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
      int64_t u = __shfl_up(v, o);
      if (lane >= o) v = u > v ? u : v;
    }
    if (lane == 63) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    int64_t pre = running;
    for (int j = 0; j < (int)(threadIdx.x >> 6); ++j) pre = wsum[j] > pre ? wsum[j] : pre;
    int64_t incl = v > pre ? v : pre;
    int64_t excl = __shfl_up(incl, 1);
    if (lane == 0) excl = pre;
    if (i < nb) carry[i] = excl;
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) running = incl;
    __syncthreads();
  }
}

// state[f] = decision of the last decisive frame <= f (0 if none): block max-scan of positions + carry.
__global__ void k_frame_state(const int8_t* __restrict__ dec, const int64_t* __restrict__ carry, int64_t nf,
                              uint8_t* __restrict__ state) {
  __shared__ int64_t wlast[kSignalThreads / kWave];
  constexpr int kPer = kFramesPerBlock / kSignalThreads;  // 4 consecutive frames per thread
  const int64_t f0 = (int64_t)blockIdx.x * kFramesPerBlock + (int64_t)threadIdx.x * kPer;
  int64_t pos[kPer];
  int64_t run = -1;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    int64_t f = f0 + j;
    if (f < nf && dec[f] >= 0) run = f;
    pos[j] = run;
  }
  // exclusive max-scan of the per-thread last position across the block
  const int lane = threadIdx.x & 63;
  int64_t v = run;
  for (int o = 1; o < 64; o <<= 1) {
    int64_t u = __shfl_up(v, o);
    if (lane >= o) v = u > v ? u : v;
  }
  if (lane == 63) wlast[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t pre = carry[blockIdx.x];
  for (int j = 0; j < (int)(threadIdx.x >> 6); ++j) pre = wlast[j] > pre ? wlast[j] : pre;
  int64_t ex = __shfl_up(v, 1);
  if (lane == 0) ex = -1;
  pre = ex > pre ? ex : pre;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    int64_t f = f0 + j;
    if (f >= nf) break;
    int64_t p = pos[j] >= 0 ? pos[j] : pre;
    state[f] = p >= 0 ? (uint8_t)dec[p] : (uint8_t)0;
  }
}

// ranges[p] = (signal · mask)[reflect(p)] for p < nr·rs (fractal.py:1079, 1095-1097).
__global__ void k_form_ranges(const float* __restrict__ sig, int64_t n, int frame, const uint8_t* __restrict__ state,
                              int64_t total, float* __restrict__ ranges, uint8_t* __restrict__ mask_out) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= total) return;
  int64_t src = reflect_idx(p, n);
  uint8_t m = state[src / frame];
  ranges[p] = sig[src] * (float)m;
  if (mask_out != nullptr && p < n) mask_out[p] = m;
}

// Σ (signal·mask)² exactly as np.sum evaluates it on the reference's f32 array (fractal.py:1083): squares rounded to
// f32, numpy's reduction loop over buffers of 8192 elements, each buffer a pairwise_sum (fwav_common.h pw_leaf: 128-
// element leaves, halves split at n/2 − (n/2)%8), the buffer sums added in order into the f32 accumulator (which
// starts at 0).  Phase 1: one wave per full buffer — a complete tree of 64 leaves, one leaf per lane, combined by
// shuffles in the tree's (left + right) order; the last, partial buffer is evaluated by one lane with the general
// recursion.  Phase 2: one lane adds the buffer sums in order.
constexpr int kNpBuf = 8192;

// The leaves of numpy's pairwise recursion over n elements (pw_rec's splits), in order: offsets and lengths.
// Depth: 8191 → ≤ 6 halvings to reach ≤ 128.
template <int D>
__device__ void pw_leaf_list(int off, int n, int* loff, int* llen, int& k) {
  if constexpr (D > 0) {
    if (n > 128) {
      int n2 = n / 2;
      n2 -= n2 % 8;
      pw_leaf_list<D - 1>(off, n2, loff, llen, k);
      pw_leaf_list<D - 1>(off + n2, n - n2, loff, llen, k);
      return;
    }
  }
  loff[k] = off;
  llen[k] = n;
  ++k;
}
// The same recursion with the leaves' sums given (in order): left + right at every node.
template <int D>
__device__ float pw_tree_from_leaves(int n, const float* lsum, int& k) {
  if constexpr (D > 0) {
    if (n > 128) {
      int n2 = n / 2;
      n2 -= n2 % 8;
      const float a = pw_tree_from_leaves<D - 1>(n2, lsum, k);
      const float c = pw_tree_from_leaves<D - 1>(n - n2, lsum, k);
      return a + c;
    }
  }
  return lsum[k++];
}

// One 256-thread workgroup per full buffer: the 8192 elements are loaded coalesced (two float4 per thread and step)
// into LDS, leaf-major with a one-float skew (leaf l at l·129, so the 64 lanes reading element i of their leaves hit
// 64 different banks), then wave 0 evaluates one leaf per lane and combines the 64 leaves by shuffles.  (Reading the
// leaves straight from global memory, lane l at x[128 l + i], touched 64 lines per load: 161 µs at cfg2.)
constexpr int kLeafSkew = 129;
__global__ __launch_bounds__(256) void k_energy_buffers(const float* __restrict__ x, int64_t n,
                                                        float* __restrict__ bufsum) {
  __shared__ float lds[64 * kLeafSkew];
  const int64_t b = blockIdx.x;
  const int64_t off = b * kNpBuf;
  const int64_t len = n - off < kNpBuf ? n - off : kNpBuf;
  const int lane = threadIdx.x & 63;
  if (len < kNpBuf) {
    // the partial last buffer: the pairwise recursion's leaves (≤ 128 of ≤ 128 elements) are listed by one lane,
    // summed one per thread, and combined in the recursion's order by one lane (evaluating the whole recursion on one
    // lane took ≈ 160 µs at cfg2)
    __shared__ int loff[128], llen[128], nleaf;
    __shared__ float lsum[128];
    if (threadIdx.x == 0) {
      int k = 0;
      pw_leaf_list<7>(0, (int)len, loff, llen, k);
      nleaf = k;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nleaf; i += blockDim.x) {
      const float* p = x + off + loff[i];
      lsum[i] = pw_leaf([&](int j) { return p[j] * p[j]; }, 0, llen[i]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int k = 0;
      bufsum[b] = pw_tree_from_leaves<7>((int)len, lsum, k);
    }
    return;
  }
  const float4* x4 = reinterpret_cast<const float4*>(x + off);
#pragma unroll
  for (int k = 0; k < kNpBuf / 4 / 256; ++k) {
    const int e4 = k * 256 + threadIdx.x;  // float4 index: elements 4·e4 .. 4·e4 + 3, all in leaf (4·e4) / 128
    const float4 v = x4[e4];
    const int e = 4 * e4, leaf = e >> 7, pos = e & 127;
    float* d = lds + leaf * kLeafSkew + pos;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const float* leaf = lds + lane * kLeafSkew;
  float v = pw_leaf([&](int i) { return leaf[i] * leaf[i]; }, 0, 128);
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) {
    const float right = __shfl_down(v, w);
    if ((lane & (2 * w - 1)) == 0) v = v + right;  // node = left half + right half
  }
  if (lane == 0) bufsum[b] = v;
}

// The buffer sums added in order into the f32 accumulator: one wave loads 64 sums at a time, lane 0's chain adds them
// in order (readlane).
__global__ void k_energy_chain(const float* __restrict__ bufsum, int64_t nb, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  float acc = 0.0f;
  for (int64_t c = 0; c < nb; c += 64) {
    const float v = c + lane < nb ? bufsum[c + lane] : 0.0f;
    const int m = nb - c < 64 ? (int)(nb - c) : 64;
    for (int j = 0; j < m; ++j) acc = acc + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
  }
  if (lane == 0) out[0] = acc;
}

// Energy prune + degenerate queries + active list (fractal.py:598-622, quirk Q1/Q3/Q11).
//   pruned            → cand row all −1
//   query row all 0   → every score is 0 and the reference's candidates are whatever order numpy's introselect
//                       (argpartition) + argsort leave equal keys in (fractal.py:537-541, quirk Q11): the caller
//                       passes that order once per (n_domains, K) in zero_cand (K entries, −1 padded); NULL gives
//                       0..min(K,nd)−1
//   otherwise         → appended to `active` for the similarity search
// RS > 0: compile-time range size (row in registers, unrolled pairwise sum); RS == 0: runtime rs.
template <int RS>
__global__ void k_prune(const float* __restrict__ ranges, int64_t nr, int64_t q_offset, int rs_rt, float thr,
                        int fast_mode, const float* __restrict__ emb, int64_t nd, int k,
                        const int32_t* __restrict__ zero_cand, int32_t* __restrict__ cand,
                        int32_t* __restrict__ active, int32_t* __restrict__ n_active) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  const int rs = RS > 0 ? RS : rs_rt;
  const float* r = ranges + i * rs;
  float mean_sq;
  if constexpr (RS > 0) {
    float v[RS];
    if constexpr (RS % 4 == 0) {
#pragma unroll
      for (int j = 0; j < RS / 4; ++j) {
        const float4 t = reinterpret_cast<const float4*>(r)[j];
        v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < RS; ++j) v[j] = r[j];
    }
    auto sq = [&](int j) { return v[j] * v[j]; };
    mean_sq = pw_sum_n<RS>(sq) / (float)RS;
  } else {
    auto sq = [&](int j) { return r[j] * r[j]; };
    mean_sq = pw_sum(sq, rs) / (float)rs;
  }
  bool pruned = fast_mode && (mean_sq < thr);
  bool zero = true;
  if (!pruned) {
    const float4* q = reinterpret_cast<const float4*>(emb + (i + q_offset) * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float4 v = q[j];
      zero = zero && v.x == 0.0f && v.y == 0.0f && v.z == 0.0f && v.w == 0.0f;
    }
  }
  int32_t* c = cand + i * (int64_t)k;
  if (pruned) {
    for (int j = 0; j < k; ++j) c[j] = -1;
  } else if (zero) {
    if (zero_cand != nullptr) {
      for (int j = 0; j < k; ++j) c[j] = zero_cand[j];
    } else {
      for (int j = 0; j < k; ++j) c[j] = j < nd ? j : -1;
    }
  }
  // append the searchable ranges: one counter atomic per wave (not per range), index order kept within a wave
  const bool act = !pruned && !zero;
  const uint64_t m = __ballot(act);
  if (m == 0ull) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if (lane == leader) base = atomicAdd(n_active, __popcll(m));
  base = __shfl(base, leader);
  if (act) active[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)i;
}

}  // namespace fwav

using namespace fwav;

extern "C" {

size_t fwav_voiced_workspace_size(int64_t n, int frame) {
  const int64_t nf = cdiv(n, frame);
  const int64_t nb = cdiv(nf, kFramesPerBlock);
  return (size_t)(2 * nb * sizeof(int64_t) + nf * sizeof(float) + 2 * nf + 64);
}

// Voiced mask + ranges.  ranges: f32[nr*rs] with nr = ceil(n/rs); mask_out: optional u8[n].
int fwav_voiced_ranges(const float* sig, int64_t n, int rs, int frame, int smooth_window, float hi, float lo,
                       float* ranges, int64_t nr, uint8_t* mask_out, void* workspace, size_t ws_bytes,
                       void* stream) {
  FWAV_CHECK_ARG(sig && ranges && n > 0 && rs > 0 && frame > 0, FWAV_ERR_ARG, "fwav_voiced_ranges: bad args");
  FWAV_CHECK_ARG(nr == cdiv(n, rs), FWAV_ERR_SHAPE, "fwav_voiced_ranges: nr != ceil(n/rs)");
  FWAV_CHECK_ARG(frame <= kMaxPairwise, FWAV_ERR_SHAPE, "fwav_voiced_ranges: frame > %d", kMaxPairwise);
  const int64_t nf = cdiv(n, frame);
  FWAV_CHECK_ARG(smooth_window >= 1 && smooth_window <= 11, FWAV_ERR_SHAPE,
                 "fwav_voiced_ranges: need 1 <= smooth_window <= 11");
  FWAV_CHECK_ARG(ws_bytes >= fwav_voiced_workspace_size(n, frame), FWAV_ERR_WORKSPACE,
                 "fwav_voiced_ranges: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nb = cdiv(nf, kFramesPerBlock);
  char* w = (char*)workspace;
  int64_t* blast = (int64_t*)w;
  int64_t* carry = blast + nb;
  float* energy = (float*)(carry + nb);
  int8_t* dec = (int8_t*)(energy + nf);
  uint8_t* state = (uint8_t*)(dec + nf);
  // smoothing kernel weights: np.ones(w, f32) / w
  const float kw = 1.0f / (float)smooth_window;
  k_frame_energy<<<cdiv(nf, kSignalThreads), kSignalThreads, 0, st>>>(sig, n, frame, nf, energy);
  k_voiced_decide<<<nb, kSignalThreads, 0, st>>>(energy, nf, smooth_window, kw, hi, lo, dec, blast);
  k_voiced_carry<<<1, 1024, 0, st>>>(blast, nb, carry);
  k_frame_state<<<nb, kSignalThreads, 0, st>>>(dec, carry, nf, state);
  const int64_t total = nr * rs;
  k_form_ranges<<<cdiv(total, kSignalThreads), kSignalThreads, 0, st>>>(sig, n, frame, state, total, ranges,
                                                                          mask_out);
  FWAV_LAUNCH_CHECK("fwav_voiced_ranges");
  return FWAV_OK;
}

size_t fwav_weighted_energy_workspace_size(int64_t n) { return (size_t)(cdiv(n > 0 ? n : 1, kNpBuf) * 4 + 64); }

__global__ void k_smooth_debug(const float* __restrict__ e, int64_t nf, int w, float k, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nf) out[i] = smooth_at(e, nf, i, w, k);
}

// Diagnostic (tests): the smoothed frame energies of fwav_voiced_ranges, out[i] for i < nf.
int fwav_debug_smooth(const float* energy, int64_t nf, int smooth_window, float* out, void* stream) {
  FWAV_CHECK_ARG(energy && out && nf >= 0 && smooth_window >= 1 && smooth_window <= 11, FWAV_ERR_ARG,
                 "fwav_debug_smooth: bad args");
  if (nf == 0) return FWAV_OK;
  k_smooth_debug<<<cdiv(nf, kSignalThreads), kSignalThreads, 0, (hipStream_t)stream>>>(
      energy, nf, smooth_window, 1.0f / (float)smooth_window, out);
  FWAV_LAUNCH_CHECK("fwav_debug_smooth");
  return FWAV_OK;
}

// np.sum(ranges[0:n] ** 2) in float32, bit-exact (see k_energy_buffers); the result lands in sum[0].
int fwav_weighted_energy(const float* ranges, int64_t n, float* sum, void* workspace, size_t ws_bytes, void* stream) {
  FWAV_CHECK_ARG(ranges && sum && n >= 0, FWAV_ERR_ARG, "fwav_weighted_energy: bad args");
  FWAV_CHECK_ARG(workspace && ws_bytes >= fwav_weighted_energy_workspace_size(n), FWAV_ERR_WORKSPACE,
                 "fwav_weighted_energy: workspace too small");
  FWAV_CHECK_ARG(((uintptr_t)ranges & 15) == 0, FWAV_ERR_ARG, "fwav_weighted_energy: ranges must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nb = cdiv(n, kNpBuf);
  float* bufsum = (float*)workspace;
  if (nb > 0) k_energy_buffers<<<nb, 256, 0, st>>>(ranges, n, bufsum);
  k_energy_chain<<<1, 64, 0, st>>>(bufsum, nb, sum);
  FWAV_LAUNCH_CHECK("fwav_weighted_energy");
  return FWAV_OK;
}

// Ranges [q_offset, q_offset + nr) of the whole signal: ranges/cand/active are shard-local (row i), the
// query embedding of local range i is emb row q_offset + i.
int fwav_prune(const float* ranges, int64_t nr, int64_t q_offset, int rs, float prune_thr, int fast_mode,
               const float* emb, int64_t nd, int k, const int32_t* zero_cand, int32_t* cand, int32_t* active,
               int32_t* n_active, void* stream) {
  FWAV_CHECK_ARG(ranges && emb && cand && active && n_active && k > 0, FWAV_ERR_ARG, "fwav_prune: bad args");
  FWAV_CHECK_ARG(q_offset >= 0 && q_offset + nr <= nd, FWAV_ERR_SHAPE,
                 "fwav_prune: query rows past n_domains (query rows are domain rows, quirk Q1)");
  FWAV_CHECK_ARG(rs <= kMaxPairwise, FWAV_ERR_SHAPE, "fwav_prune: rs too large");
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(n_active, 0, sizeof(int32_t), st);
  if (nr == 0) return FWAV_OK;
  const int64_t grid = cdiv(nr, kSignalThreads);
  switch (rs) {
#define FWAV_PRUNE(RSV)                                                                                      \
  k_prune<RSV><<<grid, kSignalThreads, 0, st>>>(ranges, nr, q_offset, rs, prune_thr, fast_mode, emb, nd, k,     \
                                                zero_cand, cand, active, n_active)
    case 4: FWAV_PRUNE(4); break;
    case 8: FWAV_PRUNE(8); break;
    case 16: FWAV_PRUNE(16); break;
    default: FWAV_PRUNE(0);
#undef FWAV_PRUNE
  }
  FWAV_LAUNCH_CHECK("fwav_prune");
  return FWAV_OK;
}

}  // extern "C"
