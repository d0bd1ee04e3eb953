// fwav_topk_large.hip — exact similarity top-K for K > 64 (up to fwav_topk_max_k()).
//
// Replaces the same reference code as fwav_topk.hip for the module-global top_k > 64 (fractal.py:77, 535-552,
// 544-552), including K >= n_domains (the reference then returns every domain, sorted, −1-padded to K).
// Same contract: per active query, the K largest f32 scores emb[d]·q in the reference's sgemv order
// (fwav_common.h sgemv16), in (score desc, index asc) order.
//
// Not the benchmark path (K = 64 runs k_sim_topk_f16).  Queries are processed in batches of B: k_scores_batch
// materialises the B × nd score rows in the workspace (embedding table read once per batch, coalesced row
// writes), then k_select runs one workgroup per query:
//   1. sample 2048 scores at a fixed stride, sort them, and take as threshold t the sample whose rank
//      corresponds to ≈ 2K of nd;
//   2. one pass counts the scores ≥ t and appends them (wave-aggregated, one LDS atomic per wave and step)
//      to an LDS list of kCap entries;
//   3. if K ≤ count ≤ kCap, every member of the top K is in the list (the K-th largest score is ≥ t):
//      bitonic-sort the list on (score key, ~index) and emit the first K.  Otherwise lower / raise t and
//      retry; after the retries, an exact radix select (4 × 8-bit passes on the score key) finds the K-th
//      largest score T, takes every score > T and the lowest-index scores == T in index order (ties).
#include "fwav_common.h"
#include "../../include/fwav.h"

namespace fwav {

constexpr int kLargeMaxK = 4096;
constexpr int kSelThreads = 512;
constexpr int kCap = 2 * kLargeMaxK;  // LDS list entries (u64) = 64 KB
constexpr int kSample = 2048;
constexpr int kScoreThreads = 256;
constexpr int kScoreQ = 32;            // queries per k_scores_batch pass (q vectors in LDS)
constexpr size_t kLargeBudget = size_t(1) << 30;  // score-row workspace budget (bytes)

__device__ __forceinline__ float score_chain(const float (&e)[16], const float* __restrict__ q, int kind) {
  return sgemv16([&](int k) { return e[k]; }, [&](int k) { return q[k]; }, kind);
}

// S[j·nd + d] = score(domain d, query active[qb + j]) for j < B (rows of queries past n_active untouched).
__global__ __launch_bounds__(kScoreThreads) void k_scores_batch(const float* __restrict__ emb, int64_t nd,
                                                                const int32_t* __restrict__ active,
                                                                const int32_t* __restrict__ n_active_p,
                                                                int64_t qb, int B, int64_t q_offset, SgemvSplit sp,
                                                                float* __restrict__ S) {
  __shared__ float qv[kScoreQ][16];
  const int n_active = *n_active_p;
  if (qb >= n_active) return;
  const int nb = (int)min<int64_t>(B, n_active - qb);
  const int64_t d = (int64_t)blockIdx.x * kScoreThreads + threadIdx.x;
  float e[16];
  if (d < nd) {
    const float4* p = reinterpret_cast<const float4*>(emb + d * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 v = p[j];
      e[4 * j] = v.x; e[4 * j + 1] = v.y; e[4 * j + 2] = v.z; e[4 * j + 3] = v.w;
    }
  }
  for (int j0 = 0; j0 < nb; j0 += kScoreQ) {
    const int m = min(kScoreQ, nb - j0);
    __syncthreads();
    for (int t = threadIdx.x; t < m * 16; t += kScoreThreads) {
      const int64_t q = (int64_t)active[qb + j0 + t / 16] + q_offset;
      qv[t / 16][t % 16] = emb[q * 16 + t % 16];
    }
    __syncthreads();
    if (d < nd) {
      const int kind = sgemv_kind((uint32_t)d, sp);
      for (int j = 0; j < m; ++j) S[(int64_t)(j0 + j) * nd + d] = score_chain(e, qv[j], kind);
    }
  }
}

// S[i·nd + d] = score(domain d, query row q_offset + rows[i]), i < n_rows (fwav_score_rows).
__global__ __launch_bounds__(kScoreThreads) void k_score_rows(const float* __restrict__ emb, int64_t nd,
                                                              const int32_t* __restrict__ rows, int n_rows,
                                                              int64_t q_offset, SgemvSplit sp, float* __restrict__ S) {
  __shared__ float qv[kScoreQ][16];
  const int64_t d = (int64_t)blockIdx.x * kScoreThreads + threadIdx.x;
  float e[16];
  if (d < nd) {
    const float4* p = reinterpret_cast<const float4*>(emb + d * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 v = p[j];
      e[4 * j] = v.x; e[4 * j + 1] = v.y; e[4 * j + 2] = v.z; e[4 * j + 3] = v.w;
    }
  }
  const int kind = d < nd ? sgemv_kind((uint32_t)d, sp) : 0;
  for (int j0 = 0; j0 < n_rows; j0 += kScoreQ) {
    const int m = min(kScoreQ, n_rows - j0);
    __syncthreads();
    for (int t = threadIdx.x; t < m * 16; t += kScoreThreads) {
      const int64_t q = (int64_t)rows[j0 + t / 16] + q_offset;
      qv[t / 16][t % 16] = emb[q * 16 + t % 16];
    }
    __syncthreads();
    if (d < nd)
      for (int j = 0; j < m; ++j) S[(int64_t)(j0 + j) * nd + d] = score_chain(e, qv[j], kind);
  }
}

// Block-wide descending bitonic sort of n (power of two, ≤ kCap) u64 keys in LDS.
__device__ void block_sort_desc(uint64_t* v, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < n / 2; i += kSelThreads) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint64_t a = v[lo], b = v[hi];
        if (desc ? (a < b) : (a > b)) {
          v[lo] = b;
          v[hi] = a;
        }
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ uint64_t key64(uint32_t k32, int64_t d) {
  return ((uint64_t)k32 << 32) | (uint64_t)(~(uint32_t)d);
}

struct SelSmem {
  uint64_t list[kCap];
  uint32_t hist[256];
  int cnt;
  int tflag;  // tie_flags of the query (fwav_topk.hip): 1 = equal scores inside the top K, 2 = at the K-th place
  int wtot[kSelThreads / 64];
  uint32_t bcast[4];
};

// Append every d with key32(row[d]) >= t to sm.list (while it fits); returns the total count (all threads).
__device__ int collect_ge(const float* __restrict__ row, int64_t nd, uint32_t t, SelSmem& sm) {
  if (threadIdx.x == 0) sm.cnt = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int64_t base = 0; base < nd; base += kSelThreads) {
    const int64_t d = base + threadIdx.x;
    const uint32_t k = d < nd ? f2key(row[d]) : 0u;
    const bool take = d < nd && k >= t;
    const uint64_t m = __ballot(take);
    if (m != 0ull) {
      int b = 0;
      if (lane == 0) b = atomicAdd(&sm.cnt, __popcll(m));
      b = __shfl(b, 0);
      const int pos = b + __popcll(m & ((1ull << lane) - 1ull));
      if (take && pos < kCap) sm.list[pos] = key64(k, d);
    }
  }
  __syncthreads();
  return sm.cnt;
}

// Exact K-th largest score key by radix select; then the list = {key > T} ∪ {lowest-index `need` keys == T}.
__device__ void radix_select_collect(const float* __restrict__ row, int64_t nd, int K, SelSmem& sm) {
  uint32_t prefix = 0, pmask = 0;
  int krem = K;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = threadIdx.x; i < 256; i += kSelThreads) sm.hist[i] = 0;
    __syncthreads();
    for (int64_t d = threadIdx.x; d < nd; d += kSelThreads) {
      const uint32_t k = f2key(row[d]);
      if ((k & pmask) == prefix) atomicAdd(&sm.hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int above = 0, b = 255;
      for (; b > 0; --b) {
        if (above + (int)sm.hist[b] >= krem) break;
        above += (int)sm.hist[b];
      }
      sm.bcast[0] = (uint32_t)b;
      sm.bcast[1] = (uint32_t)above;
    }
    __syncthreads();
    prefix |= sm.bcast[0] << shift;
    pmask |= 255u << shift;
    krem -= (int)sm.bcast[1];
    // last pass: hist[b] keys equal T exactly; more of them than the top K takes → the set is numpy's choice
    if (pass == 3 && threadIdx.x == 0 && (int)sm.hist[sm.bcast[0]] > krem) sm.tflag |= 2;
    __syncthreads();
  }
  const uint32_t T = prefix;
  const int need = krem;  // keys == T to take, lowest indices first
  const int greater = K - need;
  // keys > T (exactly `greater` of them)
  if (threadIdx.x == 0) sm.cnt = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t base = 0; base < nd; base += kSelThreads) {
    const int64_t d = base + threadIdx.x;
    const uint32_t k = d < nd ? f2key(row[d]) : 0u;
    const bool take = d < nd && k > T;
    const uint64_t m = __ballot(take);
    if (m != 0ull) {
      int b = 0;
      if (lane == 0) b = atomicAdd(&sm.cnt, __popcll(m));
      b = __shfl(b, 0);
      if (take) sm.list[b + __popcll(m & ((1ull << lane) - 1ull))] = key64(k, d);
    }
  }
  __syncthreads();
  // ties in index order: block-ordered prefix count per 512-element step
  int taken = 0;
  for (int64_t base = 0; base < nd && taken < need; base += kSelThreads) {
    const int64_t d = base + threadIdx.x;
    const bool tie = d < nd && f2key(row[d]) == T;
    const uint64_t m = __ballot(tie);
    if (lane == 0) sm.wtot[wave] = __popcll(m);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < kSelThreads / 64; ++w) {
      if (w < wave) before += sm.wtot[w];
      total += sm.wtot[w];
    }
    const int pos = taken + before + __popcll(m & ((1ull << lane) - 1ull));
    if (tie && pos < need) sm.list[greater + pos] = key64(T, d);
    taken += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) sm.cnt = K;
  __syncthreads();
}

__global__ __launch_bounds__(kSelThreads) void k_select(const float* __restrict__ S, int64_t nd,
                                                        const int32_t* __restrict__ active,
                                                        const int32_t* __restrict__ n_active_p, int64_t qb, int K,
                                                        int32_t* __restrict__ cand, int32_t* __restrict__ ties) {
  __shared__ SelSmem sm;
  const int n_active = *n_active_p;
  const int64_t qi = qb + blockIdx.x;
  if (qi >= n_active) return;
  if (threadIdx.x == 0) sm.tflag = 0;
  __syncthreads();
  const float* row = S + (int64_t)blockIdx.x * nd;
  int32_t* out = cand + (int64_t)active[qi] * K;
  int n;  // valid entries in sm.list
  if (nd <= K) {
    // every domain, sorted (the reference's full argsort branch), −1 padded
    for (int64_t d = threadIdx.x; d < nd; d += kSelThreads) sm.list[d] = key64(f2key(row[d]), d);
    n = (int)nd;
  } else {
    // 1. sampled threshold
    // (the samples live in the list region until the first collect overwrites it; as u64 with a zero low
    // word so the list's sort orders them)
    uint64_t* s64 = sm.list;
    for (int i = threadIdx.x; i < kSample; i += kSelThreads) s64[i] = (uint64_t)f2key(row[(int64_t)i * nd / kSample]) << 32;
    block_sort_desc(s64, kSample);
    // rank for ≈ 2K of nd, then widen / tighten until K ≤ count ≤ kCap
    int64_t want = 2 * (int64_t)K;
    int cnt = -1;
    for (int attempt = 0; attempt < 4; ++attempt) {
      int64_t rank = (want * kSample + nd - 1) / nd + 8;
      if (rank > kSample - 1) rank = kSample - 1;
      __syncthreads();
      if (threadIdx.x == 0) sm.bcast[2] = (uint32_t)(s64[rank] >> 32);
      __syncthreads();
      const uint32_t t = sm.bcast[2];
      if (rank == kSample - 1) {
        cnt = -1;  // sample exhausted: no threshold below the sample minimum is known
        break;
      }
      __syncthreads();
      cnt = collect_ge(row, nd, t, sm);
      if (cnt >= K && cnt <= kCap) break;
      // the list region held the samples: rebuild them for the next attempt
      if (attempt + 1 < 4) {
        for (int i = threadIdx.x; i < kSample; i += kSelThreads)
          s64[i] = (uint64_t)f2key(row[(int64_t)i * nd / kSample]) << 32;
        block_sort_desc(s64, kSample);
      }
      want = cnt < K ? want * 4 : want / 2;
      if (want < K) want = K;
      cnt = -1;
    }
    if (cnt < K || cnt > kCap) {
      radix_select_collect(row, nd, K, sm);
      cnt = K;
    }
    n = cnt;
  }
  // pad to a power of two and sort
  int p2 = 1;
  while (p2 < n) p2 <<= 1;
  for (int i = n + threadIdx.x; i < p2; i += kSelThreads) sm.list[i] = 0ull;
  block_sort_desc(sm.list, p2);
  // exactly equal scores among the first K + 1 (for nd ≤ K: among all), listed for fwav_tie_check
  for (int e = threadIdx.x; e + 1 < n && e + 1 <= K; e += kSelThreads)
    if (key2f((uint32_t)(sm.list[e] >> 32)) == key2f((uint32_t)(sm.list[e + 1] >> 32)))
      atomicOr(&sm.tflag, e + 1 < K ? 1 : 2);
  __syncthreads();
  if (threadIdx.x == 0 && ties != nullptr && sm.tflag != 0) {
    const int pos = atomicAdd(ties, 1);
    ties[1 + (int64_t)kTieRec * pos] = 2 * active[qi] + ((sm.tflag >> 1) & 1);
    ties[2 + (int64_t)kTieRec * pos] = -1;  // tie group not collected (K > 64 rows are all resolved on the host)
  }
  for (int e = threadIdx.x; e < K; e += kSelThreads) out[e] = e < n ? (int32_t)(~(uint32_t)(sm.list[e] & 0xffffffffu)) : -1;
}

int64_t large_batch(int64_t nd, int64_t max_q) {
  int64_t b = (int64_t)(kLargeBudget / (4 * (size_t)(nd > 0 ? nd : 1)));
  if (b > 256) b = 256;
  if (b < 1) b = 1;
  if (max_q > 0 && b > max_q) b = max_q;
  return b;
}

size_t large_workspace_bytes(int64_t nd, int64_t max_q) { return (size_t)large_batch(nd, max_q) * nd * 4; }

int launch_topk_large(const float* emb, int64_t nd, const int32_t* active, const int32_t* n_active, int64_t max_q,
                      int64_t q_offset, int K, int32_t* cand, float* S, SgemvSplit sp, int32_t* ties, hipStream_t st) {
  const int64_t B = large_batch(nd, max_q);
  for (int64_t qb = 0; qb < max_q; qb += B) {
    k_scores_batch<<<cdiv(nd, kScoreThreads), kScoreThreads, 0, st>>>(emb, nd, active, n_active, qb, (int)B,
                                                                       q_offset, sp, S);
    k_select<<<B, kSelThreads, 0, st>>>(S, nd, active, n_active, qb, K, cand, ties);
  }
  FWAV_LAUNCH_CHECK("fwav_sim_topk (large K)");
  return FWAV_OK;
}

int launch_score_rows(const float* emb, int64_t nd, const int32_t* rows, int64_t n_rows, int64_t q_offset,
                      SgemvSplit sp, float* S, hipStream_t st) {
  for (int64_t r0 = 0; r0 < n_rows; r0 += 4096) {
    const int m = (int)std::min<int64_t>(4096, n_rows - r0);
    k_score_rows<<<cdiv(nd, kScoreThreads), kScoreThreads, 0, st>>>(emb, nd, rows + r0, m, q_offset, sp,
                                                                     S + r0 * nd);
  }
  FWAV_LAUNCH_CHECK("fwav_score_rows");
  return FWAV_OK;
}

}  // namespace fwav
