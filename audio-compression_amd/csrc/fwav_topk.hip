// fwav_topk.hip — fused similarity GEMM + streaming exact top-K on MFMA (gfx950).
//
// Replaces (reference /root/reference/fractal.py):
//   cpu_worker                          :556-632  per range: q = emb[i] (quirk Q1), linear search, pad to K
//   range_candidates_from_embedding_emb :535-541  scores = E_dom @ q ; argpartition top-K ; sort desc
//   pad_candidates                      :544-552
//
// Contract: for every active query q (a range index; its query vector is domain-embedding row q), write
// the K domains with the largest f32 score s(q,d) = emb[d]·emb[q] evaluated in the reference's own order (numpy →
// OpenBLAS sgemv_t: its 4-column microkernel, and for the last columns of each BLAS thread's chunk the 4x2 / 4x1
// tail kernels — fwav_common.h sgemv16 / sgemv_kind, pinned column by column against numpy), in (score desc,
// index asc) order, −1-padded when nd < K.  The scores being the reference's bit for bit, the result can differ from
// the reference's only among exactly equal scores, whose order (and, at the K-th place, set) numpy's introselect /
// argsort decide: every such query is listed in `ties` (record_tie) for fwav_tie_check / fwav.ties.
//
// The n_ranges × n_domains score matrix (4.4e11 entries at cfg2) is never materialised.
//
// Production path (emb16 != NULL), in file order: the work plan (query blocks, table pieces, query halves);
// k_sim_topk_f16 — 8 waves × 32 queries per workgroup (16 waves, one per CU, above 8 Mi domains), the fp16 table
// streamed through LDS by LDS-DMA in groups of 4 chunks, one fp16 MFMA per 32-domain tile and a max-fold per lane
// (stream_group), fired chunks replayed at window ends into per-query two-ended key buffers with inline compaction
// (replay_window / append_tile / compact16_s16), band limits seeded from each query's own domain window
// (seed_limit) and shared between the table pieces of a query (atomicMax), an exact f32 final pass in the
// reference's sgemv order (compact16) or a band hand-off to k_merge_pieces (piece_band); then the device-side
// overflow lists relaunch the same kernel in the narrower HL and exact modes.  Measurements behind every constant:
// DESIGN.md §3.1.
//
// k_sim_topk_f32 (emb16 == NULL; tests and a reference for the production kernel below): workgroup = 4 waves × 32
// queries; each 256-domain chunk is staged row-major in LDS and every lane scores its query against 16 domain rows
// of each 32-domain tile with sgemv16 (VALU), keeps a running threshold θ (one register per lane), and appends
// (score, index) keys that beat θ to the query's LDS buffer; a nearly full buffer is sorted (64-lane bitonic), cut
// to its top K and θ set to the K-th score.  Domains stream in increasing index order, so a later domain whose
// score equals θ can never displace an earlier one: strict '>' is exact.
#include <algorithm>
#include <cstring>
#include <type_traits>
#include "fwav_common.h"
#include "../../include/fwav.h"

// Every compile-time knob below (-DFWAV_TOPK_*: geometry, tuning and experiment code paths) builds A/B variants of
// the DEBUG library only (tools/ab_build.sh adds -DFWAV_DEBUG_API): a product build that sets one stops here, so
// libfwav.so is always the measured default.
#if !defined(FWAV_DEBUG_API) && (defined(FWAV_TOPK_ABL) || defined(FWAV_TOPK_APPOFF) || defined(FWAV_TOPK_CAP) || \
    defined(FWAV_TOPK_CB) || defined(FWAV_TOPK_CENT) || defined(FWAV_TOPK_CENTWIDE) || defined(FWAV_TOPK_CENT_HL) || \
    defined(FWAV_TOPK_CENT_MINQ) || defined(FWAV_TOPK_CG) || defined(FWAV_TOPK_CHAINS) || \
    defined(FWAV_TOPK_CPDBL) || defined(FWAV_TOPK_CPMIN) || defined(FWAV_TOPK_CSHARE) || defined(FWAV_TOPK_BANDB) || defined(FWAV_TOPK_CVACC) || \
    defined(FWAV_TOPK_CW) || defined(FWAV_TOPK_CWPE) || defined(FWAV_TOPK_DELTA) || defined(FWAV_TOPK_EXGROW) || \
    defined(FWAV_TOPK_EXWPE) || defined(FWAV_TOPK_FIRST) || defined(FWAV_TOPK_G) || defined(FWAV_TOPK_GROW) || \
    defined(FWAV_TOPK_HLDELTA) || defined(FWAV_TOPK_HLPRE) || defined(FWAV_TOPK_INTERLEAVE) || \
    defined(FWAV_TOPK_MAXP) || defined(FWAV_TOPK_PMAJOR) || defined(FWAV_TOPK_PRIO) || defined(FWAV_TOPK_QS) || \
    defined(FWAV_TOPK_RB) || defined(FWAV_TOPK_SEEDHALF) || defined(FWAV_TOPK_SMALLSORT) || defined(FWAV_TOPK_W) || \
    defined(FWAV_TOPK_WARM) || defined(FWAV_TOPK_WIDE_MIN) || defined(FWAV_TOPK_WIN) || defined(FWAV_TOPK_WPE) || \
    defined(FWAV_FLOOR_PILOTS) || defined(FWAV_FLOOR_RANK) || defined(FWAV_TOPK_YOUNG) || defined(FWAV_TOPK_TAIL))
#error "experiment switches build the debug library only (-DFWAV_DEBUG_API)"
#endif

namespace fwav {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kTopkWaves = 4;
constexpr int kTopkQ = 32 * kTopkWaves;  // queries per workgroup
constexpr int kChunk = 256;              // domains staged per LDS chunk (16 KB of f32 embeddings)
constexpr int kTopkThreads = 64 * kTopkWaves;

__device__ __forceinline__ uint64_t make_key(float s, int32_t idx) {
  return ((uint64_t)f2key(s) << 32) | (uint64_t)(~(uint32_t)idx);
}
__device__ __forceinline__ int32_t key_idx(uint64_t k) { return (int32_t)(~(uint32_t)(k & 0xffffffffu)); }
__device__ __forceinline__ float key_score(uint64_t k) { return key2f((uint32_t)(k >> 32)); }

// Descending bitonic sort of E*64 keys held as v[j] = element j*64 + lane.
template <int E>
__device__ __forceinline__ void wave_sort_desc(uint64_t (&v)[E]) {
  const int lane = threadIdx.x & 63;
  constexpr int N = E * 64;
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int js = stride >> 6;
#pragma unroll
        for (int j = 0; j < E; ++j) {
          if ((j & js) == 0) {
            const int jp = j | js;
            const int e = j * 64 + lane;
            const bool desc = (e & size) == 0;
            uint64_t a = v[j], b = v[jp];
            bool sw = desc ? (a < b) : (a > b);
            v[j] = sw ? b : a;
            v[jp] = sw ? a : b;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) {
          const int e = j * 64 + lane;
          uint64_t o = __shfl_xor(v[j], stride);
          const bool lower = (lane & stride) == 0;
          const bool desc = (e & size) == 0;
          uint64_t mx = v[j] > o ? v[j] : o;
          uint64_t mn = v[j] > o ? o : v[j];
          v[j] = (lower == desc) ? mx : mn;
        }
      }
    }
  }
}

// Exactly equal scores among the first K + 1 entries of a sorted key list (entry e = j·64 + lane, n valid entries):
// bit 0 — two equal scores inside the top K (numpy's argpartition/argsort decide their order), bit 1 — the K-th and
// (K+1)-th scores are equal (numpy decides the set).  Scores compare as floats (−0 == +0).  Whole wave; the result
// is wave-uniform.
template <int E>
__device__ __forceinline__ int tie_flags(const uint64_t (&v)[E], int n, int K) {
  const int lane = threadIdx.x & 63;
  bool in = false, bd = false;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    uint64_t nx = __shfl_down(v[j], 1);
    const uint64_t first_next = __shfl(v[j + 1 < E ? j + 1 : j], 0);
    if (lane == 63) nx = j + 1 < E ? first_next : 0ull;
    const int e = j * 64 + lane;
    if (e + 1 < n && e + 1 <= K && key_score(nx) == key_score(v[j])) {
      if (e + 1 < K) in = true;
      else bd = true;
    }
  }
  return (__ballot(in) != 0ull ? 1 : 0) | (__ballot(bd) != 0ull ? 2 : 0);
}

// Lists query qid for the tie check (fwav_tie_check): ties[0] = count; record i = ties[1 + kTieRec·i ..]:
// [0] = 2·qid + (boundary tie), and for a boundary tie [1] = the number of domains outside the emitted K whose score
// equals the K-th (−1: not known), [2 ..] = those domains.  `v` (sorted, n valid entries) is the query's final band:
// when `group` is set it holds every domain scoring at least the K-th score, so the tie group is complete.  Whole
// wave (wave-uniform arguments).
template <int E>
__device__ __forceinline__ void record_tie(int32_t* ties, int32_t qid, int flags, const uint64_t (&v)[E], int n,
                                           int K, bool group) {
  if (ties == nullptr || flags == 0) return;
  const int lane = threadIdx.x & 63;
  int pos = 0;
  if (lane == 0) pos = atomicAdd(ties, 1);
  pos = __shfl(pos, 0);
  int32_t* rec = ties + 1 + (int64_t)kTieRec * pos;
  if (lane == 0) rec[0] = 2 * qid + ((flags >> 1) & 1);
  if (!(flags & 2)) return;
  int total = -1;
  if (group) {
    uint64_t kth = 0;
#pragma unroll
    for (int j = 0; j < E; ++j)
      if (j == ((K - 1) >> 6)) kth = __shfl(v[j], (K - 1) & 63);
    const float S = key_score(kth);
    total = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const int e = j * 64 + lane;
      const bool in = e >= K && e < n && key_score(v[j]) == S;  // sorted: positions K, K + 1, … of the group
      if (in && e - K < kTieRec - 2) rec[2 + e - K] = key_idx(v[j]);
      total += __popcll(__ballot(in));
    }
    if (total > kTieRec - 2) total = -1;
  }
  if (lane == 0) rec[1] = total;
}
template <int E>
__device__ __forceinline__ void record_tie(int32_t* ties, int32_t qid, int flags, const uint64_t (&v)[E], int n,
                                           int K) {
  record_tie<E>(ties, qid, flags, v, n, K, false);
}

// Sort query ql's buffer, keep the top K, update count and θ; returns tie_flags of the sorted buffer (a (K+1)-th
// entry equal to the K-th, about to be dropped, sets bit 1).  Whole wave, uniform ql.
template <int C>
__device__ __forceinline__ int compact(uint64_t* __restrict__ keys, int* __restrict__ cnt, float* __restrict__ theta,
                                       int ql, int K) {
  constexpr int E = C / 64;
  const int lane = threadIdx.x & 63;
  const int n = cnt[ql];
  uint64_t v[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < n ? keys[ql * C + e] : 0ull;
  }
  wave_sort_desc<E>(v);
  const int tf = tie_flags<E>(v, n, K);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    if (e < K && e < n) keys[ql * C + e] = v[j];
  }
  // K-th key (position K-1) lives in lane (K-1)&63, slot (K-1)>>6
  const int kl = (K - 1) & 63, kj = (K - 1) >> 6;
  uint64_t kth = 0;
#pragma unroll
  for (int j = 0; j < E; ++j)
    if (j == kj) kth = __shfl(v[j], kl);
  if (lane == 0) {
    cnt[ql] = n < K ? n : K;
    theta[ql] = n >= K ? key_score(kth) : -INFINITY;
  }
  return tf;
}

template <int C>
__global__ __launch_bounds__(kTopkThreads) void k_sim_topk_f32(const float* __restrict__ emb, int64_t nd,
                                                               const int32_t* __restrict__ active,
                                                               const int32_t* __restrict__ n_active_p,
                                                               int64_t q_offset, int K, int32_t* __restrict__ cand,
                                                               SgemvSplit sp, int32_t* __restrict__ ties) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* keys = (uint64_t*)smem;                            // [kTopkQ][C]
  float* lda = (float*)(keys + (size_t)kTopkQ * C);            // [kChunk][16] (row-major domain rows)
  int* cnt = (int*)(lda + 16 * kChunk);                        // [kTopkQ]
  float* theta = (float*)(cnt + kTopkQ);                       // [kTopkQ]
  // [kTopkQ] f2key of the largest θ that a domain of equal score was not kept at (0: none); the set among equal
  // scores is numpy's choice only if that θ is the final K-th score (θ rises, so earlier ones are superseded)
  uint32_t* tieb = (uint32_t*)(theta + kTopkQ);

  const int n_active = *n_active_p;
  const int qbase = blockIdx.x * kTopkQ;
  if (qbase >= n_active) return;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int col = lane & 31;
  const int h = lane >> 5;
  const int ql = wave * 32 + col;  // local query slot
  const int qi = qbase + ql;
  const int32_t q = qi < n_active ? active[qi] : -1;

  float qf[16];  // the whole query vector (sgemv16)
#pragma unroll
  for (int k = 0; k < 16; ++k) qf[k] = q >= 0 ? emb[((int64_t)q + q_offset) * 16 + k] : 0.0f;
  float th = q >= 0 ? -INFINITY : INFINITY;  // invalid lanes never append
  if (tid < kTopkQ) {
    cnt[tid] = 0;
    theta[tid] = -INFINITY;
    tieb[tid] = 0;
  }

  const int64_t nchunks = cdiv(nd, kChunk);
  // prefetch chunk 0: thread t holds the 16 floats of domain chunk*kChunk + t
  float4 pf[4];
  auto load_chunk = [&](int64_t c) {
    const int64_t d = c * kChunk + tid;
    if (d < nd) {
      const float4* p = reinterpret_cast<const float4*>(emb + d * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) pf[j] = p[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) pf[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  load_chunk(0);

  for (int64_t c = 0; c < nchunks; ++c) {
    __syncthreads();  // previous chunk fully consumed (and cnt/theta init visible)
#pragma unroll
    for (int j = 0; j < 4; ++j) reinterpret_cast<float4*>(lda)[tid * 4 + j] = pf[j];
    __syncthreads();
    if (c + 1 < nchunks) load_chunk(c + 1);
    const int64_t dbase = c * kChunk;

    for (int t = 0; t < kChunk / 32; ++t) {
      // the tile's sgemv kernels (fwav_common.h): all kind 0 unless it holds the tail of a BLAS thread chunk
      const uint32_t tf0 = (uint32_t)(dbase + t * 32);
      const uint32_t tl = (uint32_t)min<int64_t>(dbase + t * 32 + 31, nd - 1);
      const bool plain = sgemv_kind(tl, sp) == 0 && tf0 >= sgemv_chunk_start(tl, sp);
      // the lane's 16 rows of the tile (the row ↔ domain map of the MFMA tiles: d0 + (r&3) + 8*(r>>2))
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float4* row = reinterpret_cast<const float4*>(lda) + (t * 32 + 4 * h + (r & 3) + 8 * (r >> 2)) * 4;
        float dv[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 v = row[j];
          dv[4 * j] = v.x; dv[4 * j + 1] = v.y; dv[4 * j + 2] = v.z; dv[4 * j + 3] = v.w;
        }
        const uint32_t dr = (uint32_t)(dbase + t * 32 + 4 * h + (r & 3) + 8 * (r >> 2));
        acc[r] = sgemv16([&](int k) { return dv[k]; }, [&](int k) { return qf[k]; },
                         plain || dr >= (uint32_t)nd ? 0 : sgemv_kind(dr, sp));
      }
      const int64_t d0 = dbase + t * 32 + 4 * h;  // domain of acc[r] = d0 + (r&3) + 8*(r>>2)
      // mask rows past nd
      if (dbase + t * 32 + 32 > nd) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (d0 + (r & 3) + 8 * (r >> 2) >= nd) acc[r] = -INFINITY;
      }
      float mx = acc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, acc[r]);
      if (__ballot(mx >= th) != 0ull) {
        uint64_t* kq = keys + (size_t)ql * C;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (acc[r] > th) {
            const int slot = atomicAdd(&cnt[ql], 1);
            kq[slot] = make_key(acc[r], (int32_t)(d0 + (r & 3) + 8 * (r >> 2)));
          } else if (acc[r] == th && th != -INFINITY) {
            atomicMax(&tieb[ql], f2key(th));  // equal to θ but later in index order: not kept
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        uint64_t need = __ballot(lane < 32 && cnt[ql] > C - 32);
        while (need != 0ull) {
          const int l = __builtin_ctzll(need);
          need &= need - 1;
          if ((compact<C>(keys, cnt, theta, wave * 32 + l, K) & 2) && lane == 0)
            atomicMax(&tieb[wave * 32 + l], f2key(theta[wave * 32 + l]));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (q >= 0) th = theta[ql];
      }
    }
  }

  // final: sort every query of this wave and write its top K
  for (int l = 0; l < 32; ++l) {
    const int qs = wave * 32 + l;
    const int qq = qbase + qs;
    if (qq >= n_active) break;
    const int32_t qid = active[qq];
    const int tf = compact<C>(keys, cnt, theta, qs, K);
    const uint32_t tv = tieb[qs];
    const uint64_t none[1] = {0ull};
    record_tie<1>(ties, qid, tf | (tv != 0u && cnt[qs] >= K && key2f(tv) == theta[qs] ? 2 : 0), none, 0, K);
    const int n = cnt[qs];
    int32_t* out = cand + (int64_t)qid * K;
    for (int e = lane; e < K; e += 64) out[e] = e < n ? key_idx(keys[(size_t)qs * C + e]) : -1;
  }
}

// ------------------------------------------------------------------ fp16 pre-filter + exact f32 rescoring
// Same contract and results as k_sim_topk_f32 (the production K ≤ 64 search).
//
// Exactness.  Three scores per (query, domain): s32 the exact f32 score (sgemv16), s16 = ONE
// v_mfma_f32_32x32x16_f16 of the fp16 high parts (x_hi = f16(x)), shl = s16 + MFMA(d_hi, q_lo) + MFMA(d_lo, q_hi)
// (x_lo = f16(x − x_hi), f32 accumulation).  |s16 − s32| ≤ (2u + u²)·Σ|q_k d_k| + f32 accumulation ≤ 1.9584e-3
// (u = 2^-11; Σ|q_k d_k| ≤ ‖q‖‖d‖ ≤ 2, the tonal and transient heads each having norm ≤ 1) < δ = 2.0e-3;
// |shl − s32| ≤ 3u²·2 + fp16-subnormal low parts (≈ 3e-7) + three MFMAs' f32 accumulation (≤ 48 roundings of ≤ 2,
// 5.7e-6) + s32's own rounding (≈ 1e-6) < δ' = 1e-5 (measured max 6e-7: tools/micro/hilo_err.hip).
// The stream scores every tile with s16 only and fires a tile when some s16 > lim − δ − 2δ'; the replay of a fired
// tile adds the two low-part MFMAs and appends (shl, index) keys with shl > lim to the query's buffer.  A
// compaction takes S = its K-th largest shl and keeps the band shl > lim = S − 2δ' (K domains have s32 ≥ S − δ', so
// every exact top-K member has shl ≥ S − 2δ').  The final pass rescores the band in exact f32 (sgemv16), sorts
// (score desc, index asc) and emits K — identical to the all-f32 kernel whatever the processing order.  A band that
// would not leave 64 free slots (≥ 192 domains within 2δ' of the K-th: runs of identical tiles, periodic signals)
// flags the query for the exact-mode relaunch.
//
// Geometry.  8 waves × 32 queries per workgroup, two workgroups per CU (4 waves per SIMD).  Lane l owns query
// l & 31 (the MFMA's B column, in registers for the whole run) and 16 domain rows of each tile.  The fp16
// table streams through LDS in groups of 4 chunks (256 domains = 8 KB each) with one barrier per group: group
// g+1 goes global → LDS by LDS-DMA (global_load_lds_dwordx4, 8 wave-instructions per chunk) into the other
// half while group g is consumed.  Per chunk a wave issues 8 ds_read_b128 + 8 MFMAs and folds each tile's 16
// outputs into its own integer-max chain (8 × v_max3 per tile), then takes ballots against its integer filter.
// Chunks with a firing chain are recorded (chunk, chain mask) and replayed at the window end (every 32 groups;
// every group during the first 32 chunks) from L2/MALL in batches of 8 tiles: recompute the tile's three MFMAs,
// append survivors to the query's two-ended global key buffer (C = 256 entries), compact a buffer inline when
// it is nearly full.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
// Native 16-byte vector for the chunk stream (a uint4 struct copy lowers to memcpy, which keeps the prefetch
// array out of registers).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// δ ≥ max |s16 − s32| (see "Exactness" above): 1.9536e-3 (f16 rounding of both operands) + ≈ 5e-6 (f32
// accumulation of both sums, f16 subnormals) = 1.9584e-3.  2.5e-3 → 2.0e-3: cfg3 792 → 719 ms, cfg2 unchanged.
#ifndef FWAV_TOPK_DELTA
#define FWAV_TOPK_DELTA 2.0e-3f
#endif
constexpr float kF16Delta = FWAV_TOPK_DELTA;
// δ' ≥ max |shl − s32| (see "Exactness"); the stream fires a tile when s16 > lim − kStreamMargin
#ifndef FWAV_TOPK_HLDELTA
#define FWAV_TOPK_HLDELTA 1.0e-5f
#endif
constexpr float kHLDelta = FWAV_TOPK_HLDELTA;
constexpr float kStreamMargin = kF16Delta + 2.0f * kHLDelta;
// Search modes (template MODE of k_sim_topk_f16; launched as a chain, each relaunch on the previous pass's overflow
// list, seeded with its band limits):
//   kModeS16: band on s16 (width 2δ), keys s16 — no low-part MFMAs in the replays;
//   kModeHL : band on shl (width 2.5δ'), keys shl — three MFMAs per replayed tile, overflows only on ≥ 192 domains
//             within ≈ 2δ' of the K-th (runs of identical tiles);
//   kModeEX : exact keys (sgemv16 on the VALU for rows passing the s16 filter), a compaction keeps exactly the top K,
//             so nothing can overflow.
constexpr int kModeS16 = 0, kModeHL = 1, kModeEX = 2;
// The first pass's mode: S16 (→ HL → EX relaunches) for tables of at most kHLFirstMinDomains domains, HL (→ EX) for
// larger ones.  Same-box A/B (tools/ab_topk.py, identical outputs): cfg2 (1.3 M domains, noise) S16 20.0–20.1 ms vs
// HL 20.7–21.0 — its bands never overflow, and HL's three-MFMA replays cost more; cfg3 (6.6 M, speech-like) S16
// 254–258 ms vs HL 186–189 (30.5 % of the queries overflow the S16 band and are searched again); a cfg4 shard (86 M,
// noise) S16 1,135 ms vs HL 960.  FWAV_TOPK_FIRST=0/1 forces S16/HL (A/B builds).
#ifndef FWAV_TOPK_FIRST
#define FWAV_TOPK_FIRST -1
#endif
constexpr int64_t kHLFirstMinDomains = int64_t(1) << 22;
#ifdef FWAV_DEBUG_API
static int g_first_mode = -1;  // fwav_debug_topk_mode (debug library only): force S16 / HL
#else
constexpr int g_first_mode = -1;  // the product library has no process-global knobs
#endif
__host__ inline int first_mode(int64_t nd) {
  if (g_first_mode >= 0) return g_first_mode;
  return FWAV_TOPK_FIRST >= 0 ? FWAV_TOPK_FIRST : (nd > kHLFirstMinDomains ? kModeHL : kModeS16);
}
// HL replays test the tile's s16 against the current limit before the two low-part MFMAs (A/B at cfg2: 21.38 vs
// 20.98 ms without — the test lengthens each tile's dependent chain; cfg3 192.8 vs 188.5)
#ifndef FWAV_TOPK_HLPRE
#define FWAV_TOPK_HLPRE 0
#endif
#define FWAV_TRACE(qid, a, b, c, d) do { } while (0)

// Diagnostic counters (fwav_debug_sim_topk only; stays nullptr in production launches), summed over waves:
//   [0] replayed chunks  [1] firing tiles  [2] appends  [3] streaming compactions
//   [4] ticks in window replays (incl. their compactions)  [5] ticks in streaming compactions
//   [6] ticks per wave (whole kernel)  [7] ticks waiting at the group barrier  [8] ticks in the final pass
//   [9] ticks streaming (MFMA + filter, between barrier and window end)   (s_memrealtime ticks, 100 MHz)
// `stats` inside the kernel is the wave's own LDS counter row (lane 0 adds; flushed once per wave at the end),
// so the instrumentation adds no global atomics to the measured loop.
// [12] ticks waiting for the group's own chunk DMA (vmcnt at the group top; [7] is then the barrier alone),
//   [13] centroid level-1 ticks, [14] centroid level-2 (tile, set) pairs
constexpr int kStats = 16;
__device__ __forceinline__ void stat_add_p(unsigned long long* stats, int i, unsigned long long v) {
  if (stats != nullptr && (threadIdx.x & 63) == 0) stats[i] += v;
}
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);
#define stat_add(i, v) stat_add_p(stats, (i), (v))
// Production geometry (the -D overrides build A/B variants: tools/ab_topk.py)
#ifndef FWAV_TOPK_G
#define FWAV_TOPK_G 4
#endif
#ifndef FWAV_TOPK_W
#define FWAV_TOPK_W 8
#endif
#ifndef FWAV_TOPK_QS
#define FWAV_TOPK_QS 1
#endif
#ifndef FWAV_TOPK_WPE
#define FWAV_TOPK_WPE 4  // launch bound: waves per SIMD the register allocation must allow
#endif
// Centroid geometry (cent_level1): FWAV_TOPK_CENT query sets per wave (0: off), FWAV_TOPK_CW waves per
// workgroup, FWAV_TOPK_CG chunks per barrier, FWAV_TOPK_CWPE waves per SIMD for the register allocation
// Same-box A/B (tools/ab_topk.py, identical outputs; profiles/r04/ab_cent_*.log), search ms base → centroid:
//   cfg2 (330,750 queries) 20.36 → 17.47 (QS 2, G 4, 2 workgroups per CU, 4 waves per SIMD), QS 4 / G 3 18.49,
//   QS 4 / G 4 (one workgroup per CU: 2 waves per SIMD) 25.3 — the base kernel held to the same occupancy 25.6;
//   165,375 queries 10.94 → 9.93, 82,688 5.92 → 5.69, 41,344 (one rank's eighth) 3.32 → 3.53 (fewer, longer items:
//   the base geometry is kept below FWAV_TOPK_CENT_MINQ); cfg3 (hi/lo band, 6.6 M domains) 180 → 195 (kept base).
#ifndef FWAV_TOPK_CENT
#define FWAV_TOPK_CENT 2
#endif
#ifndef FWAV_TOPK_CW
#define FWAV_TOPK_CW 8
#endif
#ifndef FWAV_TOPK_CG
#define FWAV_TOPK_CG 4
#endif
#ifndef FWAV_TOPK_CWPE
#define FWAV_TOPK_CWPE 4
#endif
#ifndef FWAV_TOPK_CB
#define FWAV_TOPK_CB 2  // centroid level 2: (tile, set) pairs in flight together (4: +0.8 % cfg2, +10 % at 82,688 queries; 6, 8: spills)
#endif
#ifndef FWAV_TOPK_APPOFF
#define FWAV_TOPK_APPOFF 1  // appends: running byte offset and a one-op key low word (else slot arithmetic per row)
#endif
#ifndef FWAV_TOPK_CVACC
#define FWAV_TOPK_CVACC 1  // centroid level 1: firing tiles accumulated per lane in a VGPR (else scalar masks per set)
#endif
#ifndef FWAV_TOPK_PRIO
// wave priorities (bits): 1 waves W/2.. at prio 1, 2 compactions at prio 2, 4 centroid level 2 + appends at prio 1
// (the part of a group whose length varies from wave to wave: the group barrier waits for it), 8 the base geometry's
// window-end replays at prio 1.  Same-box A/B, identical outputs (profiles/r05/ab_prio.log): cfg2 17.46 → 17.24 /
// 17.27 ms with 4 (2: 17.33 / 17.38, 6: 17.39 / 17.44, 1: +0.5 %, 3: +2.5 %), 165,375 queries 9.77 → 9.61; adding 8:
// cfg3 179.8 → 178.3 ms, one rank's eighth and quarter within ±0.5 %
#define FWAV_TOPK_PRIO 12
#endif
#ifndef FWAV_TOPK_CSHARE
#define FWAV_TOPK_CSHARE 1  // centroid geometry: read the pieces' shared limits every group (else at window ends)
#endif
// Ablation builds (tools/ab_build.sh NAME -DFWAV_TOPK_ABL=<dbg bits>): the production kernel with the given `dbg`
// bits fixed at compile time — the STATS kernel's counters cost registers (it spills), which skews its timings.
#ifndef FWAV_TOPK_ABL
#define FWAV_TOPK_ABL 0
#endif
// Exact mode (overflow relaunch) compacts every FWAV_TOPK_EXGROW appends, so its K-th exact key — the store filter —
// and band limit rise sooner (cfg3 at δ = 2.5e-3: 32 / 64 / 96 / 128 / full buffer 859 / 861 / 870 / 887 / 898 ms;
// at δ = 2.0e-3: 16 / 24 / 32 / 64 / 128 → 690 / 702 / 695–704 / 711–725 / 727 ms)
#ifndef FWAV_TOPK_EXGROW
#define FWAV_TOPK_EXGROW 32
#endif
// Exact-mode occupancy (waves per SIMD): 2 avoids its register spills but halves the workgroups per CU (856 vs 785 ms)
#ifndef FWAV_TOPK_EXWPE
#define FWAV_TOPK_EXWPE 4
#endif
constexpr int kGroup = FWAV_TOPK_G;     // chunks per barrier
constexpr int k16Waves = FWAV_TOPK_W;   // waves per workgroup
constexpr int k16Sets = FWAV_TOPK_QS;   // query sets of 32 per wave (each LDS fragment feeds k16Sets MFMAs)
// final passes: bands of at most 128 keys rescored and sorted as 128 (A/B builds: 0 = always C)
#ifndef FWAV_TOPK_SMALLSORT
#define FWAV_TOPK_SMALLSORT 1
#endif
#ifndef FWAV_TOPK_CAP
#define FWAV_TOPK_CAP 256
#endif
constexpr int k16Cap = FWAV_TOPK_CAP;  // key-buffer entries per query (global workspace)
#ifndef FWAV_TOPK_GROW
#define FWAV_TOPK_GROW 64
#endif
// (A/B: triggers at 128 / 160 entries, cfg2 18.85 / 18.18 vs 17.50 ms, profiles/r04/ab_trig_*.log)
constexpr int kTrig = k16Cap - 32;  // early compaction: buffer size ...
constexpr int kGrow = FWAV_TOPK_GROW;  // ... and growth since the last compaction
static_assert(k16Cap >= 128 && (k16Cap & (k16Cap - 1)) == 0, "the final bitonic sort needs a power-of-two buffer");
// (A/B at cfg2: 512 entries 24.4 ms vs 21.2 ms for 256 — fewer compactions do not pay for the longer final sort)
constexpr int k16QB = 32 * k16Waves * k16Sets;  // queries per block (one workgroup's query set)
#ifndef FWAV_TOPK_MAXP
#define FWAV_TOPK_MAXP 8
#endif
// a first pass's table pieces per split block (merge: P·(C − 64) keys per query at most) ...
constexpr int kPlanMaxPieces = FWAV_TOPK_MAXP;
// ... and any plan's, the floor's later passes included (k_merge_pieces is instantiated for ≤ 8, 16 and 32 pieces)
constexpr int kMaxPieces = 64;
static_assert(kPlanMaxPieces <= kMaxPieces, "first-pass plans stay within the merge's widest instantiation");

// Work plan of the fp16 search.  The n_blocks query blocks are items of one launch, dispatched in order: the first
// F = nb − R blocks stream the whole table, then each of the last R = min(nb, rt) blocks is split into P pieces of
// the table (contiguous chunk ranges) so that the launch's tail is made of short items: without the split the last
// round of whole-table workgroups runs on a fraction of the slots and takes ≈ 1/5 of the kernel.  A piece ends with
// its exact top K (f32 keys, sorted), and k_merge_pieces merges a split block's P lists.  Each item owns one
// key-buffer region (QB queries × C entries).  Every workgroup recomputes the plan from the device-side active
// count, so the launch needs no host sync; the grid and workspace cover the plan of max_q.
// P < 0 selects query halves instead of table pieces: each of the last R blocks becomes two items of half its
// queries (W/2 waves, the other waves exit at once) that stream the whole table — no merge, no restarted limits, and a
// half block on a CU of its own runs its waves faster than a full block.
// Piece-major order (pm) of the split blocks: split item j is piece j / R of block F + j % R, so the first round runs
// the first pieces of all blocks and a later piece of a block starts after its earlier pieces have published their
// limits (A/B builds: FWAV_TOPK_PMAJOR=0 keeps block-major order everywhere).
#ifndef FWAV_TOPK_PMAJOR
#define FWAV_TOPK_PMAJOR 1
#endif
constexpr int kOldWeight = 17, kYoungWeight = 15;  // piece_chunks: a CU's older / younger workgroup
struct TopkPlan {
  int64_t nb, F, R;
  int P, qb;
  // two-class table split (piece_chunks): pieces [0, young) weigh wa, [young, P) wb (young 0: an even split)
  int young, wa, wb;
  // one-round plans (bit 30 of P): the first item index that starts as its CU's younger workgroup (0: none); each
  // block's pieces weigh kOldWeight / kYoungWeight by their own items' side of it
  int ybound;
  bool halves, pm;
  __host__ __device__ int64_t items() const { return F + R * P; }
  // the item of table piece p of split block b
  __host__ __device__ int64_t item_of(int64_t b, int p) const { return pm ? F + (int64_t)p * R + (b - F) : F + (b - F) * P + p; }
};
// Speculative band floor of a first pass (launch_topk): *key = f2key of a filter floor f on the pass's own score scale
// (s16 or shl; 0 = no floor).  Every query's band limit starts at f, so the pass skips the rise of its limit from the
// seed; a query whose exact K-th score does not clear f + δ (δ ≥ |s16 − s32|, ≥ |shl − s32|: when it does, every exact
// top-K member had a filter score above f, and the result is exact) is listed in miss[0 .. *n_miss) for the
// floor-free second pass instead of being emitted.
// alt_rt / alt_p: the work plan when *key is 0 — the floor did not apply (fewer active queries on the device than the
// floor's minimum, or no finite pilot estimate): the launch then runs the plan of a floor-free pass (its grid covers
// both plans), not the floor's fewer, longer table pieces.
struct FloorCtl {
  const uint32_t* key;
  int32_t* miss;
  int32_t* n_miss;
  int alt_rt = -1, alt_p = 1;
};
// Whole wave: true (and the query listed for the second pass) when the floor may have cut a member of its top K:
// fewer than K band entries, or a K-th exact score (kth: key) not above f + δ.  Every domain whose filter score
// (s16, or shl in HL mode: within δ of s32) beats f was appended, and compactions drop only what the band rule drops;
// a member of the exact top K scores s32 ≥ the exact K-th ≥ the band's K-th > f + δ, so its filter score beat f.
// (Round 5 tested f + 2δ: 8,225 misses per cfg2 call instead of ≈ 2/3 of that.)
__device__ __forceinline__ bool floor_miss(uint32_t fkey, const FloorCtl& fl, int n, int K, uint64_t kth, int32_t qid) {
  if (fkey == 0u) return false;
  const bool miss = !(n >= K && key_score(kth) > key2f(fkey) + kF16Delta);
  if (miss && (threadIdx.x & 63) == 0) fl.miss[atomicAdd(fl.n_miss, 1)] = qid;
  return miss;
}
// P: table pieces per split block, −1 for query halves; bits 8 and up: TopkPlan::young (plan_young)
__host__ __device__ inline TopkPlan make_plan(int64_t n_queries, int rt, int P, int qb) {
  TopkPlan pl;
  pl.qb = qb;
  pl.nb = cdiv(n_queries > 0 ? n_queries : 0, qb);
  const bool by_item = P > 0 && ((P >> 30) & 1);
  pl.ybound = by_item ? ((P >> 8) & 0xFFF) : 0;  // bits 8–19
  pl.young = P > 0 && !by_item ? ((P >> 8) & 0xFF) : 0;
  pl.wb = P > 0 && !by_item ? ((P >> 16) & 0x1F) : 0;  // bits 16–20 / 21–25: the weights (0: the younger pair)
  pl.wa = P > 0 && !by_item ? ((P >> 21) & 0x1F) : 0;
  if (pl.wa == 0 || pl.wb == 0) {
    pl.wa = kOldWeight;
    pl.wb = kYoungWeight;
  }
  P = P > 0 ? (P & 0xFF) : P;
  pl.halves = P < 0;
  pl.P = pl.halves ? 2 : (P < 1 ? 1 : (P > kMaxPieces ? kMaxPieces : P));
  pl.R = pl.P == 1 ? 0 : (pl.nb < rt ? pl.nb : (int64_t)rt);
  pl.F = pl.nb - pl.R;
  pl.pm = FWAV_TOPK_PMAJOR && !pl.halves && pl.P > 1 && pl.R > 0;
  return pl;
}
// Chunk range [c0, c1) of table piece `piece` of `np`.  Even, unless the plan is one round of workgroups two to a CU
// (TopkPlan::young): a CU's younger workgroup loses the issue arbitration to its older one (oldest-first) and ran
// its piece 13 % longer (41,344 queries, pieces 3–5 vs 0–2: 1.95 vs 1.72 ms median, tools/topk_timeline.py TL_R,
// profiles/r06/timeline_pieces_eighth.log), so the older pieces take 17 / 16 of the mean and the younger 15 / 16.
__host__ __device__ inline void piece_chunks(const TopkPlan& pl, int64_t block, int piece, int np, int nchunks, int& c0,
                                             int& c1) {
  if (pl.ybound > 0 && np == pl.P && block >= pl.F) {
    // by each piece's own item: older (item < ybound) kOldWeight, younger kYoungWeight
    int64_t a = 0, tot = 0;
    for (int p = 0; p < np; ++p) {
      const int w = pl.item_of(block, p) < pl.ybound ? kOldWeight : kYoungWeight;
      if (p < piece) a += w;
      tot += w;
    }
    const int w = pl.item_of(block, piece) < pl.ybound ? kOldWeight : kYoungWeight;
    c0 = (int)((int64_t)nchunks * a / tot);
    c1 = (int)((int64_t)nchunks * (a + w) / tot);
    return;
  }
  if (pl.young <= 0 || pl.young >= np || np != pl.P) {
    c0 = (int)((int64_t)nchunks * piece / np);
    c1 = (int)((int64_t)nchunks * (piece + 1) / np);
    return;
  }
  auto cum = [&](int p) -> int64_t {
    return p <= pl.young ? (int64_t)p * pl.wa : (int64_t)pl.young * pl.wa + (int64_t)(p - pl.young) * pl.wb;
  };
  const int64_t tot = cum(np);
  c0 = (int)((int64_t)nchunks * cum(piece) / tot);
  c1 = (int)((int64_t)nchunks * cum(piece + 1) / tot);
}
// Query (position in the active list) of slot ql = group·32 + col of query block `block`.  INTERLEAVE: a block's
// query groups come from different regions of the list (group g of block b is query group g·nb + b), so every block
// mixes regions and block run times even out, which shortens the launch's tail.
#ifndef FWAV_TOPK_INTERLEAVE
#define FWAV_TOPK_INTERLEAVE 1
#endif
__host__ __device__ inline int64_t slot_query(int64_t block, int ql, int64_t nb, int qb) {
#if FWAV_TOPK_INTERLEAVE
  (void)qb;
  return ((int64_t)(ql >> 5) * nb + block) * 32 + (ql & 31);
#else
  return block * qb + ql;
#endif
}
// item → (block, table piece, table pieces, query half: −1 = the whole block)
__host__ __device__ inline void plan_item(const TopkPlan& pl, int64_t item, int64_t& block, int& piece, int& np,
                                          int& qhalf) {
  qhalf = -1;
  if (item < pl.F) {
    block = item; piece = 0; np = 1;
  } else {
    const int64_t j = item - pl.F;
    block = pl.F + j / pl.P;
    if (pl.halves) {
      piece = 0; np = 1; qhalf = (int)(j % 2);
    } else if (pl.pm) {
      // items past this plan (the grid covers the plan of max_q, the device count may be smaller) map to no block
      block = j < pl.R * pl.P ? pl.F + j % pl.R : pl.nb;
      piece = j < pl.R * pl.P ? (int)(j / pl.R) : 0; np = pl.P;
    } else {
      piece = (int)(j % pl.P); np = pl.P;
    }
  }
}
// Window schedule (A/B at cfg2 with 8 chains: 16 groups / 64 warm chunks 21.17 ms, 32 / 64 20.92, 16 / 32 20.85,
// 32 / 32 20.67, 32 / 16 20.70; 8 groups 20.68 vs 20.26 on a faster box)
#ifndef FWAV_TOPK_WIN
#define FWAV_TOPK_WIN 32
#endif
#ifndef FWAV_TOPK_WARM
#define FWAV_TOPK_WARM 32
#endif
constexpr int kWindowGroups = FWAV_TOPK_WIN;  // after the warm-up, fired chunks are replayed every 32 groups (128 chunks)
// fired-chunk FIFO per query group (a ring; power of two).  Measured and rejected (cfg2 A/B, identical outputs):
// replaying B ≤ 4 pending tiles per group with prefetched fragments instead of whole windows (27–32 ms vs 22.9:
// the band limit then rises too late), and windows at doubling stream lengths (28.0 vs 21.7 ms).
constexpr int kFifo = kWindowGroups * 4;
static_assert((kFifo & (kFifo - 1)) == 0, "the fired-chunk ring needs a power-of-two size");
constexpr int kWarmChunks = FWAV_TOPK_WARM;   // ... and after every group during the first 32 chunks


// Component c (a compile-time constant after unrolling) of a float4.
__device__ __forceinline__ float f4c(const float4& v, int c) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); }

// Max of the 16 scores of a lane as an int over the float bits (v_max3_i32; a float max would be preceded
// by canonicalising v_max_f32 x,x on every MFMA output).  For a threshold t >= 0, (int)x > (int)t ⟺ x > t
// for every non-NaN x (negative floats are negative ints); callers use it only in that regime.
__device__ __forceinline__ int imax16(const floatx16& a) {
  auto I = [&](int i) { return __float_as_int(a[i]); };
  auto mx = [](int x, int y) { return x > y ? x : y; };
  const int m0 = mx(mx(I(0), I(1)), I(2));
  const int m1 = mx(mx(I(3), I(4)), I(5));
  const int m2 = mx(mx(I(6), I(7)), I(8));
  const int m3 = mx(mx(I(9), I(10)), I(11));
  const int m4 = mx(mx(I(12), I(13)), I(14));
  return mx(mx(mx(m0, m1), mx(m2, m3)), mx(m4, I(15)));
}

// Does any score in this lane's imax beat the filter thf?  Exact for thf >= 0; always true for thf < 0
// (then the exact per-score test in the slow path decides).
__device__ __forceinline__ bool may_pass(int imx, float thf) {
  return thf < 0.0f || imx > __float_as_int(thf);
}

// NG = query groups of 32 per workgroup (W waves × QS sets).  Kept small: two workgroups (2 × 64 KB of chunk
// slots + this) must fit one CU's 160 KB of LDS.
template <int NG, bool STATS, bool FIFO = true, int NW = NG>
struct Topk16SmemT {
  int cnt[32 * NG];   // final pass: entries at the front of the query's buffer (its h = 0 lane's appends)
  int cnt1[32 * NG];  // ... and at the back (its h = 1 lane's)
  int ovf[32 * NG];  // band overflowed the buffer (f2key of its band limit, else 0): recompute in exact mode
  // exact mode: f2key of the largest K-th score that a domain of equal score was not kept at (0: none) — a boundary
  // tie (tie_flags bit 1) only if it is the final K-th score
  uint32_t tie[32 * NG];
  int64_t qrow[32 * NG];
  int32_t qpos[32 * NG];  // position of the slot's query in the active list (index of its shared band limit)
  uint32_t fired[FIFO ? NG : 1][kFifo];            // deferred work: ring of fired chunk entries (not in CENT)
  unsigned long long wstat[STATS ? NW : 1][kStats];  // STATS builds only (one row per wave)
};

// Streaming compaction on shl keys (no f32 rescoring, no table loads, no sort): S = the K-th largest shl in the
// buffer; every exact top-K member has shl ≥ S − 2δ' (K domains have s32 ≥ S − δ'), so keep the band shl > S − 2.5δ'
// (unsorted; the final pass rescores and sorts) and filter new domains with it.  A greedy bitwise radix select over
// the 32 key bits finds key(S) with ballots and scalar popcounts (no sort).  If the band would not leave 64 free
// slots the query is flagged (ovf) and searched again in exact mode.
// Key-buffer reads: L2-served (sc1), never a possibly stale L1 copy of a line this wave loaded before its later
// appends to it.
__device__ __forceinline__ uint64_t ld_key(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Entry e of a two-ended buffer holding n0 entries at the front and n1 at the back (append_tile).
template <int C>
__device__ __forceinline__ int two_end_slot(int e, int n0) {
  return e < n0 ? e : C - 1 - (e - n0);
}

template <int C, bool HL, class SM>
__device__ __forceinline__ void compact16_s16(uint64_t* __restrict__ kq, int n0, int n1, SM& sm, int ql, int K,
                                              unsigned long long* stats, int& m_out, float& lim_out) {
  constexpr int E = C / 64;
  const unsigned long long t_start = stats ? __builtin_amdgcn_s_memrealtime() : 0;
  const int lane = threadIdx.x & 63;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int n = min(n0 + n1, C);
  uint64_t v[E];
  uint32_t hi[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < n ? ld_key(kq + two_end_slot<C>(e, n0)) : 0ull;
    hi[j] = (uint32_t)(v[j] >> 32);  // 0 for empty slots; f2key of any real score is > 0
  }
  float lim = -INFINITY;
  if (n >= K) {
    uint32_t T = 0;
    // HL: full precision; S16: the top 20 key bits (S16 is needed only as a lower bound at ≈ 2^-11 resolution)
    for (int bit = 31; bit >= (HL ? 0 : 12); --bit) {
      const uint32_t Tc = T | (1u << bit);
      int c = 0;
#pragma unroll
      for (int j = 0; j < E; ++j) c += __popcll(__ballot(hi[j] >= Tc));
      if (c >= K) T = Tc;
    }
    lim = HL ? key2f(T) - 2.5f * kHLDelta : key2f(T) - 2.0f * kF16Delta;
  }
  // keep: every real entry with shl > lim, written densely in (j, lane) order
  int m = 0;
  int ovf = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const bool keep = hi[j] != 0u && key_score(v[j]) > lim;
    const uint64_t bm = __ballot(keep);
    const int pos = m + __popcll(bm & ((1ull << lane) - 1ull));
    if (keep && pos < C - 64) kq[pos] = v[j];
    m += __popcll(bm);
  }
  if (m > C - 64) {
    m = C - 64;
    ovf = 1;
  }
  // the flag carries the band limit at overflow (f2key, never 0): a valid lower bound on the s16 of every domain of
  // the query's exact top K, so it seeds the exact-mode relaunch
  if (lane == 0 && ovf) sm.ovf[ql] = (int)f2key(lim);
  if (lane == 0) FWAV_TRACE(sm.qrow[ql], 2u, (uint32_t)n, __float_as_uint(lim), (uint32_t)((ovf << 16) | m));
  m_out = m;
  lim_out = lim;
  if (stats) {
    stat_add(3, 1);
    stat_add(5, __builtin_amdgcn_s_memrealtime() - t_start);
  }
}

// Final pass of query ql (a whole-table item): rescore its two-ended buffer (sm.cnt entries at the front, sm.cnt1 at
// the back) in exact f32 (sgemv16), sort, emit the top K to `out`.  Whole wave.  Every per-query buffer and
// counter is owned by one wave, so no cross-wave fences are needed; the wave's own appended stores are drained
// once (vmcnt(0)), then all key loads and all row loads are issued together (two memory round trips in total).
template <int C, int E, class SM>
__device__ __forceinline__ void compact16_e(uint64_t* __restrict__ kq, SM& sm, int ql, int K,
                                            const float* __restrict__ emb, int32_t* __restrict__ out,
                                            const SgemvSplit& sp, int32_t* __restrict__ ties, int32_t qid,
                                            uint32_t fkey, const FloorCtl& fl) {
  const int lane = threadIdx.x & 63;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int n0 = sm.cnt[ql];
  const int n = min(n0 + sm.cnt1[ql], C);
  const float4* qp = reinterpret_cast<const float4*>(emb + sm.qrow[ql] * 16);
  uint64_t v[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < n ? ld_key(kq + two_end_slot<C>(e, n0)) : 0ull;
  }
  float qv[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 w = qp[i];
    qv[4 * i] = w.x; qv[4 * i + 1] = w.y; qv[4 * i + 2] = w.z; qv[4 * i + 3] = w.w;
  }
  // rescore the entries two slots at a time (8 row loads in flight per lane)
#pragma unroll
  for (int j0 = 0; j0 < E; j0 += 2) {
    float4 row[2][4];
    int32_t dd[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = j0 + jj;
      const int e = j * 64 + lane;
      dd[jj] = (j < E && e < n) ? key_idx(v[j < E ? j : 0]) : 0;
      const float4* p = reinterpret_cast<const float4*>(emb + (int64_t)dd[jj] * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) row[jj][i] = p[i];
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = j0 + jj;
      const int e = j * 64 + lane;
      if (j < E && e < n) {
        const float acc = sgemv16([&](int k) { return f4c(row[jj][k >> 2], k & 3); }, [&](int k) { return qv[k]; },
                                  sgemv_kind((uint32_t)dd[jj], sp));
        v[j] = make_key(acc, dd[jj]);
      }
    }
  }
  wave_sort_desc<E>(v);
  // exactly tied scores at the top: listed for fwav_tie_check (not for a query about to be searched again)
  uint64_t kth = 0;
#pragma unroll
  for (int j = 0; j < E; ++j)
    if (j == ((K - 1) >> 6)) kth = __shfl(v[j], (K - 1) & 63);
  // a speculative floor that may have cut a member: the query goes to the second pass, nothing is emitted here
  if (sm.ovf[ql] == 0 && floor_miss(fkey, fl, n, K, kth, qid)) return;
  const uint32_t tv = sm.tie[ql];
  const int tf = tie_flags<E>(v, n, K) | (tv != 0u && n >= K && key2f(tv) == key_score(kth) ? 2 : 0);
  // the band of the S16 / HL modes holds every domain within the band margin of the K-th score, so the K-th's whole
  // tie group; exact mode keeps only the top K (a tied domain seen later was dropped: tv)
  if (sm.ovf[ql] == 0) record_tie<E>(ties, qid, tf, v, n, K, tv == 0u);
  // Emit straight from registers (never read back what was just stored: a load issued right behind the stores
  // of the same addresses can return the old contents): the K candidate indices, −1-padded.
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    if (e < K) out[e] = e < n ? key_idx(v[j]) : -1;
  }
}

// A buffer of at most 128 entries (the usual case: the band kept by the last compaction plus the few appends after
// it) is rescored two entries per lane and sorted as 128 keys; a fuller one as C.  Same outputs either way.
template <int C, class SM>
__device__ __forceinline__ void compact16(uint64_t* __restrict__ kq, SM& sm, int ql, int K,
                                          const float* __restrict__ emb, int32_t* __restrict__ out,
                                          const SgemvSplit& sp, int32_t* __restrict__ ties, int32_t qid,
                                          uint32_t fkey, const FloorCtl& fl) {
  const int n = __builtin_amdgcn_readfirstlane(sm.cnt[ql] + sm.cnt1[ql]);
  if (FWAV_TOPK_SMALLSORT && C > 128 && n <= 128)
    compact16_e<C, 2, SM>(kq, sm, ql, K, emb, out, sp, ties, qid, fkey, fl);
  else
    compact16_e<C, C / 64, SM>(kq, sm, ql, K, emb, out, sp, ties, qid, fkey, fl);
}

// End of a table piece (split block): no rescoring and no sort here — the piece keeps the entries of its band whose
// key beats the query's shared limit (Lk, the f2key of the largest band limit any piece of the query has published;
// every exact top-K member's key is above it), written densely at the front of its buffer, and a header in the last
// slot: (overflow key << 32) | count.  k_merge_pieces rescores and sorts the union of the pieces' bands once per
// query.  A band that would not leave 64 slots is flagged as overflowed (the query goes to the exact-mode relaunch).
// The band's keys of query ql (n = its entries, 0 past them), loaded by piece_band_load — for kBandBatch queries at
// once, so that the final loop of a table piece pays one memory round trip per batch instead of two per query
// (round 6, same process, identical candidates, profiles/r06/ab_band_batch.log: 330,750 / 165,375 / 82,688 / 41,344
// queries 14.49 → 14.38 / 8.07 → 7.86 / 4.48 → 4.37 / 2.82 → 2.72 ms)
#ifndef FWAV_TOPK_BANDB
#define FWAV_TOPK_BANDB 4
#endif
constexpr int kBandBatch = FWAV_TOPK_BANDB;
template <int C, class SM>
__device__ __forceinline__ int piece_band_load(const uint64_t* __restrict__ kq, SM& sm, int ql,
                                               uint64_t (&v)[C / 64]) {
  constexpr int E = C / 64;
  const int lane = threadIdx.x & 63;
  const int n0 = sm.cnt[ql];
  const int n = min(n0 + sm.cnt1[ql], C);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < n ? ld_key(kq + two_end_slot<C>(e, n0)) : 0ull;
  }
  return n;
}
// sh0: the query's shared limit read with its keys (any earlier value is a valid, smaller lower bound)
template <int C, bool HL, class SM>
__device__ __forceinline__ void piece_band(uint64_t* __restrict__ kq, SM& sm, int ql, int K,
                                           uint32_t* __restrict__ share_q, uint64_t (&v)[C / 64], int n,
                                           uint32_t sh0) {
  constexpr int E = C / 64;
  const int lane = threadIdx.x & 63;
  // the piece's own limit now (a last compaction's select over its whole buffer), published before the filter so
  // that the pieces still streaming and k_merge_pieces see it
  uint32_t Lk = 0u;
  if (n >= K) {
    uint32_t T = 0;
    for (int bit = 31; bit >= (HL ? 0 : 12); --bit) {
      const uint32_t Tc = T | (1u << bit);
      int c = 0;
#pragma unroll
      for (int j = 0; j < E; ++j) c += __popcll(__ballot((uint32_t)(v[j] >> 32) >= Tc));
      if (c >= K) T = Tc;
    }
    Lk = f2key(HL ? key2f(T) - 2.5f * kHLDelta : key2f(T) - 2.0f * kF16Delta);
    if (lane == 0) atomicMax(share_q, Lk);
  }
  Lk = max(Lk, sh0);
  int m = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const bool keep = v[j] != 0ull && (uint32_t)(v[j] >> 32) > Lk;
    const uint64_t bm = __ballot(keep);
    const int pos = m + __popcll(bm & ((1ull << lane) - 1ull));
    if (keep && pos < C - 64) kq[pos] = v[j];
    m += __popcll(bm);
  }
  uint32_t ovf = (uint32_t)sm.ovf[ql];
  if (m > C - 64) {
    m = C - 64;
    if (ovf == 0u) ovf = Lk != 0u ? Lk : 1u;  // any nonzero flag; the limit (if any) is a valid relaunch seed
  }
  if (lane == 0) kq[C - 1] = ((uint64_t)ovf << 32) | (uint32_t)m;
}

// Integer filter threshold for the fold-max test: (int)x > thi ⟺ x > thf for non-NaN x when thf >= 0;
// for thf < 0 every tile goes to the exact per-score test.
__device__ __forceinline__ int int_threshold(float thf) {
  return thf < 0.0f ? (int)0x80000000 : __float_as_int(thf);
}

__device__ __forceinline__ int fold16(int r, const floatx16& a) {
  auto I = [&](int i) { return __float_as_int(a[i]); };
  auto m3 = [](int x, int y, int z) { return max(max(x, y), z); };
  r = m3(r, I(0), I(1));
  r = m3(r, I(2), I(3));
  r = m3(r, I(4), I(5));
  r = m3(r, I(6), I(7));
  r = m3(r, I(8), I(9));
  r = m3(r, I(10), I(11));
  r = m3(r, I(12), I(13));
  return m3(r, I(14), I(15));
}

// One recomputed tile of a replay (acc = the tile's fp16 MFMA scores, domains dt .. dt+31): append the
// survivors (s16 keys) to the wave-owned global key buffers — one LDS atomic per lane reserves the slots,
// the stores are fire-and-forget — and compact a buffer inline only when it is about to overflow.
// Exact-mode compaction (the overflow relaunch, EX): the buffer holds exact f32 keys, so it keeps exactly its top K
// (a sort of the ≤ C keys; entries are distinct (score, index) keys, so no tie group can overflow), written sorted at
// the front.  New domains can only matter with s32 > S32_K (a later domain of equal score has a larger index), i.e.
// s16 > S32_K − δ: that is the returned filter limit.
template <int C>
__device__ __forceinline__ void compact_exact(uint64_t* __restrict__ kq, int n0, int n1, int K, int& m_out,
                                              float& lim_out, uint64_t& kth_out, uint32_t* __restrict__ tie_slot) {
  constexpr int E = C / 64;
  const int lane = threadIdx.x & 63;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int n = min(n0 + n1, C);
  uint64_t v[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < n ? ld_key(kq + two_end_slot<C>(e, n0)) : 0ull;
  }
  wave_sort_desc<E>(v);
  const int kl = (K - 1) & 63, kj = (K - 1) >> 6;
  uint64_t kth = 0;
#pragma unroll
  for (int j = 0; j < E; ++j)
    if (j == kj) kth = __shfl(v[j], kl);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    if (e < K && e < n) kq[e] = v[j];
  }
  // a dropped (K+1)-th entry with the K-th's score: the set among the equal scores is numpy's choice
  const int kl1 = K & 63, kj1 = K >> 6;
  uint32_t kh = 0u, k1h = 0u;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int hj = (int)(uint32_t)(v[j] >> 32);
    const int a = __shfl(hj, kl), b = __shfl(hj, kl1);
    if (j == kj) kh = (uint32_t)a;
    if (j == kj1) k1h = (uint32_t)b;
  }
  if (lane == 0 && n > K && key2f(k1h) == key2f(kh)) atomicMax(tie_slot, kh);
  m_out = n < K ? n : K;
  lim_out = n >= K ? key_score(kth) - kF16Delta : -INFINITY;
  kth_out = n >= K ? kth : 0ull;
}

template <int C, bool STATS, class SM, int MODE>
__device__ __forceinline__ float append_tile(const floatx16& acc, float thf, int& qcnt, int& kept, int64_t dt, int64_t nd,
                                             uint64_t* __restrict__ gkeys, SM& sm, int qg, int K, int upd,
                                             unsigned long long* stats, const SgemvSplit& sp,
                                             const float* __restrict__ emb = nullptr,
                                             const float* qv = nullptr, uint64_t* kthp = nullptr,
                                             uint32_t* __restrict__ share = nullptr) {
  constexpr bool EX = MODE == kModeEX;
  const int lane = threadIdx.x & 63;
  const int col = lane & 31;
  const int h = lane >> 5;
  const int ql = qg * 32 + col;  // qg: the wave-uniform query group (32 queries) of this tile
  if (__ballot(fold16((int)0x80000000, acc) > int_threshold(thf)) == 0ull) return thf;
  if (STATS) stat_add(1, 1);
  const unsigned long long t_a0 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
  // Two-ended buffer: the h = 0 lane of a query appends at the front (slots 0, 1, …), the h = 1 lane at the back
  // (C−1, C−2, …), so a lane stores each survivor at its own running slot as soon as its compare passes: one
  // compare, the key and one exec-masked store per row, and no per-tile exchange of counts before the stores.
  // Byte offsets from the item's key region stay 32-bit (≤ 32·NG·C·8 B).
  const uint32_t nd0 = ~(uint32_t)(dt + 4 * h);  // key low word of row r: ~(domain index) = nd0 − offset(r)
  floatx16 a = acc;
  if (dt + 32 > nd) {  // wave-uniform: the table's last tile; rows past the end never pass
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (dt + 4 * h + (r & 3) + 8 * (r >> 2) >= nd) a[r] = -INFINITY;
  }
  const int before = qcnt;
  int slot = h ? C - 1 - qcnt : qcnt;
  const int step = h ? -1 : 1;
  char* kbase = reinterpret_cast<char*>(gkeys);
  if constexpr (EX) {
    // EX: exact f32 keys (sgemv16, the final pass's score) of the rows whose s16 passes the filter — typically one
    // or none per lane and tile, so they are computed on the VALU from the rows' f32 embeddings, two rows per lane
    // and memory round trip, in increasing row order (the order of the stores below)
    uint32_t pm = 0u;
#pragma unroll
    for (int r = 0; r < 16; ++r) pm |= (a[r] > thf ? 1u : 0u) << r;
    while (__ballot(pm != 0u) != 0ull) {
      int rr[2];
      bool on[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        on[u] = pm != 0u;
        rr[u] = on[u] ? __builtin_ctz(pm) : 0;
        if (on[u]) pm &= pm - 1u;
      }
      float4 row[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t d = dt + 4 * h + (rr[u] & 3) + 8 * (rr[u] >> 2);
        const float4* p = reinterpret_cast<const float4*>(emb + (on[u] ? d : dt) * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) row[u][i] = p[i];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (on[u]) {
          const int r = rr[u];
          FWAV_TRACE(sm.qrow[ql], 1u, (uint32_t)dt, (uint32_t)((h << 16) | r), (uint32_t)slot);
          const int64_t dr = dt + 4 * h + (r & 3) + 8 * (r >> 2);
          const float sc = sgemv16([&](int k) { return f4c(row[u][k >> 2], k & 3); }, [&](int k) { return qv[k]; },
                                   sgemv_kind((uint32_t)dr, sp));
          const uint32_t uu = __float_as_uint(sc);
          const uint32_t key = uu ^ ((uint32_t)((int32_t)uu >> 31) | 0x80000000u);
          const uint64_t k64 = ((uint64_t)key << 32) | (uint64_t)(nd0 - (uint32_t)((r & 3) + 8 * (r >> 2)));
          // a domain that does not beat the query's current K-th exact key can never enter its top K (groups of
          // equal scores — repeated or silent tiles — are decided here, without stores or compactions)
          if (k64 > *kthp) {
            *reinterpret_cast<uint64_t*>(kbase + (uint32_t)((ql * C + slot) * 8)) = k64;
            slot += step;
          } else if (key_score(k64) == key_score(*kthp)) {
            // equal to the K-th exact score, later in index order: numpy decides whether it is in
            atomicMax(&sm.tie[ql], (uint32_t)(*kthp >> 32));
          }
        }
      }
    }
  } else if constexpr (FWAV_TOPK_APPOFF) {
    // a running byte offset (one add per stored row, the store's own VGPR offset) and the key's low word as one
    // subtraction from an opaque nd0 (the compiler otherwise derives it from dt's known low bits in two ops)
    uint32_t off = (uint32_t)((ql * C + slot) * 8);
    const uint32_t dstep = h ? (uint32_t)-8 : 8u;
    uint32_t nd0o = nd0;
    asm volatile("" : "+v"(nd0o));
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (a[r] > thf) {
        FWAV_TRACE(sm.qrow[ql], 1u, (uint32_t)dt, (uint32_t)((h << 16) | r), (uint32_t)(off / 8 - ql * C));
        const uint32_t u = __float_as_uint(a[r]);
        const uint32_t key = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
        const uint64_t k64 = ((uint64_t)key << 32) | (uint64_t)(nd0o - (uint32_t)((r & 3) + 8 * (r >> 2)));
        *reinterpret_cast<uint64_t*>(kbase + off) = k64;
        off += dstep;
      }
    }
    slot = (int)(off / 8) - ql * C;
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (a[r] > thf) {
        FWAV_TRACE(sm.qrow[ql], 1u, (uint32_t)dt, (uint32_t)((h << 16) | r), (uint32_t)slot);
        // f2key of the shl score, branch-free: negative → ~u, else u | sign
        const uint32_t u = __float_as_uint(a[r]);
        const uint32_t key = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
        const uint64_t k64 = ((uint64_t)key << 32) | (uint64_t)(nd0 - (uint32_t)((r & 3) + 8 * (r >> 2)));
        *reinterpret_cast<uint64_t*>(kbase + (uint32_t)((ql * C + slot) * 8)) = k64;
        slot += step;
      }
    }
  }
  qcnt = h ? C - 1 - slot : slot;  // this lane's entries; ≤ C in total: see the compaction trigger below
  // the query's total (both lanes) in every lane, by one cross-half swap
  const auto sw = __builtin_amdgcn_permlane32_swap((uint32_t)qcnt, (uint32_t)qcnt, false, false);
  const int total = (int)(sw[0] + sw[1]);
  if (STATS) {
    stat_add(2, __ockl_wfred_add_u32((uint32_t)(qcnt - before)));
    stat_add(10, __builtin_amdgcn_s_memrealtime() - t_a0);
  }
  // compact when fewer than 32 free slots remain (a tile adds ≤ 16 per lane, ≤ 32 per query) — or, to raise the band
  // limit sooner, once the buffer passes kTrig and has grown by kGrow since its last compaction
  uint64_t need = __ballot(lane < 32 && (total > C - 32 || (total > kTrig && total >= kept + kGrow) ||
                                         (EX && FWAV_TOPK_EXGROW > 0 && total >= kept + FWAV_TOPK_EXGROW)));
  if ((FWAV_TOPK_PRIO & 2) && need != 0ull) __builtin_amdgcn_s_setprio(2);  // the barrier's critical path
  while (need != 0ull) {
    const int l = __builtin_ctzll(need);
    need &= need - 1;
    int m;
    float lim;
    uint64_t kth_l = 0;
    if constexpr (EX)
      compact_exact<C>(gkeys + (size_t)(qg * 32 + l) * C, __builtin_amdgcn_readlane(qcnt, l),
                       __builtin_amdgcn_readlane(qcnt, l + 32), K, m, lim, kth_l, &sm.tie[qg * 32 + l]);
    else
      compact16_s16<C, MODE == kModeHL>(gkeys + (size_t)(qg * 32 + l) * C, __builtin_amdgcn_readlane(qcnt, l),
                       __builtin_amdgcn_readlane(qcnt, l + 32), sm, qg * 32 + l, K, STATS ? stats : nullptr, m, lim);
    if (col == l) {
      qcnt = h ? 0 : m;  // the kept band is written densely at the front
      kept = m;
      if (upd) thf = fmaxf(thf, lim);  // the seed may be above a buffer's own limit
      // a table piece publishes its limit to the query's other pieces (shared_limit below)
      if (share != nullptr && h == 0 && lim > -INFINITY) atomicMax(share + sm.qpos[qg * 32 + l], f2key(lim));
      // a query whose band overflowed is searched again in exact mode: stop appending for it here
      if (!EX && sm.ovf[qg * 32 + l]) thf = INFINITY;
      if (EX) *kthp = kth_l;
    }
  }
  if (FWAV_TOPK_PRIO & 2) {  // back to the wave's base priority
    if ((FWAV_TOPK_PRIO & 1) && (threadIdx.x >> 6) >= (blockDim.x >> 7)) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
  return thf;
}

// Window end: replay what this wave recorded.  An entry is (chunk << 8 | chain mask); with 4 chains chain j covers tiles j
// and j + 4.  The recorded tiles are walked with a wave-uniform cursor in batches of kReplayBatch: all of a
// batch's fragment loads (from the fp16 table, L2/MALL-resident) are issued together, so a window costs
// ~one memory round trip per batch instead of one per chunk, and tiles of quiet chains are not recomputed.
#ifndef FWAV_TOPK_RB
#define FWAV_TOPK_RB 8
#endif
constexpr int kReplayBatch = FWAV_TOPK_RB;
// Cursor over a query group's pending fired tiles: FIFO entries [head, tail) of `fired` (a ring), the entry being
// expanded (chunk cc, tiles rem).  Wave-uniform.
struct ReplayCursor {
  int head;
  int64_t cc;
  uint32_t rem;
};
// Fold chains per 256-domain chunk: tile t folds into chain t % kChains; a fired chunk is recorded as
// (chunk << 8 | chain mask) and its replay recomputes the tiles of the firing chains (8 / kChains tiles per chain).
#ifndef FWAV_TOPK_CHAINS
#define FWAV_TOPK_CHAINS 8
#endif
constexpr int kChains = FWAV_TOPK_CHAINS;
static_assert(kChains == 4 || kChains == 8, "4 or 8 chains per chunk");
// Next pending tile (its first domain), or −1.
__device__ __forceinline__ int64_t next_tile(ReplayCursor& cur, int tail, const uint32_t* fired) {
  while (cur.rem == 0u && cur.head < tail) {
    const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane(fired[cur.head++ & (kFifo - 1)]);
    cur.cc = e >> 8;
    cur.rem = kChains == 8 ? (e & 255u) : ((e & 15u) | ((e & 15u) << 4));
  }
  if (cur.rem == 0u) return -1;
  const int t = __builtin_ctz(cur.rem);
  cur.rem &= cur.rem - 1;
  return cur.cc * kChunk + t * 32;
}
__device__ __forceinline__ half8 tile_fragment(const _Float16* __restrict__ emb16, int64_t dt, int h, int col) {
  const int64_t c = dt / kChunk, t = (dt % kChunk) / 32;
  return *reinterpret_cast<const half8*>(emb16 + ((c * 2 + h) * kChunk + col) * 8 + t * 256);
}

template <int C, bool STATS, class SM, int MODE>
__device__ __forceinline__ float replay_window(const _Float16* __restrict__ emb16, const _Float16* __restrict__ emb16lo,
                                               half8 b, half8 bl, float thf, int& qcnt,
                                               int& kept, ReplayCursor& cur, int tail, int64_t nd, uint64_t* __restrict__ gkeys,
                                               SM& sm, int qg, int K, int upd, unsigned long long* stats,
                                               const SgemvSplit& sp, const float* __restrict__ emb = nullptr,
                                               const float* qv = nullptr, uint64_t* kthp = nullptr,
                                               uint32_t* __restrict__ share = nullptr) {
  constexpr bool HL = MODE == kModeHL;
  const int lane = threadIdx.x & 63;
  const int col = lane & 31;
  const int h = lane >> 5;
  if (STATS) stat_add(0, tail - cur.head);
  while (true) {
    int64_t ct[kReplayBatch];  // tile start domain, −1 = none
#pragma unroll
    for (int u = 0; u < kReplayBatch; ++u) ct[u] = next_tile(cur, tail, sm.fired[qg]);
    if (ct[0] < 0) break;
    half8 af[kReplayBatch], afl[HL ? kReplayBatch : 1];
#pragma unroll
    for (int u = 0; u < kReplayBatch; ++u)  // unconditional loads (no wait on the spot)
      af[u] = tile_fragment(emb16, ct[u] < 0 ? ct[0] : ct[u], h, col);
    if constexpr (HL) {  // the low parts of the fired tiles' domains (shl)
#pragma unroll
      for (int u = 0; u < kReplayBatch; ++u) afl[u] = tile_fragment(emb16lo, ct[u] < 0 ? ct[0] : ct[u], h, col);
    }
    if (STATS) {  // time the fragment round trip (timing build only: forces the wait here)
      const unsigned long long t_l0 = __builtin_amdgcn_s_memrealtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stat_add(11, __builtin_amdgcn_s_memrealtime() - t_l0);
    }
#pragma unroll
    for (int u = 0; u < kReplayBatch; ++u) {
      if (ct[u] < 0) break;
      floatx16 acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[u], b, floatx16{}, 0, 0, 0);
      if constexpr (HL) {
        // The limit may have risen since the tile fired: refine (shl = s16 + d_hi·q_lo + d_lo·q_hi, f32
        // accumulation) only if some s16 of the tile can still pass (s16 > lim − δ − 2δ')
#if FWAV_TOPK_HLPRE
        if (__ballot(fold16((int)0x80000000, acc) > int_threshold(thf - kStreamMargin)) == 0ull) continue;
#endif
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[u], bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(afl[u], b, acc, 0, 0, 0);
      }
      thf = append_tile<C, STATS, SM, MODE>(acc, thf, qcnt, kept, ct[u], nd, gkeys, sm, qg, K, upd, stats, sp, emb,
                                          qv, kthp, share);
    }
    if (ct[kReplayBatch - 1] < 0) break;
  }
  return thf;
}

// Seed of a query's band limit before the stream: the K-th largest s16 among the domains of its own window
// [qrow − 64, qrow + 64).  Consecutive domains are windows 2 samples apart, so this window holds close matches and
// its K-th score is far above what the first streamed chunks give; a valid start for the rising limit (K domains
// have s16 ≥ T, so s32 ≥ T − δ: every exact top-K member has shl > T − δ − 2δ', and s16 > T − 2δ for the exact
// mode's s16-scale limit), it removes the first compactions and ≈ 1/4 of the appends.  The wave's window tiles (6 × 32 domains from a tile-aligned base, read from L2/MALL) are scored with
// the stream's own MFMA, recomputed per radix step (a greedy bitwise select over the non-negative keys, ballots
// free: each query's two lanes combine their counts by one shuffle).  Returns −∞ when fewer than K window scores
// are ≥ 0.
#ifndef FWAV_TOPK_SEEDHALF
#define FWAV_TOPK_SEEDHALF 64
#endif
constexpr int kSeedHalf = FWAV_TOPK_SEEDHALF;
constexpr int kSeedTiles = (2 * kSeedHalf + 62) / 32 + 1;  // the wave's 32 windows from a tile-aligned base
template <int MODE>
__device__ __forceinline__ float seed_limit(const _Float16* __restrict__ emb16, int64_t nd, half8 b, int64_t qrow,
                                            int64_t wbase, int K) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 31;
  const int h = lane >> 5;
  const half8* afp[kSeedTiles];
  uint32_t wm[kSeedTiles];  // per tile: the lane's 16 outputs that are in its query's window (and the table)
#pragma unroll
  for (int t = 0; t < kSeedTiles; ++t) {
    const int64_t dt = wbase + 32 * t;
    const bool ok = dt >= 0 && dt < nd;
    const int64_t c = ok ? dt / kChunk : 0, tt = ok ? (dt % kChunk) / 32 : 0;
    afp[t] = reinterpret_cast<const half8*>(emb16 + ((c * 2 + h) * kChunk + col) * 8 + tt * 256);
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t d = dt + 4 * h + (r & 3) + 8 * (r >> 2);
      m |= (ok && d < nd && d >= qrow - kSeedHalf && d < qrow + kSeedHalf) ? (1u << r) : 0u;
    }
    wm[t] = m;
  }
  auto count_ge = [&](float thr) {
    int c = 0;
    half8 af[kSeedTiles];  // re-read per step (L2): keeps the prologue's register peak below the stream's
#pragma unroll
    for (int t = 0; t < kSeedTiles; ++t) af[t] = *afp[t];
#pragma unroll
    for (int t = 0; t < kSeedTiles; ++t) {
      const floatx16 acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[t], b, floatx16{}, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) c += ((wm[t] >> r) & 1u) && acc[r] >= thr ? 1 : 0;
    }
    return c + __shfl_xor(c, 32);
  };
  // No per-lane branches here: the MFMAs and shuffles need the whole wave active (a per-lane early return let the
  // compiler run the select loop under a partial EXEC, which corrupts both)
  const bool ok = count_ge(0.0f) >= K;
  uint32_t T = 0x80000000u;  // key of +0.0
  for (int bit = 30; bit >= 12; --bit) {
    const uint32_t Tc = T | (1u << bit);
    const int c = count_ge(key2f(Tc));
    T = c >= K ? Tc : T;
  }
  return ok ? (MODE == kModeHL ? key2f(T) - kF16Delta - 2.0f * kHLDelta : key2f(T) - 2.0f * kF16Delta) : -INFINITY;
}

// NC chunks from the LDS slots as a single unrolled software pipeline over their 8·NC tiles: fragments are read
// 3 tiles ahead and each MFMA is issued one tile before its fold, across chunk boundaries (a per-chunk loop waits
// on its first ds_reads and on its last MFMA at every chunk — half the wave time was parked in those waits).
// With QS query sets per wave each fragment read feeds QS MFMAs (set s: B operand b[s]).  Tile t of a chunk
// folds into max chain t % kChains of its set (8 chains: one per tile); at each chunk end one ballot tests the
// chains' maximum, and a firing chunk is recorded in its set's row as (chunk << 8 | chain mask).
// MODE (timing ablations, STATS builds only): 1 = fold but no ballots/records, 2 = MFMA with a 2-output fold
// (one v_max3 per tile instead of 8; results kept alive through `sink`).
template <int NC, int QS, int MODE = 0>
__device__ __forceinline__ void stream_group(const _Float16* __restrict__ lda0, const half8 (&b)[QS],
                                             const int (&thi)[QS], int cbase, uint32_t (*fired)[kFifo],
                                             int (&nfired)[QS], int lane, int* sink = nullptr) {
  constexpr int NT = 8 * NC;
  constexpr int kChunkHalfs = 512 * 8;  // one 8 KB chunk slot
  auto chunk_of = [](int i) { return i >> 3; };
  auto rd = [&](int i) {
    return *reinterpret_cast<const half8*>(lda0 + chunk_of(i) * kChunkHalfs + (i & 7) * 256);
  };
  half8 a[NT];
  floatx16 acc[NT][QS];
#pragma unroll
  for (int i = 0; i < 3 && i < NT; ++i) a[i] = rd(i);
#pragma unroll
  for (int s = 0; s < QS; ++s) acc[0][s] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[s], floatx16{}, 0, 0, 0);
  int r[QS][kChains];
#pragma unroll
  for (int s = 0; s < QS; ++s)
#pragma unroll
    for (int c = 0; c < kChains; ++c) r[s][c] = (int)0x80000000;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i + 3 < NT) a[i + 3] = rd(i + 3);
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      if (i + 1 < NT) acc[i + 1][s] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i + 1], b[s], floatx16{}, 0, 0, 0);
      constexpr int cm = kChains - 1;
      if (MODE & 2)
        r[s][i & cm] = max(max(r[s][i & cm], __float_as_int(acc[i][s][0])), __float_as_int(acc[i][s][15]));
      else
        r[s][i & cm] = fold16(r[s][i & cm], acc[i][s]);
    }
    if (MODE != 0) {
      if (i == NT - 1) {
#pragma unroll
        for (int s = 0; s < QS; ++s)
#pragma unroll
          for (int c = 0; c < kChains; ++c) *sink ^= r[s][c];
      }
      continue;
    }
    if ((i & 7) == 7) {
#pragma unroll
      for (int s = 0; s < QS; ++s) {
        const int t = thi[s];
        // one test of the max of the chains first: most chunks fire none
        int rm = r[s][0];
#pragma unroll
        for (int c = 1; c < kChains; ++c) rm = max(rm, r[s][c]);
        if (__ballot(rm > t) != 0ull) {
          uint32_t mk = 0u;
#pragma unroll
          for (int c = 0; c < kChains; ++c) mk |= __ballot(r[s][c] > t) != 0ull ? (1u << c) : 0u;
          if (lane == 0) fired[s][nfired[s] & (kFifo - 1)] = ((uint32_t)(cbase + chunk_of(i)) << 8) | mk;
          ++nfired[s];
        }
#pragma unroll
        for (int c = 0; c < kChains; ++c) r[s][c] = (int)0x80000000;
      }
    }
  }
}

__device__ __forceinline__ int ctz_mask(uint32_t x) { return __builtin_ctz(x); }
__device__ __forceinline__ int ctz_mask(uint64_t x) { return __builtin_ctzll(x); }
// f(std::integral_constant<int, I>) for I = 0 .. N−1: loops over per-set register arrays with compile-time indices
// where the body is too large for the unroller
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// ---- Centroid pre-filter (CENT geometry): QS query sets of 32 per wave, one centroid per QS consecutive queries.
// Centroid column j of a wave belongs to set j % QS and stands for its members, the columns QS·(j / QS) + k (k < QS)
// of that set — QS consecutive positions of the active list, i.e. (unpruned) ranges a few samples apart, whose
// embeddings lie close together.  With c the centroid's fp16 vector and ρ_h = max over members |q_hi,h − c_h| per
// head h (the tonal and transient halves of the embedding, each of norm ≤ 1 in the table), every member's fp16 score
// obeys s16(q, d) = (q_hi − c)·d_hi + c·d_hi ≤ s16(c, d) + (ρ_0 + ρ_1)(1 + 2⁻⁹) + 1e-5 (d_hi's heads have norm
// ≤ 1 + 2⁻¹¹; both MFMA accumulations ≤ 16 roundings of ≤ 2).  So one MFMA of the 32 centroids per 32-domain tile
// — a 4:1 (QS = 4) reduction of the fold, the stream's issue bound — decides which sets need their own MFMA and fold
// for that tile: a set is scored only where some centroid of it reaches the smallest member threshold minus the
// centroid's slack.  Exact: a tile skipped for a set holds no domain above any member's threshold.
constexpr int kCentBatch = FWAV_TOPK_CB;
template <int QS>
__device__ __forceinline__ uint64_t cent_set_mask(int s) {
  static_assert(QS == 2 || QS == 4 || QS == 8, "centroid sets: 2, 4 or 8 query sets per wave");
  constexpr uint64_t m = QS == 2 ? 0x5555555555555555ull : (QS == 4 ? 0x1111111111111111ull : 0x0101010101010101ull);
  return m << s;
}
// The lane's centroid (column col = lane & 31, half h = lane >> 5): the fp16 mean of its members' query fragments and
// the slack (ρ_0 + ρ_1)(1 + 2⁻⁹) + 1e-5 added to every member bound.  `qrow_of(k)` = member k's table row, or −1.
template <int QS, class RowOf>
__device__ __forceinline__ void centroid_setup(const _Float16* __restrict__ emb16, RowOf qrow_of, half8& bc,
                                               float& slack) {
  typedef float floatx8 __attribute__((ext_vector_type(8)));
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  auto frag = [&](int64_t r) {  // the member's fp16 high parts of head h (re-read from L2 in the second pass)
    return *reinterpret_cast<const half8*>(emb16 + (((r >> 8) * 2 + h) * 256 + (r & 255)) * 8);
  };
  floatx8 sum = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int nv = 0;
#pragma unroll
  for (int k = 0; k < QS; ++k) {
    const int64_t r = qrow_of(k);
    if (r >= 0) {
      const half8 m = frag(r);
      ++nv;
#pragma unroll
      for (int i = 0; i < 8; ++i) sum[i] += (float)m[i];
    }
  }
  half8 c;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = (_Float16)(nv > 0 ? sum[i] / (float)nv : 0.0f);
  float rho = 0.0f;
#pragma unroll
  for (int k = 0; k < QS; ++k) {
    const int64_t r = qrow_of(k);
    if (r >= 0) {
      const half8 m = frag(r);
      float d2 = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = (float)m[i] - (float)c[i];  // exact: a difference of two fp16 values
        d2 += d * d;
      }
      rho = fmaxf(rho, __builtin_sqrtf(d2));
    }
  }
  rho += __shfl_xor(rho, 32);  // both heads
  bc = c;
  slack = rho * (1.0f + 0x1p-9f) + 1e-5f;
}
// The lane's centroid filter threshold: the smallest stream threshold (float) of its members minus the slack
// (+∞ when no member takes appends; −∞ members make the centroid fire on every tile).
template <int QS>
__device__ __forceinline__ int centroid_threshold(const float (&tv)[QS], float slack) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 31;
  const int sj = col % QS, base = (lane & 32) + QS * (col / QS);
  float mn = INFINITY;
#pragma unroll
  for (int k = 0; k < QS; ++k) {
    float v = INFINITY;
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      const float x = __shfl(tv[s], base + k);
      v = s == sj ? x : v;
    }
    mn = fminf(mn, v);
  }
  return int_threshold(mn - slack);
}
// Level 1 of the centroid pre-filter over one group of NC chunks: the 32 centroids scored against every tile (the
// stream's software pipeline: fragments 3 tiles ahead, MFMAs one tile ahead); pend[s] bit i marks tile i of the group
// where some centroid of set s reaches its threshold.  The marked (tile, set) pairs are then scored with the set's
// own queries and their survivors appended at once (k_sim_topk_f16, CENT): no fired-chunk ring, no replay.
template <int NC, int QS>
__device__ __forceinline__ void cent_level1(const _Float16* __restrict__ lda0, half8 bc, int thc,
                                            uint64_t (&pend)[QS]) {
  constexpr int NT = 8 * NC;
  static_assert(NT <= 64, "tile masks are 64-bit");
  constexpr int kChunkHalfs = 512 * 8;
  auto rd = [&](int i) {
    return *reinterpret_cast<const half8*>(lda0 + (i >> 3) * kChunkHalfs + (i & 7) * 256);
  };
#pragma unroll
  for (int s = 0; s < QS; ++s) pend[s] = 0ull;
  half8 a[NT];
  floatx16 acc[NT];
#pragma unroll
  for (int i = 0; i < 3 && i < NT; ++i) a[i] = rd(i);
  acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bc, floatx16{}, 0, 0, 0);
if constexpr (FWAV_TOPK_CVACC && NT <= 32) {
  // the lane's firing tiles accumulated in a VGPR (bits = 2·bits + fired, one v_addc per tile: tile i at bit NT−1−i),
  // then OR-reduced over the lanes of each set once per group — instead of 4 scalar ops per set and tile
  uint32_t bits = 0u;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i + 3 < NT) a[i + 3] = rd(i + 3);
    if (i + 1 < NT) acc[i + 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i + 1], bc, floatx16{}, 0, 0, 0);
    const uint64_t m = __ballot(fold16((int)0x80000000, acc[i]) > thc);
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(bits), "=s"(co) : "v"(bits), "s"(m));
  }
#pragma unroll
  for (int off = QS; off < 64; off <<= 1) bits |= (uint32_t)__shfl_xor((int)bits, off);
#pragma unroll
  for (int s = 0; s < QS; ++s)
    pend[s] = (uint64_t)(__builtin_bitreverse32((uint32_t)__builtin_amdgcn_readlane((int)bits, s)) >> (32 - NT));
} else {
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i + 3 < NT) a[i + 3] = rd(i + 3);
    if (i + 1 < NT) acc[i + 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i + 1], bc, floatx16{}, 0, 0, 0);
    const uint64_t m = __ballot(fold16((int)0x80000000, acc[i]) > thc);
#pragma unroll
    for (int s = 0; s < QS; ++s)
      if (m & cent_set_mask<QS>(s)) pend[s] |= 1ull << i;
  }
}
}

template <int C, bool STATS, int MODE, int W = k16Waves, int G = kGroup, int QS = k16Sets, bool CENT = false>
__global__ __launch_bounds__(64 * W, MODE == kModeEX ? FWAV_TOPK_EXWPE : (CENT ? FWAV_TOPK_CWPE : FWAV_TOPK_WPE)) void k_sim_topk_f16(const _Float16* __restrict__ emb16,
                                                                const float* __restrict__ emb, int64_t nd,
                                                                const int32_t* __restrict__ active,
                                                                const int32_t* __restrict__ n_active_p,
                                                                int64_t q_offset, int K, int32_t* __restrict__ cand,
                                                                uint64_t* __restrict__ gkeys_all,
                                                                int32_t* __restrict__ ovf_list,
                                                                int32_t* __restrict__ n_ovf,
                                                                uint32_t* __restrict__ share_lim,
                                                                const uint32_t* __restrict__ seeds_in,
                                                                float seed_shift, int plan_rt,
                                                                int plan_p, int dbg, unsigned long long* gstats,
                                                                SgemvSplit sp, int32_t* __restrict__ ties,
                                                                FloorCtl fl) {
  constexpr bool EX = MODE == kModeEX;
  constexpr bool HL = MODE == kModeHL;
  constexpr int NG = W * QS;  // query groups of 32 per workgroup; wave w owns groups w·QS .. w·QS + QS − 1
  constexpr bool ABL = STATS || FWAV_TOPK_ABL != 0;  // ablation bits honoured
  // 2 × G chunk slots: group g is consumed from one half while group g+1 streams into the other.
  // ALL of the kernel's LDS is one __shared__ object: beside a second one, hipcc waits vmcnt(0) for the in-flight
  // LDS DMA before the first ds_read of every chunk (cdna_hip_programming.md, "three .s-level traps" (a)).
  // (Measured and rejected, tools/experiments/ring_and_knobs.patch: a ring of NB slots with LDS ready/free counters
  // instead of the group barrier)
  constexpr int NB = 2;
  struct Lds {
    u32x4 slots[NB * G][512];
    Topk16SmemT<NG, STATS, !CENT, W> sm;
  };
  __shared__ __attribute__((aligned(16))) Lds lds_all;
  u32x4(*slots)[512] = lds_all.slots;
  Topk16SmemT<NG, STATS, !CENT, W>& sm = lds_all.sm;

  const int n_active = *n_active_p;
  constexpr int QB = 32 * NG;  // queries per block
  // a first pass's speculative floor (FloorCtl): every band limit starts there; none applied → the floor-free plan
  const uint32_t fkey = (!EX && fl.key != nullptr) ? __builtin_amdgcn_readfirstlane(*fl.key) : 0u;
  const bool alt = fl.key != nullptr && fkey == 0u;
  const TopkPlan plan = make_plan(n_active, alt ? fl.alt_rt : plan_rt, alt ? fl.alt_p : plan_p, QB);
  int64_t block;
  int piece, npieces, qhalf;
  plan_item(plan, blockIdx.x, block, piece, npieces, qhalf);
  if (block >= plan.nb) return;
  const int Wact = qhalf < 0 ? W : W / 2;  // waves with queries
  if ((int)(threadIdx.x >> 6) >= Wact) return;
  const int qslot0 = qhalf > 0 ? (W / 2) * QS * 32 : 0;  // the second half block's first query slot
  uint64_t* gkeys = gkeys_all + (size_t)blockIdx.x * 32 * NG * C;  // this item's key-buffer region
  const unsigned long long t_kernel = STATS ? __builtin_amdgcn_s_memrealtime() : 0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform: scalar control flow below
  unsigned long long* stats = nullptr;
  if (STATS) {
    if (lane < kStats) sm.wstat[wave][lane] = 0;
    stats = sm.wstat[wave];
  }
  const int col = lane & 31;
  const int h = lane >> 5;
  // dbg (STATS builds only; timing ablations, outputs invalid): 1 = never take the slow path,
  // 2 = skip MFMA + threshold test, 4 = no global chunk loads, 128 = DMA only every other chunk,
  // 256 = no group barrier, 512 = fold without ballots, 1024 = MFMA without fold, 4096 = record the workgroup
  // timeline (combinable with the others), 8192 = no seeded band limits
  if (!STATS) dbg = FWAV_TOPK_ABL;  // production: 0; ablation builds (-DFWAV_TOPK_ABL=bits) fix the bits at compile time
  half8 b[QS], bl[QS];  // the query's fp16 high and low parts (MFMA B operands)
  float thf[QS];        // band limit: on shl (first pass), on s16 (exact mode)
  int upd[QS];
  float qv[QS][EX ? 16 : 1];  // EX: the exact query vector (sgemv16 keys)
  const int64_t n16 = (int64_t)cdiv(nd, kChunk) * kChunk * 16;  // halfs per fp16 table
  const _Float16* emb16lo = emb16 + n16;
  uint64_t kth[QS];           // EX: the query's current K-th exact key (0 until K entries)
  float inseed[QS];           // relaunch: the previous pass's band limit at overflow, in this mode's scale
  int32_t qpos[QS];           // the slot's query position in the active list
  // Table pieces of one query block share their band limits: a piece's compaction limit is a valid lower bound for
  // the whole query (K domains of its own chunk range beat it), so every piece filters with the largest limit any
  // piece has found (atomicMax on the f2key, read back at window ends) instead of restarting its own rise.
  uint32_t* share = (npieces > 1 && !EX) ? share_lim : nullptr;
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    const int ql = (wave * QS + s) * 32 + col;
    const int64_t qi = slot_query(block, qslot0 + ql, plan.nb, QB);
    const int32_t q = qi < n_active ? active[qi] : -1;
    const int64_t qrow = (int64_t)(q < 0 ? 0 : q) + q_offset;
    b[s] = *reinterpret_cast<const half8*>(emb16 + (((qrow >> 8) * 2 + h) * 256 + (qrow & 255)) * 8);
    bl[s] = *reinterpret_cast<const half8*>(emb16lo + (((qrow >> 8) * 2 + h) * 256 + (qrow & 255)) * 8);
    upd[s] = (q >= 0 && !(dbg & 1)) ? 1 : 0;
    thf[s] = upd[s] ? -INFINITY : INFINITY;  // slots past n_active never take appends
    qpos[s] = (int32_t)(qi < n_active ? qi : 0);
    if (h == 0) {
      sm.ovf[ql] = 0;
      sm.tie[ql] = 0;
      sm.qrow[ql] = qrow;
      sm.qpos[ql] = qpos[s];
    }
    kth[s] = 0ull;
    // relaunch: active = the previous pass's overflow list, whose position qi holds this query's seed (that pass's
    // band limit); seed_shift converts it to this mode's scale (S16 → HL: −(δ + 2δ'); HL → EX: −(δ + 2δ'))
    inseed[s] = seeds_in != nullptr && q >= 0 ? key2f(seeds_in[qi]) - seed_shift : -INFINITY;
    if constexpr (EX) {
      const float* qp = emb + qrow * 16;
#pragma unroll
      for (int i = 0; i < 16; ++i) qv[s][i] = qp[i];
    }
  }

  // seed the band limits from the queries' own domain windows (tiles from the wave's first query row)
  if (!(ABL && (dbg & 8192))) {  // ablation 8192: no seed
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      // whole wave (MFMA + shuffles); lanes of unused query slots discard the result
      const int64_t wbase =
          (int64_t)((__builtin_amdgcn_readfirstlane((int)sm.qrow[(wave * QS + s) * 32]) - kSeedHalf) >> 5) << 5;
      const float seed = seed_limit<MODE>(emb16, nd, b[s], sm.qrow[(wave * QS + s) * 32 + col], wbase, K);
      if (upd[s]) thf[s] = seed;
      if (STATS && (dbg & 32768) && gstats != nullptr && h == 0 && upd[s])  // diagnostics: the seeds
        gstats[16 + slot_query(block, qslot0 + (wave * QS + s) * 32 + col, plan.nb, QB)] = __float_as_uint(seed);
    }
  }
  if (seeds_in != nullptr) {
#pragma unroll
    for (int s = 0; s < QS; ++s)
      if (upd[s]) thf[s] = fmaxf(thf[s], inseed[s]);
  }
  if (fkey != 0u) {
#pragma unroll
    for (int s = 0; s < QS; ++s)
      if (upd[s]) thf[s] = fmaxf(thf[s], key2f(fkey));
  }
  // the query sets this wave works on: set position s holds logical set lid[s] (its slots lid[s]·32 + col, its key
  // buffers and LDS rows) — wave w's own sets w·QS + s (dealing sets to other waves between groups by their recent
  // work measured slower: tools/experiments/set_repairing.patch)
  int lid[QS];
#pragma unroll
  for (int s = 0; s < QS; ++s) lid[s] = wave * QS + s;
  half8 bc{};          // CENT: the lane's centroid (fp16, MFMA B operand) ...
  float cslack = 0.0f;  // ... and its slack
  auto setup_centroids = [&]() {
    const int sj = col % QS, mcol0 = QS * (col / QS);
    int ls = lid[0];
#pragma unroll
    for (int s = 1; s < QS; ++s) ls = sj == s ? lid[s] : ls;
    centroid_setup<QS>(emb16, [&](int k) -> int64_t {
      const int64_t qi = slot_query(block, qslot0 + ls * 32 + mcol0 + k, plan.nb, QB);
      return qi < n_active ? (int64_t)active[qi] + q_offset : (int64_t)-1;
    }, bc, cslack);
  };
  if constexpr (CENT) setup_centroids();
  const int nchunks = (int)cdiv(nd, kChunk);  // < 2^31 / 256: chunk arithmetic stays 32-bit (scalar)
  if ((FWAV_TOPK_PRIO & 1) && wave >= W / 2) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half
  // this item's chunk range [c0, c1) (the whole table unless the block is split)
  int c0, c1;
  piece_chunks(plan, block, piece, npieces, nchunks, c0, c1);
  const int ngroups = (c1 - c0 + G - 1) / G;
  const u32x4* src = reinterpret_cast<const u32x4*>(emb16);
  // Chunk stream: global → LDS directly (global_load_lds_dwordx4: no staging registers, no ds_write).  The
  // destination of one wave-instruction is wave-uniform base + lane × 16 B, which is exactly the slot layout
  // (thread t ↔ bytes [16t, 16t + 16) of the 8 KB chunk).  Chunks past the end re-read the last one (never
  // consumed).  Group g+1 is issued right after the barrier that retires group g and frees its half.
  auto issue_group = [&](int gg) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      int c_ = c0 + gg * G + j;
      c_ = c_ < c1 ? c_ : c1 - 1;
      if (ABL && (dbg & 4)) c_ = 0;  // ablation: no streaming traffic beyond one L2-resident chunk
      if (ABL && (dbg & 128) && (j & 1)) continue;  // ablation: DMA only every other chunk
      // the chunk's 8 KB = 8 wave-instructions of 64 × 16 B, dealt round-robin over the active waves
      for (int k = wave; k < 8; k += Wact) {
        // inline asm, not the builtin: hipcc would otherwise wait for this DMA (vmcnt(0)) before every ds_read
        // of the other half; completion is counted by hand at the group top
        const unsigned lds_dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(
            (__attribute__((address_space(3))) void*)(&slots[(gg % NB) * G + j][k * 64])));
        const u32x4* gsrc = src + (int64_t)c_ * 512 + k * 64 + lane;
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
      }
    }
  };
  // retire the prologue's ordinary loads (query fragments, active list) before the stream, visibly to hipcc
  // (a load still pending at the loop head is waited on, vmcnt(0), inside every chunk iteration)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  if (ngroups > 0) issue_group(0);

  int sink = 0;     // ablation builds: keeps the MFMA / fold results of dbg 512/1024 alive
  int nfired[QS];  // wave-uniform FIFO tail: chunks recorded in sm.fired[group] so far
  ReplayCursor cur[QS];
  int qcnt[QS];    // this lane's entries in its query's two-ended buffer (h = 0: front, h = 1: back)
  int kept[QS];    // the query's buffer size after its last compaction
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    nfired[s] = qcnt[s] = kept[s] = 0;
    cur[s] = ReplayCursor{0, 0, 0u};
  }
  // CENT: the pieces' shared limits, loaded before each group's top wait and applied before the next group's DMA is
  // issued.  (Read after that issue, as rounds 4–5 did, the compiler's wait for the loaded value, vmcnt(0), also
  // waited for the whole next group's DMA: every group's level 1 started only once the group after it had landed.)
  uint32_t shv[QS];
  for (int g = 0; g < ngroups; ++g) {
    u32x4(*half)[512] = slots + (g % NB) * G;
    const int cg = c0 + g * G;  // first chunk of group g
    const int c_end = cg + G < c1 ? cg + G : c1;
    const bool window_end =
        (c_end - c0 <= kWarmChunks) || ((g + 1) % (kWindowGroups * 4 / G) == 0) || (g + 1 == ngroups);
    if (CENT && FWAV_TOPK_CSHARE && share != nullptr) {
#pragma unroll
      for (int s = 0; s < QS; ++s)
        shv[s] = __hip_atomic_load(share + qpos[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t_b0 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    // RAW: own DMA of group g retired, then every wave's (barrier).  WAR: the other half was last read in
    // iteration g−1, whose ds_reads were all consumed before its waves reached this barrier.
    if (!(ABL && (dbg & 256))) {  // ablation 256: no group barrier (LDS races; timing only)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      if (STATS) stat_add(12, __builtin_amdgcn_s_memrealtime() - t_b0);
      if (FWAV_TOPK_PRIO & 4) __builtin_amdgcn_s_setprio(0);
      if (!(ABL && (dbg & 16384))) __builtin_amdgcn_s_barrier();  // 16384: own DMA wait, no barrier
      asm volatile("" ::: "memory");
    }
    const unsigned long long t_b1 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    if (STATS) stat_add(7, t_b1 - t_b0);
    if (CENT && FWAV_TOPK_CSHARE && share != nullptr) {
      // CENT: the pieces' shared limits every group (a filter threshold that rises sooner skips more level-2 work),
      // retired by the wait above
#pragma unroll
      for (int s = 0; s < QS; ++s)
        if (upd[s] && shv[s] != 0u) thf[s] = fmaxf(thf[s], key2f(shv[s]));
    }
    // (the DMA issued after level 1 or level 2 instead measured no better: profiles/r04/ab_prefix_dma_barrier.log)
    if (g + 1 < ngroups) issue_group(g + 1);
    if (ABL && (dbg & 2)) continue;
    int thi[QS];
#pragma unroll
    for (int s = 0; s < QS; ++s) thi[s] = int_threshold(HL ? thf[s] - kStreamMargin : thf[s]);
    const _Float16* lda0 = reinterpret_cast<const _Float16*>(half[0]) + ((h * kChunk) + col) * 8;
    if constexpr (CENT) {
      float tv[QS];
#pragma unroll
      for (int s = 0; s < QS; ++s) tv[s] = HL ? thf[s] - kStreamMargin : thf[s];
      const int thc = centroid_threshold<QS>(tv, cslack);
      uint64_t pend[QS];
      const unsigned long long t_l1 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
      if (c_end - cg == G) {
        cent_level1<G, QS>(lda0, bc, thc, pend);
      } else {
#pragma unroll
        for (int s = 0; s < QS; ++s) pend[s] = 0ull;
        for (int c = cg; c < c_end; ++c) {
          uint64_t pc[QS];
          cent_level1<1, QS>(lda0 + (c - cg) * 512 * 8, bc, thc, pc);
#pragma unroll
          for (int s = 0; s < QS; ++s) pend[s] |= pc[s] << (8 * (c - cg));
        }
      }
      if (STATS) {
        stat_add(13, __builtin_amdgcn_s_memrealtime() - t_l1);
        unsigned long long np = 0;
#pragma unroll
        for (int s = 0; s < QS; ++s) np += __popcll(pend[s]);
        stat_add(14, np);
      }
      if (FWAV_TOPK_PRIO & 4) __builtin_amdgcn_s_setprio(1);
      // level 2: the marked (tile, set) pairs scored with the set's queries, kCentBatch at a time (their fragments and
      // MFMAs in flight together).  S16: survivors appended at once.  HL: the pairs whose s16 can pass are collected
      // first, then refined in batches of kReplayBatch with their low-part fragments fetched from L2 together (one
      // memory round trip per batch, as the base geometry's replays) and appended.
      static_for<QS>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        using TMask = uint64_t;  // (32-bit masks for ≤ 32-tile groups: 17.15 vs 16.88 ms)
        TMask pm = (TMask)pend[s];
        TMask pass = 0;  // HL: tiles whose s16 passes the set's stream threshold
        while (pm != 0) {
          int t[kCentBatch];
          bool on[kCentBatch];
#pragma unroll
          for (int u = 0; u < kCentBatch; ++u) {
            on[u] = pm != 0;
            t[u] = on[u] ? ctz_mask(pm) : t[0];
            if (on[u]) pm &= pm - 1;
          }
          half8 af[kCentBatch];
          floatx16 acc[kCentBatch];
#pragma unroll
          for (int u = 0; u < kCentBatch; ++u)
            af[u] = *reinterpret_cast<const half8*>(lda0 + (t[u] >> 3) * (512 * 8) + (t[u] & 7) * 256);
#pragma unroll
          for (int u = 0; u < kCentBatch; ++u)
            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[u], b[s], floatx16{}, 0, 0, 0);
#pragma unroll
          for (int u = 0; u < kCentBatch; ++u) {
            if (!on[u]) break;
            if constexpr (HL) {
              if (__ballot(fold16((int)0x80000000, acc[u]) > thi[s]) != 0ull) pass |= (TMask)1 << t[u];
            } else {
              const int64_t dt = (int64_t)(cg + (t[u] >> 3)) * kChunk + (t[u] & 7) * 32;
              thf[s] = append_tile<C, STATS, Topk16SmemT<NG, STATS, !CENT, W>, MODE>(acc[u], thf[s], qcnt[s], kept[s],
                                                                                 dt, nd, gkeys, sm, lid[s], K,
                                                                                 upd[s], stats, sp, emb, qv[s],
                                                                                 &kth[s], share);
            }
          }
        }
        if constexpr (HL) {  // shl = s16 + d_hi·q_lo + d_lo·q_hi for the passing tiles, batched
          while (pass != 0) {
            int t[kReplayBatch];
            bool on[kReplayBatch];
#pragma unroll
            for (int u = 0; u < kReplayBatch; ++u) {
              on[u] = pass != 0;
              t[u] = on[u] ? ctz_mask(pass) : t[0];
              if (on[u]) pass &= pass - 1;
            }
            half8 afl[kReplayBatch];
#pragma unroll
            for (int u = 0; u < kReplayBatch; ++u)
              afl[u] = tile_fragment(emb16lo, (int64_t)(cg + (t[u] >> 3)) * kChunk + (t[u] & 7) * 32, h, col);
#pragma unroll
            for (int u = 0; u < kReplayBatch; ++u) {
              if (!on[u]) break;
              const half8 af = *reinterpret_cast<const half8*>(lda0 + (t[u] >> 3) * (512 * 8) + (t[u] & 7) * 256);
              floatx16 a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, b[s], floatx16{}, 0, 0, 0);
              a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bl[s], a2, 0, 0, 0);
              a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(afl[u], b[s], a2, 0, 0, 0);
              const int64_t dt = (int64_t)(cg + (t[u] >> 3)) * kChunk + (t[u] & 7) * 32;
              thf[s] = append_tile<C, STATS, Topk16SmemT<NG, STATS, !CENT, W>, MODE>(a2, thf[s], qcnt[s], kept[s], dt,
                                                                                 nd, gkeys, sm, lid[s], K,
                                                                                 upd[s], stats, sp, emb, qv[s],
                                                                                 &kth[s], share);
            }
          }
        }
      });
    } else if (ABL && (dbg & (512 | 1024)) && c_end - cg == G) {
      // ablations 512: fold without ballots, 1024: MFMA without fold (outputs invalid)
      if (dbg & 1024)
        stream_group<G, QS, 2>(lda0, b, thi, cg, sm.fired + wave * QS, nfired, lane, &sink);
      else
        stream_group<G, QS, 1>(lda0, b, thi, cg, sm.fired + wave * QS, nfired, lane, &sink);
    } else if (c_end - cg == G) {
      stream_group<G, QS>(lda0, b, thi, cg, sm.fired + wave * QS, nfired, lane);
    } else {
      for (int c = cg; c < c_end; ++c)
        stream_group<1, QS>(lda0 + (c - cg) * 512 * 8, b, thi, c, sm.fired + wave * QS, nfired, lane);
    }
    const unsigned long long t_c = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    if (STATS) stat_add(9, t_c - t_b1);
    if (window_end) {
      // the largest limit the query's pieces have published (CENT reads it every group, above)
      if (share != nullptr && !(CENT && FWAV_TOPK_CSHARE)) {
#pragma unroll
        for (int s = 0; s < QS; ++s) {
          const uint32_t v = __hip_atomic_load(share + qpos[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (upd[s] && v != 0u) thf[s] = fmaxf(thf[s], key2f(v));
        }
      }
      // each wave replays its own fired chunks (compacting inline when a buffer fills); compile-time set indices
      // (static_for): a runtime-indexed per-set array would live in scratch / LDS
      if (!CENT && (FWAV_TOPK_PRIO & 8)) __builtin_amdgcn_s_setprio(1);
      static_for<QS>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (!CENT) {
          if (nfired[s] > cur[s].head || cur[s].rem != 0u)
            thf[s] = replay_window<C, STATS, Topk16SmemT<NG, STATS, !CENT, W>, MODE>(emb16, emb16lo, b[s], bl[s], thf[s],
                                             qcnt[s], kept[s], cur[s], nfired[s], nd, gkeys, sm, lid[s], K, upd[s],
                                             stats, sp, emb, qv[s], &kth[s], share);
        }
      });
      if (!CENT && (FWAV_TOPK_PRIO & 8)) __builtin_amdgcn_s_setprio(0);
      if (STATS) stat_add(4, __builtin_amdgcn_s_memrealtime() - t_c);
      // retire the replay's loads and stores here, visibly to hipcc's wait bookkeeping (vmcnt(0) expcnt(7)
      // lgkmcnt(15)): otherwise it keeps them "pending" at the loop head and waits on them before the next
      // chunk's ds_reads — which, at run time, also drains the in-flight chunk DMA
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
  }
  const unsigned long long t_final = STATS ? __builtin_amdgcn_s_memrealtime() : 0;
  // the final pass reads the counts from LDS (same wave: program order)
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    if (h == 0)
      sm.cnt[lid[s] * 32 + col] = qcnt[s];
    else
      sm.cnt1[lid[s] * 32 + col] = qcnt[s];
  }

  auto slot_of = [&](int l) {  // the wave's l-th query slot
    int ls = lid[0];
#pragma unroll
    for (int s = 1; s < QS; ++s) ls = (l >> 5) == s ? lid[s] : ls;
    return ls * 32 + (l & 31);
  };
  if (npieces > 1) {
    // a table piece hands each query's filtered band to k_merge_pieces: kBandBatch queries' keys and shared limits
    // loaded together (the wave's own appends drained once)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int l0 = 0; l0 < 32 * QS; l0 += kBandBatch) {
      uint64_t v[kBandBatch][C / 64];
      int nb_[kBandBatch];
      uint32_t sh[kBandBatch];
#pragma unroll
      for (int b = 0; b < kBandBatch; ++b) {
        const int qs = slot_of(l0 + b);
        const int64_t qq = slot_query(block, qslot0 + qs, plan.nb, QB);
        const bool ok = l0 + b < 32 * QS && qq < n_active;
        nb_[b] = ok ? piece_band_load<C>(gkeys + (size_t)qs * C, sm, qs, v[b]) : -1;
        sh[b] = ok ? __hip_atomic_load(share_lim + qq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      }
#pragma unroll
      for (int b = 0; b < kBandBatch; ++b) {
        if (nb_[b] < 0) continue;
        const int qs = slot_of(l0 + b);
        const int64_t qq = slot_query(block, qslot0 + qs, plan.nb, QB);
        if (lane == 0) FWAV_TRACE(sm.qrow[qs], 3u, (uint32_t)sm.cnt[qs], (uint32_t)sm.ovf[qs], (uint32_t)sm.cnt1[qs]);
        piece_band<C, HL>(gkeys + (size_t)qs * C, sm, qs, K, share_lim + qq, v[b], nb_[b], sh[b]);
      }
    }
  }
  for (int l = 0; l < (npieces > 1 ? 0 : 32 * QS); ++l) {
    const int qs = slot_of(l);
    const int64_t qq = slot_query(block, qslot0 + qs, plan.nb, QB);
    if (qq >= n_active) continue;
    const int32_t qid = active[qq];
    uint64_t* kq = gkeys + (size_t)qs * C;
    if (lane == 0) FWAV_TRACE(sm.qrow[qs], 3u, (uint32_t)sm.cnt[qs], (uint32_t)sm.ovf[qs], (uint32_t)sm.cnt1[qs]);
    // exact f32 rescoring of the kept band + sort
    compact16<C>(kq, sm, qs, K, emb, cand + (int64_t)qid * K, sp, ties, qid, fkey, fl);
    // overflowed: listed for the exact-mode relaunch with its band limit as the seed (same list position)
    if (lane == 0 && sm.ovf[qs]) {
      const int pos = atomicAdd(n_ovf, 1);
      ovf_list[pos] = qid;
      reinterpret_cast<uint32_t*>(n_ovf + 1)[pos] = (uint32_t)sm.ovf[qs];
    }
  }
  if (ABL && sink == 0x7fffffff) cand[0] = sink;
  if (STATS) {
    stat_add(8, __builtin_amdgcn_s_memrealtime() - t_final);
    stat_add(6, __builtin_amdgcn_s_memrealtime() - t_kernel);
    // [15]: per workgroup, the busiest wave's time outside the group barrier (Σ over workgroups; against the mean
    // Σ([6] − [7]) / waves it tells a systematic per-wave imbalance from a per-group one)
    __syncthreads();
    if (gstats != nullptr && threadIdx.x == 0) {
      unsigned long long mx = 0;
      for (int w = 0; w < Wact; ++w) mx = max(mx, sm.wstat[w][6] - sm.wstat[w][7]);
      atomicAdd(gstats + 15, mx);
    }
    if (gstats != nullptr && lane < kStats && lane != 15) atomicAdd(gstats + lane, sm.wstat[wave][lane]);
    // dbg 4096: workgroup timeline (start of its first wave, end of its last) at gstats[16 + 2·block]
    if (gstats != nullptr && (dbg & 4096) && lane == 0) {
      atomicMin(gstats + 16 + 2 * blockIdx.x, t_kernel);
      atomicMax(gstats + 17 + 2 * blockIdx.x, __builtin_amdgcn_s_memrealtime());
    }
  }
}

// Merge the pieces of split blocks: per query, the union of its P pieces' bands (piece_band: entries whose key beats
// the shared limit at the piece's end) is filtered once more by the query's final shared limit Lk, rescored in exact
// f32 (sgemv16, the order of every other final pass), sorted (score desc, index asc) and cut to K.  Every exact top-K
// member lies in one piece's chunk range with a key above every limit, so it is in the union; the piece that
// published Lk holds K entries above it, so the union has at least K whenever Lk != 0.  A query flagged by any piece,
// or whose union would not fit one sort (C entries), goes to the exact-mode relaunch list once, seeded with the
// largest flag key (each a valid band limit) or Lk.  One wave per query.
// k_merge_pieces' last step: the band's mb ≤ 64·E keys (staged in LDS) rescored in exact f32 (sgemv16), sorted
// (score desc, index asc), listed if tied, the first K emitted.
template <int E>
__device__ __forceinline__ void merge_band(const uint64_t* __restrict__ sw, int mb, int K, const float* __restrict__ emb,
                                           int64_t qrow, const SgemvSplit& sp, int32_t* __restrict__ ties, int32_t qid,
                                           int32_t* __restrict__ out, uint32_t fkey, const FloorCtl& fl) {
  const int lane = threadIdx.x & 63;
  uint64_t v[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    v[j] = e < mb ? sw[e] : 0ull;
  }
  const float4* qp = reinterpret_cast<const float4*>(emb + qrow * 16);
  float qv[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 x = qp[i];
    qv[4 * i] = x.x; qv[4 * i + 1] = x.y; qv[4 * i + 2] = x.z; qv[4 * i + 3] = x.w;
  }
  // rescore two slots at a time (8 row loads in flight per lane; all E at once held 4·E float4 rows and doubled the
  // kernel's registers)
#pragma unroll
  for (int j0 = 0; j0 < E; j0 += 2) {
    float4 row[2][4];
    int32_t dd[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = j0 + jj < E ? j0 + jj : E - 1;
      dd[jj] = (j0 + jj < E && v[j] != 0ull) ? key_idx(v[j]) : 0;
      const float4* rp = reinterpret_cast<const float4*>(emb + (int64_t)dd[jj] * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) row[jj][i] = rp[i];
    }
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = j0 + jj;
      if (j < E && v[j] != 0ull) {
        const float acc = sgemv16([&](int k) { return f4c(row[jj][k >> 2], k & 3); }, [&](int k) { return qv[k]; },
                                  sgemv_kind((uint32_t)dd[jj], sp));
        v[j] = make_key(acc, dd[jj]);
      }
    }
  }
  wave_sort_desc<E>(v);
  if (fkey != 0u) {
    uint64_t kth = 0;
#pragma unroll
    for (int j = 0; j < E; ++j)
      if (j == ((K - 1) >> 6)) kth = __shfl(v[j], (K - 1) & 63);
    if (floor_miss(fkey, fl, mb, K, kth, qid)) return;
  }
  record_tie<E>(ties, qid, tie_flags<E>(v, mb, K), v, mb, K, true);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int e = j * 64 + lane;
    if (e < K) out[e] = v[j] != 0ull ? key_idx(v[j]) : -1;
  }
}

// One split-block query of k_merge_pieces (defined below the kernel); MP ≥ the plan's pieces.
template <int C, int QB, bool HL, int MP>
__device__ __forceinline__ void merge_query(const TopkPlan& plan, int64_t w, int lane, uint64_t* sw, uint32_t* sh,
                                            const uint64_t* __restrict__ gkeys_all, const int32_t* __restrict__ active,
                                            int n_active, int K, int32_t* __restrict__ cand,
                                            int32_t* __restrict__ ovf_list, int32_t* __restrict__ n_ovf,
                                            const uint32_t* __restrict__ share, const float* __restrict__ emb,
                                            int64_t q_offset, const SgemvSplit& sp, int32_t* __restrict__ ties,
                                            uint32_t fkey, const FloorCtl& fl);

// k_merge_pieces' union: the pieces' bands hold n = Σ counts entries (cfg2: mean 174, max 268 over 60,416 queries;
// those above the shared limit Lk mean 163; the band kept after the select mean 78, max 113: tools/diag/
// merge_inputs.py, profiles/r06/merge_inputs_cfg2.log).  The entries above Lk are compacted into the wave's LDS row
// and, up to merge_fast(MP)·64 of them, selected from registers; a wider union (long runs of near-equal scores) is
// selected by re-reading it from L2 once per key bit instead, so the register budget — and the occupancy — no longer
// scale with the widest plan's P·(C − 64).
// (The floor's second pass merges 16, 32 or 64 pieces of a low floor: its unions above Lk run to ≈ 800 entries and
// more — thousands with 64 pieces; there the union's key words, merge_hi_rows(MP) rows of them, are selected from LDS
// before the L2 tier: a 64-piece merge of 580 queries 786 µs with 32 rows, 145 with 64.)
constexpr int kMergeFast = 8;
constexpr int merge_hi_rows(int MP) { return MP <= 8 ? 1 : (MP <= 32 ? 32 : 64); }
template <int C, int QB, bool HL, int MP>
__global__ __launch_bounds__(256) void k_merge_pieces(const uint64_t* __restrict__ gkeys_all,
                                                      const int32_t* __restrict__ active,
                                                      const int32_t* __restrict__ n_active_p, int plan_rt, int plan_p,
                                                      int K, int32_t* __restrict__ cand, int32_t* __restrict__ ovf_list,
                                                      int32_t* __restrict__ n_ovf, const uint32_t* __restrict__ share,
                                                      const float* __restrict__ emb, int64_t q_offset, SgemvSplit sp,
                                                      int32_t* __restrict__ ties, FloorCtl fl) {
  const int n_active = *n_active_p;
  const uint32_t fkey = fl.key != nullptr ? __builtin_amdgcn_readfirstlane(*fl.key) : 0u;
  const bool alt = fl.key != nullptr && fkey == 0u;  // the floor did not apply: the floor-free plan (FloorCtl)
  const TopkPlan plan = make_plan(n_active, alt ? fl.alt_rt : plan_rt, alt ? fl.alt_p : plan_p, QB);
  if (plan.R == 0 || plan.halves) return;
  const int lane = threadIdx.x & 63;
  __shared__ uint64_t stage[4][kMergeFast * 64];  // per wave: the union above Lk, then the band (≤ C of it)
  __shared__ uint32_t hstage[4][merge_hi_rows(MP) * 64];  // per wave (16 / 32 pieces): the union's key words
  uint64_t* sw = stage[threadIdx.x >> 6];
  uint32_t* sh = hstage[threadIdx.x >> 6];
  // one wave per split-block query.  (Persistent waves looping over the queries measured the same, cfg2 search 17.40
  // vs 17.39 ms, profiles/r05/ab_merge_persistent.log, but the loop made the compiler hoist per-lane invariants of
  // the body out of it: 131 VGPRs, 3 waves per SIMD.)
  // (wave-uniform values in scalar registers: the query's row, limit and addresses load through the scalar cache)
  const int64_t w = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (w < plan.R * QB)
    merge_query<C, QB, HL, MP>(plan, w, lane, sw, sh, gkeys_all, active, n_active, K, cand, ovf_list, n_ovf, share,
                               emb, q_offset, sp, ties, fkey, fl);
}

// One split-block query w of k_merge_pieces (whole wave; sw: the wave's LDS row).
template <int C, int QB, bool HL, int MP>
__device__ __forceinline__ void merge_query(const TopkPlan& plan, int64_t w, int lane, uint64_t* sw, uint32_t* sh,
                                            const uint64_t* __restrict__ gkeys_all, const int32_t* __restrict__ active,
                                            int n_active, int K, int32_t* __restrict__ cand,
                                            int32_t* __restrict__ ovf_list, int32_t* __restrict__ n_ovf,
                                            const uint32_t* __restrict__ share, const float* __restrict__ emb,
                                            int64_t q_offset, const SgemvSplit& sp, int32_t* __restrict__ ties,
                                            uint32_t fkey, const FloorCtl& fl) {
  constexpr int E = C / 64;
  constexpr int kBit0 = HL ? 0 : 12;  // the select's resolution (S16 needs the K-th only at ≈ 2^-11)
  constexpr int kHiRows = merge_hi_rows(MP);
  const int64_t block = plan.F + w / QB;
  const int ql = (int)(w % QB);
  const int64_t qq = slot_query(block, ql, plan.nb, QB);
  if (qq >= n_active) return;
  const int P = plan.P;
  // piece headers ((overflow key << 32) | count), lane p < P loading piece p's: one vector load for all of them
  // key region of piece p: base0 + p·pstride (item_of is linear in the piece)
  const int64_t base0 = ((int64_t)plan.item_of(block, 0) * QB + ql) * C;
  const int64_t pstride = (plan.item_of(block, 1) - plan.item_of(block, 0)) * (int64_t)QB * C;
  const uint64_t hdr = lane < P ? gkeys_all[base0 + (int64_t)lane * pstride + C - 1] : 0ull;
  const uint32_t Lk = __builtin_amdgcn_readfirstlane(share[qq]);
  const int32_t qid = __builtin_amdgcn_readfirstlane(active[qq]);
  // prefix of the counts and the largest overflow flag.  Up to 16 pieces: wave-uniform, in SGPRs, and a piece found by
  // comparing against each prefix; 32 / 64 pieces: lane p holds piece p's exclusive prefix and an entry's piece is
  // found by a binary search over the lanes (6 shuffles instead of MP − 1 compares and selects per entry)
  constexpr bool kLanePre = MP > 16;
  int pre[kLanePre ? 1 : MP + 1];
  uint32_t seed = 0u;
  int n = 0, pre_l = 0;
  if constexpr (kLanePre) {
    static_assert(MP <= 64, "one piece per lane");
    const int cnt = lane < P ? (int)(uint32_t)hdr : 0;
    int inc = cnt;  // inclusive prefix over the lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    pre_l = inc - cnt;
    n = __builtin_amdgcn_readlane(inc, 63);
    uint32_t sd = lane < P ? (uint32_t)(hdr >> 32) : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sd = max(sd, (uint32_t)__shfl_xor((int)sd, off));
    seed = __builtin_amdgcn_readfirstlane(sd);
  } else {
    pre[0] = 0;
#pragma unroll
    for (int p = 0; p < MP; ++p) {
      const uint64_t h = p < P ? (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)hdr, p) |
                                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hdr >> 32), p) << 32)
                               : 0ull;
      seed = max(seed, (uint32_t)(h >> 32));
      pre[p + 1] = pre[p] + (int)(uint32_t)h;
    }
    n = pre[MP];
  }
  // entry e of the union: piece p (pre[p] ≤ e < pre[p + 1]) at offset e − pre[p]; 0 past the end
  auto entry = [&](int e) -> uint64_t {
    int p = 0, start = 0;
    if constexpr (kLanePre) {
      // the largest p < P with pre[p] ≤ e (a piece of count 0 shares its prefix with the next one, which wins)
#pragma unroll
      for (int step = 32; step > 0; step >>= 1) {
        const int mid = p + step;
        const int pm = __shfl(pre_l, mid < 64 ? mid : 63);
        if (mid < P && pm <= e) p = mid;
      }
      start = __shfl(pre_l, p);
    } else {
#pragma unroll
      for (int pp = 1; pp < MP; ++pp)
        if (pp < P && e >= pre[pp]) {
          p = pp;
          start = pre[pp];
        }
    }
    return e < n ? gkeys_all[base0 + (int64_t)p * pstride + (e - start)] : 0ull;
  };
  const int nu = (n + 63) >> 6;  // 64-entry rows of the union (wave-uniform)
  uint32_t L = Lk;
  int mb = 0;
  if (seed == 0u) {
    // the union's entries above Lk, compacted into the wave's LDS row (kMergeFast rows of loads in flight: one
    // memory round trip for a union of up to kMergeFast·64 entries), with the key bits they all share (a AND, o OR)
    int m = 0;
    uint32_t a = ~0u, o = 0u;
    for (int u0 = 0; u0 < nu; u0 += kMergeFast) {
      uint64_t y[kMergeFast];
#pragma unroll
      for (int i = 0; i < kMergeFast; ++i) y[i] = u0 + i < nu ? entry((u0 + i) * 64 + lane) : 0ull;
#pragma unroll
      for (int i = 0; i < kMergeFast; ++i) {
        const bool in = (uint32_t)(y[i] >> 32) > Lk;
        const uint64_t bm = __ballot(in);
        const int pos = m + __popcll(bm & ((1ull << lane) - 1ull));
        if (in) {
          if (pos < kMergeFast * 64) sw[pos] = y[i];
          if (kHiRows > 1 && pos < kHiRows * 64) sh[pos] = (uint32_t)(y[i] >> 32);
          a &= (uint32_t)(y[i] >> 32);
          o |= (uint32_t)(y[i] >> 32);
        }
        m += __popcll(bm);
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      a &= (uint32_t)__shfl_xor((int)a, off);
      o |= (uint32_t)__shfl_xor((int)o, off);
    }
    const uint32_t d = a ^ o;
    const int top = d == 0u ? -1 : 31 - __builtin_clz(d);
    uint32_t T = (top < 0 ? a : a & ~((2u << top) - 1u)) & ~((1u << kBit0) - 1u);
    const int mu = (m + 63) >> 6;
    if (m <= kMergeFast * 64) {
      // the usual case: the union above Lk in registers; its K-th key T by a greedy bitwise select that starts below
      // the bits every entry shares, and the band above T − margin compacted back into the LDS row
      uint64_t x[kMergeFast];
#pragma unroll
      for (int u = 0; u < kMergeFast; ++u) x[u] = u * 64 + lane < m ? sw[u * 64 + lane] : 0ull;
      if (m > K) {
        for (int bit = top; bit >= kBit0; --bit) {
          const uint32_t Tc = T | (1u << bit);
          int c = 0;
#pragma unroll
          for (int u = 0; u < kMergeFast; ++u)
            if (u < mu) c += __popcll(__ballot((uint32_t)(x[u] >> 32) >= Tc));
          if (c >= K) T = Tc;
        }
        L = max(L, f2key(HL ? key2f(T) - 2.5f * kHLDelta : key2f(T) - 2.0f * kF16Delta));
      }
#pragma unroll
      for (int u = 0; u < kMergeFast; ++u) {
        if (u < mu) {
          const bool keep = x[u] != 0ull && (uint32_t)(x[u] >> 32) > L;
          const uint64_t bm = __ballot(keep);
          const int pos = mb + __popcll(bm & ((1ull << lane) - 1ull));
          if (keep && pos < C) sw[pos] = x[u];
          mb += __popcll(bm);
        }
      }
    } else if (kHiRows > 1 && m <= kHiRows * 64) {
      // a wider union (16 / 32 pieces): the select over its key words in LDS, then the band re-streamed from L2
      if (m > K) {
#pragma unroll 1
        for (int bit = top; bit >= kBit0; --bit) {
          const uint32_t Tc = T | (1u << bit);
          // the lane's count over the rows, 8 LDS reads in flight, then one wave sum per bit
          int c = 0;
#pragma unroll 1
          for (int u0 = 0; u0 < mu; u0 += 8) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int e = (u0 + i) * 64 + lane;
              c += (e < m && sh[e < kHiRows * 64 ? e : 0] >= Tc) ? 1 : 0;
            }
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
          if (c >= K) T = Tc;
        }
        L = max(L, f2key(HL ? key2f(T) - 2.5f * kHLDelta : key2f(T) - 2.0f * kF16Delta));
      }
      for (int u0 = 0; u0 < nu; u0 += kMergeFast) {
        uint64_t y[kMergeFast];
#pragma unroll
        for (int i = 0; i < kMergeFast; ++i) y[i] = u0 + i < nu ? entry((u0 + i) * 64 + lane) : 0ull;
#pragma unroll
        for (int i = 0; i < kMergeFast; ++i) {
          const bool keep = (uint32_t)(y[i] >> 32) > L;
          const uint64_t bm = __ballot(keep);
          const int pos = mb + __popcll(bm & ((1ull << lane) - 1ull));
          if (keep && pos < C) sw[pos] = y[i];
          mb += __popcll(bm);
        }
      }
    } else {
      // a wide union (long runs of near-equal scores): the same select, its entries re-read from L2 for every key bit
#pragma unroll 1
      for (int bit = top; bit >= kBit0; --bit) {
        const uint32_t Tc = T | (1u << bit);
        int c = 0;
#pragma unroll 1
        for (int u = 0; u < nu; ++u) {
          const uint32_t h = (uint32_t)(entry(u * 64 + lane) >> 32);
          c += __popcll(__ballot(h > Lk && h >= Tc));
        }
        if (c >= K) T = Tc;
      }
      L = max(L, f2key(HL ? key2f(T) - 2.5f * kHLDelta : key2f(T) - 2.0f * kF16Delta));
#pragma unroll 1
      for (int u = 0; u < nu; ++u) {
        const uint64_t y = entry(u * 64 + lane);
        const bool keep = (uint32_t)(y >> 32) > L;
        const uint64_t bm = __ballot(keep);
        const int pos = mb + __popcll(bm & ((1ull << lane) - 1ull));
        if (keep && pos < C) sw[pos] = y;
        mb += __popcll(bm);
      }
    }
  }
  if (seed != 0u || mb > C) {
    // a piece overflowed, or the band would not fit one sort: the exact-mode relaunch, seeded with a valid limit
    if (lane == 0) {
      const int pos = atomicAdd(n_ovf, 1);
      ovf_list[pos] = qid;
      reinterpret_cast<uint32_t*>(n_ovf + 1)[pos] = max(seed, L);
    }
    return;
  }
  // same wave: its own ds_writes are ordered before merge_band's reads
  if (FWAV_TOPK_SMALLSORT && C > 128 && mb <= 128)
    merge_band<2>(sw, mb, K, emb, (int64_t)qid + q_offset, sp, ties, qid, cand + (int64_t)qid * K, fkey, fl);
  else
    merge_band<E>(sw, mb, K, emb, (int64_t)qid + q_offset, sp, ties, qid, cand + (int64_t)qid * K, fkey, fl);
}

// Host-side plan: default policy from the device's workgroup slots, or a diagnostic override.
#ifdef FWAV_DEBUG_API
static int g_plan_rt = -1, g_plan_p = -1;  // fwav_debug_topk_plan (debug library only)
static int g_tail_wb = -1;  // fwav_debug_topk_tail (debug library only): the last piece's weight in 1/16
#else
constexpr int g_plan_rt = -1, g_plan_p = -1;
constexpr int g_tail_wb = -1;
#endif
// Per-device caches (the caller makes the stream's device current: fwav.engine wraps every call in
// torch.cuda.device); kMaxDev bounds the device ordinal.
constexpr int kMaxDev = 64;
static int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
  return dev;
}
// First-pass geometry.  Tables of more than kWideMinDomains domains (an fp16 table of > 128 MB, on its way past the
// 256 MB Infinity Cache) take the wide workgroup: kWideW = 16 waves × 32 queries, one workgroup per CU (its LDS holds
// 2 × 8 chunk slots, one barrier per 8 chunks), so a CU streams the table once for 512 queries where the base
// geometry streams it twice for 2 × 256.  Same-box A/B on a cfg4 shard (86.4 M domains × 337,500 queries, identical
// outputs): base 973.8 ms, W = 16 / G = 4 963.3, W = 16 / G = 8 944.0, QS = 2 (233 VGPRs: 2 waves per SIMD) 1,088;
// cfg2 (1.3 M domains, MALL-resident table): base 20.7 ms, wide 21.7; cfg3 (6.6 M, a 212 MB table): base 187.6,
// wide 193.4; cfg4 shard again: base 962.2, wide 945.6 — so the wide geometry is used only where the table (32 B per
// domain) no longer fits the Infinity Cache.  Relaunches on overflow lists keep the base geometry (few queries).
#ifndef FWAV_TOPK_WIDE_MIN
#define FWAV_TOPK_WIDE_MIN (int64_t(1) << 23)
#endif
constexpr int kWideW = 16, kWideG = 8;
constexpr int kWideQB = 32 * kWideW;
constexpr int kCentQS = FWAV_TOPK_CENT > 0 ? FWAV_TOPK_CENT : 4, kCentW = FWAV_TOPK_CW, kCentG = FWAV_TOPK_CG;
constexpr int kCentQB = 32 * kCentW * kCentQS;
constexpr int kCentWideQS = 2;  // the centroid filter in the wide geometry: 16 waves × 2 sets, 8 chunks per barrier
constexpr int kCentWideQB = 32 * kWideW * kCentWideQS;
#ifdef FWAV_DEBUG_API
static int g_wide = -1;  // fwav_debug_topk_geometry (debug library only): force base / wide / centroid
#else
constexpr int g_wide = -1;
#endif
// first-pass geometries
constexpr int kGeoBase = 0, kGeoWide = 1, kGeoCent = 2, kGeoCentWide = 3;
#ifndef FWAV_TOPK_CPDBL
#define FWAV_TOPK_CPDBL 4  // centroid geometry, blocks on at most half the slots: pieces doubled below this count
#endif
#ifndef FWAV_TOPK_TAIL
#define FWAV_TOPK_TAIL 12  // multi-round plans of split blocks: the last piece's table share in 1/16 (16, 0: even)
#endif
#ifndef FWAV_TOPK_YOUNG
#define FWAV_TOPK_YOUNG 1  // one-round plans: smaller table pieces for the CUs' younger workgroups (piece_chunks)
#endif
#ifndef FWAV_TOPK_CENTWIDE
// tables past the Infinity Cache: the centroid filter in the wide geometry (16 waves × 2 sets of 32, 8-chunk groups,
// one workgroup per CU).  A cfg4 shard (337,500 queries × 86.4 M domains, hi/lo band, identical outputs): wide
// 920 ms → centroid wide 632 ms (profiles/r04/ab_centwide_cfg4_q337500.log)
#define FWAV_TOPK_CENTWIDE 1
#endif
#ifndef FWAV_TOPK_CPMIN
#define FWAV_TOPK_CPMIN 6  // centroid geometry, up to 1.5 rounds of blocks: at least this many table pieces each
#endif
constexpr int kCentFloorPieces = 3;  // ... and this many with the speculative floor (profiles/r05/plan_floor_ab*.log)
#ifndef FWAV_TOPK_CENT_HL
#define FWAV_TOPK_CENT_HL 0  // the centroid geometry for hi/lo first passes too (cfg3: 195 vs 180 ms base)
#endif
#ifndef FWAV_TOPK_CENT_MINQ
// the centroid geometry for first passes of at least this many queries.  Below the speculative floor's minimum the
// centroid geometry lost to the base one (cold limits: 41,344 queries 3.42 vs 3.26 ms); with the floor it wins from
// 32,768 queries on (round 6, tools/ab/eighth_geo_prof.sh, profiles/r06/eighth_geo_*.log, floor on / base geometry,
// floor off, base geometry → floor on, centroid: 32,768 queries 2.73 / 2.80 → 2.42 ms, 41,344 2.93 / 3.22 → 2.88,
// 55,000 4.38 / 4.35 → 3.75), not at 20,672 (2.12 / 2.07 → 2.36: 41 blocks of 512 fill 328 of the 512 slots)
#define FWAV_TOPK_CENT_MINQ 32768
#endif
static int first_geometry(int64_t nd, int64_t max_q) {
  if (g_wide >= 0) return g_wide;
  if (nd > (int64_t)FWAV_TOPK_WIDE_MIN)
    return FWAV_TOPK_CENTWIDE && max_q >= (int64_t)FWAV_TOPK_CENT_MINQ ? kGeoCentWide : kGeoWide;
  const bool cent = FWAV_TOPK_CENT > 0 && max_q >= (int64_t)FWAV_TOPK_CENT_MINQ &&
                    (FWAV_TOPK_CENT_HL || first_mode(nd) == kModeS16);
  return cent ? kGeoCent : kGeoBase;
}
static int geometry_qb(int geo) {
  return geo == kGeoWide ? kWideQB : (geo == kGeoCent ? kCentQB : (geo == kGeoCentWide ? kCentWideQB : k16QB));
}

static void topk_device_slots(int geo, int& cus, int& per_cu) {
  static int cs[4][kMaxDev] = {{0}}, ws[4][kMaxDev] = {{0}};
  const int dev = current_device();
  int& c = cs[geo][dev];
  int& w = ws[geo][dev];
  if (c == 0) {
    const hipError_t occ =
        geo == kGeoWide
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&w, k_sim_topk_f16<k16Cap, false, kModeHL, kWideW, kWideG, 1>,
                                                           64 * kWideW, 0)
        : geo == kGeoCent
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &w, k_sim_topk_f16<k16Cap, false, kModeS16, kCentW, kCentG, kCentQS, true>, 64 * kCentW, 0)
        : geo == kGeoCentWide
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &w, k_sim_topk_f16<k16Cap, false, kModeHL, kWideW, kWideG, kCentWideQS, true>, 64 * kWideW, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&w, k_sim_topk_f16<k16Cap, false, kModeS16>, 64 * k16Waves,
                                                           0);
    if (!(hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && occ == hipSuccess &&
          c > 0 && w > 0)) {
      c = 256;  // MI355X: 256 CUs × 2 base (1 wide) workgroups
      w = (geo == kGeoBase || geo == kGeoCent) ? 2 : 1;
    }
  }
  cus = c;
  per_cu = w;
}
// Default policy.  Whole-table items, dispatched in order, fill the slots round after round; the last round's
// workgroups run faster when they have a CU to themselves, but once that round holds more blocks than there are
// CUs, the surplus doubles up on a few CUs and finishes last (cfg2: 1292 blocks on 256 CUs × 2 → the last 268 blocks
// include 12 that ran 3.5 ms past the rest).  So the last 2·(surplus) blocks are split into 4 table pieces, which
// fill in beside the lone workgroups (cfg2 A/B: 24.9 → 22.6 ms; splitting more blocks costs more than it saves,
// since every piece restarts the rising limit: 268 blocks in 2 pieces 24.2 ms, 512 in 2 25.3 ms).  Few blocks
// (at most half the slots) are each split into up to 8 pieces so that the table passes use the idle CUs.
static bool floor_by_default(int64_t max_q, int64_t nd);  // (defined with the floor, below)
// floored: whether the first pass runs with the speculative floor (−1: as the launch decides, floor_by_default)
static void host_plan_for(int64_t max_q, int64_t nd, int geo, int& rt, int& P, int floored = -1) {
  if (g_plan_rt >= 0) {  // diagnostic override
    rt = g_plan_rt;
    P = g_plan_p;
  } else {
    int cus, per_cu;
    topk_device_slots(geo, cus, per_cu);
    const int64_t slots = (int64_t)cus * per_cu;
    const int64_t nb = cdiv(max_q > 0 ? max_q : 1, geometry_qb(geo));
    rt = 0;
    P = 1;
    if (2 * nb <= slots) {
      // every block split, pieces in piece-major order (TopkPlan::pm): the later pieces of a block start from the
      // limits its earlier pieces published, so twice the pieces that fit one round pay (one process per
      // configuration, identical outputs: 41,344 queries 3.60 → 3.35 ms with 6 pieces instead of 3 block-major;
      // 65,536: 5.29 → 4.83 with 4 instead of 2; 20,672: 2.25 → 2.08 with 6, block-major before)
      rt = (int)nb;
      int64_t p = slots / nb;
      if (FWAV_TOPK_PMAJOR && p < (geo == kGeoCent ? FWAV_TOPK_CPDBL : 4)) p *= 2;
      P = (int)(p < kPlanMaxPieces ? p : kPlanMaxPieces);
    } else if (FWAV_TOPK_PMAJOR && 2 * nb <= 3 * slots) {
      // up to 1.5 rounds of blocks: every block in max(3, ⌊2·slots / nb⌋) pieces, piece-major — later rounds start
      // from the earlier pieces' limits (82,688 queries: 6.43 → 5.92 ms with 3 pieces; 165,375: 11.27 → 10.81 with
      // 3, 10.72 with 4; the tail split below stays for more blocks: all of cfg2 in 2 / 3 / 4 piece-major pieces
      // 20.8 / 20.5 / 20.7 vs 20.2–20.4 ms)
      // The centroid geometry takes at least 6 (its first pass is cheap, so the table pieces' restarted limits weigh
      // less than the balance of ≈ 4–8 rounds of short items: cfg2 646 blocks in 3 / 4 / 5 / 6 / 8 pieces 17.37 /
      // 16.94 / 17.02 / 16.89 / 17.40 ms, 165,375 queries in 3 / 4 / 6 10.04 / 9.92 / 9.68;
      // profiles/r04/plan_sweep_cent_cfg2.log)
      rt = (int)nb;
      int64_t p = 2 * slots / nb;
      // With the speculative floor (§3.1b of DESIGN) no piece starts cold, and fewer, longer pieces pay: cfg2 in 3 / 4 /
      // 6 pieces 15.72 / 15.95 / 16.02 ms, 165,375 queries 8.66 / 8.89 / 8.75 (profiles/r05/plan_floor_ab*.log)
      const bool fl = floored < 0 ? floor_by_default(max_q, nd) : floored != 0;
      const int64_t pmin = (geo == kGeoCent) ? (fl ? kCentFloorPieces : FWAV_TOPK_CPMIN) : 3;
      if (p < pmin) p = pmin;
      P = (int)(p < kPlanMaxPieces ? p : kPlanMaxPieces);
    } else {
      const int64_t last = nb % slots == 0 ? slots : nb % slots;  // blocks in the last round
      if (last > cus) {
        // piece-major: the whole last round in 4 pieces (cfg2, one process per plan: 20.29–20.49 → 19.93 ms; the
        // block-major plan split only its 2·(surplus) doubled-up blocks)
        rt = (int)(FWAV_TOPK_PMAJOR ? last : (2 * (last - cus) < nb ? 2 * (last - cus) : nb));
        P = 4;
      } else if (5 * last <= 3 * cus) {
        // a last round of lone workgroups on at most 60 % of the CUs: its blocks as 4 table pieces each.  Same-box
        // A/B (identical outputs), last-round blocks → ms unsplit / split: 60 → 12.45 / 9.39, 134 (one rank's half
        // of cfg2) 12.54 / 11.24, 200 12.60 / 12.74, 250 13.13 / 13.33
        rt = (int)last;
        P = 4;
        // piece-major (base geometry): the round before it too, so that the short round's pieces follow pieces of
        // their own blocks (cfg3, one process per plan: 177.1–177.6 → 175.3–175.7 ms)
        if (FWAV_TOPK_PMAJOR && geo == kGeoBase && nb >= last + slots) rt = (int)(last + slots);
      }
    }
  }
  // every piece streams at least 16 chunks (4,096 domains)
  const int64_t pmax = cdiv(nd, kChunk) / 16;
  if (P > pmax) P = (int)(pmax > 1 ? pmax : 1);
  // one round of split blocks, two workgroups to a CU: the pieces whose items start in the round's second half run as
  // their CU's younger workgroup and get the smaller share of the table (piece_chunks)
  if (g_plan_rt < 0 && P > 1 && P <= 0xFF) {
    const int tail_wb = g_tail_wb >= 0 ? g_tail_wb : FWAV_TOPK_TAIL;
    int cus, per_cu;
    topk_device_slots(geo, cus, per_cu);
    const int64_t slots = (int64_t)cus * per_cu;
    const int64_t nb = cdiv(max_q > 0 ? max_q : 1, geometry_qb(geo));
    const TopkPlan pl = make_plan(max_q, rt, P, geometry_qb(geo));
    if (FWAV_TOPK_YOUNG && per_cu == 2 && pl.F == 0 && pl.R == nb && pl.pm && pl.items() <= slots &&
        2 * pl.items() > slots) {
      // every block's pieces weighed by their own items' side of slots / 2 (TopkPlan::ybound).  (Round 6 first
      // weighed whole pieces, from the first piece past slots / 2 on: one rank's eighth of cfg2, 81 blocks × 6
      // pieces in one round, 2.56 → 2.53 ms, profiles/r06/ab_young.log)
      if (slots / 2 < 0xFFF) P |= (1 << 30) | (int)((slots / 2) << 8);
    } else if (tail_wb > 0 && tail_wb != 16 && pl.F == 0 && pl.R == nb && pl.pm && pl.items() > slots) {
      // several rounds of split blocks, piece-major: the items that start last are the blocks' last pieces, and the
      // launch ends with the slowest of them, so the last piece of every block takes tail_wb / 16 of the others'
      // share of the table.  Same process (tools/diag/topk_reps.py, FWAV_DEBUG_TOPK_TAIL, profiles/r06/tail_sweep.log):
      // cfg2 (646 centroid blocks × 3 pieces) 14.26–14.46 ms even, 13.98 / 14.02–14.06 / 14.16 / 14.22 at 11 / 12 /
      // 13 / 14; 165,375 queries 7.72 → 7.57 at 12
      P |= ((P - 1) << 8) | (tail_wb << 16) | (16 << 21);
    }
  }
}
// ---------------------------------------------------------------------------------------- speculative floor
// A first pass of at least kFloorMinQ queries over at least kFloorMinD domains starts every band
// limit at a floor guessed from kFloorPilots pilot queries (FloorCtl); the queries it cuts are searched again.
// Measured (tools/seed_ab.py, profiles/r05/seed_floor_cfg2.log): cfg2's search 17.01 ms unseeded, 15.27 / 14.71 /
// 14.12 ms with one floor of 1.80 / 1.85 / 1.88 for every query (0.05 / 0.38 / 1.7 % of the queries below it, their
// misses not counted), 12.20 ms with each query's own exact K-th score.
// The later passes cost a round of table pieces whatever their size (≈ 0.5–1 ms: a piece's cost is mostly the rise
// of its limit), so the floor pays only where it saves more than that (tools/floor_pass_ab.py, pilots' 10th-smallest
// estimate, same box): 330,750 queries 18.15 → 15.90 ms, 165,375 9.70 → 8.65, 82,688 6.14 → 5.33, but 41,344 (one
// rank's share at N = 8) 3.40 → 3.94 (profiles/r05/floor_pass_ab.log, floor_pass_ab_mid.log) — in the base
// geometry; with the centroid geometry the floor pays from 32,768 queries on (round 6, FWAV_TOPK_CENT_MINQ)
constexpr int64_t kFloorMinQ = 32768, kFloorMinD = 65536;
// ... and tables of at most kFloorMaxD domains: the later passes' pieces grow with the table, and at cfg4's
// 86.4 M domains the second pass took 204 ms after a 511 ms first pass (a 262,144-query search, profiles/r05/
// kernel_stats_bench_cfg2.txt: the cfg4 affine-roofline extra of bench.py)
constexpr int64_t kFloorMaxD = int64_t(1) << 22;
// the second pass's table pieces per split block: the most of 64 / 32 / 16 with which the misses expected at the
// floor's rank (≈ 2 % of the launch) fill at most one round of workgroup slots (the pass's latency is the length of
// one piece: 82,688 queries 4.86 → 4.60 ms with 32 instead of 16, profiles/r06/ab_floor_p2_quarter.log; 41,344: 64
// pieces 370 → 231 µs, their merge 67 → 145 µs, profiles/r06/timeline_eg_41344_f-_g-_p{32,64}.txt); cfg2's ≈ 5,000
// misses in 21 blocks × 16 pieces fill one round, 32 pieces would take two
constexpr int kFloorP2 = 16, kFloorP2Few = 32, kFloorP2Fewest = 64;
// Pilot count and floor rank (A/B builds may override): 256 pilots at rank 5 (the same ≈ 2 % quantile) against
// round 5's 512 at rank 10, same process, identical candidates (profiles/r06/ab_pilots256/): cfg2 14.03 → 14.01
// ms, 165,375 queries 7.83 → 7.87, 82,688 4.55 → 4.48, 41,344 2.85 → 2.80 — the pilots' half of the work (≈ 55 µs)
#ifndef FWAV_FLOOR_PILOTS
#define FWAV_FLOOR_PILOTS 256
#endif
#ifndef FWAV_FLOOR_RANK
#define FWAV_FLOOR_RANK 5
#endif
constexpr int kFloorPilots = FWAV_FLOOR_PILOTS;  // pilot queries (evenly spaced over the active list)
constexpr int kFloorJ = 8;  // the pilot's estimate: its j-th best score over every (K/j)-th domain ≈ its K-th
constexpr int kFloorRank = FWAV_FLOOR_RANK;  // the floor: the pilots' kFloorRank-th smallest estimate (≈ 2 % quantile)
static_assert(kFloorPilots % 64 == 0 && kFloorPilots <= 1024, "pilots: whole waves, one k_floor_reduce workgroup");
// second pass: up to kFloorSplit blocks (of 256 misses) split into kFloorP2 pieces, any further ones
// whole-table (a floor that cut more than 5 % of cfg2's queries)
constexpr int kFloorSplit = 64;
// The second pass runs at a lower floor, the pilots' smallest estimate − kFloor2Margin, meant to lie below every K-th
// score (cfg2: the smallest of all 330,750 is 1.720; the pilots' smallest estimate is 1.75–1.85 depending on which
// queries they are — with fwav_prune's active-list order margins of 0.06 / 0.10 still cut 11 / 15 queries, and each
// call then paid a cold third pass: tools/diag/floor_misses.py, profiles/r05/floor_misses*.log), so that its table
// pieces do not start cold either; the queries that one cuts (normally none) take a floor-free third pass.  (Full
// score rows for them, launch_topk_large, measured 3.6 ms per launch: one workgroup per row streams it repeatedly.)
constexpr float kFloor2Margin = 0.15f;
// (The later passes in the centroid geometry, on the miss list in its atomic order, measured slower: 330,750 /
// 165,375 / 82,688 / 41,344 queries 14.14 → 14.70 / 7.72 → 8.13 / 4.38 → 4.78 / 2.69 → 3.20 ms, round 6,
// profiles/r06/ab_floor_geo2.log — consecutive misses are unrelated queries, so the centroids' slack is large.)
static_assert(kFloorP2 >= 1 && kFloorP2Fewest <= kMaxPieces, "second-pass pieces outside the merge");
#ifdef FWAV_DEBUG_API
static int g_floor_mode = -1;      // fwav_debug_topk_floor: −1 auto, 0 off, 1 / 3 forced value, 2 pilot at any size
static uint32_t g_floor_key = 0u;
static int g_floor_rank = kFloorRank;
static float g_floor2_margin = kFloor2Margin;
#else
constexpr int g_floor_mode = -1;
constexpr uint32_t g_floor_key = 0u;
constexpr int g_floor_rank = kFloorRank;
constexpr float g_floor2_margin = kFloor2Margin;
#endif
static int floor_mode() { return g_floor_mode; }
// the first pass of max_q queries over nd domains runs with the floor (K ≤ 64, the fp16 search)
static bool floor_by_default(int64_t max_q, int64_t nd) {
  const int fmode = floor_mode();
  return fmode != 0 && (fmode > 0 || (max_q >= kFloorMinQ && nd >= kFloorMinD && nd <= kFloorMaxD));
}
// second-pass plan (base geometry) for a miss list of at most max_q queries: every piece streams ≥ 16 chunks
#ifdef FWAV_DEBUG_API
static int g_floor_p2 = 0;  // fwav_debug_topk_floor_pieces (debug library only; 0: by the launch's size)
#else
constexpr int g_floor_p2 = 0;
#endif
static void floor_plan(int64_t max_q, int64_t nd, int& rt, int& P) {
  rt = kFloorSplit;
  const int64_t pmax = cdiv(nd, kChunk) / 16;
  int cus, per_cu;
  topk_device_slots(kGeoBase, cus, per_cu);
  const int64_t blocks = cdiv(cdiv(max_q > 0 ? max_q : 1, 50), k16QB);  // ≈ 2 % of the launch, in 256-query blocks
  const int64_t slots = (int64_t)cus * per_cu;
  // 64 pieces where they fit one round, else as many from 16 to 32 as fit it (cfg2, ≈ 4,200–5,600 misses, 21–26
  // blocks expected: 19 pieces 13.82 vs 13.87–13.92 ms with 16, and 23 / 26 / 30 faster still on the misses of that
  // run, 17 blocks — but the floor's miss count varies run to run, so the round is sized for the 2 % estimate;
  // profiles/r06/floor_p2_sweep.log)
  const int64_t per = blocks > 0 ? slots / blocks : kFloorP2Fewest;
  const int p2 = g_floor_p2 > 0 ? g_floor_p2
                                : (per >= kFloorP2Fewest ? kFloorP2Fewest
                                                         : (int)std::max<int64_t>(kFloorP2, std::min<int64_t>(per, kFloorP2Few)));
  P = (int)std::max<int64_t>(1, std::min<int64_t>(p2, pmax));
}

// The pilots' sampled scores: workgroup (g, s) = (blockIdx.x % kPilotGroups, blockIdx.x / kPilotGroups) scores the 64
// pilots g·64 + lane (pilot p at active position p·n/kFloorPilots) against slice s of the sampled domains m·stride
// (1/kFloorSlices of them; its rows staged in LDS 256 at a time, every 4th row to each of the 4 waves), keeps each
// pilot's kFloorJ best per wave, merges the 4 waves' lists in LDS and writes them to scratch[(p·kFloorSlices + s)·kFloorJ
// + i] (pilot-major: k_floor_est reads a pilot's entries contiguously).  The dot products in packed f32 FMAs (a guess
// only: no reference order needed).  Round 5 put 2 pilots on each thread of 1,024 one-dimensional slices and wrote
// 16 MB of pilot-major entries in 32-B pieces 32 KB apart: 136 µs, plus 47 µs in k_floor_est.
constexpr int kPilotGroups = kFloorPilots / 64, kFloorSlices = 128;
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_floor_pilot(const float* __restrict__ emb, int64_t nd,
                                                     const int32_t* __restrict__ active,
                                                     const int32_t* __restrict__ n_active_p, int64_t q_offset,
                                                     int stride, float* __restrict__ scratch) {
  __shared__ float4 rows[256][4];
  __shared__ float lists[4][64][kFloorJ + 1];
  const int na = *n_active_p;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = blockIdx.x % kPilotGroups, sl = blockIdx.x / kPilotGroups;
  const int p = g * 64 + lane;
  const int64_t M = (nd + stride - 1) / stride;
  const int64_t m0 = M * sl / kFloorSlices, m1 = M * (sl + 1) / kFloorSlices;
  f32x2 q[8];
  {
    const int64_t pos = na > 0 ? (int64_t)p * na / kFloorPilots : 0;
    const int64_t row = na > 0 ? (int64_t)active[pos] + q_offset : 0;
    const float4* qp = reinterpret_cast<const float4*>(emb + row * 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 v = qp[k];
      q[2 * k] = f32x2{v.x, v.y};
      q[2 * k + 1] = f32x2{v.z, v.w};
    }
  }
  float top[kFloorJ];
#pragma unroll
  for (int k = 0; k < kFloorJ; ++k) top[k] = -INFINITY;
  for (int64_t mb = m0; mb < m1; mb += 256) {
    const int nr = (int)min<int64_t>(256, m1 - mb);
    __syncthreads();
    if ((int)threadIdx.x < nr) {
      const float4* rp = reinterpret_cast<const float4*>(emb + (mb + threadIdx.x) * stride * 16);
#pragma unroll
      for (int k = 0; k < 4; ++k) rows[threadIdx.x][k] = rp[k];
    }
    __syncthreads();
    for (int r = wave; r < nr; r += 4) {
      f32x2 acc = f32x2{0.0f, 0.0f};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 d = rows[r][k];
        acc = __builtin_elementwise_fma(q[2 * k], f32x2{d.x, d.y}, acc);
        acc = __builtin_elementwise_fma(q[2 * k + 1], f32x2{d.z, d.w}, acc);
      }
      float x = acc.x + acc.y;
      // sorted insertion into the pilot's top kFloorJ (descending), only for a score that enters it
      if (x > top[kFloorJ - 1]) {
#pragma unroll
        for (int k = 0; k < kFloorJ; ++k) {
          const float hi = fmaxf(top[k], x);
          x = fminf(top[k], x);
          top[k] = hi;
        }
      }
    }
  }
  // the 4 waves' lists of each pilot merged by wave 0
#pragma unroll
  for (int k = 0; k < kFloorJ; ++k) lists[wave][lane][k] = top[k];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int w = 1; w < 4; ++w)
#pragma unroll
      for (int i = 0; i < kFloorJ; ++i) {
        float x = lists[w][lane][i];
        if (x > top[kFloorJ - 1]) {
#pragma unroll
          for (int k = 0; k < kFloorJ; ++k) {
            const float hi = fmaxf(top[k], x);
            x = fminf(top[k], x);
            top[k] = hi;
          }
        }
      }
    float4* out = reinterpret_cast<float4*>(scratch + ((int64_t)p * kFloorSlices + sl) * kFloorJ);
    static_assert(kFloorJ == 8, "two float4 per list");
    out[0] = make_float4(top[0], top[1], top[2], top[3]);
    out[1] = make_float4(top[4], top[5], top[6], top[7]);
  }
}

// One wave per pilot (block = pilot): its j-th best score over all nwg slices (its estimate of its K-th score), to
// est[pilot].  Each lane keeps the top kFloorJ of its slices' entries; then kFloorJ rounds take the wave's largest
// head (the lowest lane holding it pops it).
__global__ __launch_bounds__(64) void k_floor_est(const float* __restrict__ scratch, int nwg, int j,
                                                  float* __restrict__ est) {
  const int lane = threadIdx.x;
  const float* sp = scratch + (int64_t)blockIdx.x * nwg * kFloorJ;
  float top[kFloorJ];
#pragma unroll
  for (int k = 0; k < kFloorJ; ++k) top[k] = -INFINITY;
  for (int e = lane; e < nwg * kFloorJ; e += 64) {
    float x = sp[e];
    if (x > top[kFloorJ - 1]) {
#pragma unroll
      for (int k = 0; k < kFloorJ; ++k) {
        const float hi = fmaxf(top[k], x);
        x = fminf(top[k], x);
        top[k] = hi;
      }
    }
  }
  float got = -INFINITY;
  for (int r = 0; r < j; ++r) {
    float m = top[0];
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    const uint64_t who = __ballot(top[0] == m);
    if (lane == __builtin_ctzll(who)) {
#pragma unroll
      for (int k = 0; k + 1 < kFloorJ; ++k) top[k] = top[k + 1];
      top[kFloorJ - 1] = -INFINITY;
    }
    got = m;
  }
  if (lane == 0) est[blockIdx.x] = got;
}

// The floors from the pilots' estimates: the rank-th smallest (key in f2key order; 0 = no floor: fewer than min_q
// active queries, or no finite estimate) and the smallest − kFloor2Margin for the second pass.
__global__ __launch_bounds__(kFloorPilots) void k_floor_reduce(const float* __restrict__ est_g, int rank,
                                                               const int32_t* __restrict__ n_active_p, int min_q,
                                                               float margin2, uint32_t* __restrict__ floor_key) {
  __shared__ float est[kFloorPilots];
  const int p = threadIdx.x;
  // a NaN estimate ranks as +inf (after every number), so each place 0 … kFloorPilots − 1 has exactly one owner and
  // both keys are always written (a non-finite one as 0: no floor)
  const float e0 = est_g[p];
  const float e = e0 == e0 ? e0 : INFINITY;
  est[p] = e;
  __syncthreads();
  // every pilot's place in (estimate, pilot) order: the one at place rank − 1 is the floor, the one at place 0 the
  // second pass's floor (+ kFloor2Margin)
  int place = 0;
  // (unrolled: the LDS reads are independent — the rolled loop waited on each one, 15 µs for 512 pilots)
#pragma unroll 32
  for (int i = 0; i < kFloorPilots; ++i) {
    const float x = est[i];
    place += (x < e || (x == e && i < p)) ? 1 : 0;
  }
  const int na = *n_active_p;
  const bool ok = na >= min_q && na > 0 && e > -INFINITY && e < INFINITY;
  if (place == rank - 1) floor_key[0] = ok ? f2key(e) : 0u;
  if (place == 0) floor_key[1] = ok ? f2key(e - margin2) : 0u;
}

// ------------------------------------------------------------------------------------ the active list in order
// The search works on its own copy of the active list in ascending query order, whatever order the caller's list is
// in: fwav_prune appends each wave's ranges (ascending) at an atomic offset, so its list is runs of 64 ascending
// ranges in arbitrary run order, and with it the first pass ran 2.30 instead of 1.90 ms for 41,344 queries at the
// same floor (round 6, tools/diag/topk_reps.py AB_RUNS=1 against ascending ranges, profiles/r06/active_order.log;
// the counters of the two runs' work — appends, level-2 pairs — are equal, so it is how the work lands on the
// workgroups, not how much of it there is: with ascending ids the interleaved query groups of every block are spread
// evenly over the queries, with runs in random order each block draws its 16 groups at random and the slowest block
// sets the launch).  A bitmap of the listed ids (duplicates collapse), one count per 8,192 ids, then every block
// writes its ids at its prefix: three small kernels, no host synchronisation.  A list holding an id outside
// [0, max_q) (max_q bounds the list's length, not its ids: a slice of a longer list) is used as given.
constexpr int kOrderWords = 256;  // bitmap words (8,192 query ids) per block of k_order_sum / k_order_emit
__host__ __device__ inline int64_t order_words(int64_t max_q) { return cdiv(max_q > 0 ? max_q : 1, 32); }
// n_order[1] (zeroed with the bitmap): set when an id lies outside [0, max_q)
__global__ __launch_bounds__(256) void k_order_mark(const int32_t* __restrict__ active,
                                                    const int32_t* __restrict__ n_active_p, int64_t max_q,
                                                    uint32_t* __restrict__ bits, int32_t* __restrict__ n_order) {
  const int64_t n = *n_active_p;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int32_t v = active[i];
    if (v >= 0 && v < max_q) atomicOr(bits + (v >> 5), 1u << (v & 31));
    else n_order[1] = 1;
  }
}
// an id outside [0, max_q): the caller's list as given
__global__ __launch_bounds__(256) void k_order_copy(const int32_t* __restrict__ active,
                                                    const int32_t* __restrict__ n_active_p,
                                                    int32_t* __restrict__ order, int32_t* __restrict__ n_order) {
  if (n_order[1] == 0) return;
  const int64_t n = *n_active_p;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) order[i] = active[i];
  if (blockIdx.x == 0 && threadIdx.x == 0) n_order[0] = (int32_t)n;
}
__device__ __forceinline__ int block_sum256(int c, int* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if (lane == 0) red[wave] = c;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
__global__ __launch_bounds__(256) void k_order_sum(const uint32_t* __restrict__ bits, int64_t nwords,
                                                   uint32_t* __restrict__ bsum) {
  __shared__ int red[4];
  const int64_t w = (int64_t)blockIdx.x * kOrderWords + threadIdx.x;
  const int t = block_sum256(w < nwords ? __popc(bits[w]) : 0, red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = (uint32_t)t;
}
__global__ __launch_bounds__(256) void k_order_emit(const uint32_t* __restrict__ bits, int64_t nwords,
                                                    const uint32_t* __restrict__ bsum, int32_t* __restrict__ order,
                                                    int32_t* __restrict__ n_order) {
  __shared__ int red[4], wsum[4];
  if (n_order[1] != 0) return;  // k_order_copy writes the list
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int before = 0;  // ids in the blocks before this one
  for (int b = tid; b < (int)blockIdx.x; b += 256) before += (int)bsum[b];
  before = block_sum256(before, red);
  const int64_t w = (int64_t)blockIdx.x * kOrderWords + tid;
  const uint32_t word = w < nwords ? bits[w] : 0u;
  const int c = __popc(word);
  int inc = c;  // inclusive prefix over the wave's lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int pos = before + inc - c;
  for (int k = 0; k < wave; ++k) pos += wsum[k];
  for (uint32_t m = word; m != 0u; m &= m - 1u) order[pos++] = (int32_t)(w * 32 + __builtin_ctz(m));
  if (blockIdx.x == gridDim.x - 1 && tid == 255) *n_order = pos;
}
// the caller's active list → order[0 .. *n_order), ascending (workspace regions of TopkLayout)
static void order_active(const int32_t* active, const int32_t* n_active, int64_t max_q, uint32_t* bits, uint32_t* bsum,
                         int32_t* order, int32_t* n_order, hipStream_t st) {
  const int64_t nw = order_words(max_q);
  const int64_t nb = cdiv(nw, kOrderWords);
  (void)hipMemsetAsync(bits, 0, (size_t)nw * sizeof(uint32_t), st);
  (void)hipMemsetAsync(n_order + 1, 0, sizeof(int32_t), st);
  const int64_t gm = std::min<int64_t>(cdiv(max_q > 0 ? max_q : 1, 256), 2048);
  k_order_mark<<<gm, 256, 0, st>>>(active, n_active, max_q, bits, n_order);
  k_order_sum<<<nb, 256, 0, st>>>(bits, nw, bsum);
  k_order_emit<<<nb, 256, 0, st>>>(bits, nw, bsum, order, n_order);
  k_order_copy<<<gm, 256, 0, st>>>(active, n_active, order, n_order);
}

// Key-buffer bytes: enough for the first pass in either geometry (a diagnostic override may switch it between the
// size query and the launch), for the relaunches' base plan and for the floor's second pass.
static size_t f16_keys_bytes(int64_t max_q, int64_t nd) {
  const int64_t q = max_q > 0 ? max_q : 1;
  size_t items_q = (size_t)make_plan(q, 0, 1, k16QB).items() * k16QB;
  {
    int rt2, P2;
    floor_plan(q, nd, rt2, P2);
    const size_t n2 = (size_t)make_plan(q, rt2, P2, k16QB).items() * k16QB;
    items_q = n2 > items_q ? n2 : items_q;
  }
  for (int geo = 0; geo < 8; ++geo) {  // each geometry with and without the floor (a debug knob may switch it)
    int rt, P;
    host_plan_for(q, nd, geo & 3, rt, P, geo >> 2);
    const int qb = geometry_qb(geo & 3);
    const size_t n = (size_t)make_plan(q, rt, P, qb).items() * qb;
    items_q = n > items_q ? n : items_q;
  }
  return items_q * k16Cap * sizeof(uint64_t);
}

// The fp16 search's workspace (K ≤ 64), in byte offsets from its start; one definition for the launch, the size query
// and fwav_debug_sim_topk_layout (tests read the tail through it, never by arithmetic of their own).
//   keys      u64 key buffers (f16_keys_bytes)        share   u32[q] shared band limits of split blocks
//   ovf2      i32[q] overflow list of the HL relaunch  n_ovf2  i32 count, then seeds2 u32[q]
//   ovf1      i32[q] overflow list of the first pass   n_ovf1  i32 count, then seeds1 u32[q]
//   miss      i32[q] floor misses of the first pass    n_miss  i32
//   miss2     i32[q] floor misses of the second pass   n_miss2 i32
//   floor_key u32[2]
//   order     i32[q] the active list in ascending query order (k_order_*), n_order i32[2] its length, a flag
//   order_bits u32[⌈q/32⌉] its bitmap                  order_bsum u32 per 8,192 queries: the bitmap's block counts
//   pilot     f32 pilot scores + estimates (only when the floor can run: floor_by_default, or any size in the debug
//             library)
struct TopkLayout {
  size_t keys, share, ovf2, n_ovf2, seeds2, ovf1, n_ovf1, seeds1, miss, n_miss, miss2, n_miss2, floor_key, order,
      n_order, order_bits, order_bsum, pilot, total;
};
constexpr size_t kPilotBytes = ((size_t)kFloorPilots * kFloorSlices * kFloorJ + kFloorPilots) * sizeof(float);
static TopkLayout topk_layout(int64_t max_q, int64_t nd) {
  const size_t q = (size_t)(max_q > 0 ? max_q : 1);
  TopkLayout L;
  L.keys = 0;
  L.share = f16_keys_bytes(max_q, nd);
  L.ovf2 = L.share + 4 * q;
  L.n_ovf2 = L.ovf2 + 4 * q;
  L.seeds2 = L.n_ovf2 + 4;
  L.ovf1 = L.seeds2 + 4 * q;
  L.n_ovf1 = L.ovf1 + 4 * q;
  L.seeds1 = L.n_ovf1 + 4;
  L.miss = L.seeds1 + 4 * q;
  L.n_miss = L.miss + 4 * q;
  L.miss2 = L.n_miss + 4;
  L.n_miss2 = L.miss2 + 4 * q;
  L.floor_key = L.n_miss2 + 4;
  L.order = L.floor_key + 8;
  L.n_order = L.order + 4 * q;
  L.order_bits = L.n_order + 8;
  L.order_bsum = L.order_bits + 4 * (size_t)order_words(q);
  L.pilot = L.order_bsum + 4 * (size_t)cdiv((int64_t)order_words(q), kOrderWords);
#ifdef FWAV_DEBUG_API
  const bool pilots = true;  // a debug knob may force the floor after the size query
#else
  const bool pilots = floor_by_default(max_q, nd);
#endif
  L.total = L.pilot + (pilots ? kPilotBytes : 0);
  return L;
}

template <int C>
static size_t topk_lds_bytes() {
  return (size_t)kTopkQ * C * sizeof(uint64_t) + 16 * kChunk * sizeof(float) + 3 * kTopkQ * sizeof(int);
}

template <int C>
static int launch_topk(const float* emb, const _Float16* emb16, int64_t nd, const int32_t* active,
                       const int32_t* n_active, int64_t max_q, int64_t q_offset, int K, int32_t* cand, hipStream_t st,
                       uint64_t* gkeys, SgemvSplit sp, int32_t* ties, int dbg = 0,
                       unsigned long long* stats = nullptr) {
  const int64_t grid = cdiv(max_q, kTopkQ);
  if (ties != nullptr) (void)hipMemsetAsync(ties, 0, sizeof(int32_t), st);
  if (grid == 0) return FWAV_OK;
  if (emb16 != nullptr) {
    if (gkeys == nullptr) {
      set_error("fwav_sim_topk: fp16 search needs its key workspace (fwav_sim_topk_workspace_size)");
      return FWAV_ERR_WORKSPACE;
    }
    const int64_t q1 = max_q > 0 ? max_q : 1;
    // workspace tail (TopkLayout): two overflow lists, each list[q], count, seeds u32[q] (seeds[i] = f2key of the
    // band limit of list[i]), the floor's miss lists, its keys and the pilots' scores
    const TopkLayout lay = topk_layout(max_q, nd);
    char* const wb = reinterpret_cast<char*>(gkeys);
    uint32_t* share = reinterpret_cast<uint32_t*>(wb + lay.share);  // u32[q]: shared band limits of split blocks
    int32_t* ovf2 = reinterpret_cast<int32_t*>(wb + lay.ovf2);
    int32_t* n_ovf2 = reinterpret_cast<int32_t*>(wb + lay.n_ovf2);
    int32_t* ovf1 = reinterpret_cast<int32_t*>(wb + lay.ovf1);
    int32_t* n_ovf1 = reinterpret_cast<int32_t*>(wb + lay.n_ovf1);
    const uint32_t* seeds1 = reinterpret_cast<const uint32_t*>(wb + lay.seeds1);
    const uint32_t* seeds2 = reinterpret_cast<const uint32_t*>(wb + lay.seeds2);
    (void)hipMemsetAsync(n_ovf1, 0, sizeof(int32_t), st);
    (void)hipMemsetAsync(n_ovf2, 0, sizeof(int32_t), st);
    // Geometry: k16Waves waves × k16Sets query sets of 32 per workgroup.  Measured at cfg2 (W, QS=1): W = 8
    // 27.9 ms, W = 7 31.6 ms, W = 6 44.5 ms — an even 4 waves per SIMD beats a fuller last round of workgroups.
#ifdef FWAV_DEBUG_API
    const bool stats_first = (stats != nullptr && !(dbg & (1 << 17))) || (dbg & 65535) != 0;
#else
    constexpr bool stats_first = false;  // counter / ablation launches: debug library only
    (void)dbg;
#endif
    // counter builds run the base geometry, or with dbg bit 18 the product's own (centroid) geometry
    const int geo = stats_first && !(dbg & (1 << 18)) ? kGeoBase : first_geometry(nd, max_q);
    const int mode1 = first_mode(nd);
    // the floor's miss lists (first and second pass), its two keys, the pilots' scores
    int32_t* miss = reinterpret_cast<int32_t*>(wb + lay.miss);
    int32_t* n_miss = reinterpret_cast<int32_t*>(wb + lay.n_miss);
    int32_t* miss2 = reinterpret_cast<int32_t*>(wb + lay.miss2);
    int32_t* n_miss2 = reinterpret_cast<int32_t*>(wb + lay.n_miss2);
    uint32_t* floor_key = reinterpret_cast<uint32_t*>(wb + lay.floor_key);
    float* pilot = reinterpret_cast<float*>(wb + lay.pilot);
    // One first pass (search + merge of split blocks) over act[0 .. *nact) in geometry g with plan (rt, P) and floor
    // fl; `diag`: the debug library's counter / ablation launches may replace the search
    // (with a floor the device runs the floor-free plan fl.alt_* when the floor did not apply: the grid, the shared
    // limits and the merge cover both plans)
    auto first_pass = [&](const int32_t* act, const int32_t* nact, int g, int rt, int P, FloorCtl fl, bool diag) {
      const TopkPlan pl0 = make_plan(max_q, rt, P, geometry_qb(g));
      const TopkPlan pla = fl.key != nullptr ? make_plan(max_q, fl.alt_rt, fl.alt_p, geometry_qb(g)) : pl0;
      struct {
        int64_t n, R;
        int P;
        int64_t items() const { return n; }
      } pl{std::max(pl0.items(), pla.items()), std::max(pl0.R, pla.R), std::max(pl0.P, pla.P)};
      if ((pl0.R > 0 && !pl0.halves) || (pla.R > 0 && !pla.halves))
        (void)hipMemsetAsync(share, 0, (size_t)q1 * sizeof(uint32_t), st);
#define FWAV_FIRST(MODE_, STATS_, DBG_, ST_)                                                                    \
  k_sim_topk_f16<k16Cap, STATS_, MODE_><<<pl.items(), 64 * k16Waves, 0, st>>>(                                  \
      emb16, emb, nd, act, nact, q_offset, K, cand, gkeys, ovf1, n_ovf1, share, nullptr, 0.0f, rt, P, DBG_, ST_,  \
      sp, ties, fl)
#define FWAV_FIRST_GEO(MODE_, W_, G_, QS_, CENT_)                                                               \
  k_sim_topk_f16<k16Cap, false, MODE_, W_, G_, QS_, CENT_><<<pl.items(), 64 * W_, 0, st>>>(                     \
      emb16, emb, nd, act, nact, q_offset, K, cand, gkeys, ovf1, n_ovf1, share, nullptr, 0.0f, rt, P, 0, nullptr, \
      sp, ties, fl)
      bool done = false;
      (void)diag;
#ifdef FWAV_DEBUG_API
      if (!done && diag && stats_first && g == kGeoCent) {
        if (mode1 == kModeHL)
          k_sim_topk_f16<k16Cap, true, kModeHL, kCentW, kCentG, kCentQS, true><<<pl.items(), 64 * kCentW, 0, st>>>(
              emb16, emb, nd, act, nact, q_offset, K, cand, gkeys, ovf1, n_ovf1, share, nullptr, 0.0f, rt, P,
              dbg & 65535, stats, sp, ties, fl);
        else
          k_sim_topk_f16<k16Cap, true, kModeS16, kCentW, kCentG, kCentQS, true><<<pl.items(), 64 * kCentW, 0, st>>>(
              emb16, emb, nd, act, nact, q_offset, K, cand, gkeys, ovf1, n_ovf1, share, nullptr, 0.0f, rt, P,
              dbg & 65535, stats, sp, ties, fl);
        done = true;
      } else if (!done && diag && stats_first) {
        if (mode1 == kModeHL) FWAV_FIRST(kModeHL, true, dbg & 65535, stats);
        else FWAV_FIRST(kModeS16, true, dbg & 65535, stats);
        done = true;
      }
#endif
      if (!done) {
        if (g == kGeoWide) {
          if (mode1 == kModeHL) FWAV_FIRST_GEO(kModeHL, kWideW, kWideG, 1, false);
          else FWAV_FIRST_GEO(kModeS16, kWideW, kWideG, 1, false);
        } else if (g == kGeoCent) {
          if (mode1 == kModeHL) FWAV_FIRST_GEO(kModeHL, kCentW, kCentG, kCentQS, true);
          else FWAV_FIRST_GEO(kModeS16, kCentW, kCentG, kCentQS, true);
        } else if (g == kGeoCentWide) {
          if (mode1 == kModeHL) FWAV_FIRST_GEO(kModeHL, kWideW, kWideG, kCentWideQS, true);
          else FWAV_FIRST_GEO(kModeS16, kWideW, kWideG, kCentWideQS, true);
        } else {
          if (mode1 == kModeHL) FWAV_FIRST(kModeHL, false, 0, nullptr); else FWAV_FIRST(kModeS16, false, 0, nullptr);
        }
      }
#undef FWAV_FIRST
#undef FWAV_FIRST_GEO
      if (pl.R > 0) {
        // one merge wave per split-block query
#define FWAV_MERGE_MP(QB_, HL_, MP_)                                                                            \
  k_merge_pieces<k16Cap, QB_, HL_, MP_><<<cdiv(pl.R * QB_, 4), 256, 0, st>>>(                                 \
      gkeys, act, nact, rt, P, K, cand, ovf1, n_ovf1, share, emb, q_offset, sp, ties, fl)
#define FWAV_MERGE(QB_, HL_)                                                                                    \
  do {                                                                                                          \
    if (pl.P <= 8) FWAV_MERGE_MP(QB_, HL_, 8);                                                                  \
    else if (pl.P <= 16) FWAV_MERGE_MP(QB_, HL_, 16);                                                           \
    else if (pl.P <= 32) FWAV_MERGE_MP(QB_, HL_, 32);                                                           \
    else FWAV_MERGE_MP(QB_, HL_, kMaxPieces);                                                                   \
  } while (0)
        if (g == kGeoWide) {
          if (mode1 == kModeHL) FWAV_MERGE(kWideQB, true); else FWAV_MERGE(kWideQB, false);
        } else if (g == kGeoCent) {
          if (mode1 == kModeHL) FWAV_MERGE(kCentQB, true); else FWAV_MERGE(kCentQB, false);
        } else if (g == kGeoCentWide) {
          if (mode1 == kModeHL) FWAV_MERGE(kCentWideQB, true); else FWAV_MERGE(kCentWideQB, false);
        } else {
          if (mode1 == kModeHL) FWAV_MERGE(k16QB, true); else FWAV_MERGE(k16QB, false);
        }
#undef FWAV_MERGE
#undef FWAV_MERGE_MP
      }
    };
    // Speculative floor (FloorCtl): from the exact scores of kFloorPilots evenly spaced queries against every
    // (K/8)-th domain (k_floor_pilot), a guess at the lowest K-th score of the search; the queries it may cut are
    // searched again at a lower floor, and the few that one cuts without any (base geometry, table pieces).
    // the centroid geometry's passes on the search's own ascending copy of the caller's active list (order_active;
    // every pass below reads it), where it was measured; the other geometries on the caller's order (ascending ids
    // are not better everywhere: cfg3's sliced search on ascending slices ran 373 instead of 347 ms per step,
    // profiles/r06/active_order/cfg3_*.log)
    const int32_t* order = active;
    const int32_t* n_order = n_active;
    if (geo == kGeoCent) {
      int32_t* const ord = reinterpret_cast<int32_t*>(wb + lay.order);
      int32_t* const n_ord = reinterpret_cast<int32_t*>(wb + lay.n_order);
      order_active(active, n_active, max_q, reinterpret_cast<uint32_t*>(wb + lay.order_bits),
                   reinterpret_cast<uint32_t*>(wb + lay.order_bsum), ord, n_ord, st);
      order = ord;
      n_order = n_ord;
    }
    const int fmode = floor_mode();
    // (counter launches run without the floor unless dbg bit 19 asks for the product's floor too)
    const bool use_floor = (!stats_first || (dbg & (1 << 19))) && K <= 64 && floor_by_default(max_q, nd);
    int rt, P;
    host_plan_for(max_q, nd, geo, rt, P, use_floor ? 1 : 0);
    FloorCtl fl{nullptr, nullptr, nullptr};
    if (use_floor) {
      (void)hipMemsetAsync(n_miss, 0, sizeof(int32_t), st);
      (void)hipMemsetAsync(n_miss2, 0, sizeof(int32_t), st);
      if (fmode == 1 || fmode == 3) {  // debug: a forced floor value (3: the second pass's too)
        (void)hipMemsetD32Async((hipDeviceptr_t)floor_key, (int)g_floor_key, 1, st);
        (void)hipMemsetD32Async((hipDeviceptr_t)(floor_key + 1), fmode == 3 ? (int)g_floor_key : 0, 1, st);
      } else {
        const int j = K < kFloorJ ? K : kFloorJ, stride = K / j;
        float* est = pilot + (size_t)kFloorPilots * kFloorSlices * kFloorJ;
        k_floor_pilot<<<kPilotGroups * kFloorSlices, 256, 0, st>>>(emb, nd, order, n_order, q_offset, stride, pilot);
        k_floor_est<<<kFloorPilots, 64, 0, st>>>(pilot, kFloorSlices, j, est);
        k_floor_reduce<<<1, kFloorPilots, 0, st>>>(est, g_floor_rank, n_order, fmode == 2 ? 0 : (int)kFloorMinQ,
                                                   g_floor2_margin, floor_key);
      }
      int rt_nf, P_nf;  // the plan when the device finds the floor does not apply
      host_plan_for(max_q, nd, geo, rt_nf, P_nf, 0);
      fl = FloorCtl{floor_key, miss, n_miss, rt_nf, P_nf};
    }
    first_pass(order, n_order, geo, rt, P, fl, true);
    if (use_floor) {
      int rt2, P2;
      floor_plan(max_q, nd, rt2, P2);
      first_pass(miss, n_miss, kGeoBase, rt2, P2, FloorCtl{floor_key + 1, miss2, n_miss2, rt2, P2}, false);
      first_pass(miss2, n_miss2, kGeoBase, rt2, P2, FloorCtl{nullptr, nullptr, nullptr}, false);
    }
    // Queries whose band overflowed the buffer (large groups of equal or nearly equal scores) are searched again by
    // the same kernel in a narrower mode, on the device-side overflow list (no host sync; a relaunch exits at once
    // when its list is empty): after an S16 first pass the HL mode, then the exact mode for what still overflows;
    // after an HL first pass the exact mode, whose compactions keep exactly the top K, so nothing overflows.
    const TopkPlan pl_re = make_plan(max_q, 0, 1, k16QB);
    const int32_t* ex_in = ovf1;
    const int32_t* ex_n = n_ovf1;
    const uint32_t* ex_seeds = seeds1;
    if (mode1 == kModeS16) {
      k_sim_topk_f16<k16Cap, false, kModeHL><<<pl_re.items(), 64 * k16Waves, 0, st>>>(
          emb16, emb, nd, ovf1, n_ovf1, q_offset, K, cand, gkeys, ovf2, n_ovf2, nullptr, seeds1, kStreamMargin, 0, 1, 0,
          nullptr, sp, ties, FloorCtl{nullptr, nullptr, nullptr});
      ex_in = ovf2;
      ex_n = n_ovf2;
      ex_seeds = seeds2;
    }
#ifdef FWAV_DEBUG_API
    if (stats != nullptr && (dbg & (1 << 17)))  // diagnostic: counters of the exact-mode relaunch only
      k_sim_topk_f16<k16Cap, true, kModeEX><<<pl_re.items(), 64 * k16Waves, 0, st>>>(
          emb16, emb, nd, ex_in, ex_n, q_offset, K, cand, gkeys, ovf2, n_ovf2, nullptr, ex_seeds, kStreamMargin, 0, 1, 0,
          stats, sp, ties, FloorCtl{nullptr, nullptr, nullptr});
    else
#endif
      k_sim_topk_f16<k16Cap, false, kModeEX><<<pl_re.items(), 64 * k16Waves, 0, st>>>(
          emb16, emb, nd, ex_in, ex_n, q_offset, K, cand, gkeys, ovf2, n_ovf2, nullptr, ex_seeds, kStreamMargin, 0, 1, 0,
          nullptr, sp, ties, FloorCtl{nullptr, nullptr, nullptr});
  } else {
    const size_t lds = topk_lds_bytes<C>();
    static bool attr32[kMaxDev] = {false};  // a function attribute is set per device
    const int dev = current_device();
    if (!attr32[dev]) {
      (void)hipFuncSetAttribute((const void*)k_sim_topk_f32<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr32[dev] = true;
    }
    k_sim_topk_f32<C><<<grid, kTopkThreads, lds, st>>>(emb, nd, active, n_active, q_offset, K, cand, sp, ties);
  }
  FWAV_LAUNCH_CHECK("fwav_sim_topk");
  return FWAV_OK;
}

// fwav_topk_large.hip (K > 64)
int64_t large_batch(int64_t nd, int64_t max_q);
size_t large_workspace_bytes(int64_t nd, int64_t max_q);
int launch_topk_large(const float* emb, int64_t nd, const int32_t* active, const int32_t* n_active, int64_t max_q,
                      int64_t q_offset, int K, int32_t* cand, float* S, SgemvSplit sp, int32_t* ties, hipStream_t st);
int launch_score_rows(const float* emb, int64_t nd, const int32_t* rows, int64_t n_rows, int64_t q_offset,
                      SgemvSplit sp, float* S, hipStream_t st);

}  // namespace fwav

using namespace fwav;

extern "C" {

int fwav_topk_max_k(void) { return 4096; }

int64_t fwav_tie_list_size(int64_t max_q) { return 1 + (int64_t)kTieRec * (max_q > 0 ? max_q : 1); }

// Workspace of fwav_sim_topk: for K <= 64 the fp16 search's global key buffers (max_q queries), for K > 64
// the score rows of one query batch (≤ 1 GiB).
size_t fwav_sim_topk_workspace_size(int64_t max_q, int64_t n_domains, int k) {
  const int64_t q = max_q > 0 ? max_q : 1;
  if (k > 64) return large_workspace_bytes(n_domains, q);
  // key buffers, shared limits u32[q], two overflow lists (list, count, seeds), the floor's two miss lists (list,
  // count), its two keys, the pilots' scores when the floor can run (TopkLayout)
  return topk_layout(q, n_domains).total;
}

// Exact top-K over all nd domains for the local queries listed in active[0 .. *n_active) (device count,
// at most max_q); local query i uses embedding row q_offset + i and writes cand row i.  Rows of queries
// not listed are not touched.  emb16 (tiled fp16 copy from fwav_pool_embed) selects the fp16 pre-filter
// kernel; NULL runs the all-f32-MFMA kernel.  Both return identical candidates.
int fwav_sim_topk(const float* emb, const void* emb16, int64_t nd, const int32_t* active, const int32_t* n_active,
                  int64_t max_q, int64_t q_offset, int K, int blas_threads, int32_t* cand, int32_t* ties,
                  void* workspace, size_t ws_bytes, void* stream) {
  FWAV_CHECK_ARG(emb && active && n_active && cand && nd > 0 && max_q >= 0, FWAV_ERR_ARG, "fwav_sim_topk: bad args");
  FWAV_CHECK_ARG(blas_threads >= 1 && blas_threads <= 4096, FWAV_ERR_ARG, "fwav_sim_topk: blas_threads outside [1, 4096]");
  FWAV_CHECK_ARG(K >= 1 && K <= fwav_topk_max_k(), FWAV_ERR_K, "fwav_sim_topk: K=%d outside [1, %d]", K,
                 fwav_topk_max_k());
  FWAV_CHECK_ARG(nd < (int64_t)0x7fffffff, FWAV_ERR_SHAPE, "fwav_sim_topk: nd too large");
  hipStream_t st = (hipStream_t)stream;
  if (K > 64) {
    FWAV_CHECK_ARG(workspace && ws_bytes >= fwav_sim_topk_workspace_size(max_q, nd, K), FWAV_ERR_WORKSPACE,
                   "fwav_sim_topk: workspace too small");
    if (ties != nullptr) (void)hipMemsetAsync(ties, 0, sizeof(int32_t), st);
    if (max_q == 0) return FWAV_OK;
    return launch_topk_large(emb, nd, active, n_active, max_q, q_offset, K, cand, (float*)workspace,
                             make_sgemv_split(nd, blas_threads), ties, st);
  }
  FWAV_CHECK_ARG(emb16 == nullptr || (workspace && ws_bytes >= fwav_sim_topk_workspace_size(max_q, nd, K)),
                 FWAV_ERR_WORKSPACE, "fwav_sim_topk: workspace too small");
  return launch_topk<128>(emb, (const _Float16*)emb16, nd, active, n_active, max_q, q_offset, K, cand, st,
                          (uint64_t*)workspace, make_sgemv_split(nd, blas_threads), ties);
}

// Exact reference score rows for the host's tie resolution: scores[i·nd + d] = emb[d] · emb[q_offset + rows[i]] in
// the reference's sgemv order for `blas_threads` OpenBLAS threads (fractal.py:537).
int fwav_score_rows(const float* emb, int64_t nd, const int32_t* rows, int64_t n_rows, int64_t q_offset,
                    int blas_threads, float* scores, void* stream) {
  FWAV_CHECK_ARG(emb && rows && scores && nd > 0 && nd < (int64_t)0x7fffffff && n_rows >= 0, FWAV_ERR_ARG,
                 "fwav_score_rows: bad args");
  FWAV_CHECK_ARG(blas_threads >= 1 && blas_threads <= 4096, FWAV_ERR_ARG, "fwav_score_rows: blas_threads outside [1, 4096]");
  if (n_rows == 0) return FWAV_OK;
  return launch_score_rows(emb, nd, rows, n_rows, q_offset, make_sgemv_split(nd, blas_threads), scores,
                           (hipStream_t)stream);
}

#ifdef FWAV_DEBUG_API  // ---- debug library only (include/fwav_debug.h)
// Diagnostic ablations of the fp16 search kernel (timing only; see k_sim_topk_f16 `dbg`).
int fwav_debug_sim_topk(const float* emb, const void* emb16, int64_t nd, const int32_t* active, const int32_t* n_active,
                        int64_t max_q, int64_t q_offset, int K, int32_t* cand, void* workspace, size_t ws_bytes, int dbg,
                        unsigned long long* stats, void* stream) {
  FWAV_CHECK_ARG(emb && emb16 && workspace && K >= 1 && K <= 64, FWAV_ERR_ARG, "fwav_debug_sim_topk: bad args");
  // the key buffers depend on the work plan of THIS max_q (a split plan for fewer queries can need more than a
  // whole-block plan for more): a workspace sized for another query count once ran off its end
  FWAV_CHECK_ARG(ws_bytes >= fwav_sim_topk_workspace_size(max_q, nd, K), FWAV_ERR_WORKSPACE,
                 "fwav_debug_sim_topk: workspace too small for max_q=%lld", (long long)max_q);
  return launch_topk<128>(emb, (const _Float16*)emb16, nd, active, n_active, max_q, q_offset, K, cand,
                          (hipStream_t)stream, (uint64_t*)workspace, make_sgemv_split(nd, 1), nullptr, dbg, stats);
}

// Diagnostic override of the first pass's mode: 0 = S16 (→ HL → exact relaunches), 1 = HL (→ exact), −1 = by table
// size (default).  Every mode returns the same candidates.
int fwav_debug_topk_mode(int mode) {
  FWAV_CHECK_ARG(mode >= -1 && mode <= 1, FWAV_ERR_ARG, "fwav_debug_topk_mode: mode outside [-1, 1]");
  g_first_mode = mode;
  return FWAV_OK;
}

// Diagnostic override of the first pass's geometry: 0 = base (8 waves, 256 queries per workgroup), 1 = wide (16
// waves, 512 queries, one workgroup per CU), −1 = by table size (default).  Both return the same candidates.
int fwav_debug_topk_geometry(int wide) {
  FWAV_CHECK_ARG(wide >= -1 && wide <= 3, FWAV_ERR_ARG, "fwav_debug_topk_geometry: outside [-1, 3]");
  g_wide = wide;
  return FWAV_OK;
}

// Diagnostic override of the speculative floor (include/fwav_debug.h).
int fwav_debug_topk_floor(int mode, float value) {
  FWAV_CHECK_ARG(mode >= -1 && mode <= 4, FWAV_ERR_ARG, "fwav_debug_topk_floor: mode outside [-1, 4]");
  FWAV_CHECK_ARG(mode != 4 || (value >= 0.0f && value < 4.0f), FWAV_ERR_ARG,
                 "fwav_debug_topk_floor: the second pass's margin must lie in [0, 4)");
  FWAV_CHECK_ARG((mode != 1 && mode != 3) || (value == value && value > -INFINITY && value < INFINITY), FWAV_ERR_ARG,
                 "fwav_debug_topk_floor: the forced floor must be finite");
  g_floor_mode = mode == 4 ? 2 : mode;
  g_floor2_margin = mode == 4 ? value : kFloor2Margin;
  g_floor_rank = mode == 2 && value >= 1.0f && value <= (float)kFloorPilots ? (int)value : kFloorRank;
  uint32_t u;
  std::memcpy(&u, &value, sizeof u);
  g_floor_key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // f2key
  return FWAV_OK;
}

// Diagnostic override of the floor's second-pass table pieces per split block (1 … 32; 0: by the launch's size, the
// default).  Re-query fwav_sim_topk_workspace_size afterwards.
int fwav_debug_topk_floor_pieces(int p2) {
  FWAV_CHECK_ARG(p2 >= 0 && p2 <= kMaxPieces, FWAV_ERR_ARG, "fwav_debug_topk_floor_pieces: outside [0, %d]", kMaxPieces);
  g_floor_p2 = p2;
  return FWAV_OK;
}

// Host-side check of the work plan (no device needed): for every item of the plan of n queries (rt, pieces as in
// fwav_debug_topk_plan; wide: the 16-wave geometry) and every query slot its workgroup runs, count[position] += 1.
// A query of a whole-table block or a query half must be counted once, one of a block split into P table pieces P
// times.  *items = the launch's grid.
int fwav_debug_topk_plan_cover(int64_t n, int rt, int pieces, int wide, int32_t* count, int64_t* items) {
  FWAV_CHECK_ARG(n >= 0 && count && items && wide >= 0 && wide <= 3 &&
                     (pieces == -1 || (pieces >= 1 && pieces <= kMaxPieces)), FWAV_ERR_ARG,
                 "fwav_debug_topk_plan_cover: bad args");  // (any plan's pieces: the floor's later passes take 16)
  const int geo = wide;  // 0 base, 1 wide, 2 centroid, 3 centroid wide
  const int W = (geo == kGeoWide || geo == kGeoCentWide) ? kWideW : (geo == kGeoCent ? kCentW : k16Waves);
  const int sets = geo == kGeoCent ? kCentQS : (geo == kGeoCentWide ? kCentWideQS : k16Sets), qb = 32 * W * sets;
  const TopkPlan pl = make_plan(n, rt, pieces, qb);
  *items = pl.items();
  for (int64_t it = 0; it < pl.items(); ++it) {
    int64_t block;
    int piece, np, qhalf;
    plan_item(pl, it, block, piece, np, qhalf);
    if (block >= pl.nb) continue;
    const int wact = qhalf < 0 ? W : W / 2;
    const int qslot0 = qhalf > 0 ? (W / 2) * sets * 32 : 0;
    for (int ql = 0; ql < wact * sets * 32; ++ql) {
      const int64_t qi = slot_query(block, qslot0 + ql, pl.nb, qb);
      if (qi < n) ++count[qi];
    }
  }
  return FWAV_OK;
}

// The first pass fwav_sim_topk would launch for max_q queries over nd domains on the current device (no launch):
// geometry (1 = wide), first-pass mode (0 = S16, 1 = HL), whole-table blocks F, split blocks R, pieces P (−1: query
// halves), grid.
// The default first-pass plan's chunk range of every table piece of split block `block` (mod the split blocks;
// piece_chunks, with the floor as the launch would decide it): c01[2p], c01[2p + 1] = [c0, c1) of piece p < *np (at
// most kMaxPieces); *np = 1 for an unsplit plan.
int fwav_debug_topk_piece_chunks(int64_t max_q, int64_t nd, int64_t block, int32_t* c01, int32_t* np) {
  FWAV_CHECK_ARG(max_q > 0 && nd > 0 && block >= 0 && c01 && np, FWAV_ERR_ARG, "fwav_debug_topk_piece_chunks: bad args");
  const int geo = first_geometry(nd, max_q);
  int rt, P;
  host_plan_for(max_q, nd, geo, rt, P);
  const TopkPlan pl = make_plan(max_q, rt, P, geometry_qb(geo));
  const int n = pl.halves || pl.R == 0 ? 1 : pl.P;
  const int nchunks = (int)cdiv(nd, kChunk);
  const int64_t b = pl.F + (pl.R > 0 ? block % pl.R : 0);  // a split block
  for (int p = 0; p < n; ++p) piece_chunks(pl, b, p, n, nchunks, c01[2 * p], c01[2 * p + 1]);
  *np = n;
  return FWAV_OK;
}

int fwav_debug_topk_plan_info(int64_t max_q, int64_t nd, int32_t* info, int64_t* blocks) {
  FWAV_CHECK_ARG(max_q >= 0 && nd > 0 && info && blocks, FWAV_ERR_ARG, "fwav_debug_topk_plan_info: bad args");
  const int geo = first_geometry(nd, max_q);
  int rt, P;
  host_plan_for(max_q, nd, geo, rt, P);
  const TopkPlan pl = make_plan(max_q, rt, P, geometry_qb(geo));
  info[0] = geo;
  info[1] = first_mode(nd);
  info[2] = pl.halves ? -1 : pl.P;
  blocks[0] = pl.F;
  blocks[1] = pl.R;
  blocks[2] = pl.items();
  return FWAV_OK;
}

// Queries per block (one workgroup's query slots) of first-pass geometry geo (0 base, 1 wide, 2 centroid).
int64_t fwav_debug_topk_qb(int geo) { return geo >= 0 && geo <= 3 ? geometry_qb(geo) : -1; }

// Byte offsets of the fp16 search's workspace regions for max_q queries over nd domains (K ≤ 64), in the order of
// TopkLayout: keys, share, ovf2, n_ovf2, seeds2, ovf1, n_ovf1, seeds1, miss, n_miss, miss2, n_miss2, floor_key,
// pilot, total (15 values; total = fwav_sim_topk_workspace_size of this library).
int fwav_debug_sim_topk_layout(int64_t max_q, int64_t nd, int64_t* offsets) {
  FWAV_CHECK_ARG(max_q >= 0 && nd > 0 && offsets, FWAV_ERR_ARG, "fwav_debug_sim_topk_layout: bad args");
  const TopkLayout L = topk_layout(max_q > 0 ? max_q : 1, nd);
  const size_t v[19] = {L.keys,      L.share, L.ovf2,    L.n_ovf2,     L.seeds2,     L.ovf1,  L.n_ovf1,
                        L.seeds1,    L.miss,  L.n_miss,  L.miss2,      L.n_miss2,    L.floor_key, L.order,
                        L.n_order,   L.order_bits,       L.order_bsum, L.pilot,      L.total};
  for (int i = 0; i < 19; ++i) offsets[i] = (int64_t)v[i];
  return FWAV_OK;
}

// Diagnostic override of the fp16 search's work plan (rt < 0: default policy).  Re-query
// fwav_sim_topk_workspace_size after changing it.
int fwav_debug_topk_tail(int wb) {
  FWAV_CHECK_ARG(wb >= -1 && wb <= 31, FWAV_ERR_ARG, "fwav_debug_topk_tail: weight outside [-1, 31]");
  g_tail_wb = wb;
  return FWAV_OK;
}

int fwav_debug_topk_plan(int rt, int pieces) {
  FWAV_CHECK_ARG(pieces == -1 || (pieces >= 1 && pieces <= kMaxPieces), FWAV_ERR_ARG,
                 "fwav_debug_topk_plan: pieces outside [1, %d] (or -1: query halves)", kMaxPieces);
  g_plan_rt = rt;
  g_plan_p = rt < 0 ? -1 : pieces;
  return FWAV_OK;
}

#endif  // FWAV_DEBUG_API

}  // extern "C"
