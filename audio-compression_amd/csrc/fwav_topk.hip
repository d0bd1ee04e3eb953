// fwav_topk.hip — fused similarity GEMM + streaming exact top-K on MFMA (gfx950).
//
// Replaces (reference /root/reference/fractal.py):
//   cpu_worker                          :556-632  per range: q = emb[i] (quirk Q1), linear search, pad to K
//   range_candidates_from_embedding_emb :535-541  scores = E_dom @ q ; argpartition top-K ; sort desc
//   pad_candidates                      :544-552
//
// Contract: for every active query q (a range index; its query vector is domain-embedding row q), write
// the K domains with the largest f32 score  s(q,d) = fma-chain_{k=0..15}(emb[d][k]·emb[q][k])  in order
// (score desc, index asc), −1-padded when nd < K.  The reference scores with BLAS sgemv, whose summation
// order differs, so candidate parity is defined up to near-ties (SURVEY Appendix A rule 3).
//
// The n_ranges × n_domains score matrix (4.4e11 entries at cfg2) is never materialised.
// Workgroup = 4 waves × 32 queries.  Per wave and 32-domain tile:
//   * MFMA f32 32x32x2 ×8 (k = 16), domains as A rows (staged transposed in LDS, shared by the 4 waves),
//     queries as B columns (registers for the whole stream): lane l owns query l&31 and 16 domain rows,
//     so the running threshold θ is ONE register per lane.
//   * threshold test: max of the lane's 16 scores vs θ (v_max3 tree + 1 compare); only when some lane
//     passes does the wave append (score, index) keys to that query's LDS buffer (capacity C).
//   * when a buffer holds more than C − 32 entries the wave sorts it (64-lane bitonic on 64-bit keys),
//     keeps the top K and sets θ to the K-th score.  Domains stream in increasing index order, so a
//     later domain whose score equals θ can never displace an earlier one: strict '>' is exact.
// The chunk for the next iteration is prefetched into registers while the current one is consumed.
#include "fwav_common.h"

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

// Sort query ql's buffer, keep the top K, update count and θ.  Whole wave, uniform ql.
template <int C>
__device__ __forceinline__ void compact(uint64_t* __restrict__ keys, int* __restrict__ cnt, float* __restrict__ theta,
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
}

template <int C>
__global__ __launch_bounds__(kTopkThreads) void k_sim_topk_f32(const float* __restrict__ emb, int64_t nd,
                                                               const int32_t* __restrict__ active,
                                                               const int32_t* __restrict__ n_active_p,
                                                               int64_t q_offset, int K, int32_t* __restrict__ cand) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* keys = (uint64_t*)smem;                            // [kTopkQ][C]
  float* lda = (float*)(keys + (size_t)kTopkQ * C);            // [16][kChunk]
  int* cnt = (int*)(lda + 16 * kChunk);                        // [kTopkQ]
  float* theta = (float*)(cnt + kTopkQ);                       // [kTopkQ]

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

  float b[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) b[s] = q >= 0 ? emb[((int64_t)q + q_offset) * 16 + 2 * s + h] : 0.0f;
  float th = q >= 0 ? -INFINITY : INFINITY;  // invalid lanes never append
  if (tid < kTopkQ) {
    cnt[tid] = 0;
    theta[tid] = -INFINITY;
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
    for (int j = 0; j < 4; ++j) {
      lda[(4 * j + 0) * kChunk + tid] = pf[j].x;
      lda[(4 * j + 1) * kChunk + tid] = pf[j].y;
      lda[(4 * j + 2) * kChunk + tid] = pf[j].z;
      lda[(4 * j + 3) * kChunk + tid] = pf[j].w;
    }
    __syncthreads();
    if (c + 1 < nchunks) load_chunk(c + 1);
    const int64_t dbase = c * kChunk;

    for (int t = 0; t < kChunk / 32; ++t) {
      floatx16 acc = {};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const float a = lda[(2 * s + h) * kChunk + t * 32 + col];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[s], acc, 0, 0, 0);
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
      if (__ballot(mx > th) != 0ull) {
        uint64_t* kq = keys + (size_t)ql * C;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (acc[r] > th) {
            const int slot = atomicAdd(&cnt[ql], 1);
            kq[slot] = make_key(acc[r], (int32_t)(d0 + (r & 3) + 8 * (r >> 2)));
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        uint64_t need = __ballot(lane < 32 && cnt[ql] > C - 32);
        while (need != 0ull) {
          const int l = __builtin_ctzll(need);
          need &= need - 1;
          compact<C>(keys, cnt, theta, wave * 32 + l, K);
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
    compact<C>(keys, cnt, theta, qs, K);
    const int n = cnt[qs];
    int32_t* out = cand + (int64_t)qid * K;
    for (int e = lane; e < K; e += 64) out[e] = e < n ? key_idx(keys[(size_t)qs * C + e]) : -1;
  }
}

template <int C>
static size_t topk_lds_bytes() {
  return (size_t)kTopkQ * C * sizeof(uint64_t) + 16 * kChunk * sizeof(float) + 2 * kTopkQ * sizeof(int);
}

template <int C>
static int launch_topk(const float* emb, int64_t nd, const int32_t* active, const int32_t* n_active, int64_t max_q,
                       int64_t q_offset, int K, int32_t* cand, hipStream_t st) {
  const size_t lds = topk_lds_bytes<C>();
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_sim_topk_f32<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const int64_t grid = cdiv(max_q, kTopkQ);
  if (grid == 0) return FWAV_OK;
  k_sim_topk_f32<C><<<grid, kTopkThreads, lds, st>>>(emb, nd, active, n_active, q_offset, K, cand);
  FWAV_LAUNCH_CHECK("fwav_sim_topk");
  return FWAV_OK;
}

}  // namespace fwav

using namespace fwav;

extern "C" {

int fwav_topk_max_k(void) { return 64; }

// Exact top-K over all nd domains for the local queries listed in active[0 .. *n_active) (device count,
// at most max_q); local query i uses embedding row q_offset + i and writes cand row i.  Rows of queries
// not listed are not touched.
int fwav_sim_topk(const float* emb, int64_t nd, const int32_t* active, const int32_t* n_active, int64_t max_q,
                  int64_t q_offset, int K, int32_t* cand, void* stream) {
  FWAV_CHECK_ARG(emb && active && n_active && cand && nd > 0 && max_q >= 0, FWAV_ERR_ARG, "fwav_sim_topk: bad args");
  FWAV_CHECK_ARG(K >= 1 && K <= 64, FWAV_ERR_K, "fwav_sim_topk: K=%d outside [1, 64] (use fwav_sim_topk_large)", K);
  FWAV_CHECK_ARG(nd < (int64_t)0x7fffffff, FWAV_ERR_SHAPE, "fwav_sim_topk: nd too large");
  hipStream_t st = (hipStream_t)stream;
  return launch_topk<128>(emb, nd, active, n_active, max_q, q_offset, K, cand, st);
}

}  // extern "C"
