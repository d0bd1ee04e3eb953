// fwav_decode.hip — iterative decompression (apply-transform loop), bit-exact, device-side convergence.
//
// Replaces (reference /root/reference/fractal.py):
//   decompress_audio :1378-1473
//     setup  :1391-1408  idx/s/o/sym; sentinel idx < 0 → tile 0 zeroed, s = o = 0, sym = False
//     loop   :1411-1467  T = D[idx] (mirrored per sym); s_opt = <rec − mean rec, T − mean T> / ‖T − mean T‖²
//                        where ‖·‖² > 1e-12 else 0; s_used = damping > 0 ? (1−d)s_st + d·s_opt
//                        : (valid ? s_opt : s_st); clip ±s_clip; next = s_used·T + o (bincount → +0.0 + x);
//                        Δ = ‖next − rec‖ / (‖rec‖ or 1); stop when Δ < eps.
//
// T, mean(T), ‖T − mean T‖² and `valid` do not change across iterations: k_decode_prepare computes them
// once.  Each iteration is one k_decode_iter launch (thread per range, f64 block partials of ‖rec‖² and
// ‖next − rec‖²) and one single-block k_decode_check that sums the partials in a fixed order, records Δ and
// raises a device flag; every later launch sees the flag and exits, so all `iterations` launches are
// queued with no host synchronisation.  Δ is f64 here (BLAS sdot in the reference): only the early-exit
// decision can differ, and only when Δ lies within rounding of eps.
// Bytes per range per iteration: 4·rs (rec) + 4·rs (next) + 4·rs (T) + 16 (mean, den, s, o) + 1 (valid).
#include "fwav_common.h"
#include "../../include/fwav.h"

namespace fwav {

constexpr int kDecThreads = 256;

template <int RS>
__global__ void k_decode_prepare(const int32_t* __restrict__ idx, const float* __restrict__ s_in,
                                 const float* __restrict__ o_in, const uint8_t* __restrict__ sym_in, int64_t nr,
                                 int rs_rt, const float* __restrict__ pool, float* __restrict__ T,
                                 float* __restrict__ md, float* __restrict__ den, float* __restrict__ sst,
                                 float* __restrict__ ost, uint8_t* __restrict__ valid) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  const int rs = RS > 0 ? RS : rs_rt;
  const int32_t i0 = idx[r];
  const bool inval = i0 < 0;
  const bool sym = inval ? false : (sym_in[r] != 0);
  const float* D = pool + (int64_t)(inval ? 0 : i0) * rs;
  float* Tr = T + r * rs;
  for (int i = 0; i < rs; ++i) Tr[i] = inval ? 0.0f : (sym ? D[rs - 1 - i] : D[i]);
  auto ft = [&](int i) { return Tr[i]; };
  const float m = pw_sum(ft, rs) / (float)rs;
  auto fd = [&](int i) {
    const float t = Tr[i] - m;
    return t * t;
  };
  const float dd = pw_sum(fd, rs);
  md[r] = m;
  den[r] = dd;
  valid[r] = dd > 1e-12f;
  sst[r] = inval ? 0.0f : s_in[r];
  ost[r] = inval ? 0.0f : o_in[r];
}

template <int RS>
__global__ __launch_bounds__(kDecThreads) void k_decode_iter(
    const float* __restrict__ T, const float* __restrict__ md, const float* __restrict__ den,
    const float* __restrict__ sst, const float* __restrict__ ost, const uint8_t* __restrict__ valid, int64_t nr,
    int rs_rt, float s_clip, float c_keep, float c_opt, int use_damping, const float* __restrict__ rec,
    float* __restrict__ nxt, double* __restrict__ partial, const int* __restrict__ done) {
  __shared__ double red[2][kDecThreads / kWave];
  if (*done) return;
  const int rs = RS > 0 ? RS : rs_rt;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double rn = 0.0, dn = 0.0;
  if (r < nr) {
    const float* Tr = T + r * rs;
    const float* Rr = rec + r * rs;
    float* Nr = nxt + r * rs;
    const float m = md[r];
    auto fr = [&](int i) { return Rr[i]; };
    const float mr = pw_sum(fr, rs) / (float)rs;
    auto fn = [&](int i) { return (Rr[i] - mr) * (Tr[i] - m); };
    const float num = pw_sum(fn, rs);
    const bool v = valid[r] != 0;
    const float s_opt = v ? num / den[r] : 0.0f;
    float su = use_damping ? c_keep * sst[r] + c_opt * s_opt : (v ? s_opt : sst[r]);
    su = clip_sym(su, s_clip);
    const float o = ost[r];
    for (int i = 0; i < rs; ++i) {
      const float x = 0.0f + (su * Tr[i] + o);
      const float old = Rr[i];
      const float df = x - old;
      Nr[i] = x;
      rn += (double)old * (double)old;
      dn += (double)df * (double)df;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    rn += __shfl_xor(rn, o);
    dn += __shfl_xor(dn, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = rn;
    red[1][threadIdx.x >> 6] = dn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int j = 0; j < kDecThreads / kWave; ++j) {
      a += red[0][j];
      b += red[1][j];
    }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
}

// One block: Δ for iteration `it`, convergence flag, iteration counter.  state: int done, int iters_run.
__global__ void k_decode_check(const double* __restrict__ partial, int nblocks, int it, double eps,
                               int* __restrict__ state, double* __restrict__ deltas) {
  __shared__ double red[2][1024 / kWave];
  if (state[0]) return;
  double a = 0.0, b = 0.0;
  for (int j = threadIdx.x; j < nblocks; j += blockDim.x) {
    a += partial[2 * j];
    b += partial[2 * j + 1];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double rn = 0.0, dn = 0.0;
    for (int j = 0; j < (int)(blockDim.x / kWave); ++j) {
      rn += red[0][j];
      dn += red[1][j];
    }
    const double nrm = sqrt(rn);
    const double delta = sqrt(dn) / (nrm > 0.0 ? nrm : 1.0);
    deltas[it] = delta;
    state[1] = it + 1;
    if (delta < eps) state[0] = 1;
  }
}

}  // namespace fwav

using namespace fwav;

extern "C" {

size_t fwav_decode_workspace_size(int64_t nr, int rs, int iterations) {
  const int64_t nb = cdiv(nr > 0 ? nr : 1, kDecThreads);
  return (size_t)(nr * rs * 4 * 3 + nr * 4 * 4 + nr + 64 + nb * 2 * 8 + 64);
}

// Full decode loop.  recon_a / recon_b: f32[nr*rs] ping-pong buffers (recon_a is zeroed here); after the
// call, iteration count state[1] = t selects the result: t odd → recon_b, t even → recon_a.
// deltas: f64[iterations].  state: int[2] on device.
int fwav_decode(const int32_t* idx, const float* s_in, const float* o_in, const uint8_t* sym, int64_t nr, int rs,
                const float* pool, int64_t nd, int iterations, double eps, float s_clip, double s_damping,
                float* recon_a, float* recon_b, double* deltas, int* state, void* workspace, size_t ws_bytes,
                void* stream) {
  FWAV_CHECK_ARG(idx && s_in && o_in && sym && pool && recon_a && recon_b && state, FWAV_ERR_ARG,
                 "fwav_decode: null pointer");
  FWAV_CHECK_ARG(nr >= 0 && rs >= 1 && rs <= kMaxPairwise && iterations >= 0, FWAV_ERR_SHAPE, "fwav_decode: shape");
  FWAV_CHECK_ARG(ws_bytes >= fwav_decode_workspace_size(nr, rs, iterations) && workspace, FWAV_ERR_WORKSPACE,
                 "fwav_decode: workspace too small");
  FWAV_CHECK_ARG(iterations == 0 || deltas, FWAV_ERR_ARG, "fwav_decode: deltas required");
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(state, 0, 2 * sizeof(int), st);
  if (nr == 0) return FWAV_OK;
  (void)hipMemsetAsync(recon_a, 0, (size_t)nr * rs * sizeof(float), st);
  char* w = (char*)workspace;
  float* T = (float*)w;
  float* md = T + nr * rs;
  float* den = md + nr;
  float* sst = den + nr;
  float* ost = sst + nr;
  uint8_t* valid = (uint8_t*)(ost + nr);
  double* partial = (double*)(((uintptr_t)(valid + nr) + 63) & ~(uintptr_t)63);
  const int64_t nb = cdiv(nr, kDecThreads);
  const float c_keep = (float)(1.0 - s_damping);  // Python float (1.0 - d) meets an f32 array (NEP 50)
  const float c_opt = (float)s_damping;
  const int use_d = s_damping > 0.0;
  const float clipc = fabsf(s_clip);
#define FWAV_DEC(RSV)                                                                                             \
  do {                                                                                                            \
    k_decode_prepare<RSV><<<nb, kDecThreads, 0, st>>>(idx, s_in, o_in, sym, nr, rs, pool, T, md, den, sst, ost,  \
                                                      valid);                                                     \
    for (int it = 0; it < iterations; ++it) {                                                                     \
      const float* rec = (it & 1) ? recon_b : recon_a;                                                            \
      float* nx = (it & 1) ? recon_a : recon_b;                                                                   \
      k_decode_iter<RSV><<<nb, kDecThreads, 0, st>>>(T, md, den, sst, ost, valid, nr, rs, clipc, c_keep, c_opt,  \
                                                     use_d, rec, nx, partial, state);                             \
      k_decode_check<<<1, 1024, 0, st>>>(partial, (int)nb, it, eps, state, deltas);                               \
    }                                                                                                             \
  } while (0)
  switch (rs) {
    case 4: FWAV_DEC(4); break;
    case 8: FWAV_DEC(8); break;
    case 16: FWAV_DEC(16); break;
    default: FWAV_DEC(0); break;
  }
#undef FWAV_DEC
  FWAV_LAUNCH_CHECK("fwav_decode");
  return FWAV_OK;
}

}  // extern "C"
