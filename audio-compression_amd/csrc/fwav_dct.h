// fwav_dct.h — scipy.fftpack.dct(x, type=2, norm='ortho') for n = 4, 8, 16, bit-exact in float32 and float64.
//
// The reference embeds every domain with scipy's DCT-II (fractal.py:186 tonal head in float32, :158 transient head in
// float64).  scipy (1.15) runs pocketfft's T_dcst23 (FFTPACK's cosqb): pre-butterflies, a backward real FFT (rfftp
// radix passes radb4 / radb2 over the factors 4 → [4], 8 → [2, 4], 16 → [4, 4]) scaled by fct = 1/sqrt(2n), the
// twiddle post-pass and the orthonormal c[0]·sqrt2/2.  The same operations in the same order, each rounded in T, give
// scipy's outputs bit for bit; the constants (twiddles, fct, sqrt2) are pocketfft's own values, computed on the host
// by dct_constants() exactly as pocketfft computes them (sincos_2pibyn in double, long-double π and 1/sqrt).
// Pinned: tests/test_capi.py::test_dct_is_scipy_bitexact (fwav_debug_dct2, the host instantiation of this header)
// against scipy on random inputs of every size and both precisions; the device instantiation is the same source.
// Requires -ffp-contract=off (every a*b+c two roundings, as pocketfft compiled for baseline x86-64).
#pragma once

#ifdef __HIPCC__
#define FWAV_HD __host__ __device__ __forceinline__
#else
#define FWAV_HD inline
#endif

namespace fwav {

// One precision's constants for length N (pocketfft's values rounded to T).  rtw: the first rfftp factor's twiddles
// (N = 8: radb2 with ido 4 → 3 used; N = 16: radb4 with ido 4 → 9 used; N = 4: none).  w: np.linspace(1, 2, N).
template <class T, int N>
struct DctK {
  T tw[N];
  T rtw[9];
  T w[N];
  T fct;
  T sqrt2;
};
// doubles per precision in the constant block: tw N, rtw 9, w N, fct, sqrt2
constexpr int dct_block(int n) { return 2 * n + 11; }

template <class T, int N>
FWAV_HD void dct_load(DctK<T, N>& k, const double* p) {
  for (int i = 0; i < N; ++i) k.tw[i] = (T)p[i];
  for (int i = 0; i < 9; ++i) k.rtw[i] = (T)p[N + i];
  for (int i = 0; i < N; ++i) k.w[i] = (T)p[N + 9 + i];
  k.fct = (T)p[2 * N + 9];
  k.sqrt2 = (T)p[2 * N + 10];
}

template <class T>
FWAV_HD void pm(T& a, T& b, T c, T d) {
  a = c + d;
  b = c - d;
}

// pocketfft rfftp::radb4 (backward radix-4 pass), ido / l1 fixed at compile time.
template <class T, int IDO, int L1>
FWAV_HD void radb4(const T* cc, T* ch, const T* wa, T sqrt2) {
  auto CC = [&](int a, int b, int c) { return cc[a + IDO * (b + 4 * c)]; };
  auto CH = [&](int a, int b, int c) -> T& { return ch[a + IDO * (b + L1 * c)]; };
  auto WA = [&](int x, int i) { return wa[i + x * (IDO - 1)]; };
  for (int k = 0; k < L1; ++k) {
    T tr1, tr2;
    pm(tr2, tr1, CC(0, 0, k), CC(IDO - 1, 3, k));
    const T tr3 = (T)2 * CC(IDO - 1, 1, k);
    const T tr4 = (T)2 * CC(0, 2, k);
    pm(CH(0, k, 0), CH(0, k, 2), tr2, tr3);
    pm(CH(0, k, 3), CH(0, k, 1), tr1, tr4);
  }
  if ((IDO & 1) == 0) {
    for (int k = 0; k < L1; ++k) {
      T tr1, tr2, ti1, ti2;
      pm(ti1, ti2, CC(0, 3, k), CC(0, 1, k));
      pm(tr2, tr1, CC(IDO - 1, 0, k), CC(IDO - 1, 2, k));
      CH(IDO - 1, k, 0) = tr2 + tr2;
      CH(IDO - 1, k, 1) = sqrt2 * (tr1 - ti1);
      CH(IDO - 1, k, 2) = ti2 + ti2;
      CH(IDO - 1, k, 3) = -sqrt2 * (tr1 + ti1);
    }
  }
  if (IDO <= 2) return;
  for (int k = 0; k < L1; ++k) {
    for (int i = 2; i < IDO; i += 2) {
      const int ic = IDO - i;
      T ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
      pm(tr2, tr1, CC(i - 1, 0, k), CC(ic - 1, 3, k));
      pm(ti1, ti2, CC(i, 0, k), CC(ic, 3, k));
      pm(tr4, ti3, CC(i, 2, k), CC(ic, 1, k));
      pm(tr3, ti4, CC(i - 1, 2, k), CC(ic - 1, 1, k));
      pm(CH(i - 1, k, 0), cr3, tr2, tr3);
      pm(CH(i, k, 0), ci3, ti2, ti3);
      pm(cr4, cr2, tr1, tr4);
      pm(ci2, ci4, ti1, ti4);
      // MULPM(a, b, c, d, e, f): a = c·e + d·f, b = c·f − d·e
      CH(i, k, 1) = WA(0, i - 2) * ci2 + WA(0, i - 1) * cr2;
      CH(i - 1, k, 1) = WA(0, i - 2) * cr2 - WA(0, i - 1) * ci2;
      CH(i, k, 2) = WA(1, i - 2) * ci3 + WA(1, i - 1) * cr3;
      CH(i - 1, k, 2) = WA(1, i - 2) * cr3 - WA(1, i - 1) * ci3;
      CH(i, k, 3) = WA(2, i - 2) * ci4 + WA(2, i - 1) * cr4;
      CH(i - 1, k, 3) = WA(2, i - 2) * cr4 - WA(2, i - 1) * ci4;
    }
  }
}

// pocketfft rfftp::radb2.
template <class T, int IDO, int L1>
FWAV_HD void radb2(const T* cc, T* ch, const T* wa) {
  auto CC = [&](int a, int b, int c) { return cc[a + IDO * (b + 2 * c)]; };
  auto CH = [&](int a, int b, int c) -> T& { return ch[a + IDO * (b + L1 * c)]; };
  auto WA = [&](int x, int i) { return wa[i + x * (IDO - 1)]; };
  for (int k = 0; k < L1; ++k) pm(CH(0, k, 0), CH(0, k, 1), CC(0, 0, k), CC(IDO - 1, 1, k));
  if ((IDO & 1) == 0) {
    for (int k = 0; k < L1; ++k) {
      CH(IDO - 1, k, 0) = (T)2 * CC(IDO - 1, 0, k);
      CH(IDO - 1, k, 1) = (T)-2 * CC(0, 1, k);
    }
  }
  if (IDO <= 2) return;
  for (int k = 0; k < L1; ++k) {
    for (int i = 2; i < IDO; i += 2) {
      const int ic = IDO - i;
      T ti2, tr2;
      pm(CH(i - 1, k, 0), tr2, CC(i - 1, 0, k), CC(ic - 1, 1, k));
      pm(ti2, CH(i, k, 0), CC(i, 0, k), CC(ic, 1, k));
      CH(i, k, 1) = WA(0, i - 2) * ti2 + WA(0, i - 1) * tr2;
      CH(i - 1, k, 1) = WA(0, i - 2) * tr2 - WA(0, i - 1) * ti2;
    }
  }
}

// pocketfft rfftp::exec(c, fct, r2hc = false): the radix passes in factor order, then copy_and_norm (c = fct·p).
template <class T, int N>
FWAV_HD void rfftb(T (&c)[N], const DctK<T, N>& k) {
  static_assert(N == 4 || N == 8 || N == 16, "exact DCT for n = 4, 8, 16");
  T ch[N];
  if constexpr (N == 4) {
    radb4<T, 1, 1>(c, ch, k.rtw, k.sqrt2);  // result in ch (p1 after one swap)
    for (int i = 0; i < N; ++i) c[i] = k.fct * ch[i];
  } else if constexpr (N == 8) {
    radb2<T, 4, 1>(c, ch, k.rtw);            // → ch
    radb4<T, 1, 2>(ch, c, nullptr, k.sqrt2);  // → c (two swaps: p1 == c)
    for (int i = 0; i < N; ++i) c[i] *= k.fct;
  } else {
    radb4<T, 4, 1>(c, ch, k.rtw, k.sqrt2);
    radb4<T, 1, 4>(ch, c, nullptr, k.sqrt2);
    for (int i = 0; i < N; ++i) c[i] *= k.fct;
  }
}

// T_dcst23::exec(c, fct, ortho = true, type = 2, cosine = true) — scipy.fftpack.dct(c, norm='ortho') in place.
template <class T, int N>
FWAV_HD void dct2_ortho(T (&c)[N], const DctK<T, N>& k) {
  constexpr int NS2 = (N + 1) / 2;
  c[0] *= (T)2;
  if ((N & 1) == 0) c[N - 1] *= (T)2;
  for (int i = 1; i < N - 1; i += 2) {  // MPINPLACE(c[i+1], c[i])
    const T t = c[i + 1];
    c[i + 1] -= c[i];
    c[i] += t;
  }
  rfftb<T, N>(c, k);
  for (int i = 1, ic = N - 1; i < NS2; ++i, --ic) {
    const T t1 = k.tw[i - 1] * c[ic] + k.tw[ic - 1] * c[i];
    const T t2 = k.tw[i - 1] * c[i] - k.tw[ic - 1] * c[ic];
    c[i] = (T)0.5 * (t1 + t2);
    c[ic] = (T)0.5 * (t1 - t2);
  }
  if ((N & 1) == 0) c[NS2] *= k.tw[NS2 - 1];
  c[0] *= k.sqrt2 * (T)0.5;
}

}  // namespace fwav
