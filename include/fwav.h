/* fwav.h — C ABI of libfwav.so, the MI355X (gfx950) hot path of the fractal WAV codec.
 *
 * Drop-in boundary for xavenordu/Audio-Compression (reference: /root/reference/fractal.py).  The reference is
 * pure Python; its hot path is the xp (NumPy/CuPy) code inside compress_audio / decompress_audio.  Each entry
 * point below replaces one of those stages and cites the lines it replaces.  The Python host
 * (audio-compression_amd/fwav) binds these with ctypes; INTEGRATION.md shows that binding.
 *
 * Conventions
 *   - All array pointers are DEVICE pointers (HBM) owned by the caller; sizes are element counts.
 *   - `stream` is a hipStream_t passed as void*; every call only enqueues work on it (no host sync, no
 *     allocation) unless stated otherwise, so a caller may capture the sequence in a hipGraph.
 *   - Return value: 0 = FWAV_OK, negative = error; fwav_last_error() returns a thread-local message.
 *     No exception, abort or exit crosses the ABI.
 *   - Workspaces are caller-allocated; *_workspace_size() gives the byte count.
 *   - Results are deterministic for identical inputs.
 *   - No entry point reads or writes process-global state: the test and experiment knobs of the search live in the
 *     separate debug library (libfwav_debug.so, include/fwav_debug.h).
 */
#ifndef FWAV_H
#define FWAV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FWAV_OK 0
#define FWAV_ERR_ARG (-1)       /* null pointer / invalid argument */
#define FWAV_ERR_SHAPE (-2)     /* sizes inconsistent or outside supported range */
#define FWAV_ERR_K (-3)         /* top-K outside the supported range */
#define FWAV_ERR_HIP (-4)       /* HIP runtime / launch error */
#define FWAV_ERR_WORKSPACE (-5) /* workspace missing or too small */

/* ---------------------------------------------------------------------------------------- plumbing */
const char* fwav_last_error(void);
int fwav_abi_version(void);
/* SHA-256 (hex) of the sources and compiler flags this library was built from (__graft_entry__.build writes it in;
 * fwav/_lib.py refuses a library whose digest differs from the sources beside it). */
const char* fwav_build_digest(void);
/* Blocks until `stream` is idle; surfaces asynchronous kernel faults as FWAV_ERR_HIP. */
int fwav_stream_sync(void* stream);

/* ------------------------------------------------------------- voiced detection + range formation
 * Replaces voiced_detection (fractal.py:880-909) and the range setup of compress_audio
 * (fractal.py:1074-1112): frame energies (frame = 2·range_size, reflect-padded, numpy pairwise mean),
 * `smooth_window`-tap moving average (np.convolve 'same' order), hysteresis hi/lo (float32 compares),
 * ranges[p] = (signal·mask)[reflect(p)] for p < n_ranges·range_size, n_ranges = ceil(n / range_size).
 * hi = float32(energy_thresh), lo = float32(0.5·energy_thresh).  mask_out (u8[n]) may be NULL. */
size_t fwav_voiced_workspace_size(int64_t n, int frame);
int fwav_voiced_ranges(const float* sig, int64_t n, int range_size, int frame, int smooth_window, float hi, float lo,
                       float* ranges, int64_t n_ranges, uint8_t* mask_out, void* workspace, size_t ws_bytes,
                       void* stream);

/* Silent-input test of compress_audio (fractal.py:1083): sum[0] = np.sum(ranges[0:n] ** 2) in float32, bit-exact
 * (numpy's 8192-element reduction buffers, each a pairwise sum); the caller compares it with float32(1e-8).
 * ranges must be 16-B aligned. */
size_t fwav_weighted_energy_workspace_size(int64_t n);
int fwav_weighted_energy(const float* ranges, int64_t n, float* sum, void* workspace, size_t ws_bytes, void* stream);
/* Diagnostic (tests): out[i] = the smoothed energy of frame i (i < nf) exactly as fwav_voiced_ranges computes it —
 * np.convolve(energy, ones(w)/w, 'same')[:nf] in numpy's own arithmetic (nf < w included). */
int fwav_debug_smooth(const float* energy, int64_t nf, int smooth_window, float* out, void* stream);

/* ------------------------------------------------------------------- domain pool + embeddings
 * Replaces build_domains_memmap (fractal.py:285-334) and build_domain_embeddings → multi_head_embedding →
 * tile_embedding / transient_embedding (fractal.py:238-280, 166-208, 154-164).
 * pool f32[n_domains·range_size] (bit-exact), emb f32[n_domains·16] (bit-exact for range_size 4, 8, 16: scipy's own
 * pocketfft DCT sequence in f32 and f64 and numpy's BLAS norm orders; |Δ| ≤ 1e-6 for other range sizes),
 * emb16 (optional) fp16 copies in the search's tiled layout, f16[fwav_emb16_elems(n_domains)]: the high part
 * f16(emb) then the low part f16(emb − f16(emb)), ceil(n_domains/256)·256·16 halfs each.
 * n_domains = (n − tile) / step + 1.  tab = device copy of fwav_embed_tables(range_size) (host call, tab_host holds
 * fwav_embed_tables_size(range_size) doubles). */
size_t fwav_emb16_elems(int64_t n_domains);
/* The fp16 search tables (hi/lo parts, f16[fwav_emb16_elems(n_domains)]) of embedding rows emb f32[n_domains·16],
 * exactly as fwav_pool_embed writes them — for embeddings that did not come from fwav_pool_embed (tests). */
int fwav_emb16_from_emb(const float* emb, int64_t n_domains, void* emb16, void* stream);
size_t fwav_embed_tables_size(int range_size);
int fwav_embed_tables(int range_size, double* tab_host);
/* Test hook (host, no device): scipy.fftpack.dct(x, norm='ortho') for n = 4, 8, 16 in float32 (dbl = 0) or float64
 * through the embedding kernel's own code (x and out are doubles). */
int fwav_debug_dct2(int n, int dbl, const double* x, double* out);
size_t fwav_pool_workspace_size(int64_t n, int tile, int range_size, int step);
int fwav_pool_embed(const float* sig, int64_t n, int tile, int range_size, int step, const double* tab, float* pool,
                    float* emb, void* emb16, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------- energy prune + degenerate queries
 * Replaces the per-range prefix of cpu_worker (fractal.py:598-622) for ranges [q_offset, q_offset + n):
 *   mean(r²) < prune_thr (= float32(0.75·energy_thresh), fast_mode) → cand row all −1;
 *   query embedding (domain row q_offset + i, quirk Q1 fractal.py:1190-1195) all zero → every score is 0, and the
 *     reference's row is the order numpy's argpartition + argsort leave equal keys in (fractal.py:537-541, quirk
 *     Q11): cand row = zero_cand[0..K) (device, −1 padded; the host computes it once per (n_domains, K) with the
 *     reference's own numpy calls), or 0..K−1 when zero_cand is NULL;
 *   otherwise local index i is appended to active[] (*n_active, device counter) for fwav_sim_topk. */
int fwav_prune(const float* ranges, int64_t n, int64_t q_offset, int range_size, float prune_thr, int fast_mode,
               const float* emb, int64_t n_domains, int k, const int32_t* zero_cand, int32_t* cand, int32_t* active,
               int32_t* n_active, void* stream);

/* ------------------------------------------------------------------- similarity top-K
 * Replaces range_candidates_from_embedding_emb + pad_candidates (fractal.py:535-552, 617-622): for each
 * local query listed in active[0 .. *n_active) (at most max_q entries; max_q bounds their number, not their
 * values — a listed i only needs its cand row), the K domains with the largest f32 score emb[d]·emb[q_offset+i]
 * evaluated in the reference's own BLAS order (OpenBLAS sgemv_t over `blas_threads` threads: the thread split
 * decides which columns its tail kernels score; fwav_common.h), in (score desc, index asc) order, −1-padded when
 * n_domains < K, into cand[i·K .. i·K+K).  ties (device int32[fwav_tie_list_size(max_q)], may be NULL): ties[0] =
 * the number of queries whose top K + 1 scores hold exactly equal values; record j = ties[1 + 9·j .. 10 + 9·j):
 * [0] = 2·i + (1 if the K-th and (K+1)-th are equal), and for such a K-th place tie [1] = the number of domains
 * outside the K with the K-th's score (−1: not collected, at most 7), [2 ..] = those domains — the rows whose order
 * (or set) the reference leaves to numpy's argpartition/argsort; see fwav_tie_check.
 * K ≤ 64: emb16 != NULL selects the fp16 MFMA pre-filter + exact f32 rescoring
 * kernel, emb16 == NULL the all-f32 MFMA kernel; both return identical candidates.  (For at least 32,768 queries
 * over 65,536 to 4 Mi domains the fp16 search starts every band limit at a floor guessed from pilot queries and
 * searches again, without it, the queries the floor may have cut — all on `stream`, no host synchronisation, the
 * same candidates.)  K > 64 (the module-global
 * top_k is unrestricted in the reference; K ≥ n_domains returns every domain sorted): batched exact score
 * rows + per-query select and sort (fwav_topk_large.hip).  `workspace` holds
 * fwav_sim_topk_workspace_size(max_q, n_domains, k) bytes (unused for K ≤ 64 with emb16 == NULL).
 * 1 ≤ K ≤ fwav_topk_max_k(). */
int fwav_topk_max_k(void);
int64_t fwav_tie_list_size(int64_t max_q);
size_t fwav_sim_topk_workspace_size(int64_t max_q, int64_t n_domains, int k);
int fwav_sim_topk(const float* emb, const void* emb16, int64_t n_domains, const int32_t* active,
                  const int32_t* n_active, int64_t max_q, int64_t q_offset, int k, int blas_threads, int32_t* cand,
                  int32_t* ties, void* workspace, size_t ws_bytes, void* stream);
/* Exact reference score rows (for resolving ties on the host with numpy's own calls): scores[i·n_domains + d] =
 * emb[d]·emb[q_offset + rows[i]] in the order of fwav_sim_topk, i < n_rows (device f32[n_rows·n_domains]).
 * Replaces `scores = domain_embs @ q` (fractal.py:537). */
int fwav_score_rows(const float* emb, int64_t n_domains, const int32_t* rows, int64_t n_rows, int64_t q_offset,
                    int blas_threads, float* scores, void* stream);
/* ------------------------------------------------------------------- batched affine solve
 * Replaces _flush_gpu_batch / _process_gpu_batch (fractal.py:852-870, 757-850): per range, over the K
 * candidates and their mirrors, s = Σd̃r̃/(Σd̃²+1e-12), o = r̄ − s·d̄, err = ‖s·D+o−R‖₂ (+inf for cand < 0),
 * first minimum over [K | K mirrored]; outputs (cand clamped to ≥ 0, clip(s, ±s_clip), o, sym, err),
 * bit-exact with the reference's float32 numpy arithmetic. */
int fwav_affine(const float* ranges, int64_t n_ranges, int range_size, const int32_t* cand, int k, const float* pool,
                int64_t n_domains, float s_clip, int32_t* out_idx, float* out_s, float* out_o, uint8_t* out_sym,
                float* out_err, void* stream);
/* Tie check (after fwav_affine on the same rows): for every query listed in ties (fwav_sim_topk), decide whether the
 * reference's numpy tie order could change its match (fractal.py:816-824) — equal scores inside the top K when two
 * candidates of one run of equal scores both attain the minimum error; a tie at the K-th place when some member of
 * the K-th score's group (in the K or left out) fits no worse than the best candidate outside it, or when the group
 * was not collected; with exact_sets == 1 every K-th place tie (the candidate sets are then the reference's too), with
 * exact_sets == 2 every listed query (whole candidate rows, order included, are then the reference's).
 * resolve (device int32[1 + max_ties]): resolve[0] = count, resolve[1 + j] = local row to resolve on the host
 * (fwav.ties.resolve_rows: exact score rows, numpy's argpartition/argsort, fwav_affine on those rows). */
int fwav_tie_check(const float* ranges, int64_t n_ranges, int range_size, const int32_t* cand, int k,
                   const float* pool, int64_t n_domains, const float* emb, int64_t q_offset, int blas_threads,
                   const int32_t* ties, int64_t max_ties, int exact_sets, int32_t* resolve, void* stream);
/* Tie fix-up, in (fwav.ties.apply_rows): for j < n, row r = rows[j] (local index): cand[r·k ..] = new_cand[j·k ..]
 * (numpy's ranking of row r, fractal.py:537-541) and ranges_out[j·rs ..] = ranges[r·rs ..], the compact input of
 * the fwav_affine re-solve of those rows. */
int fwav_tie_rows_in(const int32_t* rows, int64_t n, const int32_t* new_cand, int k, int32_t* cand,
                     const float* ranges, int range_size, float* ranges_out, void* stream);
/* Tie fix-up, out: the re-solve's compact outputs (j < n) scattered to row rows[j] of the five output arrays
 * (fractal.py:816-870 for those rows). */
int fwav_tie_rows_out(const int32_t* rows, int64_t n, const int32_t* idx_in, const float* s_in, const float* o_in,
                      const uint8_t* sym_in, const float* err_in, int32_t* out_idx, float* out_s, float* out_o,
                      uint8_t* out_sym, float* out_err, void* stream);
/* Diagnostic (bench roofline, not the product path): n uniformly random rows of rs floats (rs 4/8/16, 16-B aligned
 * table of n_rows rows) gathered with nothing computed — the ceiling of fwav_affine's memory side on this device.
 * sink: one float of device memory. */
int fwav_debug_gather_rows(const float* table, int64_t n_rows, int rs, int64_t n, float* sink, void* stream);

/* ------------------------------------------------------------------- decompression loop
 * Replaces decompress_audio (fractal.py:1378-1473).  recon values are bit-exact with the reference.
 * fwav_decode runs the whole loop on one device with no host synchronisation: up to 64 iterations per launch
 * with each range's reconstruction held in registers (range_size <= 32), Δ = ‖next − rec‖/(‖rec‖ or 1) in f64 per
 * iteration from fixed-order partial sums, and a device flag that stops the loop at the first iteration where the
 * REFERENCE's Δ (float32 BLAS sdot norms, fractal.py:1460-1461) is < eps for certain — the f64 Δ and a proven bound
 * on the two measures' difference decide — or, where the bound cannot decide, stops it "for a check".
 * After the call: state[0] = 0 (every iteration ran), 1 (stopped: the reference stops here too) or 2 (stopped for the
 * exact check), state[1] = iterations run t, state[2] = result buffer (0 → recon_a, 1 → recon_b), deltas[0..t) = Δ
 * per iteration (f64 measure).  With state[0] = 2 the OTHER buffer holds the reconstruction before iteration t:
 * fwav_decode_exact(prev = other buffer, next = result buffer, n_ranges·range_size, eps, t − 1, deltas, state)
 * computes the reference's Δ in its own sdot order, stores it in deltas[t − 1] and sets state[0] = 1 (the reference
 * stops) or 3 (it goes on: continue with fwav_decode_from, recon_init = a copy of the result buffer, the remaining
 * iterations).  state: int[4]; deltas: f64[iterations].  So with state[0] = 2 fwav_decode ALONE has run fewer
 * iterations than the reference: a caller that does not run that check loop uses fwav_decode_all (below). */
size_t fwav_decode_workspace_size(int64_t n_ranges, int range_size, int iterations);
int fwav_decode(const int32_t* idx, const float* s, const float* o, const uint8_t* sym, int64_t n_ranges,
                int range_size, const float* pool, int64_t n_domains, int iterations, double eps, float s_clip,
                double s_damping, float* recon_a, float* recon_b, double* deltas, int* state, void* workspace,
                size_t ws_bytes, void* stream);
/* fwav_decode starting from the reconstruction recon_init (device f32[n_ranges·range_size], not recon_a/recon_b;
 * NULL = zeros, the reference's start) instead of zeros: the loop resumed after an exact check (iterations = the
 * iterations left). */
/* fwav_decode run to the reference's own stop in ONE call, for callers that do not run the exact-check loop above
 * themselves: wherever fwav_decode stops for the check it runs fwav_decode_exact and, when the reference goes on,
 * fwav_decode_from the checked reconstruction (kept in the workspace's tail) for the iterations left.  Synchronises
 * `stream` (to read the state after each launch of the loop) — the only decode entry point that does.  On return
 * state[0] = 1 (stopped) or 0 (every iteration ran), state[1] = iterations run, state[2] = result buffer (0 → recon_a,
 * 1 → recon_b), deltas[0 .. state[1]) = Δ per iteration (the reference's own Δ at a checked iteration). */
size_t fwav_decode_all_workspace_size(int64_t n_ranges, int range_size, int iterations);
int fwav_decode_all(const int32_t* idx, const float* s, const float* o, const uint8_t* sym, int64_t n_ranges,
                    int range_size, const float* pool, int64_t n_domains, int iterations, double eps, float s_clip,
                    double s_damping, float* recon_a, float* recon_b, double* deltas, int* state, void* workspace,
                    size_t ws_bytes, void* stream);
int fwav_decode_from(const int32_t* idx, const float* s, const float* o, const uint8_t* sym, int64_t n_ranges,
                     int range_size, const float* pool, int64_t n_domains, int iterations, double eps, float s_clip,
                     double s_damping, const float* recon_init, float* recon_a, float* recon_b, double* deltas,
                     int* state, void* workspace, size_t ws_bytes, void* stream);
/* The early-exit check (only when state[0] == 2; a no-op otherwise): Δ_ref = f32(‖next − prev‖)/(‖prev‖ or 1), both
 * norms sqrt of numpy's BLAS sdot in its own order (fractal.py:1460-1461) over n values — one workgroup, since each
 * of the sdot's 64 accumulators is a sequential fma chain (≈ 10 ms at cfg5's 172.8 M values).  deltas[t] = Δ_ref;
 * state[0] = 1 if Δ_ref < eps, else 3. */
int fwav_decode_exact(const float* prev, const float* next, int64_t n, double eps, int t, double* deltas, int* state,
                      void* stream);

/* Range-sharded decode (multi-GPU, fwav.dist.decompress_sharded; range_size <= 32).  A rank owns ranges
 * [lo, lo + m) of n_ranges_global (idx/s/o/sym/recon are the rank's local slices; lo and, unless the shard ends the
 * signal, m are multiples of fwav_decode_span()).  Per chunk c < fwav_decode_n_chunks(iterations, eps) (at most
 * fwav_decode_chunk_iterations() iterations each; the first is 2 iterations when eps > 0):
 *   fwav_decode_run(c)  → the rank's block partials in partials[0 .. 2·chunk_iterations·ceil(n_ranges_global/span))
 *                         (other blocks zeroed); the caller all-reduces (SUM) that prefix across ranks;
 *   fwav_decode_reduce(c) → Δ per iteration and the stop decision (as fwav_decode's), identical on every rank and
 *                         bit-identical to the single-device fwav_decode (one non-zero contributor per partial, fixed
 *                         summation order);
 * then fwav_decode_finish() once.  partials holds fwav_decode_partials_count(n_ranges_global) doubles; recon_init
 * (the rank's slice, or NULL = zeros) as fwav_decode_from.  After a stop for the check (state[0] == 2) the caller
 * gathers the ranks' slices of both buffers and runs fwav_decode_exact on the whole signal's (fwav.dist). */
int fwav_decode_span(void);
int fwav_decode_chunk_iterations(void);
int fwav_decode_n_chunks(int iterations, double eps);
size_t fwav_decode_partials_count(int64_t n_ranges_global);
int fwav_decode_run(const int32_t* idx, const float* s, const float* o, const uint8_t* sym, int64_t m, int64_t lo,
                    int64_t n_ranges_global, int range_size, const float* pool, int64_t n_domains, int iterations,
                    int chunk, double eps, float s_clip, double s_damping, const float* recon_init, float* recon_a,
                    float* recon_b, double* partials, int* state, void* stream);
int fwav_decode_reduce(const double* partials, int64_t n_ranges_global, int range_size, int iterations, int chunk,
                       double eps, double* deltas, int* state, void* stream);
int fwav_decode_finish(const int32_t* idx, const float* s, const float* o, const uint8_t* sym, int64_t m, int64_t lo,
                       int64_t n_ranges_global, int range_size, const float* pool, int64_t n_domains, int iterations,
                       double eps, float s_clip, double s_damping, const float* recon_init, float* recon_a,
                       float* recon_b, int* state, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FWAV_H */
