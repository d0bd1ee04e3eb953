/* fwav_debug.h — the debug library libfwav_debug.so: every entry point of fwav.h plus the search's test knobs and
 * diagnostics.  Built from the same sources with -DFWAV_DEBUG_API (__graft_entry__.build; tools/ab_build.sh for
 * experiment variants); the product library libfwav.so exports none of these.  Used by tests/ and tools/ only.
 */
#ifndef FWAV_DEBUG_H
#define FWAV_DEBUG_H

#include "fwav.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic ablations of the fp16 kernel (timing only, outputs invalid for dbg & 65535 != 0); stats (u64[16]
 * device, may be NULL) receives slow-path counters — of the first pass, or with dbg = 1 << 17 of the exact-mode
 * relaunch for overflowed queries only (outputs valid); dbg bit 18 counts in the product's first-pass geometry
 * (else the base one), bit 19 with the product's speculative floor (else none).  Not used by the product path. */
int fwav_debug_sim_topk(const float* emb, const void* emb16, int64_t n_domains, const int32_t* active,
                        const int32_t* n_active, int64_t max_q, int64_t q_offset, int k, int32_t* cand,
                        void* workspace, size_t ws_bytes, int dbg, unsigned long long* stats, void* stream);
/* The three overrides below (fwav_debug_topk_plan / _mode / _geometry) are PROCESS-GLOBAL test knobs, not thread-safe:
 * they change which kernels fwav_sim_topk launches and how much workspace it needs, so set them only while no search
 * is being sized or is in flight on any thread, and re-query fwav_sim_topk_workspace_size after a change (a search
 * sized before the change is rejected with FWAV_ERR_WORKSPACE when it needs more).  The product never sets them.
 *
 * Diagnostic override of the fp16 search's work plan: the last `rt` query blocks are split into `pieces` table
 * ranges, or with pieces == -1 into two query halves (rt < 0 restores the default policy).  Every plan returns the
 * same candidates.  Re-query fwav_sim_topk_workspace_size afterwards. */
int fwav_debug_topk_plan(int rt, int pieces);
/* Diagnostic: in multi-round plans whose blocks are all split, the last table piece of every block takes wb / 16 of
 * the other pieces' share (0 or 16: an even split; −1: the default, 12).  Same candidates. */
int fwav_debug_topk_tail(int wb);
/* The first pass fwav_sim_topk would launch for max_q queries over n_domains domains on the current device (host
 * only): info[0] = geometry (0 = base, 1 = wide, 2 = centroid, 3 = centroid wide), info[1] = first-pass mode (0 = fp16 band, 1 = hi/lo band), info[2] = table
 * pieces per split block (−1: query halves); blocks[0] = whole-table blocks, blocks[1] = split blocks,
 * blocks[2] = grid. */
int fwav_debug_topk_plan_info(int64_t max_q, int64_t n_domains, int32_t* info, int64_t* blocks);
/* The default plan's table pieces for max_q queries over n_domains (host only), of split block `block` (taken modulo
 * the split blocks): c01[2p .. 2p + 1] = the chunk range [c0, c1) of piece p (256-domain chunks) for p < *np (≤ 64;
 * 1 when the plan splits no block).  One-round and multi-round plans weigh some pieces unevenly; the
 * ranges always tile the table. */
int fwav_debug_topk_piece_chunks(int64_t max_q, int64_t n_domains, int64_t block, int32_t* c01, int32_t* np);
/* Host-side check of a work plan (no device): count[position] += 1 for every query slot of every item of the plan of
 * n queries (whole blocks and query halves cover a query once, a block in P table pieces P times) in first-pass
 * geometry `wide` (0 = base, 1 = wide, 2 = centroid, 3 = centroid wide); *items = grid. */
int fwav_debug_topk_plan_cover(int64_t n, int rt, int pieces, int wide, int32_t* count, int64_t* items);
/* Diagnostic override of the fp16 search's first-pass mode: 0 = fp16 band (overflowing queries relaunched with the
 * hi/lo band, then exact keys), 1 = hi/lo band (then exact keys), −1 = by table size (the default: hi/lo above 4 Mi
 * domains).  Every mode returns the same candidates. */
int fwav_debug_topk_mode(int mode);
/* Diagnostic override of the fp16 search's first-pass geometry: 0 = 8 waves × 32 queries per workgroup, 1 = 16 waves
 * × 32 queries, one workgroup per CU (the table streamed once per 512 queries), 2 = the centroid pre-filter (query
 * sets of 2 × 32 per wave), 3 = the centroid pre-filter in the wide geometry, −1 = by table size and query count (the
 * default).  All return the same candidates.  Re-query
 * fwav_sim_topk_workspace_size afterwards. */
int fwav_debug_topk_geometry(int wide);
/* Queries per block (one workgroup's query slots) of first-pass geometry geo (0 base, 1 wide, 2 centroid,
 * 3 centroid wide); −1 for another geo. */
int64_t fwav_debug_topk_qb(int geo);
/* Diagnostic override of the fp16 search's speculative floor (a first pass's band limits start at a floor guessed from
 * pilot queries; the queries it cuts are searched again without it): −1 = the default (first passes of at least
 * 32,768 queries over 65,536 to 4 Mi domains), 0 = never, 1 = every first pass, at the floor `value` (a filter score;
 * above a query's K-th score it sends the query to the second pass), 2 = every first pass, floor from the pilots
 * (`value` ≥ 1: the pilots' value-th smallest estimate instead of the default rank), 3 = as 1, and the second pass
 * at the same floor (every query the first pass cuts is cut again: the floor-free third pass takes them), 4 = as 2 at
 * the default rank, with the second pass's floor `value` (≥ 0) below the pilots' smallest estimate instead of 0.15.
 * All return the same candidates. */
int fwav_debug_topk_floor(int mode, float value);
/* Diagnostic override of the floor's second pass: table pieces per split block of misses (1 … 64; 0 = the default:
 * 64 where the expected misses fill one round of workgroups with them, else as many from 16 to 32 as do).  Re-query
 * fwav_sim_topk_workspace_size afterwards.  All return the same candidates. */
int fwav_debug_topk_floor_pieces(int pieces);
/* Byte offsets of the fp16 search's workspace regions (K <= 64) for max_q queries over n_domains domains, as this
 * library lays them out: offsets[0..18] = keys, share, ovf2, n_ovf2, seeds2, ovf1, n_ovf1, seeds1, miss, n_miss, miss2,
 * n_miss2, floor_key, order, n_order, order_bits, order_bsum (the search's ascending copy of the active list and its
 * bitmap), pilot, total (= fwav_sim_topk_workspace_size).  Every region before `pilot` sits at the same offset in
 * libfwav.so; the product library adds the pilots' scores only where its floor can run. */
int fwav_debug_sim_topk_layout(int64_t max_q, int64_t n_domains, int64_t* offsets);

#ifdef __cplusplus
}
#endif

#endif /* FWAV_DEBUG_H */
