// Host-side sanitizer check of libfwav's C ABI: the work-plan, workspace-sizing and argument-check code
// of the search and the other entry points, built with AddressSanitizer + UndefinedBehaviorSanitizer on the host side
// only (tests/test_capi.py builds it: every .hip source host-only, -Xarch_host -fsanitize=...).  No kernel is
// launched; without a GPU the occupancy queries fail and the plan falls back to the MI355X's 256 CUs.  Exit 0 = every
// check held and no sanitizer report.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/fwav_debug.h"

static int g_fail = 0;
#define CHECK(c, ...)                            \
  do {                                           \
    if (!(c)) {                                  \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);         \
      std::fprintf(stderr, "\n");                \
      ++g_fail;                                  \
    }                                            \
  } while (0)

int main() {
  long plans = 0;
  const int64_t nds[] = {1000, 21027, 1321977, 6613977, 86398977};
  const int64_t qs[] = {1, 31, 32, 33, 255, 256, 257, 1023, 1024, 1025, 20672, 41344, 65536, 82688, 165375, 330750,
                        337500, 666606, 2700000};
  for (int64_t nd : nds) {
    for (int64_t q : qs) {
      if (q > 3 * nd) continue;
      for (int geo = -1; geo <= 3; ++geo) {
        CHECK(fwav_debug_topk_geometry(geo) == FWAV_OK, "geometry %d", geo);
        int32_t info[3] = {-9, -9, -9};
        int64_t blocks[3] = {-9, -9, -9};
        CHECK(fwav_debug_topk_plan_info(q, nd, info, blocks) == FWAV_OK, "plan_info");
        const int g = info[0], P = info[2] < 0 ? -1 : info[2];
        CHECK(g >= 0 && g <= 3 && (geo < 0 || g == geo), "geometry %d for %d", g, geo);
        const int64_t F = blocks[0], R = blocks[1], items = blocks[2];
        CHECK(F >= 0 && R >= 0 && items >= F + R, "blocks F=%lld R=%lld items=%lld", (long long)F, (long long)R,
              (long long)items);
        // the plan the search would launch covers every query exactly once per table piece of its block
        std::vector<int32_t> count((size_t)q, 0);
        int64_t it = -1;
        CHECK(fwav_debug_topk_plan_cover(q, (int)R, P, g, count.data(), &it) == FWAV_OK, "plan_cover");
        CHECK(it == items, "cover items %lld vs plan %lld", (long long)it, (long long)items);
        int64_t once = 0, split = 0, bad = 0;
        for (int64_t i = 0; i < q; ++i) {
          if (count[i] == 1) ++once;
          else if (P > 1 && count[i] == P) ++split;
          else ++bad;
        }
        CHECK(bad == 0, "nd=%lld q=%lld geo=%d P=%d: %lld queries covered wrongly", (long long)nd, (long long)q, g, P,
              (long long)bad);
        // the workspace holds the plan's key buffers (256 keys of 8 B per query slot) in every geometry
        const size_t ws = fwav_sim_topk_workspace_size(q, nd, 64);
        const int qb = (int)fwav_debug_topk_qb(g);
        CHECK(qb >= 256 && qb % 256 == 0, "qb %d", qb);
        CHECK(ws >= (size_t)items * qb * 256 * 8, "workspace %zu < %lld items x %d", ws, (long long)items, qb);
        ++plans;
      }
      // the speculative floor's later passes (base geometry, ≤ 64 blocks in P2 table pieces, the rest whole-table) on
      // a miss list of up to all q queries: their plan covers it and their key buffers fit the same workspace
      const int64_t pmax = ((nd + 255) / 256) / 16;
      const int P2 = (int)(pmax < 1 ? 1 : (pmax < 16 ? pmax : 16));
      std::vector<int32_t> count2((size_t)q, 0);
      int64_t it2 = -1;
      CHECK(fwav_debug_topk_plan_cover(q, 64, P2, 0, count2.data(), &it2) == FWAV_OK, "floor plan_cover");
      int64_t bad2 = 0;
      for (int64_t i = 0; i < q; ++i) bad2 += (count2[i] == 1 || (P2 > 1 && count2[i] == P2)) ? 0 : 1;
      CHECK(bad2 == 0, "floor plan nd=%lld q=%lld: %lld queries covered wrongly", (long long)nd, (long long)q,
            (long long)bad2);
      CHECK(fwav_sim_topk_workspace_size(q, nd, 64) >= (size_t)it2 * 256 * 256 * 8, "floor plan workspace");
    }
  }
  CHECK(fwav_debug_topk_geometry(-1) == FWAV_OK, "reset");
  // every work-plan override returns a covering plan
  for (int pieces : {-1, 1, 2, 3, 5, 8}) {
    for (int rt : {0, 1, 7, 1 << 20}) {
      for (int geo = 0; geo <= 3; ++geo) {
        const int64_t n = 41344;
        std::vector<int32_t> count((size_t)n, 0);
        int64_t it = 0;
        CHECK(fwav_debug_topk_plan_cover(n, rt, pieces, geo, count.data(), &it) == FWAV_OK, "cover");
        for (int64_t i = 0; i < n; ++i) CHECK(count[i] >= 1 && count[i] <= 8, "count %d", count[i]);
      }
    }
  }
  // argument checks: rejected before any HIP call, with a message
  CHECK(fwav_debug_topk_plan_cover(-1, 0, 1, 0, nullptr, nullptr) == FWAV_ERR_ARG, "cover args");
  CHECK(fwav_debug_topk_plan_cover(10, 0, 9, 0, nullptr, nullptr) == FWAV_ERR_ARG, "cover pieces");
  CHECK(fwav_debug_topk_geometry(4) == FWAV_ERR_ARG, "geometry range");
  CHECK(fwav_debug_topk_mode(2) == FWAV_ERR_ARG, "mode range");
  CHECK(fwav_debug_topk_plan(0, 65) == FWAV_ERR_ARG, "plan pieces");
  CHECK(fwav_sim_topk(nullptr, nullptr, 10, nullptr, nullptr, 10, 0, 64, 1, nullptr, nullptr, nullptr, 0, nullptr) ==
            FWAV_ERR_ARG, "sim_topk null");
  void* p = reinterpret_cast<void*>(16);
  const float* fp = static_cast<const float*>(p);
  int32_t* ip = static_cast<int32_t*>(p);
  CHECK(fwav_sim_topk(fp, nullptr, 10, ip, ip, 10, 0, 4097, 1, ip, nullptr, nullptr, 0, nullptr) == FWAV_ERR_K, "K");
  CHECK(fwav_sim_topk(fp, p, 1000, ip, ip, 10, 0, 64, 1, ip, nullptr, p, 1, nullptr) == FWAV_ERR_WORKSPACE, "ws");
  CHECK(fwav_debug_sim_topk(fp, p, 1321977, ip, ip, 41344, 0, 64, ip, p,
                            fwav_sim_topk_workspace_size(20672, 1321977, 64) - 1, 0, nullptr, nullptr) ==
            FWAV_ERR_WORKSPACE, "debug ws");
  CHECK(fwav_affine(nullptr, 10, 8, nullptr, 64, nullptr, 100, 16.f, nullptr, nullptr, nullptr, nullptr, nullptr,
                    nullptr) == FWAV_ERR_ARG, "affine");
  CHECK(fwav_tie_rows_in(ip, -1, ip, 64, ip, fp, 8, const_cast<float*>(fp), nullptr) == FWAV_ERR_SHAPE, "rows_in");
  CHECK(fwav_score_rows(nullptr, 100, nullptr, 1, 0, 1, nullptr, nullptr) == FWAV_ERR_ARG, "score_rows");
  CHECK(fwav_voiced_ranges(nullptr, 100, 8, 16, 5, 1e-4f, 5e-5f, nullptr, 13, nullptr, nullptr, 0, nullptr) != FWAV_OK,
        "voiced");
  CHECK(fwav_decode(nullptr, nullptr, nullptr, nullptr, 10, 8, nullptr, 100, 8, 1e-3, 16.f, 0.0, nullptr, nullptr,
                    nullptr, nullptr, nullptr, 0, nullptr) != FWAV_OK, "decode");
  // workspace-size queries at the extremes stay finite and monotone where the plan is
  CHECK(fwav_sim_topk_workspace_size(0, 1000, 64) > 0, "ws0");
  CHECK(fwav_sim_topk_workspace_size(21600000, 86398977, 64) >= (size_t)21600000 * 256 * 8, "ws cfg4");
  CHECK(fwav_sim_topk_workspace_size(10, 1000, 1000) == (size_t)10 * 1000 * 4, "ws large K");
  CHECK(fwav_decode_workspace_size(21600000, 8, 50) > 0, "decode ws");
  CHECK(fwav_voiced_workspace_size(172800000, 16) > 0, "voiced ws");
  CHECK(fwav_pool_workspace_size(1000, 2048, 8, 2) == 0, "pool ws short");
  std::printf("plan_check: %ld default plans covered, %d failures\n", plans, g_fail);
  return g_fail == 0 ? 0 : 1;
}
