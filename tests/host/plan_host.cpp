// Host harness for the library's host-side planning (livox-motion-compensation-sim_amd/csrc/plan.cpp):
// the blocked-CSR batch layout / tile builder and the merged-cloud gather plan + its finishing
// copies, executed with host memcpy standing in for hipMemcpyAsync / hipMemcpy2DAsync and for the
// RCCL receives.  tests/test_sanitizers.py builds it with -fsanitize=address,undefined (every
// buffer is sized exactly, so an out-of-range copy is a heap overflow ASan reports).
// Exit status = number of failed checks (capped at 255).
#include "plan.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <vector>

using namespace mcplan;

static int bad = 0;
#define CHECK(cond, ...)                          \
  do {                                            \
    if (!(cond)) {                                \
      ++bad;                                      \
      if (bad < 20) {                             \
        std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
        std::printf(__VA_ARGS__);                 \
        std::printf("\n");                        \
      }                                           \
    }                                             \
  } while (0)

static void test_batch(std::mt19937_64& g) {
  const int64_t menu[] = {0, 1, 2, 3, 4, 5, 7, 255, 256, 257, 1023, 2047, 2048, 2049, 4096, 8191, 100003};
  for (int trial = 0; trial < 3000; ++trial) {
    const int32_t F = (int32_t)(g() % 40);
    std::vector<int64_t> counts(F);
    for (auto& c : counts) c = (g() % 3) ? menu[g() % (sizeof(menu) / sizeof(menu[0]))] : (int64_t)(g() % 300000);
    const int32_t tg = (trial % 3 == 0) ? 512 : (int32_t)(1 + g() % 600);
    BatchLayout L;
    const std::string e = plan_batch(counts.data(), F, tg, 2, &L);
    CHECK(e.empty(), "plan_batch: %s", e.c_str());
    if (!e.empty()) continue;
    CHECK(L.poff.size() == (size_t)F + 1 && L.doff.size() == (size_t)F + 1 && L.ftile.size() == (size_t)F + 1,
          "table sizes");
    CHECK(L.poff[0] == 0 && L.doff[0] == 0 && L.ftile[0] == 0, "first offsets");
    for (int32_t f = 0; f < F; ++f) {
      CHECK(L.poff[f] % kBlk == 0, "poff[%d] = %lld not block aligned", f, (long long)L.poff[f]);
      CHECK(L.poff[f + 1] - L.poff[f] == (counts[f] + kBlk - 1) / kBlk * kBlk, "padded size of frame %d", f);
      CHECK(L.doff[f + 1] - L.doff[f] == counts[f], "dense size of frame %d", f);
      int64_t groups = 0;
      for (int32_t t = L.ftile[f]; t < L.ftile[f + 1]; ++t) {
        const TileRec& r = L.tiles[(size_t)t];
        CHECK(r.frame == f, "tile %d frame %d != %d", t, r.frame, f);
        CHECK(r.ngroups > 0 && r.ngroups <= tg, "tile %d ngroups %d", t, r.ngroups);
        CHECK(r.pstart == L.poff[f] + 4 * groups, "tile %d pstart", t);
        groups += r.ngroups;
      }
      CHECK(groups == (counts[f] + 3) / 4, "frame %d groups %lld != %lld", f, (long long)groups,
            (long long)((counts[f] + 3) / 4));
    }
    CHECK(L.ftile[F] == (int32_t)L.tiles.size(), "ftile[F]");
  }
  // errors: a negative count; a tile count past the int32 sub-tile index (must fail before allocating)
  BatchLayout L;
  const int64_t neg[] = {5, -1};
  CHECK(!plan_batch(neg, 2, 512, 2, &L).empty(), "negative count accepted");
  const int64_t huge[] = {int64_t(1) << 42};
  CHECK(!plan_batch(huge, 1, 512, 2, &L).empty(), "2^42-point frame accepted");
  CHECK(plan_batch(nullptr, 0, 512, 2, &L).empty() && L.tiles.empty() && L.poff.size() == 1, "empty batch");
}

// value of (rank q, shard-local padded point p, column c): exact in float32
static float tag(int q, int64_t p, int c) { return (float)(q * 1000000 + (p % 200000) * 5 + c); }

static void test_gather(std::mt19937_64& g) {
  long runs = 0, staged_runs = 0, errors = 0;
  for (int trial = 0; trial < 4000; ++trial) {
    const int32_t W = 1 + (int32_t)(g() % 8);
    const int32_t root = (int32_t)(g() % W);
    const int64_t mC = 4 + (int64_t)(g() % 2);
    const bool allow_narrow = trial % 7 == 0;   // some shards with fewer columns than merged: an error
    std::vector<int64_t> P(W), C(W);
    int64_t tot = 0;
    bool narrow = false;
    for (int32_t q = 0; q < W; ++q) {
      P[q] = kBlk * (int64_t)(g() % 4 == 0 ? 0 : g() % 6);
      C[q] = (allow_narrow || mC == 4) ? 4 + (int64_t)(g() % 2) : 5;
      if (P[q] > 0 && C[q] < mC) narrow = true;
      tot += P[q];
    }
    const bool wrong_total = trial % 11 == 0;
    GatherPlan G;
    const std::string e = plan_gather(W, root, P.data(), C.data(), tot + (wrong_total ? kBlk : 0), mC, &G);
    if (narrow || wrong_total) {
      CHECK(!e.empty(), "plan accepted narrow=%d wrong_total=%d", (int)narrow, (int)wrong_total);
      ++errors;
      continue;
    }
    CHECK(e.empty(), "plan_gather: %s", e.c_str());
    if (!e.empty()) continue;
    ++runs;
    // shards, the merged batch and the staging area, each allocated to its exact size
    std::vector<std::unique_ptr<float[]>> shard(W);
    for (int32_t q = 0; q < W; ++q) {
      shard[q].reset(new float[(size_t)std::max<int64_t>(C[q] * P[q], 1)]);
      for (int64_t p = 0; p < P[q]; ++p)
        for (int c = 0; c < C[q]; ++c) shard[q][(size_t)(((p / kBlk) * C[q] + c) * kBlk + p % kBlk)] = tag(q, p, c);
    }
    std::unique_ptr<float[]> merged(new float[(size_t)std::max<int64_t>(mC * tot, 1)]);
    std::fill(merged.get(), merged.get() + mC * tot, -1.f);
    std::unique_ptr<float[]> stage(G.stage_values > 0 ? new float[(size_t)G.stage_values] : nullptr);
    if (G.stage_values > 0) ++staged_runs;
    // the receives (RCCL on the device), then the root's copy and the re-pitches
    for (int32_t q = 0; q < W; ++q) {
      if (q == root || P[q] == 0) continue;
      float* dst = gather_dst(G, q, merged.get(), mC, stage.get());
      std::memcpy(dst, shard[q].get(), (size_t)(C[q] * P[q]) * sizeof(float));
    }
    auto copy = [](float* d, const float* s, int64_t n) {
      std::memcpy(d, s, (size_t)n * sizeof(float));
      return 0;
    };
    auto copy2d = [](float* d, int64_t dp, const float* s, int64_t sp, int64_t w, int64_t rows) {
      for (int64_t r = 0; r < rows; ++r) std::memcpy(d + r * dp, s + r * sp, (size_t)w * sizeof(float));
      return 0;
    };
    const int r = gather_finish(G, W, root, P.data(), C.data(), merged.get(), mC, shard[root].get(), stage.get(), copy,
                                copy2d);
    CHECK(r == 0, "gather_finish %d", r);
    // merged == rank-ordered concatenation of the shards' first mC columns
    int64_t o = 0;
    for (int32_t q = 0; q < W; ++q) {
      CHECK(G.off[q] == o, "off[%d]", q);
      for (int64_t p = 0; p < P[q]; ++p)
        for (int c = 0; c < mC; ++c) {
          const int64_t m = o + p;
          const float got = merged[(size_t)(((m / kBlk) * mC + c) * kBlk + m % kBlk)];
          if (got != tag(q, p, c)) {
            CHECK(false, "W=%d root=%d mC=%lld rank %d point %lld col %d: %g", W, root, (long long)mC, q, (long long)p,
                  c, (double)got);
            p = P[q];
            break;
          }
        }
      o += P[q];
    }
  }
  std::printf("gather plans: %ld executed (%ld with staging), %ld rejected\n", runs, staged_runs, errors);
  CHECK(staged_runs > 100 && errors > 100, "coverage");
}

// the merged batch's frames must be the rank-ordered concatenation of the shards'
// frames — [300, 100] and [100, 300] pad to the same total.  Exact check (one process) and the
// chained-hash check (across ranks) must agree on every split, swap and perturbation.
static void test_frame_order(std::mt19937_64& g) {
  int64_t accepted = 0, rejected = 0;
  for (int trial = 0; trial < 4000; ++trial) {
    const int32_t W = 1 + (int32_t)(g() % 8);
    const int64_t Fm = (int64_t)(g() % 30);
    std::vector<int64_t> merged(Fm);
    for (auto& c : merged) c = (int64_t)(g() % 5 == 0 ? 0 : g() % 200000);
    // a split of the merged frames over W ranks
    std::vector<int64_t> cut(W + 1, 0);
    cut[W] = Fm;
    for (int32_t q = 1; q < W; ++q) cut[q] = Fm ? (int64_t)(g() % (Fm + 1)) : 0;
    std::sort(cut.begin(), cut.end());
    std::vector<std::vector<int64_t>> sh(W);
    for (int32_t q = 0; q < W; ++q) sh[q].assign(merged.begin() + cut[q], merged.begin() + cut[q + 1]);
    const int kind = trial % 4;   // 0: correct, 1: two shards swapped, 2: one count changed, 3: a frame moved
    bool should_fail = false;
    if (kind == 1 && W >= 2) {
      const int32_t a = (int32_t)(g() % W), b = (int32_t)(g() % W);
      should_fail = sh[a] != sh[b];
      std::swap(sh[a], sh[b]);
    } else if (kind == 2 && Fm > 0) {
      const int32_t q = (int32_t)(g() % W);
      if (!sh[q].empty()) { sh[q][g() % sh[q].size()] += 1 + (int64_t)(g() % 7); should_fail = true; }
    } else if (kind == 3 && W >= 2) {
      const int32_t q = (int32_t)(g() % (W - 1));
      if (!sh[q].empty()) { sh[q + 1].insert(sh[q + 1].begin(), sh[q].back()); sh[q].pop_back(); }
    }
    std::vector<int64_t> cat;
    for (int32_t q = 0; q < W; ++q) cat.insert(cat.end(), sh[q].begin(), sh[q].end());
    should_fail = cat != merged;   // a swap of equal (or empty) neighbours leaves the concatenation alone
    std::vector<const int64_t*> ptr(W);
    std::vector<int64_t> F(W);
    std::vector<uint64_t> H(W);
    for (int32_t q = 0; q < W; ++q) {
      ptr[q] = sh[q].data();
      F[q] = (int64_t)sh[q].size();
      H[q] = counts_hash(sh[q].data(), F[q]);
    }
    const std::string e1 = check_frame_concat(W, ptr.data(), F.data(), merged.data(), Fm);
    const std::string e2 = check_frame_hashes(W, F.data(), H.data(), Fm, counts_hash(merged.data(), Fm));
    CHECK(e1.empty() == !should_fail, "exact check kind %d: '%s'", kind, e1.c_str());
    CHECK(e1.empty() == e2.empty(), "hash check disagrees (kind %d): '%s' vs '%s'", kind, e1.c_str(), e2.c_str());
    (e1.empty() ? accepted : rejected) += 1;
  }
  // the advisor's example
  const int64_t a[2] = {300, 100}, b[2] = {100, 300};
  const int64_t* one[1] = {a};
  const int64_t F1[1] = {2};
  CHECK(!check_frame_concat(1, one, F1, b, 2).empty(), "[300,100] accepted as [100,300]");
  CHECK(counts_hash(a, 2) != counts_hash(b, 2), "hash collision on the swap");
  std::printf("frame-order checks: %ld accepted, %ld rejected\n", accepted, rejected);
  CHECK(accepted > 500 && rejected > 500, "coverage");
}

int main() {
  std::mt19937_64 g(12345);
  test_batch(g);
  test_gather(g);
  test_frame_order(g);
  std::printf("bad %d\n", bad);
  return bad > 255 ? 255 : bad;
}
