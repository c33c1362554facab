// gather.cpp — mcgather::run, the merged-cloud gather sequence (gather.hpp).  Host-only C++.
#include "gather.hpp"

#include <vector>

#include "plan.hpp"

namespace mcgather {

int run(const Transport& T, int root, const Shard& local, const Merged* merged, std::string* msg) {
  const int nr = T.nranks;
  const bool is_root = T.rank == root;
  if (root < 0 || root >= nr) {
    *msg = "bad root " + std::to_string(root);
    return kBadPlan;
  }
  // 1. every rank's (padded length, column count, frame count, hash of its frame counts) and the
  // root's merged ones: all ranks then hold the whole plan and reject a bad one together, before
  // any send (equal padded totals do not make the same frame order).  A root without a merged
  // batch still takes part (its words say so), so no rank is left waiting in a collective.
  const int64_t none = -1, missing = -2;
  const bool have = is_root && merged;
  const int64_t mine[kPlanWords] = {
      local.P, local.C, have ? merged->P : (is_root ? missing : none), have ? merged->C : none, local.F,
      (int64_t)mcplan::counts_hash(local.counts, local.F), have ? merged->F : none,
      have ? (int64_t)mcplan::counts_hash(merged->counts, merged->F) : none};
  std::vector<int64_t> all((size_t)kPlanWords * nr);
  if (int r = T.allgather_i64(T.self, mine, kPlanWords, all.data())) return r;
  std::vector<int64_t> P(nr), C(nr), F(nr);
  std::vector<uint64_t> H(nr);
  for (int q = 0; q < nr; ++q) {
    const int64_t* w = all.data() + (size_t)kPlanWords * q;
    P[q] = w[0]; C[q] = w[1]; F[q] = w[4]; H[q] = (uint64_t)w[5];
  }
  const int64_t* wr = all.data() + (size_t)kPlanWords * root;
  if (wr[2] == missing) {
    *msg = "root needs a merged batch";
    return kBadPlan;
  }
  // 2. the plan (where each shard lands, which are staged for a re-pitch) and the frame-order check
  mcplan::GatherPlan G;
  std::string perr = mcplan::plan_gather(nr, root, P.data(), C.data(), wr[2], wr[3], &G);
  if (perr.empty()) perr = mcplan::check_frame_hashes(nr, F.data(), H.data(), wr[6], (uint64_t)wr[7]);
  if (!perr.empty()) {
    *msg = perr;
    return kBadPlan;
  }
  // 3. the data: one send per non-root rank, the root's receives grouped
  if (!is_root) {
    if (local.P > 0) {
      if (int r = T.group_start(T.self)) return r;
      if (int r = T.send(T.self, local.cols, C[T.rank] * P[T.rank], root)) return r;
      if (int r = T.group_end(T.self)) return r;
    }
    return T.sync(T.self);
  }
  float* stage = nullptr;
  if (int r = T.stage(T.self, G.stage_values, &stage)) return r;
  if (int r = T.group_start(T.self)) return r;
  for (int q = 0; q < nr; ++q) {
    if (q == root || P[q] == 0) continue;
    if (int r = T.recv(T.self, mcplan::gather_dst(G, q, merged->cols, merged->C, stage), C[q] * P[q], q)) return r;
  }
  if (int r = T.group_end(T.self)) return r;
  // 4. the root's own shard and the staged shards, re-pitched to the merged column count
  auto copy = [&](float* d, const float* s, int64_t n) { return T.copy(T.self, d, s, n); };
  auto copy2d = [&](float* d, int64_t dp, const float* s, int64_t sp, int64_t w, int64_t rows) {
    return T.copy2d(T.self, d, dp, s, sp, w, rows);
  };
  if (int r = mcplan::gather_finish(G, nr, root, P.data(), C.data(), merged->cols, merged->C, local.cols, stage, copy,
                                    copy2d))
    return r;
  return T.sync(T.self);
}

}  // namespace mcgather
