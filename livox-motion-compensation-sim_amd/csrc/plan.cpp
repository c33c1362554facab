// plan.cpp — host-only batch layout and gather planning (see plan.hpp).
#include "plan.hpp"

#include <algorithm>
#include <climits>
#include <cstdio>

namespace mcplan {

static std::string msg(const char* fmt, long long a, long long b = 0, long long c = 0, long long d = 0,
                       long long e = 0) {
  char buf[320];
  std::snprintf(buf, sizeof(buf), fmt, a, b, c, d, e);
  return buf;
}

std::string plan_batch(const int64_t* counts, int32_t F, int32_t tile_groups, int32_t sub_per_tile,
                       BatchLayout* out) {
  if (F < 0) return "n_frames must be >= 0";
  if (F > 0 && !counts) return "counts is NULL";
  if (tile_groups < 1 || sub_per_tile < 1) return "bad tile geometry";
  BatchLayout& L = *out;
  L.poff.assign((size_t)F + 1, 0);
  L.doff.assign((size_t)F + 1, 0);
  L.ftile.assign((size_t)F + 1, 0);
  L.tiles.clear();
  // every frame's tile count first: one allocation, and the int32 bound is checked before any
  // tile is built (a huge count must fail cleanly, not exhaust host memory)
  int64_t n_tiles = 0;
  for (int32_t f = 0; f < F; ++f) {
    if (counts[f] < 0) return msg("frame %lld has a negative count", f);
    if (counts[f] > (INT64_MAX / 8)) return msg("frame %lld count %lld is too large", f, counts[f]);
    const int64_t groups = (counts[f] + 3) / 4;
    n_tiles += (groups + tile_groups - 1) / tile_groups;
    if (n_tiles > (int64_t)INT32_MAX / sub_per_tile) return "too many tiles";
  }
  L.tiles.reserve((size_t)n_tiles);
  for (int32_t f = 0; f < F; ++f) {
    L.ftile[f] = (int32_t)L.tiles.size();
    const int64_t groups = (counts[f] + 3) / 4;
    L.doff[f + 1] = L.doff[f] + counts[f];
    L.poff[f + 1] = L.poff[f] + (counts[f] + kBlk - 1) / kBlk * kBlk;
    for (int64_t g0 = 0; g0 < groups; g0 += tile_groups) {
      TileRec t;
      t.pstart = L.poff[f] + 4 * g0;
      t.frame = f;
      t.ngroups = (int32_t)std::min<int64_t>(tile_groups, groups - g0);
      L.tiles.push_back(t);
    }
  }
  L.ftile[F] = (int32_t)L.tiles.size();
  return "";
}

std::string plan_gather(int32_t nranks, int32_t root, const int64_t* P, const int64_t* C, int64_t merged_P,
                        int64_t merged_C, GatherPlan* out) {
  if (nranks < 1) return msg("bad rank count %lld", nranks);
  if (root < 0 || root >= nranks) return msg("bad root %lld of %lld ranks", root, nranks);
  if (!P || !C) return "shard sizes are NULL";
  if (merged_C != 4 && merged_C != 5) return msg("merged batch has %lld columns (4 or 5 expected)", merged_C);
  GatherPlan& G = *out;
  G.off.assign((size_t)nranks, 0);
  G.stage_off.assign((size_t)nranks, -1);
  G.stage_values = 0;
  int64_t o = 0;
  for (int32_t q = 0; q < nranks; ++q) {
    if (P[q] < 0 || P[q] % kBlk != 0) return msg("rank %lld sent %lld padded points (not a block multiple)", q, P[q]);
    if (C[q] != 4 && C[q] != 5) return msg("rank %lld sent %lld columns (4 or 5 expected)", q, C[q]);
    if (P[q] > 0 && C[q] < merged_C)
      return msg("rank %lld sent %lld columns into a %lld-column merged batch (t_ns would be undefined)", q, C[q],
                 merged_C);
    G.off[q] = o;
    if (P[q] > INT64_MAX / 8 - o) return "merged size overflows";
    o += P[q];
    if (q != root && P[q] > 0 && C[q] != merged_C) {
      G.stage_off[q] = G.stage_values;
      G.stage_values += C[q] * P[q];
    }
  }
  if (o != merged_P)
    return msg("merged batch holds %lld padded points, ranks sent %lld", merged_P, o);
  return "";
}

namespace {
constexpr uint64_t kHashBase = 0x9E3779B97F4A7C15ull;   // odd: multiplication is a bijection mod 2^64
uint64_t pow_mod(uint64_t b, int64_t e) {
  uint64_t r = 1;
  while (e > 0) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return r;
}
}  // namespace

uint64_t counts_hash(const int64_t* counts, int64_t n) {
  uint64_t h = 0;
  for (int64_t i = 0; i < n; ++i) h = h * kHashBase + (uint64_t)counts[i] + 1;
  return h;
}

uint64_t hash_concat(uint64_t ha, uint64_t hb, int64_t nb) { return ha * pow_mod(kHashBase, nb) + hb; }

std::string check_frame_concat(int32_t nranks, const int64_t* const* shard_counts, const int64_t* shard_F,
                               const int64_t* merged_counts, int64_t merged_F) {
  int64_t f = 0;
  for (int32_t q = 0; q < nranks; ++q) {
    if (shard_F[q] > merged_F - f)
      return msg("the shards hold more frames than the merged batch (%lld)", merged_F);
    for (int64_t i = 0; i < shard_F[q]; ++i, ++f)
      if (shard_counts[q][i] != merged_counts[f])
        return msg("merged frame %lld holds %lld points, shard %lld's frame %lld holds %lld (the merged batch must "
                   "be the rank-ordered concatenation of the shards)", f, merged_counts[f], q, i, shard_counts[q][i]);
  }
  if (f != merged_F) return msg("the shards hold %lld frames, the merged batch %lld", f, merged_F);
  return "";
}

std::string check_frame_hashes(int32_t nranks, const int64_t* F, const uint64_t* H, int64_t merged_F,
                               uint64_t merged_H) {
  uint64_t h = 0;
  int64_t f = 0;
  for (int32_t q = 0; q < nranks; ++q) {
    if (F[q] < 0) return msg("rank %lld sent %lld frames", q, F[q]);
    h = hash_concat(h, H[q], F[q]);
    f += F[q];
  }
  if (f != merged_F) return msg("the ranks hold %lld frames, the merged batch %lld", f, merged_F);
  if (h != merged_H)
    return "the merged batch's frame counts are not the rank-ordered concatenation of the shards' frame counts";
  return "";
}

}  // namespace mcplan
