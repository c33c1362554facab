// plan.hpp — host-only planning of the blocked-CSR batch layout and of the merged-cloud gather.
//
// Plain C++ (no HIP): the library calls it (mcdeskew.hip, comm.cpp) and tests/host/plan_host.cpp
// runs the same code under AddressSanitizer + UndefinedBehaviorSanitizer on the CPU,
// with host memcpy standing in for the device copies and the RCCL receives.
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

namespace mcplan {

constexpr int64_t kBlk = 256;   // points per block (== mc::kBlkPts)

// == mc::Tile (kernels.hpp): the device tile record, 16 bytes
struct TileRec {
  int64_t pstart;   // padded index of the tile's first point (a frame's first tile: a multiple of kBlk)
  int32_t frame;
  int32_t ngroups;  // float4 groups, <= tile_groups
};

// Blocked-CSR layout of a ragged batch: frame f's points sit at padded indices
// [poff[f], poff[f] + counts[f]), poff[f] a multiple of kBlk; dense offsets doff; tiles of at most
// tile_groups float4 groups that never cross a frame; ftile[f] = first tile of frame f (F+1).
struct BatchLayout {
  std::vector<int64_t> poff, doff;
  std::vector<TileRec> tiles;
  std::vector<int32_t> ftile;
};

// "" on success, else the error message.  tiles * sub_per_tile must fit int32 (the per-point
// kernels' sub-tile index).
std::string plan_batch(const int64_t* counts, int32_t n_frames, int32_t tile_groups, int32_t sub_per_tile,
                       BatchLayout* out);

// The merged-cloud gather (LMC:887-889 np.vstack of the frame-ordered shards; comm.cpp): shard q
// (P[q] padded points, C[q] >= merged_C columns per block) lands at padded offset off[q] of the
// merged batch, i.e. the rank-ordered concatenation.  Shards other than the root's whose column
// count differs from the merged batch's are received into a staging area (stage_off[q] = value
// offset, -1 = received in place) and re-pitched block by block; the root's own shard is copied
// or re-pitched straight from its batch.  A shard with fewer columns than the merged batch is an
// error (its missing column would be left undefined).
struct GatherPlan {
  std::vector<int64_t> off;
  std::vector<int64_t> stage_off;
  int64_t stage_values = 0;
};
std::string plan_gather(int32_t nranks, int32_t root, const int64_t* P, const int64_t* C, int64_t merged_P,
                        int64_t merged_C, GatherPlan* out);

// The merged batch's frames must be the rank-ordered concatenation of the shards' frames, not
// merely the same padded total ([300, 100] and [100, 300] pad alike).  In one process the counts
// are compared directly (check_frame_concat); across ranks each shard sends (frame count, rolling
// hash of its counts) and the root checks the merged batch's hash against the chained shard hashes:
// H(a ++ b) = H(a) * B^len(b) + H(b) (mod 2^64).
uint64_t counts_hash(const int64_t* counts, int64_t n);
uint64_t hash_concat(uint64_t ha, uint64_t hb, int64_t nb);
std::string check_frame_concat(int32_t nranks, const int64_t* const* shard_counts, const int64_t* shard_F,
                               const int64_t* merged_counts, int64_t merged_F);
std::string check_frame_hashes(int32_t nranks, const int64_t* F, const uint64_t* H, int64_t merged_F,
                               uint64_t merged_H);

// Where rank q's C[q] * P[q] values are received: in place in the merged batch, or staged.
inline float* gather_dst(const GatherPlan& G, int32_t q, float* merged, int64_t merged_C, float* stage) {
  return G.stage_off[q] >= 0 ? stage + G.stage_off[q] : merged + G.off[q] * merged_C;
}

// After the shards arrived: the root's own shard (root_src, its batch's columns) and every staged
// shard, re-pitched to merged_C columns per block.  Primitives, in float values:
//   copy(dst, src, n)                               contiguous
//   copy2d(dst, dpitch, src, spitch, width, rows)   one row per block
// Returns the first non-zero status of a primitive.
template <class Copy, class Copy2D>
int gather_finish(const GatherPlan& G, int32_t nranks, int32_t root, const int64_t* P, const int64_t* C,
                  float* merged, int64_t merged_C, const float* root_src, const float* stage, Copy copy,
                  Copy2D copy2d) {
  auto repitch = [&](const float* src, int64_t cs, int64_t np, int64_t off) {
    const int64_t w = std::min(cs, merged_C);
    return copy2d(merged + off * merged_C, merged_C * kBlk, src, cs * kBlk, w * kBlk, np / kBlk);
  };
  if (P[root] > 0) {
    const int r = C[root] == merged_C ? copy(merged + G.off[root] * merged_C, root_src, C[root] * P[root])
                                      : repitch(root_src, C[root], P[root], G.off[root]);
    if (r) return r;
  }
  for (int32_t q = 0; q < nranks; ++q)
    if (G.stage_off[q] >= 0)
      if (const int r = repitch(stage + G.stage_off[q], C[q], P[q], G.off[q])) return r;
  return 0;
}

}  // namespace mcplan
