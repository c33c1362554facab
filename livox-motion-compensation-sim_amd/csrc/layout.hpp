// layout.hpp — the batch's blocked column index and the XCD-aware workgroup -> unit order, shared
// by the deskew, stager, scan and codec kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

// Blocked batch layout: block k = points 256k .. 256k+255 holds its C columns as C
// runs of 256 values; frames start on a block, so tiles and frame ranges are whole blocks.
constexpr int kBlkPts = 256;
__host__ __device__ __forceinline__ int64_t bidx(int C, int c, int64_t p) {
  return ((p >> 8) * C + c) * kBlkPts + (p & (kBlkPts - 1));
}

// XCD-aware unit order.  Workgroups are dealt round-robin over the 8 XCDs (observed; speed only,
// never correctness): unit order b -> contiguous runs per XCD, so the 16-byte per-unit records
// (tiles, sub-tile windows) of neighbouring units share 128-byte lines inside one XCD's L2
// instead of each workgroup fetching its own line.  A bijection on [0, n) for any n.
constexpr int kXcds = 8;
template <bool ON>
__device__ __forceinline__ int64_t xcd_unit(int64_t b, int64_t n) {
  if (!ON) return b;
  const int64_t x = b % kXcds, i = b / kXcds, per = n / kXcds, rem = n % kXcds;
  return x * per + (x < rem ? x : rem) + i;
}

}  // namespace mc
