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

// Stream order of a launch over n units (workgroup b -> unit): bit 1 = the 8 contiguous XCD ranges of
// xcd_unit<true> (else in order), bit 0 = reversed (within each range).  Codec kernels take the order
// that starts where the previous kernel over the same batch ended (mc_batch::hot_order), while those
// points may still sit in the 256 MB Infinity Cache.  A bijection on [0, n) for any n.
__device__ __forceinline__ int64_t stream_unit(int order, int64_t b, int64_t n) {
  const bool rev = (order & 1) != 0;
  if (order & 2) {
    const int64_t x = b % kXcds, i = b / kXcds, per = n / kXcds, rem = n % kXcds;
    const int64_t len = per + (x < rem ? 1 : 0), start = x * per + (x < rem ? x : rem);
    return start + (rev ? len - 1 - i : i);
  }
  return rev ? n - 1 - b : b;
}

// 64-bit integer minimum (HIP's min / max templates resolve int64_t arguments through float64
// conversions on gfx950: six VALU instructions for a wave-uniform value)
__device__ __forceinline__ int64_t min_i64(int64_t a, int64_t b) { return a < b ? a : b; }

// wave-uniform load (memory the kernel never writes) through the constant address space -> s_load_dword* into SGPRs
template <typename T>
__device__ __forceinline__ T ldu(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "ldu needs a dword-multiple type");
  struct Raw { int v[sizeof(T) / 4]; };
  typedef __attribute__((address_space(4))) const int CI;
  CI* q = (CI*)(p);
  Raw r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) r.v[i] = q[i];
  return __builtin_bit_cast(T, r);
}

// component c of a float4 / int4 (c a compile-time constant after unrolling)
__device__ __forceinline__ float& f4c(float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ float f4g(const float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ int i4c(const int4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

// ASCII PCD text bytes of a wave's float32 values (LMC:948 "%.6f" + ' ' / '\n') on the packed path,
// |v| < 4294: each value is [-] + 1..4 integer digits + '.' + 6 digits + separator = 9 + [v < 0] +
// [|v| >= 10] + [|v| >= 100] + [|v| >= 1000] bytes (a float32 never rounds across a power of ten at
// six decimals: the float32 below 10 is 9.99999905).  Any value outside the packed path (NaN, inf,
// |v| >= 4294) adds kPcdSlowValue: a block whose count reaches it holds a line for the exact
// formatter (the measure pass).  Per-lane sums (compares + adds) with one wave reduction at the end:
// a ballot per term added up on the scalar unit was slower (+15 / +36 / +47 us: the 64-bit masks
// spilled SGPRs into VGPR lanes, profiles/round3/s12).
constexpr int kPcdSlowValue = 1 << 20;
constexpr uint32_t kPcdSlowBits = 0x45863000u;   // |v| >= 4294.0f as a float32 bit pattern
struct PcdCount {
  int n = 0;          // this lane's sum
  uint32_t amax = 0;  // largest |v| bit pattern of the lane's valid values (NaN / inf above any finite)
  __device__ __forceinline__ void add(bool valid, float v) {
    const uint32_t u = (uint32_t)__float_as_int(v), ua = u & 0x7fffffffu;
    const float a = __int_as_float((int)ua);
    const int len = 9 + (int)(u >> 31) + (a >= 10.0f ? 1 : 0) + (a >= 100.0f ? 1 : 0) + (a >= 1000.0f ? 1 : 0);
    n += valid ? len : 0;
    amax = valid && ua > amax ? ua : amax;
  }
  __device__ __forceinline__ static bool lanes(bool valid) { return valid; }
  __device__ __forceinline__ int bytes() const {   // the wave total (every lane takes part)
    int t = n;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    const bool slow = __builtin_amdgcn_ballot_w64(amax >= kPcdSlowBits) != 0;
    return t + (slow ? kPcdSlowValue : 0);
  }
};

// DPP quad exchange (quad_perm): lanes 4q .. 4q + 3 of a wave form a quad.
template <int K>   // quad_perm [K, K, K, K]: lane K of each quad to all four
__device__ __forceinline__ float quad_bcast(float v) {
  // bound_ctrl: quad_perm never reads outside the quad, so no "old" value has to be set up first
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), K * 0x55, 0xF, 0xF, true));
}
// component k (= this lane's index in its quad) of lane L's float4: with L = 0 .. 3 over a quad
// whose lane c holds column c of four points, lane k gets point k's columns (a 4 x 4 transpose)
template <int L>
__device__ __forceinline__ float quad_pick(const float4& v, int k) {
  const float a = quad_bcast<L>(v.x), b = quad_bcast<L>(v.y), c = quad_bcast<L>(v.z), d = quad_bcast<L>(v.w);
  return k == 0 ? a : (k == 1 ? b : (k == 2 ? c : d));
}

}  // namespace mc
