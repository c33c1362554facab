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
// formatter (the measure pass).
//
// Two values at a time in 16-bit halves (round 6): the thresholds 10, 100 and 1000 are float32s
// whose low 16 bits are zero, so |v| >= T is a compare of the upper halves, and the upper halves of
// two values pack into one register (v_perm_b32) for the packed 16-bit ALU — each [h >= T] is a
// saturating subtract and a min (v_pk_sub_u16 clamp, v_pk_min_u16), added with v_pk_add_u16.  The
// slow test on upper halves flags |v| >= 4288 (0x4586 << 16): a value in [4288, 4294) sends its block
// to the measure pass, which formats it exactly.  Per-lane sums with one DPP wave reduction at the
// end (a ballot per term added up on the scalar unit was slower, profiles/round3/s12).
constexpr int kPcdSlowValue = 1 << 20;
constexpr uint32_t kPcdSlowBits = 0x45860000u;   // |v| >= 4288.0f: conservatively outside the packed path
// per 16-bit half of m: [m > c] (v_pk_sub_u16 clamp saturates at 0, v_pk_min_u16 caps at 1), as
// inline asm: written with clang's elementwise builtins the two became a compare + select per half
__device__ __forceinline__ uint32_t pk_gt_u16(uint32_t m, uint32_t c2) {
  uint32_t d, r;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(d) : "v"(m), "s"(c2));
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(d), "s"(0x00010001u));
  return r;
}
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_pk_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// the wave's sum, in every lane: DPP within each 16-lane row (pairs, quads, half-row and row
// mirrors), then the four rows' sums read from lanes 0, 16, 32, 48 (no LDS permutes)
__device__ __forceinline__ int wave_sum_dpp(int t) {
  t += __builtin_amdgcn_update_dpp(0, t, 0xB1, 0xF, 0xF, true);    // quad_perm [1, 0, 3, 2]
  t += __builtin_amdgcn_update_dpp(0, t, 0x4E, 0xF, 0xF, true);    // quad_perm [2, 3, 0, 1]
  t += __builtin_amdgcn_update_dpp(0, t, 0x141, 0xF, 0xF, true);   // row_half_mirror
  t += __builtin_amdgcn_update_dpp(0, t, 0x140, 0xF, 0xF, true);   // row_mirror
  return __builtin_amdgcn_readlane(t, 0) + __builtin_amdgcn_readlane(t, 16) + __builtin_amdgcn_readlane(t, 32) +
         __builtin_amdgcn_readlane(t, 48);
}
struct PcdCount {
  uint32_t acc = 0;    // two 16-bit halves: signs + integer digits beyond the first, of the lane's values
  uint32_t amax = 0;   // two 16-bit halves: the largest |v| upper 16 bits
  int n = 0;           // the lane's valid values (9 bytes each before the counts)
  // two values (the upper halves packed by v_perm_b32, b's low); an invalid one counts as +0.0 and
  // adds no bytes
  __device__ __forceinline__ void add2(bool va, float a, bool vb, float b) {
    pack(__builtin_amdgcn_perm(va ? __float_as_uint(a) : 0u, vb ? __float_as_uint(b) : 0u, 0x07060302u));
    n += (va ? 1 : 0) + (vb ? 1 : 0);
  }
  // two values of one point (one validity)
  __device__ __forceinline__ void add2(bool v, float a, float b) {
    const uint32_t h = __builtin_amdgcn_perm(__float_as_uint(a), __float_as_uint(b), 0x07060302u);
    pack(v ? h : 0u);
    n += v ? 2 : 0;
  }
  __device__ __forceinline__ void pack(uint32_t h) {
    const uint32_t m = h & 0x7FFF7FFFu;
    acc = pk_add_u16(acc, (h >> 15) & 0x00010001u);
    acc = pk_add_u16(acc, pk_gt_u16(m, 0x411F411Fu));   // |v| >= 10
    acc = pk_add_u16(acc, pk_gt_u16(m, 0x42C742C7u));   // |v| >= 100
    acc = pk_add_u16(acc, pk_gt_u16(m, 0x44794479u));   // |v| >= 1000
    amax = pk_max_u16(amax, m);
  }
  __device__ __forceinline__ int lane_bytes() const { return 9 * n + (int)(acc & 0xFFFFu) + (int)(acc >> 16); }
  __device__ __forceinline__ bool lane_slow() const {
    const uint32_t lo = amax & 0xFFFFu, hi = amax >> 16;
    return (lo > hi ? lo : hi) >= (kPcdSlowBits >> 16);
  }
  __device__ __forceinline__ int bytes() const {   // the wave total (every lane takes part)
    const bool slow = __builtin_amdgcn_ballot_w64(lane_slow()) != 0;
    return wave_sum_dpp(lane_bytes()) + (slow ? kPcdSlowValue : 0);
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
