// codecs.hpp — gfx950 kernels for the reference's output codecs, encoding
// straight from a device-resident (N, ld) float64 AoS cloud (the array layout of LMC:770 / 776):
//
//   LVX v1.1 packer  LMC:24-272   96-point packages of 14-byte records (int32 mm + reflectivity)
//   ASCII PCD body   LMC:932-948  "%.6f %.6f %.6f %.6f\n" per point, correctly rounded
//
// Both produce byte streams whose records are not 4-byte aligned (14-byte LVX records, variable
// PCD lines).  Each workgroup therefore assembles its contiguous piece of the output in LDS at the
// same offset modulo 16 as in HBM, then stores it with 16-byte stores by consecutive lanes; only
// the two partial 16-byte chunks at the ends of the piece are written with narrow stores.
// Frames map to "units" (LVX package chunks, PCD tiles) through a per-frame prefix, so one launch
// covers every frame of a batch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

// File bytes are stored non-temporally (written once, never re-read): LVX 308.4 vs 325.2 us, PCD
// 1005.5 vs 1057.8 us with plain stores (profiles/round3/s21/ab_codec_nt.log); sc1 write-through was
// slower still (LVX 381.6 vs 302.9 us, PCD 1164.8 vs 1014.7 us, s50).  Non-temporal loads of the
// batch's columns gave nothing (1000.6 vs 1004.1 us PCD, s24).
#ifndef MC_XCD_CODEC
#define MC_XCD_CODEC 0       // PCD unit order: dealt — write pass 807.5 / 800.7 vs 832.8 / 831.0 us
                             // XCD-contiguous, fused PCD share 0.514 / 0.519 vs 0.502 / 0.500, measure +
                             // write 1012.1 vs 1024.1 us (profiles/round3/s61)
#endif
// (The LVX packer and the float32 PCD passes take their unit order at run time from the batch's hot
// end, layout.hpp stream_unit; standalone, dealt beat XCD-contiguous for LVX as well: 304.5 / 305.5 /
// 305.1 vs 310.6 / 314.9 / 319.5 us, profiles/round3/s58, s59.)

namespace mc {

constexpr int kCodecBlock = 256;
constexpr int kLvxPkgPoints = 96;
constexpr int kLvxRec = 14;
constexpr int kLvxPkgHdr = 22;
constexpr int kLvxPkg = kLvxPkgHdr + kLvxPkgPoints * kLvxRec;   // 1366 bytes
constexpr int kLvxFrameHdr = 24;
constexpr int kLvxFileHdr = 88;
constexpr int kLvxPkgPerWG = 8;                                 // one unit = up to this many packages of a frame
constexpr int kLvxUnitPoints = kLvxPkgPerWG * kLvxPkgPoints;    // 768
constexpr int kLvxLds = kLvxPkgPerWG * kLvxPkg + 16 + 24;       // + alignment shift + a frame header
constexpr int kLvxSlots = kLvxUnitPoints / kCodecBlock;         // 3 batch blocks per unit
static_assert(kLvxUnitPoints % kCodecBlock == 0, "unit = whole blocks");
#ifndef MC_PCD_MEASURE_SCALAR
#define MC_PCD_MEASURE_SCALAR 1   // float32 measure pass: wave-uniform tile arithmetic (scalar), DPP wave sum
#endif
#ifndef MC_PCD_TILES_PER_WG
#define MC_PCD_TILES_PER_WG 4   // 4 / 8 / 16 / 32: 1048.0 / 1023.5 / 1029.2 / 1054.9 us (profiles/round2/s26,
                                // XCD unit order); in the dealt order 4 wins: write pass 788.0 / 741.0 vs
                                // 822.6 / 772.1 us (SLERP / frame source), fused PCD share 0.527 / 0.561 vs
                                // 0.507 / 0.537 (profiles/round3/s66, s67)
#endif
constexpr int kPcdTilesPerWG = MC_PCD_TILES_PER_WG;             // PCD tiles per measure / byte-path workgroup
constexpr int kPcdBlock = 256;   // PCD: threads per workgroup = lines per tile (512: 1088 / 1085 vs 1080 us, profiles/round2/s40)
constexpr int kPcdTileText = kPcdBlock * 64;                     // LDS text buffer per tile (packed lines <= 52 B)
constexpr int kPcdPackedText = kPcdBlock * 52 + 16;              // a packed tile's text + its HBM offset mod 16

struct CodecFrames {
  const double* aos; int64_t ld;   // (N, ld) float64 AoS source, or
  const float* cols; int32_t C;    // a batch's blocked float32 columns (cols != null; ld = 4)
  const int64_t* poff;             // [F+1] the batch's padded frame offsets
  const int64_t* doff;       // [F+1] dense row offset of each frame
  const int64_t* unit_off;   // [F+1] prefix of per-frame units
  int32_t F;
  int64_t n_units;           // unit_off[F]
  double frames_per_unit;    // F / n_units (codec_frame_of's guess without an integer division)
};

// frame owning unit u: last f with unit_off[f] <= u (frames without units are skipped over).
// First the interpolation guess u * F / n_units with its two bounds (one round of loads when the
// frames are of similar size), the binary search (~log2 F dependent loads) otherwise.  The guess
// multiplies by the host's F / n_units in float64 (MC_CODEC_GUESS_F64): the integer quotient was a
// 64-bit division on the scalar unit, ~130 dependent instructions at the head of every workgroup.
#ifndef MC_CODEC_GUESS_F64
#define MC_CODEC_GUESS_F64 1
#endif
__device__ __forceinline__ int32_t codec_frame_of(const CodecFrames& s, int64_t u) {
  const int64_t* __restrict__ unit_off = s.unit_off;
  if (s.n_units > 0) {
    // (+1e-6: u * ratio rounds to within 2^-21 of the exact quotient, which is an integer at every
    // frame's first unit when the frames are equal)
    int64_t g = MC_CODEC_GUESS_F64 ? (int64_t)((double)u * s.frames_per_unit + 1e-6)
                                   : u * s.F / s.n_units;   // u < 2^31 and F < 2^31: no overflow
    g = g < s.F - 1 ? g : s.F - 1;
    if (ldu(unit_off + g) <= u && u < ldu(unit_off + g + 1)) return (int32_t)g;
  }
  int32_t lo = 0, hi = s.F + 1;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (ldu(unit_off + mid) <= u) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

// columns 0..3 of dense row `row` (frame f) as float64; ld == 3 leaves c[3] = 0.  A batch source
// widens its float32 values exactly, so both sources give the bytes of the reference writer applied
// to the same (N,4) float64 array (Batch.download_aos()).
__device__ __forceinline__ void codec_point(const CodecFrames& s, int32_t f, int64_t row, double c[4]) {
  if (s.cols) {
    const float* q = s.cols + bidx(s.C, 0, s.poff[f] + (row - s.doff[f]));
    c[0] = q[0]; c[1] = q[kBlkPts]; c[2] = q[2 * kBlkPts]; c[3] = q[3 * kBlkPts];
    return;
  }
  const double* q = s.aos + row * s.ld;
  if (s.ld == 4) {
    const double2 p01 = *reinterpret_cast<const double2*>(q);
    const double2 p23 = *reinterpret_cast<const double2*>(q + 2);
    c[0] = p01.x; c[1] = p01.y; c[2] = p23.x; c[3] = p23.y;
  } else {
    c[0] = q[0]; c[1] = q[1]; c[2] = q[2];
    c[3] = s.ld > 3 ? q[3] : 0.0;
  }
}

// advance a workgroup-uniform frame cursor to unit u (units of a workgroup are consecutive)
__device__ __forceinline__ int32_t codec_advance(const int64_t* __restrict__ unit_off, int32_t f, int64_t u) {
  while (ldu(unit_off + f + 1) <= u) ++f;
  return f;
}

// A text / record chunk's 16-byte store: non-temporal (sc1 write-through, the deskew kernels' policy:
// LVX 336.6 vs 304.3 us, PCD measure + write 1065.4 vs 798.9 us, profiles/round5/s02; non-temporal
// point loads: LVX +-0, PCD 776.0 vs 772.5-798.9 us across identical builds — not taken)
typedef unsigned int codec_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void codec_st16(char* p, const uint4& v) {
  __builtin_nontemporal_store(codec_v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<codec_v4u*>(p));
}
// bytes of LDS [lo, hi) outside the full chunks [f0, f1) (the partial end chunks) -> g, lanes t < 32
// of the workgroup, one byte each: lanes 0-15 the head chunk lo / 16, lanes 16-31 the tail chunk hi / 16
__device__ __forceinline__ void codec_store_edges(char* __restrict__ g, const char* lds, int lo, int hi, int f0, int f1,
                                                  int t) {
  if (t < 32) {
    const int ch = t < 16 ? lo >> 4 : hi >> 4;
    const int b = 16 * ch + (t & 15);
    const bool in = b >= lo && b < hi && !(ch >= f0 && ch < f1) && !(t >= 16 && (lo >> 4) == (hi >> 4));
    if (in) g[b] = lds[b];
  }
}

// Store LDS bytes [lo, hi) to g + [lo, hi), where lds and g agree modulo 16: whole 16-byte chunks
// with dwordx4 stores, the partial chunks at either end byte by byte.  All threads participate.
// MAXCH > 0: the piece holds at most MAXCH chunks; each lane issues all of its LDS chunk reads before
// its first store (the loop waits for every read) and 32 lanes store the end bytes at once (LVX 293.0
// vs 296.0 us, profiles/round5/s04).  MAXCH = 0: a loop (the byte path's pieces vary in size).
// (Partial chunks from one 16-byte LDS read + predicated byte stores: 50 instead of 56 VGPRs in the
// LVX kernel but LVX 310.4 vs 308.2, PCD 808.4 vs 803.3 us, profiles/round4/s12: not taken.)
template <int NT = kCodecBlock, int MAXCH = 0>   // NT: threads of the workgroup
__device__ __forceinline__ void codec_store_piece(char* __restrict__ g, const char* lds, int lo, int hi) {
  if constexpr (MAXCH > 0) {
    const int f0 = (lo + 15) >> 4, f1 = hi >> 4;
    constexpr int kIt = (MAXCH + NT - 1) / NT;
    uint4 v[kIt];
#pragma unroll
    for (int u = 0; u < kIt; ++u) {
      const int c = f0 + (int)threadIdx.x + u * NT;
      if (c < f1) v[u] = *reinterpret_cast<const uint4*>(lds + 16 * c);
    }
#pragma unroll
    for (int u = 0; u < kIt; ++u) {
      const int c = f0 + (int)threadIdx.x + u * NT;
      if (c < f1) codec_st16(g + 16 * c, v[u]);
    }
    codec_store_edges(g, lds, lo, hi, f0, f1, (int)threadIdx.x);
    return;
  }
  const int c0 = lo >> 4, c1 = (hi + 15) >> 4;
  for (int c = c0 + threadIdx.x; c < c1; c += NT) {
    const int b0 = c << 4;
    if (b0 >= lo && b0 + 16 <= hi) {
      codec_st16(g + b0, *reinterpret_cast<const uint4*>(lds + b0));
    } else {
      const int e = b0 + 16 < hi ? b0 + 16 : hi;
      for (int b = b0 > lo ? b0 : lo; b < e; ++b) g[b] = lds[b];
    }
  }
}

// ---- LVX v1.1 -------------------------------------------------------------------------------
struct LvxArgs {
  CodecFrames src;
  const int64_t* frame_pos;     // [F + 1] byte offset of each frame in the file, then the file size
  const uint64_t* frame_id;     // [F]
  const uint64_t* ts_ns;        // [F] package timestamp, int(timestamp * 1e9) (LMC:176)
  const uint8_t* has_int;       // [F] frame has an intensity column (else reflectivity 128), or null
  char* out;                    // file base
  int* err;                     // set to 1 on a NaN coordinate / intensity (LMC:259, 268 int(nan))
  int order;                    // stream_unit order of the package units
};

// int(np.clip(v * scale, lo, hi)) (LMC:259-261, 268): truncation toward zero after the clip
__device__ __forceinline__ int32_t lvx_fixed(double v, double scale, double lo, double hi, int* err) {
  const double s = v * scale;
  if (s != s) { *err = 1; return 0; }
  return (int32_t)fmin(fmax(s, lo), hi);
}

// MC_LVX_DIAG (diagnostic builds only, wrong output): 1 = no point loads (records formed from the slot
// index), 2 = no HBM stores (the assembled LDS piece is read but only a never-true test of it stores),
// 3 = both.  Naming the packer's limiter: its time with each part removed (tools/ab_codecs.py,
// profiles/round5/s02: 196.0 / 186.6 / 117.1 vs 304.3 us).
#ifndef MC_LVX_DIAG
#define MC_LVX_DIAG 0
#endif
// One unit = up to 8 consecutive packages of one frame = one contiguous byte range of the file.
// Phase 1: a thread per point slot writes its 14-byte record (7 halfwords, zero for the padding
// slots of the last package, LMC:245-248), threads 0..k*11 the 22-byte package headers
// (LMC:204-237) and, in a frame's first unit, threads 96..107 the frame header (LMC:178-193: own
// offset, next frame's offset, frame id) into LDS.  Phase 2: codec_store_piece.  k_lvx_frames writes
// the headers of frames without points (they have no unit).  Folding the frame headers in removed a
// launch: 296.0 vs 302.2 us (profiles/round5/s04).
// Rejected (tools/ab_codecs.py --source batch): 2 / 4 / 8 units per workgroup with the next unit's
// points loaded while one is stored (305.0 vs 333.9-356.4 us, profiles/round3/s69); a batch-only unit
// kernel with 32-bit scalar unit arithmetic, all 12 loads of a lane up front and branch-free records
// (336.8 vs 306.8 us, profiles/round5/s01); 768 / 512 threads per workgroup (497.8 / 384.6 vs 304.3
// us, s02); records as naturally aligned LDS stores instead of the compiler's ds_write_b96 at 2-byte
// alignment (303.5 vs 305.3, s03) and with every point load issued up front (301.2; 315.4 vs 293.0
// on top of the folded headers and unrolled stores, s04); the frame metadata loaded for the frame
// guess in the guess's own scalar round (297.9 vs 292.4, s06); a branch-free NaN flag with one error
// store per lane and each package header written by one thread (35 % fewer instructions: 299.7 vs
// 292.7; either alone 296.2 / 293.2, s12) — the packer is not issue-bound.
__global__ __launch_bounds__(kCodecBlock) void k_lvx_packages(const LvxArgs a) {
  static_assert(kCodecBlock >= 96 + 12 && kLvxPkgPerWG * (kLvxPkgHdr / 2) <= 96, "header threads");
  __shared__ uint4 s_buf[kLvxLds / 16 + 1];
  uint16_t* const s16 = reinterpret_cast<uint16_t*>(s_buf);
  const int64_t u = stream_unit(a.order, blockIdx.x, gridDim.x);   // grid = units exactly
  const int32_t f = codec_frame_of(a.src, u);
  const int64_t pkg0 = (u - a.src.unit_off[f]) * kLvxPkgPerWG;
  const int64_t frow = a.src.doff[f];
  const int64_t fcount = a.src.doff[f + 1] - frow;
  const int64_t fpkgs = (fcount + kLvxPkgPoints - 1) / kLvxPkgPoints;
  const int k = (int)((fpkgs - pkg0) < kLvxPkgPerWG ? (fpkgs - pkg0) : kLvxPkgPerWG);
  const int64_t rem = fcount - pkg0 * kLvxPkgPoints;
  const int n = (int)(rem < k * kLvxPkgPoints ? rem : k * kLvxPkgPoints);
  const int hdr = pkg0 == 0 ? kLvxFrameHdr : 0;                            // frame header bytes first
  const int64_t S = a.frame_pos[f] + kLvxFrameHdr + pkg0 * kLvxPkg - hdr;   // piece start, even
  const int shift = (int)(S & 15) + hdr;                                    // LDS offset of the first package
  const uint64_t ts = a.ts_ns[f];
  const bool hi = a.has_int ? a.has_int[f] != 0 : a.src.ld > 3;
  const int64_t row0 = frow + pkg0 * kLvxPkgPoints;

#pragma unroll
  for (int j = 0; j < kLvxSlots; ++j) {   // a unit's 768 slots: three passes of the workgroup
    const int i = j * kCodecBlock + (int)threadIdx.x;
    if (i >= k * kLvxPkgPoints) break;
    const int pk = i / kLvxPkgPoints, slot = i - pk * kLvxPkgPoints;
    uint16_t* r = s16 + ((shift + pk * kLvxPkg + kLvxPkgHdr + slot * kLvxRec) >> 1);
    uint32_t x = 0, y = 0, z = 0, refl = 0;
    if ((MC_LVX_DIAG & 1) && i < n) {
      x = (uint32_t)i; y = x * 3u; z = x ^ 0x5555u; refl = x & 255u;
    } else if (i < n) {
      double v[4];
      codec_point(a.src, f, row0 + i, v);
      x = (uint32_t)lvx_fixed(v[0], 1000.0, -2147483648.0, 2147483647.0, a.err);
      y = (uint32_t)lvx_fixed(v[1], 1000.0, -2147483648.0, 2147483647.0, a.err);
      z = (uint32_t)lvx_fixed(v[2], 1000.0, -2147483648.0, 2147483647.0, a.err);
      refl = hi ? (uint32_t)lvx_fixed(v[3], 255.0, 0.0, 255.0, a.err) : 128u;   // tag byte 0
    }
    r[0] = (uint16_t)x; r[1] = (uint16_t)(x >> 16);
    r[2] = (uint16_t)y; r[3] = (uint16_t)(y >> 16);
    r[4] = (uint16_t)z; r[5] = (uint16_t)(z >> 16);
    r[6] = (uint16_t)refl;
  }
  // dev 0, version 5 | slot 0, lidar 1 | reserved, status (4 B) | ts type 1 | data type 2 |
  // reserved (3 B) | timestamp (8 B)
  for (int h = threadIdx.x; h < k * (kLvxPkgHdr / 2); h += kCodecBlock) {
    const int pk = h / (kLvxPkgHdr / 2), w = h - pk * (kLvxPkgHdr / 2);
    uint32_t v;
    switch (w) {
      case 0: v = 0x0500u; break;
      case 1: v = 0x0100u; break;
      case 4: v = 0x0100u; break;
      case 5: v = 0x0002u; break;
      case 7: case 8: case 9: case 10: v = (uint32_t)(ts >> (16 * (w - 7))) & 0xffffu; break;
      default: v = 0u;
    }
    s16[((shift + pk * kLvxPkg) >> 1) + w] = (uint16_t)v;
  }
  if (hdr && threadIdx.x >= 96 && threadIdx.x < 96 + 12) {   // own offset, next frame's (0 after the last), id
    const int i = (int)threadIdx.x - 96;
    const uint64_t q = i < 4 ? (uint64_t)a.frame_pos[f] : i < 8 ? (f + 1 < a.src.F ? (uint64_t)a.frame_pos[f + 1] : 0ull)
                                                             : a.frame_id[f];
    s16[((shift - hdr) >> 1) + i] = (uint16_t)(q >> (16 * (i & 3)));
  }
  __syncthreads();
  if constexpr ((MC_LVX_DIAG & 2) != 0) {
    const uint4 v = s_buf[threadIdx.x];   // every LDS word is live; (almost) nothing reaches HBM
    if (v.x == 0x7eadbeefu && v.y == 0x7eadbeefu) a.out[S] = 1;
    return;
  }
  codec_store_piece<kCodecBlock, kLvxLds / 16 + 1>(a.out + (S - (shift - hdr)), reinterpret_cast<const char*>(s_buf),
                                                   shift - hdr, shift + k * kLvxPkg);
}

// LMC:178-193: frame header = own offset, next frame's offset (0 for the last), frame_id
__global__ __launch_bounds__(kCodecBlock) void k_lvx_frames(const LvxArgs a, int64_t next_of_last_frame) {
  const int32_t f = blockIdx.x * kCodecBlock + threadIdx.x;
  if (f >= a.src.F) return;
  const uint64_t q[3] = {(uint64_t)a.frame_pos[f],
                         f + 1 < a.src.F ? (uint64_t)a.frame_pos[f + 1] : (uint64_t)next_of_last_frame,
                         a.frame_id[f]};
  uint16_t* o = reinterpret_cast<uint16_t*>(a.out + a.frame_pos[f]);
#pragma unroll
  for (int i = 0; i < 12; ++i) o[i] = (uint16_t)(q[i >> 2] >> (16 * (i & 3)));
}

// ---- "%.6f" (Python's correctly rounded fixed-point float formatting) -------------------------
// v = m * 2^e exactly; N = round-half-even(|v| * 10^6) in 128-bit integer arithmetic, printed as
// ip = N / 10^6, "." and the six digits of N % 10^6.  |v| < 2^107 (~1.6e32) is supported; larger
// values set the error flag.  |v| < 4294.97 (N < 2^32, every LiDAR coordinate) stays in 32-bit
// integer arithmetic.
struct Fmt6 {
  unsigned __int128 ip;
  uint32_t fp;
  int nd;      // digits of ip
  int len;     // characters
  int kind;    // 0 finite, 1 inf, 2 nan, 3 out of range
  bool neg;
};

__device__ __forceinline__ int u32_digits(uint32_t x) {
  return 1 + (x >= 10u) + (x >= 100u) + (x >= 1000u) + (x >= 10000u) + (x >= 100000u) + (x >= 1000000u) +
         (x >= 10000000u) + (x >= 100000000u) + (x >= 1000000000u);
}

__device__ __noinline__ Fmt6 fmt6_prepare_exact(double v);

// Common case, |v| < 4294: y = |v| * 1e6 in double is within 2.4e-7 of the exact product, so
// unless y's fraction is within 1e-6 of one half the rounded integer is floor(y) or floor(y) + 1
// as decided by the fraction — no 128-bit arithmetic.  Otherwise (and for NaN / inf / large
// magnitudes) the exact path decides.
__device__ __forceinline__ Fmt6 fmt6_prepare(double v) {
  const double a = fabs(v);
  if (a < 4294.0) {
    const double y = a * 1000000.0;
    const double fl = floor(y);
    const double fr = y - fl;
    if (fabs(fr - 0.5) > 1e-6) {
      Fmt6 r;
      const uint32_t n = (uint32_t)fl + (fr > 0.5 ? 1u : 0u);
      const uint32_t ip = n / 1000000u;
      r.neg = signbit(v);
      r.kind = 0;
      r.ip = ip;
      r.fp = n - ip * 1000000u;
      r.nd = 1 + (ip >= 10u) + (ip >= 100u) + (ip >= 1000u);
      r.len = (r.neg ? 1 : 0) + r.nd + 7;
      return r;
    }
  }
  return fmt6_prepare_exact(v);
}

__device__ __noinline__ Fmt6 fmt6_prepare_exact(double v) {
  Fmt6 r;
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  r.neg = (bits >> 63) != 0;
  const int ex = (int)((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  r.ip = 0; r.fp = 0; r.nd = 1;
  if (ex == 0x7ff) {                                // "nan" (Python drops a NaN's sign) / "inf" / "-inf"
    r.kind = frac ? 2 : 1;
    r.len = 3 + (r.kind == 1 && r.neg ? 1 : 0);
    return r;
  }
  const uint64_t m = ex ? (frac | (1ull << 52)) : frac;
  const int e = ex ? ex - 1075 : -1074;
  const unsigned __int128 P = (unsigned __int128)m * 1000000u;   // < 2^73
  unsigned __int128 N = 0;
  if (e >= 0) {
    if (e > 54) { r.kind = 3; r.len = 0; return r; }
    N = P << e;
  } else if (-e < 74) {
    const int s = -e;
    const unsigned __int128 one = 1;
    unsigned __int128 q = P >> s;
    const unsigned __int128 rem = P & ((one << s) - 1);
    const unsigned __int128 half = one << (s - 1);
    if (rem > half || (rem == half && (q & 1))) ++q;
    N = q;
  }
  r.kind = 0;
  if ((uint64_t)(N >> 32) == 0) {
    const uint32_t n = (uint32_t)N;
    const uint32_t ip = n / 1000000u;
    r.ip = ip;
    r.fp = n - ip * 1000000u;
    r.nd = u32_digits(ip);
  } else {
    const unsigned __int128 ip = (uint64_t)(N >> 64) == 0 ? (unsigned __int128)((uint64_t)N / 1000000u)
                                                          : N / 1000000u;
    r.ip = ip;
    r.fp = (uint32_t)(N - ip * 1000000u);
    int d = 1;
    for (unsigned __int128 x = ip; x >= 10; x /= 10) ++d;
    r.nd = d;
  }
  r.len = (r.neg ? 1 : 0) + r.nd + 7;
  return r;
}

// the last min(n, 3) decimal digits of x < 1000 at q[3-n .. 2] (q[0..2] = hundreds, tens, units)
__device__ __forceinline__ void put3(char* q, uint32_t x, int n) {
  const uint32_t h = __umul24(x, 41u) >> 12;
  const uint32_t r = x - h * 100u;
  const uint32_t t = __umul24(r, 103u) >> 10;
  if (n >= 3) q[0] = (char)('0' + h);
  if (n >= 2) q[1] = (char)('0' + t);
  q[2] = (char)('0' + (r - t * 10u));
}

// writes f.len characters at p (generic pointer: LDS or global)
__device__ __forceinline__ void fmt6_write(const Fmt6& f, char* p) {
  if (f.kind == 3) return;
  if (f.kind == 2) { p[0] = 'n'; p[1] = 'a'; p[2] = 'n'; return; }
  if (f.neg) *p++ = '-';
  if (f.kind == 1) { p[0] = 'i'; p[1] = 'n'; p[2] = 'f'; return; }
  const int nd = f.nd;
  if (nd <= 4) {
    // ip < 10^4: 24-bit multiply-shift digit extraction ((x*41)>>12 == x/100 for x < 1000,
    // (x*103)>>10 == x/10 for x < 100, (x*8389)>>23 == x/1000 for x < 10^4)
    const uint32_t ip = (uint32_t)f.ip;
    const uint32_t th = __umul24(ip, 8389u) >> 23;
    put3(p + nd - 3, ip - th * 1000u, nd);
    if (nd == 4) p[0] = (char)('0' + th);
    p[nd] = '.';
    const uint32_t fh = f.fp / 1000u;
    put3(p + nd + 1, fh, 3);
    put3(p + nd + 4, f.fp - fh * 1000u, 3);
    return;
  }
  uint32_t fp = f.fp;
#pragma unroll
  for (int i = 6; i >= 1; --i) {
    const uint32_t q = fp / 10u;
    p[nd + i] = (char)('0' + (fp - q * 10u));
    fp = q;
  }
  p[nd] = '.';
  if ((uint64_t)(f.ip >> 32) == 0) {
    uint32_t y = (uint32_t)f.ip;
    for (int i = nd - 1; i >= 0; --i) {
      const uint32_t q = y / 10u;
      p[i] = (char)('0' + (y - q * 10u));
      y = q;
    }
  } else {
    unsigned __int128 y = f.ip;
    for (int i = nd - 1; i >= 0; --i) { p[i] = (char)('0' + (uint32_t)(y % 10)); y /= 10; }
  }
}

struct PcdArgs {
  CodecFrames src;
  int32_t* tile_bytes;          // measure: text bytes of each tile
  const int64_t* tile_pos;      // write: byte offset of each tile's text in `out`
  char* out;
  int* err;                     // 1: a value beyond the formatter's range
  int morder, worder;           // stream_unit orders of the float32 measure pass / of the write pass
};

struct PcdLine {
  Fmt6 v[4];
  int len;
};

__device__ __forceinline__ void pcd_line(const CodecFrames& s, int32_t f, int64_t row, PcdLine& L, int* err) {
  double c[4];
  codec_point(s, f, row, c);
  L.len = 4;                                       // 3 separators + newline
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    L.v[k] = fmt6_prepare(c[k]);
    if (L.v[k].kind == 3) *err = 1;
    L.len += L.v[k].len;
  }
}

__device__ __forceinline__ void pcd_emit(const PcdLine& L, char* p) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fmt6_write(L.v[k], p);
    p += L.v[k].len;
    *p++ = k < 3 ? ' ' : '\n';
  }
}

__device__ __forceinline__ int64_t pcd_row(const CodecFrames& s, int64_t u, int32_t& f, bool& valid) {
  f = codec_advance(s.unit_off, f, u);
  const int64_t d0 = ldu(s.doff + f), d1 = ldu(s.doff + f + 1);
  const int64_t row = d0 + (u - ldu(s.unit_off + f)) * kPcdBlock + threadIdx.x;
  valid = row < d1;
  return row;
}

// wave-wide inclusive sum with DPP (no LDS round trips): row_shr 1 / 2 / 4 / 8 inside each 16-lane
// row (bound_ctrl: lanes shifted in from outside the row add 0), then row_bcast:15 carries row 0's and
// row 2's totals into rows 1 and 3, row_bcast:31 the first two rows' total into rows 2 and 3
__device__ __forceinline__ int wave_scan_incl(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
  return x;
}

// block-wide inclusive sum over the kPcdBlock threads of a PCD workgroup
// (DPP instead of round 3's __shfl_up loop: measure + write 872.6 vs 892.7 us, profiles/round4/s07)
__device__ __forceinline__ int block_scan(int x, int* s_wave, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  x = wave_scan_incl(x);
  if (lane == 63) s_wave[wid] = x;
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < kPcdBlock / 64; ++w) {
    const int c = s_wave[w];
    before += w < wid ? c : 0;
    total += c;
  }
  return x + before;
}

// tens and units of two 2-digit numbers held in the 16-bit lanes of v (each < 100): v_pk_mul_lo_u16,
// v_pk_lshrrev_b16, v_pk_mad_u16 — two lanes per instruction ((x 103) >> 10 = x / 10 for x < 179)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pk_tens_units(uint32_t v, uint32_t& t, uint32_t& u) {
  const u16x2 x = __builtin_bit_cast(u16x2, v);
  const u16x2 q = (u16x2)((x * (unsigned short)103) >> (unsigned short)10);
  const u16x2 r = x - q * (unsigned short)10;
  t = __builtin_bit_cast(uint32_t, q);
  u = __builtin_bit_cast(uint32_t, r);
}

// ---- packed line path (every value of the line |v| < 4294, ties included) ----------------------
// The common LiDAR line is formatted from four 32-bit integers N = round(|v| * 10^6): the digits come
// out of 2-digit groups split with packed 16-bit arithmetic (digit_groups, value_fields), and each value
// goes to the tile's LDS text at its final byte offset (pcd_text, pcd_emit_line).  Tiles holding a line with
// any other value (NaN, inf, |v| >= 4294) take the byte path (fmt6_prepare / pcd_emit,
// k_pcd_write_bytes).  Rejected in round 4 (tools/ab_codecs.py --source batch, profiles/round4/s07,
// measure + write): digits from a 200-byte "00".."99" LDS pair table, 909.4 vs 872.6 us (fewer VALU
// instructions, but five dependent LDS reads per value with bank conflicts); each value's text as
// unaligned 8-byte LDS stores with exact line boundaries, 1084.2 us.
struct PcdFast {
  uint32_t n[4];   // round-half-even(|v| * 10^6)
  uint32_t ip[4];  // n / 10^6 (the integer part)
  uint32_t neg;    // bit k: value k is negative (signbit)
  bool ok;         // all four values took the fast path
};

// floor(N / 10^6) for N < 2^32 given as an exact float64: N 10^-6 is within 5e-13 of N / 10^6,
// whose fraction is 0 or at least 10^-6 from 1, so adding 10^-9 and truncating is exact (one
// full-rate f64 FMA + convert instead of the quarter-rate 32-bit mul_hi of N / 10^6)
// (against N / 10^6 on the integers: measure + write 812.4 vs 818.0 us, profiles/round4/s15 — within
// noise, kept for the four quarter-rate multiplies per line it removes)
__device__ __forceinline__ uint32_t fast_ip(double N) { return (uint32_t)fma(N, 1e-6, 1e-9); }

// N = round-half-even(|v| * 10^6) exactly, for |v| < 4294 (NaN / larger values fail the test).
// y = fl(a * 10^6) and e = fma(a, 10^6, -y) represent the exact product as y + e; fr = y - floor(y)
// and fr - 0.5 are exact, so d = (fr - 0.5) + e has the sign of the exact fraction minus one half
// (rounding preserves signs) and is zero only on an exact tie, which rounds to even.  Exact ties are
// common in float32-valued clouds (any odd multiple of 1/128).
__device__ __forceinline__ bool fmt6_fast(double v, uint32_t& n, uint32_t& ip) {
  const double a = fmin(fabs(v), 4294.0);
  const double y = a * 1000000.0;
  const double e = fma(a, 1000000.0, -y);
  const double fl = floor(y);
  const double d = ((y - fl) - 0.5) + e;
  const uint32_t m = (uint32_t)fl;
  n = m + ((d > 0.0 || (d == 0.0 && (m & 1u))) ? 1u : 0u);
  ip = fast_ip((double)n);
  return fabs(v) < 4294.0;
}

__device__ __forceinline__ void pcd_fast(const CodecFrames& s, int32_t f, int64_t row, PcdFast& P) {
  double c[4];
  codec_point(s, f, row, c);
  P.ok = true;
  P.neg = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    P.ok &= fmt6_fast(c[k], P.n[k], P.ip[k]);
    P.neg |= (signbit(c[k]) ? 1u : 0u) << k;
  }
}

// ---- float32 source (a batch's own columns) ----------------------------------------------------
// v = m 2^e with a 24-bit m: |v| 10^6 = m 10^6 2^e has a significand below 2^44, so the float64
// product is exact and N = rint(|v| 10^6) (round half to even) is exact with no error term.
__device__ __forceinline__ bool fmt6_fast_f32(float v, uint32_t& n, uint32_t& ip) {
  const float a = fminf(fabsf(v), 4294.0f);   // NaN -> 4294 (the line fails the test below)
  const double y = rint((double)a * 1000000.0);
  n = (uint32_t)y;
  ip = fast_ip(y);
  return fabsf(v) < 4294.0f;
}

__device__ __forceinline__ void pcd_fast_vals_f32(const float c[4], PcdFast& P) {
  P.ok = true;
  P.neg = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    P.ok &= fmt6_fast_f32(c[k], P.n[k], P.ip[k]);
    P.neg |= (signbit(c[k]) ? 1u : 0u) << k;
  }
}

// pcd_fast_vals_f32 for a tile the measure pass found packed (every value |v| < 4294): no clamp and
// no path test (a NaN cannot reach here; it would convert to 0)
__device__ __forceinline__ void pcd_fast_vals_packed(const float c[4], PcdFast& P) {
  P.ok = true;
  P.neg = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double y = rint((double)fabsf(c[k]) * 1000000.0);
    P.n[k] = (uint32_t)y;
    P.ip[k] = fast_ip(y);
    P.neg |= (signbit(c[k]) ? 1u : 0u) << k;
  }
}

// pcd_fast_len for float32 values: line length, or -1 outside the packed path
__device__ __forceinline__ int pcd_fast_len_f32(const float c[4]) {
  int len = 4 + 4 * 8;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = fabsf(c[k]);
    ok = ok && a < 4294.0f;
    len += (signbit(c[k]) ? 1 : 0) + (a >= 10.0f) + (a >= 100.0f) + (a >= 1000.0f);
  }
  return ok ? len : -1;
}

// Digit groups of N = round(|v| 10^6) < 2^32 (|v| < 4294, so ip = N / 10^6 < 2^13): the ten digits
// as five 2-digit groups, g0 = ip / 100, g1 = ip % 100, g2 = fp / 10^4, g3 = fp / 100 % 100 and
// g4 = fp % 100 (fp = N - 10^6 ip), returned as g01 = g0 | g1 << 16, g23 = g2 | g3 << 16 and g4 (two
// values' g4 are split together, pair_tu4).  g2 = (fp 429497) >> 32 is fp / 10^4 exactly for
// fp < 10^6 (the multiplier's excess adds < 6.3e-5 to a quotient whose fraction is at most 0.9999).
// The products are 24-bit multiply-adds (v_mad_i32_i24 by __mul24 with a negative constant, no
// range masks).  Against the two 3-digit halves in 32-bit SWAR: 802.8 vs 806.8 us measure + write
// (profiles/round4/s17).
__device__ __forceinline__ void digit_groups(uint32_t N, uint32_t ip, uint32_t& g01, uint32_t& g23, uint32_t& g4) {
  const uint32_t fp = N + (uint32_t)__mul24((int)ip, -1000000);                         // < 10^6
  uint32_t g2 = (uint32_t)(((uint64_t)(fp & 0xFFFFFu) * 429497ull) >> 32);             // fp / 10^4
  // opaque to the optimiser: it recognises fp - (fp / 10^4) 10^4 as fp % 10^4 and lowers that
  // through a quarter-rate 64-bit multiply-add
  asm("" : "+v"(g2));
  const uint32_t r4 = fp + (uint32_t)__mul24((int)g2, -10000);                          // < 10^4
  const uint32_t g3 = __umul24(r4, 5243u) >> 19;                                        // r4 / 100
  g4 = r4 - g3 * 100u;
  const uint32_t g0 = __umul24(ip, 5243u) >> 19;                                        // ip / 100
  const uint32_t g1 = ip - g0 * 100u;
  g01 = g0 | (g1 << 16);
  g23 = g2 | (g3 << 16);
}
// tens | units << 8 of two values' g4 at once (one packed split for both)
__device__ __forceinline__ void pair_tu4(uint32_t ga, uint32_t gb, uint32_t& tua, uint32_t& tub) {
  uint32_t T, U;
  pk_tens_units(ga | (gb << 16), T, U);
  tua = __builtin_amdgcn_perm(U, T, 0x0C0C0400u);
  tub = __builtin_amdgcn_perm(U, T, 0x0C0C0602u);
}
// Text fields of one value (bytes in text order, v_perm_b32 placement): D = the 4 integer digits
// with leading zeros as values 0..9 (byte 0 = thousands), A = ". d1 d2 d3", B = "d4 d5 d6 sep"
__device__ __forceinline__ void value_fields(uint32_t g01, uint32_t g23, uint32_t tu4, uint32_t sep, uint32_t& D,
                                             uint32_t& A, uint32_t& B) {
  uint32_t T1, U1, T2, U2;
  pk_tens_units(g01, T1, U1);
  pk_tens_units(g23, T2, U2);
  D = __builtin_amdgcn_perm(T1, U1, 0x02060004u);
  A = __builtin_amdgcn_perm(T2, U2, 0x0600040Cu) + 0x3030302Eu;
  B = __builtin_amdgcn_perm(U2, tu4, 0x0C010006u) + (0x00303030u | (sep << 24));
}
__device__ __forceinline__ void put4(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// A packed line's text: value k's fields D (ASCII), A, B, its count q of leading zero digits in D
// (4 - its integer digit count: the index of D's first non-zero digit byte, one v_ffbl_b32), the sign
// bits and the line length 4 (nd + [v < 0] + 8) summed = 48 + sum([v < 0] - q).  The digit count
// comes out of the digits themselves, so it is N >= 10^7 / 10^8 / 10^9 exactly (no compares).
struct PcdText {
  uint32_t D[4], A[4], B[4];
  int q0;      // q of value 0
  int ng[4];   // 1: value k is negative
  int d[4];    // ng - q: value k's text is 12 + d[k] bytes with its separator
  int len;
};
__device__ __forceinline__ void pcd_text(const PcdFast& P, PcdText& T) {
  uint32_t g01[4], g23[4], g4[4], tu4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) digit_groups(P.n[k], P.ip[k], g01[k], g23[k], g4[k]);
  pair_tu4(g4[0], g4[1], tu4[0], tu4[1]);
  pair_tu4(g4[2], g4[3], tu4[2], tu4[3]);
  int len = 48;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t D;
    value_fields(g01[k], g23[k], tu4[k], k == 3 ? '\n' : ' ', D, T.A[k], T.B[k]);
    const int q = (int)(__builtin_ctz(D | 0x01000000u) >> 3);   // the units byte always counts
    if (k == 0) T.q0 = q;
    T.D[k] = D + 0x30303030u;
    T.ng[k] = (int)((P.neg >> k) & 1u);
    T.d[k] = T.ng[k] - q;
    len += T.d[k];
  }
  T.len = len;
}

// One packed line at byte `off` of the tile text, OR-ed into the zeroed text buffer (pcd_tile_text) as
// naturally aligned 8-byte words: value k's 16 bytes [pa - 8, pa + 8) — H = the 8 bytes ending at its
// '.' (zeros, its '-' if negative, its integer digits with the leading zeros blanked), then A, B —
// shifted to the 8-byte grid are three ds_or_b64 whose zero bytes leave the neighbours' text (the
// line's other values, other lanes' lines) untouched.  Naturally aligned LDS stores issue at 4.6
// ticks per wave-instruction, the unaligned 8 / 12-byte stores of byte-offset text at 36
// (tools/issue_probe.hip, profiles/round5/s02); against those stores (values 3..1 as unaligned
// 12-byte fields overwriting each other's heads, value 0 byte by byte): measure + write 772.1 / 782.5
// vs 788.7 / 793.5 us, fused write pass 630.9 / 635.2 vs 639.8 / 642.7 us (profiles/round5/s03, s04;
// ds_or_b32 on 4-byte words ran alike but took more VALU).  base is 16 bytes into the buffer (value
// 0's window starts up to 7 bytes before its line).
typedef __attribute__((address_space(3))) uint64_t lds_u64;
__device__ __forceinline__ void lds_or64(uint8_t* p, uint64_t v) {
  __hip_atomic_fetch_or((lds_u64*)(void*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// one value whose '.' is at byte pa: D its 4 integer digit characters, q of them leading zeros, ng 1
// if negative
__device__ __forceinline__ void pcd_emit_value(uint8_t* base, int pa, uint32_t D, uint32_t A, uint32_t B, int q,
                                               int ng) {
  const uint32_t Dm = D & (0xFFFFFFFFu << (8 * q));
  const uint64_t H = ((uint64_t)Dm << 32) | ((uint64_t)(ng ? 0x2Du : 0u) << (24 + 8 * q));
  const uint64_t AB = ((uint64_t)B << 32) | A;
  const int s0 = pa - 8, r = s0 & 7;
  uint8_t* const w = base + (s0 - r);   // 8-byte aligned
  const int sh = 8 * r;                 // 0 .. 56
  // x >> (64 - sh) as (x >> 8) >> (56 - sh): zero at sh = 0 (one 64-bit shift takes its amount mod 64)
  lds_or64(w, H << sh);
  lds_or64(w + 8, (AB << sh) | ((H >> 8) >> (56 - sh)));
  lds_or64(w + 16, (AB >> 8) >> (56 - sh));
}
// text: the tile's text buffer as 16-byte chunks — typed uint4 so the 8-byte grid pcd_emit_value
// ORs into is the buffer's own alignment (a ds_or_b64 at a 4-byte LDS offset faults, profiles/round5/s03)
__device__ __forceinline__ void pcd_emit_line(const PcdText& T, uint4* text, int off) {
  static_assert(alignof(uint4) % 8 == 0, "the text chunks must keep the 8-byte grid of ds_or_b64");
  uint8_t* const base = reinterpret_cast<uint8_t*>(text);
  int pa = off + 4 + T.d[0];   // the '.' of value k
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k > 0) pa += 12 + T.d[k];
    pcd_emit_value(base, pa, T.D[k], T.A[k], T.B[k], T.ng[k] - T.d[k], T.ng[k]);
  }
}

// The packed line's length without its digits: "%.6f" of |v| < 4294 has 1 + [v < 0] + nd + 7
// characters with the separator, nd = 1 + [N >= 10^7] + [N >= 10^8] + [N >= 10^9] for
// N = round-half-even(|v| 10^6).  N >= T (T even) <=> |v| 10^6 >= T - 1/2 exactly; y = fl(|v| 10^6)
// decides that except when y lands on T - 1/2, where the product's error e does.  -1: a value
// outside the packed path.
__device__ __forceinline__ int pcd_fast_len(const double c[4]) {
  int len = 4 + 4 * 8;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double a = fabs(c[k]);
    ok = ok && a < 4294.0;
    const double y = a * 1000000.0;
    const bool tie_up = fma(a, 1000000.0, -y) >= 0.0;
    len += (signbit(c[k]) ? 1 : 0) + (y > 9999999.5 || (y == 9999999.5 && tie_up)) +
           (y > 99999999.5 || (y == 99999999.5 && tie_up)) + (y > 999999999.5 || (y == 999999999.5 && tie_up));
  }
  return ok ? len : -1;
}

// Tile flag: k_pcd_measure marks a tile holding any line outside the packed path by this bit of its
// byte count; the host sends those tiles to k_pcd_write_bytes and the rest to k_pcd_write.
constexpr int32_t kPcdSlowTile = 1 << 30;

// columns 0..3 of dense row `row` of a batch source as float32 (codec_point widens them)
__device__ __forceinline__ void codec_point_f32(const CodecFrames& s, int32_t f, int64_t row, float c[4]) {
  const float* q = s.cols + bidx(s.C, 0, ldu(s.poff + f) + (row - ldu(s.doff + f)));
  c[0] = q[0]; c[1] = q[kBlkPts]; c[2] = q[2 * kBlkPts]; c[3] = q[3 * kBlkPts];
}

__device__ __forceinline__ int32_t pcd_tile_word(int v) {   // scanned bytes (+ 2^20 per byte-path line)
  return (v & ((1 << 20) - 1)) | ((v >> 20) ? kPcdSlowTile : 0);
}

// Float32 source: a tile's 256 lines are one block of the batch, so one wave measures a whole tile —
// lane l takes lines 4l .. 4l + 3 from one float4 per column (16-byte lanes) and a wave reduction
// replaces the block scan: no LDS, no barrier (measure + write 893.5 / 939.0 vs 989.4 / 1022.2 us with
// a block per tile, profiles/round3/s70).  A workgroup takes kPcdTilesPerWG tiles, each wave
// kPcdTilesPerWG / 4 of them, all of whose loads are issued before the first is measured.
// (8 / 16 tiles per measure workgroup: 821.8-833.0 / 842.0 vs 812.4-827.5 us measure + write,
// profiles/round4/s14, s15)
constexpr int kPcdMeasureTiles = kPcdTilesPerWG;                       // tiles per measure workgroup
constexpr int kPcdMeasureWaveTiles = kPcdMeasureTiles / (kPcdBlock / 64);
__device__ __forceinline__ void pcd_measure_waves(const PcdArgs& a, int64_t u0) {
  static_assert(kPcdBlock == kBlkPts, "a PCD tile is one batch block");
  static_assert(kPcdMeasureTiles % (kPcdBlock / 64) == 0, "whole tiles per wave");
  constexpr int NT = kPcdMeasureWaveTiles;
  const int lane = threadIdx.x & 63;
  // the wave index as a scalar: the tile, its frame and its offsets are then wave-uniform — scalar
  // loads and branches instead of vector loads of the frame tables and a divergent frame search
  // ahead of the point loads (MC_PCD_MEASURE_SCALAR)
  const int wave = MC_PCD_MEASURE_SCALAR ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))
                                         : (int)(threadIdx.x >> 6);
  int32_t f = codec_frame_of(a.src, u0);
  int left[NT];   // lines of the tile at and after this lane's first (frame-relative, may be <= 0)
  float4 V[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int64_t u = u0 + wave * NT + j;   // a wave's tiles are consecutive
    left[j] = 0;
    if (u < a.src.n_units) {
      // tile u = block (poff_f + 256 (u - unit_off_f)) / 256: a wave-uniform base (scalar arithmetic)
      f = codec_advance(a.src.unit_off, f, u);
      const int64_t k = u - ldu(a.src.unit_off + f);
      const int64_t blk = (ldu(a.src.poff + f) >> 8) + k;
      left[j] = (int)min_i64(ldu(a.src.doff + f + 1) - ldu(a.src.doff + f) - k * kPcdBlock, kPcdBlock) - 4 * lane;
      const float* q = a.src.cols + blk * a.src.C * kBlkPts + 4 * lane;
      // the whole block is allocated (frames are padded to blocks): every lane loads, results past
      // the frame's end are ignored below
#pragma unroll
      for (int c = 0; c < 4; ++c) V[j][c] = *reinterpret_cast<const float4*>(q + c * kBlkPts);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int64_t u = u0 + wave * NT + j;
    if (u >= a.src.n_units) break;   // wave-uniform
    int v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float c[4] = {f4g(V[j][0], i), f4g(V[j][1], i), f4g(V[j][2], i), f4g(V[j][3], i)};
      const int l = pcd_fast_len_f32(c);
      // a line outside the packed path flags the tile; its exact bytes come from
      // k_pcd_measure_list (the byte formatter would double this kernel's registers)
      v += i < left[j] ? (l < 0 ? (1 << 20) : l) : 0;
    }
    // wave sum by DPP (the shuffle loop compiled to six ds_bpermute round trips)
    if (MC_PCD_MEASURE_SCALAR) {
      v = __builtin_amdgcn_readlane(wave_scan_incl(v), 63);
    } else {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    }
    if (lane == 0) a.tile_bytes[u] = pcd_tile_word(v);
  }
}

// The exact text bytes of the listed tiles (those k_pcd_measure<true> flagged): byte-path lengths
// of every line, block scan; the flag stays (k_pcd_write_bytes writes these tiles).
__global__ __launch_bounds__(kPcdBlock) void k_pcd_measure_list(const PcdArgs a, const int32_t* list) {
  __shared__ int s_wave[kPcdBlock / 64];
  const int64_t u = list[blockIdx.x];
  int32_t f = codec_frame_of(a.src, u);
  bool valid;
  const int64_t row = pcd_row(a.src, u, f, valid);
  int v = 0;
  if (valid) {
    PcdLine L;
    pcd_line(a.src, f, row, L, a.err);
    v = L.len;
  }
  int total;
  block_scan(v, s_wave, total);
  if (threadIdx.x == 0) a.tile_bytes[u] = total | kPcdSlowTile;
}

template <bool F32>
__global__ __launch_bounds__(kPcdBlock) void k_pcd_measure(const PcdArgs a) {
  if constexpr (F32) {
    pcd_measure_waves(a, stream_unit(a.morder, blockIdx.x, gridDim.x) * kPcdMeasureTiles);
  } else {
    __shared__ int s_wave[kPcdBlock / 64];
    const int64_t u0 = xcd_unit<MC_XCD_CODEC>(blockIdx.x, gridDim.x) * kPcdTilesPerWG;   // grid = units exactly
    int32_t f = codec_frame_of(a.src, u0);
    for (int j = 0; j < kPcdTilesPerWG; ++j) {
      const int64_t u = u0 + j;
      if (u >= a.src.n_units) break;
      bool valid;
      const int64_t row = pcd_row(a.src, u, f, valid);
      // scanned value: line bytes + (byte-path line ? 1 << 20 : 0); a tile's bytes stay < 2^20 and
      // its byte-path line count < 2^11, so one scan yields both (no extra barrier)
      int v = 0;
      if (valid) {
        double c[4];
        codec_point(a.src, f, row, c);
        v = pcd_fast_len(c);
        if (v < 0) {
          PcdLine L;
          pcd_line(a.src, f, row, L, a.err);
          v = L.len + (1 << 20);
        }
      }
      int total;
      block_scan(v, s_wave, total);
      if (threadIdx.x == 0) a.tile_bytes[u] = pcd_tile_word(total);
      __syncthreads();   // s_wave is reused by the next tile
    }
  }
}

// Packed tiles: every line is formatted into the tile's LDS text (which sits at its HBM offset
// modulo 16), then stored with codec_store_piece.  Tiles flagged slow are skipped
// (k_pcd_write_bytes writes them).  A packed line is at most 52 bytes, so a tile's text always fits.
// pcd_tile_text: the tile's lines in LDS, -> the tile's text bytes; pcd_tile_store: its stores.
constexpr int kPcdTextLead = 1;   // uint4 chunks before the text (pcd_emit_line's windows start early)
constexpr int kPcdTextChunks = kPcdPackedText / 16 + 1 + kPcdTextLead;
// MC_PCD_DIAG (diagnostic builds only, wrong output), bits: 1 = no text chunk stores to HBM, 4 = no
// LDS text emission (profiles/round5/s08 also ran 2 = no digit conversion and 8 = waves storing their
// own 64 lines without the tile's barriers, in the write loop this unrolled pass replaced).
#ifndef MC_PCD_DIAG
#define MC_PCD_DIAG 0
#endif
__device__ __forceinline__ void pcd_text_zero(uint4* s_text4) {
#pragma unroll
  for (int u = 0; u < (kPcdTextChunks + kPcdBlock - 1) / kPcdBlock; ++u) {
    const int c = (int)threadIdx.x + u * kPcdBlock;
    if (c < kPcdTextChunks) s_text4[c] = make_uint4(0u, 0u, 0u, 0u);
  }
}
__device__ __forceinline__ int pcd_tile_text(const PcdText& T, bool valid, int64_t G, int* s_wave, uint4* s_text4) {
  // the buffer is zeroed before the scan's barrier; the previous tile's reads of it ended before the
  // barrier that closed its stores (pcd_tile_store)
  pcd_text_zero(s_text4);
  int total;
  const int excl = block_scan(T.len, s_wave, total) - T.len;
  if (valid && !(MC_PCD_DIAG & 4)) pcd_emit_line(T, s_text4 + kPcdTextLead, (int)(G & 15) + excl);
  __syncthreads();
  return total;
}
// codec_store_piece for a tile's text: the full 16-byte chunks in a loop without per-chunk tests,
// the (at most two) partial end chunks by lanes 0 and 1
__device__ __forceinline__ void pcd_tile_store(const PcdArgs& a, int64_t G, int total, const uint4* s_text4) {
  const int lo = (int)(G & 15), hi = lo + total;
  char* const g = a.out + (G - lo);
  const char* const lds = reinterpret_cast<const char*>(s_text4);
  const int f0 = (lo + 15) >> 4, f1 = hi >> 4;   // full chunks [f0, f1)
  // (all of a lane's chunk reads before its stores, with the end bytes by 32 lanes: 816.5 vs 793.5 us,
  // profiles/round5/s04 — the LVX pieces gain from it, these do not)
  for (int c = f0 + (int)threadIdx.x; c < f1; c += kPcdBlock) {
    if constexpr ((MC_PCD_DIAG & 1) != 0) {   // diagnostic: the chunk is read, (almost) never stored
      const uint4 v = s_text4[c];
      if (v.x == 0x7eadbeefu && v.y == 0x7eadbeefu) codec_st16(g + 16 * c, v);
    } else {
      codec_st16(g + 16 * c, s_text4[c]);
    }
  }
  if (threadIdx.x < 2) {
    int b = lo, e = hi;                                    // a piece inside one chunk: lane 0 alone
    if (f0 <= f1) {
      if (threadIdx.x == 0) e = 16 * f0;                   // head: [lo, 16 f0)
      else b = 16 * f1;                                    // tail: [16 f1, hi)
    } else if (threadIdx.x == 1) {
      e = b;
    }
#pragma clang loop vectorize(disable) unroll(disable)
    for (; b < e; ++b) g[b] = lds[b];
  }
  // the next tile zeroes s_text and rewrites s_wave: this barrier closes this tile's reads of both
  __syncthreads();
}

// Tiles per write workgroup.  The float32 pass unrolls a workgroup's tiles and issues the point
// loads of two tiles before the first is converted, so that two tiles' loads are in flight and every
// vmcnt wait the compiler places is exact (no loop carries a load).  Kernel time of the previous
// pass (4 tiles in a loop, one tile's loads ahead) vs 2 tiles unrolled: 640.1 vs 588.0 us, 1 tile
// 626.4 (rocprofv3, profiles/round5/s19); measure + write 787.6 vs 739.0 us, fused write pass 722.6
// vs 671.8 us (s18).  Rejected (s13-s16, measure + write): 3 / 4 / 6 / 8 tiles unrolled with loads
// two or three tiles ahead 738.8-806.2 us; a fixed number of stores per lane (buffer stores, those
// with nothing to store dropped past the record count) so that the waits would not cover the
// previous tile's stores, 820.3 vs 787.6 us.
#ifndef MC_PCD_WRITE_TILES
#define MC_PCD_WRITE_TILES 2
#endif
constexpr int kPcdWriteTiles = MC_PCD_WRITE_TILES;

template <bool F32>
__global__ __launch_bounds__(kPcdBlock) void k_pcd_write(const PcdArgs a) {
  __shared__ int s_wave[kPcdBlock / 64];
  __shared__ alignas(16) uint4 s_text4[kPcdTextChunks];
  const int64_t u0 = stream_unit(a.worder, blockIdx.x, gridDim.x) * kPcdWriteTiles;   // grid = units exactly
  int32_t f = codec_frame_of(a.src, u0);
  if constexpr (F32) {
    // Order per tile j: loads of tile j + 2, tile j's LDS text, tile j + 1 converted, tile j's
    // stores.  vmcnt counts stores as well as loads: tile j + 1's conversion waits for its loads and
    // for tile j - 1's stores (issued before them), never for tile j's.  Tiles past the grid's end
    // load the last tile again and store nothing; a tile that is not packed is formatted all the same
    // (bounded: 36-52 bytes a line) and not stored (k_pcd_write_bytes writes it).
    constexpr int K = kPcdWriteTiles, D = K < 2 ? K : 2;
    const int64_t nu = a.src.n_units;
    float cv[K][4];
    bool vv[K];
    int32_t flag[K];
    int64_t gpos[K];
    // tile u is block (poff_f + 256 (u - unit_off_f)) / 256 of the batch: its columns start at a
    // workgroup-uniform address (scalar arithmetic), a lane's line at + threadIdx.x
    auto fetch = [&](int j) {
      const bool live = u0 + j < nu;
      const int64_t u = live ? u0 + j : nu - 1;
      f = codec_advance(a.src.unit_off, f, u);
      const int64_t k = u - ldu(a.src.unit_off + f);                       // tile of frame f
      const int64_t blk = (ldu(a.src.poff + f) >> 8) + k;
      const int left = (int)min_i64(ldu(a.src.doff + f + 1) - ldu(a.src.doff + f) - k * kPcdBlock, kPcdBlock);
      vv[j] = live && (int)threadIdx.x < left;
      // the tile's block is allocated whole: every lane loads (no branch around the loads), a lane
      // past the frame's end formats a value it never emits
      const float* q = a.src.cols + blk * a.src.C * kBlkPts + threadIdx.x;
      cv[j][0] = q[0]; cv[j][1] = q[kBlkPts]; cv[j][2] = q[2 * kBlkPts]; cv[j][3] = q[3 * kBlkPts];
      flag[j] = live ? ldu(a.tile_bytes + u) : kPcdSlowTile;
      gpos[j] = ldu(a.tile_pos + u);
    };
    auto conv = [&](int j, PcdText& T) {
      PcdFast P;
      pcd_fast_vals_packed(cv[j], P);   // (invalid lanes convert stale values: length zeroed)
      pcd_text(P, T);
      if (!vv[j]) T.len = 0;
      // pins the conversion here: the compiler would otherwise sink it below the stores, to its use
      asm volatile("" ::"v"(T.D[0]), "v"(T.D[1]), "v"(T.D[2]), "v"(T.D[3]), "v"(T.A[0]), "v"(T.A[1]),
                   "v"(T.A[2]), "v"(T.A[3]), "v"(T.B[0]), "v"(T.B[1]), "v"(T.B[2]), "v"(T.B[3]), "v"(T.len)
                   : "memory");
    };
    PcdText T0, T1;
#pragma unroll
    for (int j = 0; j < D; ++j) fetch(j);
    conv(0, T0);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      PcdText& T = (j & 1) ? T1 : T0;
      PcdText& Tn = (j & 1) ? T0 : T1;
      if (j + D < K) fetch(j + D);
      const int total = pcd_tile_text(T, vv[j], gpos[j], s_wave, s_text4);
      if (j + 1 < K) conv(j + 1, Tn);
      if (!(flag[j] & kPcdSlowTile)) pcd_tile_store(a, gpos[j], total, s_text4 + kPcdTextLead);
      else __syncthreads();   // (pcd_tile_store's closing barrier)
    }
  } else {
    for (int j = 0; j < kPcdWriteTiles; ++j) {
      const int64_t u = u0 + j;
      if (u >= a.src.n_units) break;
      if (ldu(a.tile_bytes + u) & kPcdSlowTile) continue;   // workgroup-uniform
      bool valid;
      const int64_t row = pcd_row(a.src, u, f, valid);
      PcdText T;
      T.len = 0;
      if (valid) {
        PcdFast P;
        pcd_fast(a.src, f, row, P);
        pcd_text(P, T);
      }
      const int64_t G = ldu(a.tile_pos + u);
      const int total = pcd_tile_text(T, valid, G, s_wave, s_text4);
      pcd_tile_store(a, G, total, s_text4 + kPcdTextLead);
    }
  }
}

// Byte path (any %.6f value): every tile formats its lines byte by byte into LDS and stores the
// text with codec_store_piece; a tile larger than the LDS buffer — only possible with extreme
// magnitudes — is written line by line straight to HBM instead.  Tiles: list[blockIdx.x], or, with
// list == nullptr, kPcdTilesPerWG consecutive tiles per workgroup.
__global__ __launch_bounds__(kPcdBlock) void k_pcd_write_bytes(const PcdArgs a, const int32_t* list) {
  __shared__ int s_wave[kPcdBlock / 64];
  __shared__ uint4 s_text4[kPcdTileText / 16 + 1];
  char* const s_text = reinterpret_cast<char*>(s_text4);
  const int64_t u0 = list ? (int64_t)list[blockIdx.x]
                          : xcd_unit<MC_XCD_CODEC>(blockIdx.x, gridDim.x) * kPcdTilesPerWG;
  const int per = list ? 1 : kPcdTilesPerWG;
  int32_t f = codec_frame_of(a.src, u0);
  for (int j = 0; j < per; ++j) {
    const int64_t u = u0 + j;
    if (u >= a.src.n_units) break;
    bool valid;
    const int64_t row = pcd_row(a.src, u, f, valid);
    PcdLine L;
    L.len = 0;
    if (valid) pcd_line(a.src, f, row, L, a.err);
    int total;
    const int incl = block_scan(L.len, s_wave, total);
    const int excl = incl - L.len;
    const int64_t G = a.tile_pos[u];
    const int shift = (int)(G & 15);
    if (total + shift <= kPcdTileText) {
      if (valid) pcd_emit(L, s_text + shift + excl);
      __syncthreads();
      codec_store_piece<kPcdBlock>(a.out + (G - shift), s_text, shift, shift + total);
    } else if (valid) {
      pcd_emit(L, a.out + G + excl);
    }
    __syncthreads();   // s_wave / s_text are reused by the next tile
  }
}


}  // namespace mc
