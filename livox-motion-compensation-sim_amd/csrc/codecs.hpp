// codecs.hpp — gfx950 kernels for the reference's output codecs, encoding
// straight from a device-resident (N, ld) float64 AoS cloud (the array layout of LMC:770 / 776):
//
//   LVX v1.1 packer  LMC:24-272   96-point packages of 14-byte records (int32 mm + reflectivity)
//   ASCII PCD body   LMC:932-948  "%.6f %.6f %.6f %.6f\n" per point, correctly rounded
//
// Both are byte-producing, HBM-bound passes.  Frames map to "units" (LVX packages, PCD tiles of
// kBlock points) through a per-frame prefix, so one launch covers every frame of a batch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

constexpr int kCodecBlock = 256;
constexpr int kLvxPkgPoints = 96;
constexpr int kLvxRec = 14;
constexpr int kLvxPkgHdr = 22;
constexpr int kLvxPkg = kLvxPkgHdr + kLvxPkgPoints * kLvxRec;   // 1366 bytes
constexpr int kLvxFrameHdr = 24;
constexpr int kLvxPkgWords = kLvxPkg / 2;                       // every offset in the file is even
constexpr int kLvxFileHdr = 88;
constexpr int kPcdTileText = 16384;                             // LDS text buffer per tile of kBlock lines

struct CodecFrames {
  const double* aos; int64_t ld;
  const int64_t* doff;       // [F+1] dense row offset of each frame
  const int64_t* unit_off;   // [F+1] prefix of per-frame units (LVX packages / PCD tiles)
  int32_t F;
};

// frame owning unit u: last f with unit_off[f] <= u (frames without units are skipped over)
__device__ __forceinline__ int32_t codec_frame_of(const int64_t* __restrict__ unit_off, int32_t F, int64_t u) {
  int32_t lo = 0, hi = F + 1;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (unit_off[mid] <= u) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

// ---- LVX v1.1 -------------------------------------------------------------------------------
struct LvxArgs {
  CodecFrames src;
  const int64_t* frame_pos;     // [F] byte offset of each frame in the file
  const uint64_t* frame_id;     // [F]
  const uint64_t* ts_ns;        // [F] package timestamp, int(timestamp * 1e9) (LMC:176)
  const uint8_t* has_int;       // [F] frame has an intensity column (else reflectivity 128), or null
  uint16_t* out;                // file base
  int* err;                     // set to 1 on a NaN coordinate / intensity (LMC:259, 268 int(nan))
};

// int(np.clip(v * scale, lo, hi)) (LMC:259-261, 268): truncation toward zero after the clip
__device__ __forceinline__ int32_t lvx_fixed(double v, double scale, double lo, double hi, int* err) {
  const double s = v * scale;
  if (s != s) { *err = 1; return 0; }
  return (int32_t)fmin(fmax(s, lo), hi);
}

// one workgroup per 96-point package: 683 little-endian 16-bit words (header + records + padding)
__global__ __launch_bounds__(kCodecBlock) void k_lvx_packages(const LvxArgs a) {
  const int64_t u = blockIdx.x;
  const int32_t f = codec_frame_of(a.src.unit_off, a.src.F, u);
  const int64_t p = u - a.src.unit_off[f];
  const int64_t row0 = a.src.doff[f] + p * kLvxPkgPoints;
  const int64_t rem = a.src.doff[f + 1] - row0;
  const int n = rem < kLvxPkgPoints ? (int)rem : kLvxPkgPoints;
  const int64_t word0 = (a.frame_pos[f] + kLvxFrameHdr + p * kLvxPkg) >> 1;
  const uint64_t ts = a.ts_ns[f];
  const bool hi = a.has_int ? a.has_int[f] != 0 : a.src.ld > 3;
  const double* __restrict__ aos = a.src.aos;
  const int64_t ld = a.src.ld;
  for (int w = threadIdx.x; w < kLvxPkgWords; w += kCodecBlock) {
    uint32_t v;
    if (w < kLvxPkgHdr / 2) {
      // LMC:204-237: dev 0, version 5, slot 0, lidar 1, reserved, status 0 (4 B), ts type 1,
      // data type 2, reserved (3 B), timestamp (8 B)
      constexpr uint32_t kHdr[7] = {0x0500u, 0x0100u, 0x0000u, 0x0000u, 0x0100u, 0x0002u, 0x0000u};
      v = w < 7 ? kHdr[w] : (uint32_t)(ts >> (16 * (w - 7))) & 0xffffu;
    } else {
      const int k = 2 * w - kLvxPkgHdr;
      const int r = k / kLvxRec;
      const int o = k - r * kLvxRec;
      if (r >= n) {
        v = 0;                                                  // LMC:245-248 zero padding
      } else {
        const double* q = aos + (row0 + r) * ld;
        if (o < 12) {
          const uint32_t mm = (uint32_t)lvx_fixed(q[o >> 2], 1000.0, -2147483648.0, 2147483647.0, a.err);
          v = (o & 2) ? mm >> 16 : mm & 0xffffu;
        } else {
          v = hi ? (uint32_t)lvx_fixed(q[3], 255.0, 0.0, 255.0, a.err) : 128u;   // tag byte 0
        }
      }
    }
    a.out[word0 + w] = (uint16_t)v;
  }
}

// LMC:178-193: frame header = own offset, next frame's offset (0 for the last), frame_id
__global__ __launch_bounds__(kCodecBlock) void k_lvx_frames(const LvxArgs a, int64_t next_of_last_frame) {
  const int32_t f = blockIdx.x * kCodecBlock + threadIdx.x;
  if (f >= a.src.F) return;
  const uint64_t q[3] = {(uint64_t)a.frame_pos[f],
                         f + 1 < a.src.F ? (uint64_t)a.frame_pos[f + 1] : (uint64_t)next_of_last_frame,
                         a.frame_id[f]};
  uint16_t* o = a.out + (a.frame_pos[f] >> 1);
#pragma unroll
  for (int i = 0; i < 12; ++i) o[i] = (uint16_t)(q[i >> 2] >> (16 * (i & 3)));
}

// ---- "%.6f" (Python's correctly rounded fixed-point float formatting) -------------------------
// v = m * 2^e exactly; N = round-half-even(|v| * 10^6) in 128-bit integer arithmetic, printed as
// N / 10^6 "." N % 10^6.  Finite |v| < 2^107 (~1.6e32) is supported; larger values set the error
// flag (the host reports it).
struct Fmt6 {
  unsigned __int128 N;
  int kind;    // 0 finite, 1 inf, 2 nan, 3 out of range
  bool neg;
};

__device__ __forceinline__ Fmt6 fmt6_prepare(double v) {
  Fmt6 r;
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  r.neg = (bits >> 63) != 0;
  const int ex = (int)((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  r.N = 0;
  if (ex == 0x7ff) { r.kind = frac ? 2 : 1; return r; }
  r.kind = 0;
  const uint64_t m = ex ? (frac | (1ull << 52)) : frac;
  const int e = ex ? ex - 1075 : -1074;
  const unsigned __int128 P = (unsigned __int128)m * 1000000u;   // < 2^73
  if (e >= 0) {
    if (e > 54) { r.kind = 3; return r; }
    r.N = P << e;
  } else if (-e < 74) {
    const int s = -e;
    const unsigned __int128 one = 1;
    unsigned __int128 q = P >> s;
    const unsigned __int128 rem = P & ((one << s) - 1);
    const unsigned __int128 half = one << (s - 1);
    if (rem > half || (rem == half && (q & 1))) ++q;
    r.N = q;
  }
  return r;
}

__device__ __forceinline__ int u128_digits(unsigned __int128 x) {
  int d = 1;
  if ((uint64_t)(x >> 64) == 0) {
    uint64_t y = (uint64_t)x;
    while (y >= 10) { y /= 10; ++d; }
    return d;
  }
  while (x >= 10) { x /= 10; ++d; }
  return d;
}

__device__ __forceinline__ int fmt6_len(const Fmt6& f) {
  if (f.kind == 2) return 3;                      // "nan" (Python drops a NaN's sign)
  if (f.kind == 1) return 3 + (f.neg ? 1 : 0);    // "inf" / "-inf"
  if (f.kind == 3) return 0;
  const unsigned __int128 ip = (uint64_t)(f.N >> 64) == 0 ? (unsigned __int128)((uint64_t)f.N / 1000000u)
                                                          : f.N / 1000000u;
  return (f.neg ? 1 : 0) + u128_digits(ip) + 7;
}

// writes fmt6_len(f) characters at p (generic pointer: LDS or global)
__device__ __forceinline__ void fmt6_write(const Fmt6& f, char* p) {
  if (f.kind == 3) return;
  if (f.kind == 2) { p[0] = 'n'; p[1] = 'a'; p[2] = 'n'; return; }
  if (f.neg) *p++ = '-';
  if (f.kind == 1) { p[0] = 'i'; p[1] = 'n'; p[2] = 'f'; return; }
  unsigned __int128 ip;
  uint32_t fp;
  if ((uint64_t)(f.N >> 64) == 0) {
    const uint64_t n = (uint64_t)f.N;
    ip = n / 1000000u;
    fp = (uint32_t)(n - (uint64_t)ip * 1000000u);
  } else {
    ip = f.N / 1000000u;
    fp = (uint32_t)(f.N - ip * 1000000u);
  }
  const int nd = u128_digits(ip);
  for (int i = 6; i >= 1; --i) { p[nd + i] = (char)('0' + fp % 10); fp /= 10; }
  p[nd] = '.';
  if ((uint64_t)(ip >> 64) == 0) {
    uint64_t y = (uint64_t)ip;
    for (int i = nd - 1; i >= 0; --i) { p[i] = (char)('0' + y % 10); y /= 10; }
  } else {
    for (int i = nd - 1; i >= 0; --i) { p[i] = (char)('0' + (uint32_t)(ip % 10)); ip /= 10; }
  }
}

struct PcdArgs {
  CodecFrames src;
  int32_t* tile_bytes;          // measure: text bytes of each tile
  const int64_t* tile_pos;      // write: byte offset of each tile's text in `out`
  char* out;
  int* err;                     // 1: a value beyond the formatter's range
};

struct PcdLine {
  Fmt6 v[4];
  int len;
};

__device__ __forceinline__ void pcd_line(const double* __restrict__ q, PcdLine& L, int* err) {
  L.len = 4;                                       // 3 separators + newline
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    L.v[c] = fmt6_prepare(q[c]);
    if (L.v[c].kind == 3) *err = 1;
    L.len += fmt6_len(L.v[c]);
  }
}

__device__ __forceinline__ void pcd_emit(const PcdLine& L, char* p) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    fmt6_write(L.v[c], p);
    p += fmt6_len(L.v[c]);
    *p++ = c < 3 ? ' ' : '\n';
  }
}

__device__ __forceinline__ int64_t pcd_row(const CodecFrames& s, int64_t u, int32_t& f, bool& valid) {
  f = codec_frame_of(s.unit_off, s.F, u);
  const int64_t row = s.doff[f] + (u - s.unit_off[f]) * kCodecBlock + threadIdx.x;
  valid = row < s.doff[f + 1];
  return row;
}

// block-wide inclusive sum over kCodecBlock threads (4 waves)
__device__ __forceinline__ int block_scan(int x, int* s_wave, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wave[wid] = x;
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < kCodecBlock / 64; ++w) {
    const int c = s_wave[w];
    before += w < wid ? c : 0;
    total += c;
  }
  return x + before;
}

__global__ __launch_bounds__(kCodecBlock) void k_pcd_measure(const PcdArgs a) {
  __shared__ int s_wave[kCodecBlock / 64];
  int32_t f; bool valid;
  const int64_t row = pcd_row(a.src, blockIdx.x, f, valid);
  int len = 0;
  if (valid) {
    PcdLine L;
    pcd_line(a.src.aos + row * a.src.ld, L, a.err);
    len = L.len;
  }
  int total;
  block_scan(len, s_wave, total);
  if (threadIdx.x == 0) a.tile_bytes[blockIdx.x] = total;
}

// every tile formats its lines into LDS at their block-scan offsets, then the whole tile text is
// stored with consecutive lanes on consecutive bytes (a tile larger than the LDS buffer — only
// possible with extreme magnitudes — is written line by line straight to HBM instead)
__global__ __launch_bounds__(kCodecBlock) void k_pcd_write(const PcdArgs a) {
  __shared__ int s_wave[kCodecBlock / 64];
  __shared__ char s_text[kPcdTileText];
  int32_t f; bool valid;
  const int64_t row = pcd_row(a.src, blockIdx.x, f, valid);
  PcdLine L;
  L.len = 0;
  if (valid) pcd_line(a.src.aos + row * a.src.ld, L, a.err);
  int total;
  const int incl = block_scan(L.len, s_wave, total);
  const int excl = incl - L.len;
  char* const g = a.out + a.tile_pos[blockIdx.x];
  if (total <= kPcdTileText) {
    if (valid) pcd_emit(L, s_text + excl);
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += kCodecBlock) g[i] = s_text[i];
  } else if (valid) {
    pcd_emit(L, g + excl);
  }
}

}  // namespace mc
