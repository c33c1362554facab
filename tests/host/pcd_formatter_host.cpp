// Host build of the device "%.6f" line writer in livox-motion-compensation-sim_amd/csrc/codecs.hpp
// (the section from `struct PcdFast` to `kPcdSlowTile`, spliced in by tests/test_pcd_formatter_host.py
// at FORMATTER_SECTION) with host stand-ins for the gfx950 intrinsics it uses.  Every line of a
// 256-line tile is OR-ed in reverse lane order into a zeroed buffer 16 bytes in (as the kernel's
// pcd_tile_text does), at a tile offset modulo 16, as the kernel's lanes may interleave; the text is
// compared with the C library's correctly rounded "%.6f" (the same digits as Python's formatting) and
// no byte outside the text may become non-zero.  Exit status = number of bad tiles.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define __device__
#define __forceinline__ inline
#define __noinline__
#define __ATOMIC_RELAXED 0
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
// ds_or_b64 (an LDS atomic OR): the host's plain read-modify-write
template <class T>
static inline T __hip_atomic_fetch_or(T* p, T v, int, int) {
  T o;
  std::memcpy(&o, p, sizeof o);
  const T n = o | v;
  std::memcpy(p, &n, sizeof n);
  return o;
}
static inline uint32_t __umul24(uint32_t a, uint32_t b) { return (a & 0xffffffu) * (b & 0xffffffu); }
// v_mul_i32_i24: the low 24 bits of each operand as signed integers
static inline int __mul24(int a, int b) {
  const int64_t x = (int64_t)(int32_t)((uint32_t)a << 8) >> 8, y = (int64_t)(int32_t)((uint32_t)b << 8) >> 8;
  return (int)(uint32_t)(uint64_t)(x * y);
}
// v_perm_b32: byte i of the result = byte sel[i] of {s0:s1} (0-3 = s1, 4-7 = s0), 12 -> 0x00
static inline uint32_t __builtin_amdgcn_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t v = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t c = (sel >> (8 * i)) & 0xffu;
    const uint32_t b = c < 8 ? (uint32_t)(v >> (8 * c)) & 0xffu : (c == 12 ? 0u : 0xffu);
    r |= b << (8 * i);
  }
  return r;
}
// pk_tens_units (codecs.hpp, outside the spliced section): per 16-bit lane
static inline void pk_tens_units(uint32_t v, uint32_t& t, uint32_t& u) {
  t = u = 0;
  for (int l = 0; l < 2; ++l) {
    const uint32_t x = (v >> (16 * l)) & 0xffffu;
    const uint32_t q = ((x * 103u) & 0xffffu) >> 10;
    t |= q << (16 * l);
    u |= ((x - q * 10u) & 0xffffu) << (16 * l);
  }
}
struct alignas(16) uint4 { uint32_t x, y, z, w; };   // the kernel's 16-byte text chunks
using std::fma;
using std::signbit;
using std::rint;
struct CodecFrames { const double* aos; };
static inline void codec_point(const CodecFrames& s, int32_t, int64_t row, double c[4]) {
  for (int k = 0; k < 4; ++k) c[k] = s.aos[4 * row + k];
}

namespace mc {
// FORMATTER_SECTION
}  // namespace mc
using namespace mc;

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 300000;
  int bad = 0;
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> U(-90, 90);
  std::vector<double> pts(4 * (size_t)N);
  for (size_t i = 0; i < pts.size(); ++i) {
    double x = (double)(float)(U(g) * std::pow(10.0, (double)(g() % 9) - 5));   // float32 values, 1e-5..1e3
    if (i % 5 == 0) x = (double)(int64_t)(U(g) * 1000) / 128.0;                   // exact %.6f ties
    if (i % 7 == 0) x = (double)(int64_t)(U(g) * 1e8) / 64.0 / 1e6;
    if (i % 11 == 0) x = U(g) * (1 + 1e-15 * (double)(g() % 5));                 // full float64 values
    if (i % 13 == 0) x = (g() % 2 ? -1 : 1) * (9.9999995 + 1e-9 * ((int)(g() % 200) - 100));   // digit carry
    if (i % 17 == 0) x = 99.9999995 * (1 + 1e-16 * ((int)(g() % 9) - 4));
    if (i % 19 == 0) x = (g() % 2 ? -1 : 1) * (4293.9999994 + 1e-7 * (double)(g() % 20));      // near 4294
    if (i % 23 == 0) x = -0.0;
    pts[i] = x;
  }
  const CodecFrames s{pts.data()};
  std::vector<uint32_t> buf(16400 / 4 + 4);
  // the multiply-shift divisions of digit_groups on their whole ranges
  for (uint32_t fp = 0; fp < 1000000u; ++fp)
    if ((uint32_t)(((uint64_t)(fp & 0xFFFFFu) * 4294968ull) >> 32) != fp / 1000u ||
        (uint32_t)(((uint64_t)(fp & 0xFFFFFu) * 429497ull) >> 32) != fp / 10000u) { ++bad; break; }
  for (uint32_t x = 0; x < 10000u; ++x)
    if ((__umul24(x, 5243u) >> 19) != x / 100u) { ++bad; break; }
  // fast_ip (the integer part from the float64 N) at every multiple of 10^6 and its neighbours,
  // and at a stride over all of [0, 2^32)
  for (uint64_t k = 0; k * 1000000ull < (1ull << 32); ++k)
    for (int64_t d = -2; d <= 2; ++d) {
      const int64_t N = (int64_t)(k * 1000000ull) + d;
      if (N < 0 || N >= (1ll << 32)) continue;
      if (fast_ip((double)N) != (uint32_t)(N / 1000000)) { if (++bad < 20) std::printf("fast_ip(%lld)\n", (long long)N); }
    }
  for (uint64_t N = 0; N < (1ull << 32); N += 997)
    if (fast_ip((double)N) != (uint32_t)(N / 1000000u)) { if (++bad < 20) std::printf("fast_ip(%llu)\n", (unsigned long long)N); }
  long lines = 0, fast = 0, f32_lines = 0;
  // every float32 in [0, 4294] at a stride, and every float32 within 4096 ulps of each digit-count
  // threshold (10, 100, 1000) and of 4294: the float32 path's N and length equal the float64 path's
  {
    auto check = [&](float v) {
      for (float w : {v, -v}) {
        uint32_t n32 = 0, n64 = 0, i32 = 0, i64 = 0;
        const bool k32 = fmt6_fast_f32(w, n32, i32), k64 = fmt6_fast((double)w, n64, i64);
        if (k64 && (i32 != n32 / 1000000u || i64 != n64 / 1000000u)) ++bad;
        const float c4[4] = {w, w, w, w};
        const double d4[4] = {w, w, w, w};
        if (k32 != k64 || (k64 && n32 != n64) || pcd_fast_len_f32(c4) != pcd_fast_len(d4)) {
          if (++bad < 20) std::printf("float32 value %.9g: n %u/%u ok %d/%d\n", (double)w, n32, n64, k32, k64);
        }
      }
    };
    uint32_t top;
    const float lim = 4294.5f;
    std::memcpy(&top, &lim, 4);
    for (uint32_t b = 0; b <= top; b += 97) { float v; std::memcpy(&v, &b, 4); check(v); }
    for (float t : {10.0f, 100.0f, 1000.0f, 4294.0f}) {
      float v = t;
      for (int i = 0; i < 4096; ++i) v = std::nextafter(v, 0.0f);
      for (int i = 0; i < 8192; ++i, v = std::nextafter(v, 1e9f)) check(v);
    }
    check(std::nanf(""));
    check(INFINITY);
  }
  for (int t = 0; t < N / 256; ++t) {
    std::memset(buf.data(), 0, buf.size() * 4);   // pcd_tile_text zeroes the text buffer
    const int shift = t % 16;
    int off = shift;
    std::string want;
    std::vector<PcdFast> P(256);
    std::vector<PcdText> T(256);
    std::vector<int> offs(256);
    for (int l = 0; l < 256; ++l) {
      const double* c = &pts[4 * ((size_t)t * 256 + l)];
      pcd_fast(s, 0, (int64_t)t * 256 + l, P[l]);
      pcd_text(P[l], T[l]);
      char line[160];
      std::snprintf(line, sizeof line, "%.6f %.6f %.6f %.6f\n", c[0], c[1], c[2], c[3]);
      const double cc[4] = {c[0], c[1], c[2], c[3]};
      const int lf = pcd_fast_len(cc);
      ++lines;
      // the float32-source path (k_pcd_*<true>) on float32-valued lines: same N, signs, lengths
      const float cf[4] = {(float)c[0], (float)c[1], (float)c[2], (float)c[3]};
      if ((double)cf[0] == c[0] && (double)cf[1] == c[1] && (double)cf[2] == c[2] && (double)cf[3] == c[3]) {
        PcdFast Q;
        pcd_fast_vals_f32(cf, Q);
        ++f32_lines;
        if (pcd_fast_len_f32(cf) != lf || Q.ok != P[l].ok ||
            (Q.ok && (Q.neg != P[l].neg || std::memcmp(Q.n, P[l].n, sizeof Q.n) ||
                      std::memcmp(Q.ip, P[l].ip, sizeof Q.ip)))) {
          ++bad;
          std::printf("float32 path differs (ok %d/%d) for %s", Q.ok, P[l].ok, line);
        }
        if (Q.ok) {   // the write pass's packed conversion of a measured-packed line: the same numbers
          PcdFast R;
          pcd_fast_vals_packed(cf, R);
          if (R.neg != Q.neg || std::memcmp(R.n, Q.n, sizeof R.n) || std::memcmp(R.ip, Q.ip, sizeof R.ip)) {
            ++bad;
            std::printf("packed conversion differs for %s", line);
          }
        }
      }
      if (!P[l].ok) {
        if (lf != -1) { ++bad; std::printf("pcd_fast_len accepted a byte-path line: %s", line); }
        continue;
      }
      ++fast;
      if ((int)std::strlen(line) != T[l].len || lf != T[l].len) {
        ++bad;
        std::printf("length %d / %d for %s", T[l].len, lf, line);
      }
      offs[l] = off;
      off += T[l].len;
      want += line;
    }
    for (int l = 255; l >= 0; --l)
      if (P[l].ok) pcd_emit_line(T[l], reinterpret_cast<uint4*>(buf.data()) + 1, offs[l]);
    const std::string got(reinterpret_cast<const char*>(buf.data()) + 16 + shift, off - shift);
    // nothing written outside the tile's text
    const unsigned char* bb = reinterpret_cast<const unsigned char*>(buf.data()) + 16;
    for (size_t i = 0; i + 16 < buf.size() * 4; ++i)
      if ((i < (size_t)shift || i >= (size_t)off) && bb[i] != 0) {
        ++bad;
        std::printf("tile %d: byte %zu outside the text [%d, %d) was written\n", t, i, shift, off);
        break;
      }
    if (got != want) {
      ++bad;
      size_t i = 0;
      while (i < got.size() && got[i] == want[i]) ++i;
      std::printf("tile %d: byte %zu differs: got [%s] want [%s]\n", t, i, got.substr(i > 20 ? i - 20 : 0, 60).c_str(),
                  want.substr(i > 20 ? i - 20 : 0, 60).c_str());
    }
  }
  std::printf("lines %ld packed %ld float32 %ld bad %d\n", lines, fast, f32_lines, bad);
  return bad > 255 ? 255 : bad;
}
