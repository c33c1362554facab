// scan.hpp — gfx950 kernels for scan_environment (LMC:701-770), the step before the hot path
// (SURVEY §8f row 2): every frame's local scan of a static scene, all frames in one launch.
//
// Per (frame, scene point): world distance prefilter, R^T (p - t) into the sensor frame, FOV mask
// on atan2 / asin in degrees and range_min, then in-order stream compaction and the systematic
// subsample (every (n // cap)-th visible point, at most cap).  Everything is evaluated in f64 with
// the reference's operation order: the distance sum without contraction, the rotation as numpy's
// matmul accumulates it (scan_rotate) with the pose's R from rot.cpp (scipy's, bit for bit), the
// same degree conversions — so the kept point sets and their sensor-frame coordinates are the
// reference's exactly.  The range noise (LMC:765-768) is drawn by the host from numpy's global RNG in
// frame order and added here.  Output: float32 batch columns (k_scan_emit<false>) or the reference's
// float64 rows, local and aligned in one pass (k_scan_emit<true>, mc_scan_emit_f64).
//
// A workgroup owns a tile of kScanTile scene points held in registers and tests it against
// kScanFrames frames (scene re-reads from L2 drop by that factor).  Units (tile, frame group) are
// numbered tile-major and taken in the XCD-contiguous order (scan_unit): each XCD runs a contiguous
// range of tiles with all their frame groups, so every scene tile is fetched into one XCD's L2 only
// (with the units dealt over the 8 XCDs every L2 fetched the whole scene: 2.9x the algorithmic
// bytes, profiles/pmc_traffic.json r3s65), and a frame's output runs of neighbouring tiles meet in
// one L2 instead of being written as partial lines by two.
//
// Device layout (mc_set_environment / mc_scan_count): the scene as float64 columns x, y, z (the 24
// bytes the visibility test needs, one coalesced 8-byte load per lane each; the reference's (E,4)
// rows would fetch 32) and intensity (read only for emitted points); per-frame poses {R | t} from the
// host (rot.cpp frame_poses); per-(tile, frame) counts and offsets tile-major with the frames padded
// to kScanFrames, so a workgroup's 8 frames are one 32 / 64-byte run.
#pragma once
#include "kernels.hpp"

namespace mc {

constexpr int kScanRounds = 4;                       // scene points per thread per tile
constexpr int kScanTile = kScanRounds * kBlock;      // 1024 scene points per workgroup
constexpr int kScanFrames = 8;                       // frames per workgroup

struct ScanParams {
  double range_min, range_max_sq, half_fov_h, half_fov_v;
  int64_t cap;         // points_per_frame
  double tan_h, sin_v2;        // tan / sin^2 of the half FOVs: decisions away from the edges
  double rmin2_lo, rmin2_hi;   // range_min^2 (1 -+ 1e-12)
  int fast;                    // both half FOVs in [0, 89) degrees
};

inline ScanParams make_scan_params(const double par[4], int64_t cap) {
  ScanParams sp;
  sp.range_min = par[0]; sp.range_max_sq = par[1]; sp.half_fov_h = par[2]; sp.half_fov_v = par[3];
  sp.cap = cap;
  const double d2r = 3.141592653589793 / 180.0;
  sp.fast = par[2] >= 0.0 && par[2] < 89.0 && par[3] >= 0.0 && par[3] < 89.0;
  sp.tan_h = sp.fast ? std::tan(par[2] * d2r) : 0.0;
  const double sv = sp.fast ? std::sin(par[3] * d2r) : 0.0;
  sp.sin_v2 = sv * sv;
  // a non-positive range_min passes every point (sqrt(d2) >= 0)
  sp.rmin2_lo = par[0] > 0.0 ? par[0] * par[0] * (1.0 - 1e-12) : -1.0;
  sp.rmin2_hi = par[0] > 0.0 ? par[0] * par[0] * (1.0 + 1e-12) : -1.0;
  return sp;
}

// R^T d (LMC:728: (R.T @ d.T).T) the way numpy's matmul accumulates it: per output an ascending
// FMA chain over k, fma(A[i][2], d2, fma(A[i][1], d1, A[i][0] * d0)) with A = R^T (numpy's dgemm on
// the reference's box, tools/fma_order.py).  With the pose's R from rot.cpp the sensor-frame
// coordinates equal the reference's bit for bit.
__device__ __forceinline__ void scan_rotate(const double* __restrict__ P, double dx, double dy, double dz, double& lx,
                                            double& ly, double& lz) {
#pragma clang fp contract(off)
  lx = __builtin_fma(P[6], dz, __builtin_fma(P[3], dy, P[0] * dx));
  ly = __builtin_fma(P[7], dz, __builtin_fma(P[4], dy, P[1] * dx));
  lz = __builtin_fma(P[8], dz, __builtin_fma(P[5], dy, P[2] * dx));
}

// the reference's degree comparisons (LMC:735-744), for points near an FOV edge only: kept out of
// line so the rarely taken transcendental code does not inflate the register budget of the loop
__device__ __noinline__ bool scan_fov_exact(double lx, double ly, double s, int az_in, int el_in, double half_h,
                                            double half_v) {
  if (az_in < 0 && !(fabs(atan2(ly, lx) * 180.0 / 3.141592653589793) <= half_h)) return false;
  if (el_in < 0 && !(fabs(asin(s) * 180.0 / 3.141592653589793) <= half_v)) return false;
  return true;
}

// LMC:713-745 for one scene point (ex, ey, ez); returns visibility and the sensor-frame coordinates
__device__ __forceinline__ bool scan_visible(const double* __restrict__ P, double ex, double ey, double ez,
                                             const ScanParams& sp, double& lx, double& ly, double& lz) {
#pragma clang fp contract(off)
  const double dx = ex - P[9], dy = ey - P[10], dz = ez - P[11];
  const double d2 = dx * dx + dy * dy + dz * dz;              // np.sum(.., axis=1) order
  if (!(d2 <= sp.range_max_sq)) return false;                 // LMC:718
  scan_rotate(P, dx, dy, dz, lx, ly, lz);                      // R^T (p - t), LMC:727-728
  // Away from the edges the tests of LMC:732-745 are decided without sqrt / division / atan2 /
  // asin: r >= range_min by d2 against range_min^2, |az| <= h by |ly| <= tan(h) lx (lx > 0),
  // |el| <= v by lz^2 <= sin(v)^2 d2 (both FOVs below 90 degrees, where atan2 / asin are
  // monotonic).  Within a relative 1e-9 of any edge the reference's own expressions decide.
  int r_in = -1, az_in = -1, el_in = -1;
  if (sp.fast) {
    r_in = d2 > sp.rmin2_hi ? 1 : (d2 < sp.rmin2_lo ? 0 : -1);
    const double m = 1e-9 * (fabs(lx) + fabs(ly) + fabs(lz));
    const double a = fabs(ly) - sp.tan_h * lx;
    if (lx > m) az_in = a < -m ? 1 : (a > m ? 0 : -1);
    else if (lx < -m) az_in = 0;
    if (d2 > 1e-10) {
      const double e = lz * lz - sp.sin_v2 * d2;
      const double me = 1e-9 * d2;
      el_in = e < -me ? 1 : (e > me ? 0 : -1);
    }
    if (r_in == 0 || az_in == 0 || el_in == 0) return false;
    if (r_in == 1 && az_in == 1 && el_in == 1) return true;
  }
  const double r = sqrt(d2);                                   // LMC:732
  if (!(r >= sp.range_min)) return false;                      // LMC:745
  double s = lz / fmax(r, 1e-6);                               // LMC:738-739
  s = fmin(fmax(s, -1.0), 1.0);
  return scan_fov_exact(lx, ly, s, az_in, el_in, sp.half_fov_h, sp.half_fov_v);
}

// the scene columns x, y, z, intensity (float64) in one allocation of scene_words(E) doubles
inline size_t scene_words(int64_t E) { return 4 * (size_t)E; }
struct SceneCols {
  const double* x; const double* y; const double* z; const double* w;
};
__host__ __device__ inline SceneCols scene_cols(const double* env, int64_t E) {
  return SceneCols{env, env + E, env + 2 * E, env + 3 * E};
}
__host__ __device__ inline int32_t scan_fpad(int32_t F) { return (F + kScanFrames - 1) / kScanFrames * kScanFrames; }

// the workgroup's scene tile, kScanRounds points per thread, in registers
struct ScanTile {
  double x[kScanRounds], y[kScanRounds], z[kScanRounds];
  bool in[kScanRounds];
};

__device__ __forceinline__ void scan_load_tile(const SceneCols& sc, int64_t E, int64_t tile, ScanTile& t) {
  const int64_t t0 = tile * kScanTile;
#pragma unroll
  for (int r = 0; r < kScanRounds; ++r) {
    const int64_t e = t0 + r * kBlock + threadIdx.x;
    t.in[r] = e < E;
    const int64_t i = t.in[r] ? e : 0;
    t.x[r] = sc.x[i]; t.y[r] = sc.y[i]; t.z[r] = sc.z[i];
  }
}

static_assert(kScanFrames * kScanRounds == 32, "one 32-bit visibility word per thread and workgroup");

// workgroup -> (scene tile, frame group): tile-major units, XCD-contiguous (grid = n_tiles * n_groups)
struct ScanUnit {
  int64_t tile;
  int fg;
};
__device__ __forceinline__ ScanUnit scan_unit(int32_t n_tiles) {
  const int64_t n = (int64_t)gridDim.x;
  const int64_t u = xcd_unit<1>(blockIdx.x, n);
  const int64_t n_fg = n / n_tiles;
  return ScanUnit{u / n_fg, (int)(u % n_fg)};
}

// pass 1: visible scene points per (frame, tile) -> tile_count[tile * scan_fpad(F) + f], and the
// visibility bits (bit j*kScanRounds + r: frame f0+j, round r) that pass 2 consumes
__global__ __launch_bounds__(kBlock) void k_scan_count(const double* __restrict__ env, int64_t E, int32_t n_tiles,
                                                       const double* __restrict__ pose, int32_t F, ScanParams sp,
                                                       int32_t* __restrict__ tile_count,
                                                       uint32_t* __restrict__ vis_bits) {
  __shared__ int s_cnt[kScanFrames][kBlock / 64];
  const ScanUnit su = scan_unit(n_tiles);
  ScanTile t;
  scan_load_tile(scene_cols(env, E), E, su.tile, t);
  const int f0 = su.fg * kScanFrames;
  const int nf = F - f0 < kScanFrames ? F - f0 : kScanFrames;
  uint32_t bits = 0;
  for (int j = 0; j < nf; ++j) {
    const double* P = pose + 12 * (int64_t)(f0 + j);
    int n = 0;
#pragma unroll
    for (int r = 0; r < kScanRounds; ++r) {
      double lx, ly, lz;
      if (t.in[r] && scan_visible(P, t.x[r], t.y[r], t.z[r], sp, lx, ly, lz)) {
        ++n;
        bits |= 1u << (j * kScanRounds + r);
      }
    }
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    if ((threadIdx.x & 63) == 0) s_cnt[j][threadIdx.x >> 6] = n;
  }
  vis_bits[((int64_t)su.fg * n_tiles + su.tile) * kBlock + threadIdx.x] = bits;
  __syncthreads();
  if (threadIdx.x < nf) {
    int tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) tot += s_cnt[threadIdx.x][w];
    tile_count[su.tile * scan_fpad(F) + f0 + threadIdx.x] = tot;
  }
}

// pass 2: in-order compaction + systematic subsample + noise, written into the output batch
struct ScanEmitArgs {
  const double* env; int64_t E; int32_t n_tiles;   // env: the scene columns (scene_cols)
  const double* pose; int32_t F; ScanParams sp;
  const int64_t* tile_off;   // [n_tiles][scan_fpad(F)] exclusive visible-point offset of the tile in its frame
  const int64_t* nvis;       // [F] visible points before subsampling
  const uint32_t* vis_bits;  // pass 1's visibility words
  const double* noise;       // (N_out, 3) in the batch's dense order, or nullptr
  const int64_t* poff; const int64_t* doff;
  float* cols; int32_t C;   // the output batch's blocked columns (kernels.hpp bidx)
  double* local;            // ROWS: (N_out, 4) float64 sensor-frame rows (LMC:770), dense order
  double* aligned;          // ROWS: (N_out, 4) float64 R p + t of those rows (LMC:831), or nullptr
  int32_t* pcd_len;         // columns, MC_BATCH_WITH_PCD_LEN: per-block ASCII PCD bytes (zeroed), or nullptr
};

// ROWS = false: float32 columns of a batch; ROWS = true: the reference's float64 rows (local and,
// fused, the aligned cloud of the same frame pose, LMC:826-831) with no float32 rounding anywhere
template <bool ROWS>
__global__ __launch_bounds__(kBlock) void k_scan_emit(const ScanEmitArgs a) {
  __shared__ int s_cnt[kScanRounds][kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const ScanUnit su = scan_unit(a.n_tiles);
  const SceneCols sc = scene_cols(a.env, a.E);
  ScanTile t;
  scan_load_tile(sc, a.E, su.tile, t);
  const int64_t t0 = su.tile * kScanTile;
  const int f0 = su.fg * kScanFrames;
  const int nf = a.F - f0 < kScanFrames ? a.F - f0 : kScanFrames;
  const uint32_t bits = a.vis_bits[((int64_t)su.fg * a.n_tiles + su.tile) * kBlock + threadIdx.x];
  for (int j = 0; j < nf; ++j) {
    const int f = f0 + j;
    const double* P = a.pose + 12 * (int64_t)f;
    bool vis[kScanRounds];
    double lx[kScanRounds], ly[kScanRounds], lz[kScanRounds];
    int rank[kScanRounds];
#pragma unroll
    for (int r = 0; r < kScanRounds; ++r) {
      vis[r] = (bits >> (j * kScanRounds + r)) & 1u;
      lx[r] = ly[r] = lz[r] = 0.0;
      if (vis[r]) {
        // the sensor-frame point exactly as pass 1 (and LMC:727-728) computed it
#pragma clang fp contract(off)
        const double dx = t.x[r] - P[9], dy = t.y[r] - P[10], dz = t.z[r] - P[11];
        scan_rotate(P, dx, dy, dz, lx[r], ly[r], lz[r]);
      }
      const unsigned long long m = __ballot(vis[r]);
      rank[r] = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) s_cnt[r][wid] = __popcll(m);
    }
    __syncthreads();
    const int64_t nv = a.nvis[f];
    const int64_t step = nv > a.sp.cap ? nv / a.sp.cap : 1;    // LMC:757-760
    const int64_t poff = ROWS ? 0 : a.poff[f], doff = a.doff[f];
    int64_t base = a.tile_off[su.tile * scan_fpad(a.F) + f];
#pragma unroll
    for (int r = 0; r < kScanRounds; ++r) {
      int before = 0, total = 0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) {
        const int c = s_cnt[r][w];
        before += w < wid ? c : 0;
        total += c;
      }
      if (vis[r]) {
        const int64_t idx = base + before + rank[r];          // index among the frame's visible points
        if (idx % step == 0 && idx / step < a.sp.cap) {
          const int64_t o = idx / step;
          double nx = 0, ny = 0, nz = 0;
          if (a.noise) { const double* q = a.noise + 3 * (doff + o); nx = q[0]; ny = q[1]; nz = q[2]; }
          const int64_t e = t0 + r * kBlock + threadIdx.x;
          // LMC:768 visible_points += noise (one rounding; 0 noise leaves the value unchanged)
          const double px = __dadd_rn(lx[r], nx), py = __dadd_rn(ly[r], ny), pz = __dadd_rn(lz[r], nz);
          if constexpr (ROWS) {
            double* q = a.local + 4 * (doff + o);
            *reinterpret_cast<double2*>(q) = double2{px, py};
            *reinterpret_cast<double2*>(q + 2) = double2{pz, sc.w[e]};
            if (a.aligned) {
              double ax, ay, az;
              frame_apply(P, px, py, pz, ax, ay, az, a.doff[f + 1] - doff == 1);
              double* w = a.aligned + 4 * (doff + o);
              *reinterpret_cast<double2*>(w) = double2{ax, ay};
              *reinterpret_cast<double2*>(w + 2) = double2{az, sc.w[e]};
            }
          } else {
            float* q = a.cols + bidx(a.C, 0, poff + o);
            const float v[4] = {(float)px, (float)py, (float)pz, (float)sc.w[e]};
            q[0] = v[0];
            q[kBlkPts] = v[1];
            q[2 * kBlkPts] = v[2];
            q[3 * kBlkPts] = v[3];
            if (a.pcd_len) {   // this line's text bytes (layout.hpp PcdCount), one atomic per point
              PcdCount pc;
              pc.add2(true, v[0], v[1]);
              pc.add2(true, v[2], v[3]);
              atomicAdd(a.pcd_len + ((poff + o) >> 8), pc.lane_bytes() + (pc.lane_slow() ? kPcdSlowValue : 0));
            }
          }
        }
      }
      base += total;
    }
    __syncthreads();   // s_cnt is rewritten by the next frame
  }
}

}  // namespace mc
