// scan.hpp — gfx950 kernels for scan_environment (LMC:701-770), the step before the hot path
// (SURVEY §8f row 2): every frame's local scan of a static scene, all frames in one launch.
//
// Per (frame, scene point): world distance prefilter, R^T (p - t) into the sensor frame, FOV mask
// on atan2 / asin in degrees and range_min, then in-order stream compaction and the systematic
// subsample (every (n // cap)-th visible point, at most cap).  Visibility is evaluated in f64
// with the reference's operation order (no FMA contraction in the distance sum, the same degree
// conversions), so the kept point sets are the reference's; the range noise (LMC:765-768) is drawn
// by the host from numpy's global RNG in frame order and added here.
#pragma once
#include "kernels.hpp"

namespace mc {

constexpr int kScanRounds = 4;                       // scene points per thread per tile
constexpr int kScanTile = kScanRounds * kBlock;      // 1024 scene points per workgroup

struct ScanParams {
  double range_min, range_max_sq, half_fov_h, half_fov_v;
  int64_t cap;         // points_per_frame
};

// f64 sensor pose per frame: R (row-major, 9) + position (3), pose selection as in LMC:804-812
__global__ __launch_bounds__(kBlock) void k_scan_pose(const double* time, const double* pos, const double* rpy,
                                                      int64_t T, const double* frame_time, int32_t F,
                                                      int pose_select, double* pose) {
  const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (f >= F) return;
  int64_t idx;
  if (pose_select == 1) {
    idx = f;
  } else {
    idx = lower_bound_f64(time, T, frame_time[f]);
    if (idx > T - 1) idx = T - 1;
  }
  double R[9];
  euler_xyz_matrix(rpy[3 * idx], rpy[3 * idx + 1], rpy[3 * idx + 2], R);
  for (int k = 0; k < 9; ++k) pose[12 * f + k] = R[k];
  for (int k = 0; k < 3; ++k) pose[12 * f + 9 + k] = pos[3 * idx + k];
}

// LMC:713-745 for one scene point; returns visibility and the sensor-frame coordinates
__device__ __forceinline__ bool scan_visible(const double* __restrict__ P, const double* __restrict__ e,
                                             const ScanParams& sp, double& lx, double& ly, double& lz) {
#pragma clang fp contract(off)
  const double dx = e[0] - P[9], dy = e[1] - P[10], dz = e[2] - P[11];
  const double d2 = dx * dx + dy * dy + dz * dz;              // np.sum(.., axis=1) order
  if (!(d2 <= sp.range_max_sq)) return false;                 // LMC:718
  lx = P[0] * dx + P[3] * dy + P[6] * dz;                      // R^T (p - t), LMC:727-728
  ly = P[1] * dx + P[4] * dy + P[7] * dz;
  lz = P[2] * dx + P[5] * dy + P[8] * dz;
  const double r = sqrt(d2);                                   // LMC:732
  const double az = atan2(ly, lx) * 180.0 / 3.141592653589793;
  double s = lz / fmax(r, 1e-6);
  s = fmin(fmax(s, -1.0), 1.0);
  const double el = asin(s) * 180.0 / 3.141592653589793;
  return fabs(az) <= sp.half_fov_h && fabs(el) <= sp.half_fov_v && r >= sp.range_min;
}

// pass 1: visible scene points per (frame, tile)
__global__ __launch_bounds__(kBlock) void k_scan_count(const double* __restrict__ env, int64_t ld, int64_t E,
                                                       const double* __restrict__ pose, ScanParams sp,
                                                       int32_t* __restrict__ tile_count) {
  __shared__ int s_cnt[kBlock / 64];
  const int f = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * kScanTile;
  const double* P = pose + 12 * (int64_t)f;
  int n = 0;
#pragma unroll
  for (int r = 0; r < kScanRounds; ++r) {
    const int64_t e = t0 + r * kBlock + threadIdx.x;
    double lx, ly, lz;
    if (e < E && scan_visible(P, env + e * ld, sp, lx, ly, lz)) ++n;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) tot += s_cnt[w];
    tile_count[(int64_t)f * gridDim.x + blockIdx.x] = tot;
  }
}

// pass 2: in-order compaction + systematic subsample + noise, written into the output batch
struct ScanEmitArgs {
  const double* env; int64_t ld; int64_t E;
  const double* pose; ScanParams sp;
  const int64_t* tile_off;   // [F][n_tiles] exclusive visible-point offset of the tile in its frame
  const int64_t* nvis;       // [F] visible points before subsampling
  const double* noise;       // (N_out, 3) in the batch's dense order, or nullptr
  const int64_t* poff; const int64_t* doff;
  float* cols; int64_t cap;
};

__global__ __launch_bounds__(kBlock) void k_scan_emit(const ScanEmitArgs a) {
  __shared__ int s_cnt[kBlock / 64];
  const int f = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * kScanTile;
  const double* P = a.pose + 12 * (int64_t)f;
  const int64_t nv = a.nvis[f];
  const int64_t step = nv > a.sp.cap ? nv / a.sp.cap : 1;    // LMC:757-760
  const int64_t poff = a.poff[f], doff = a.doff[f];
  int64_t base = a.tile_off[(int64_t)f * gridDim.x + blockIdx.x];
  for (int r = 0; r < kScanRounds; ++r) {
    const int64_t e = t0 + r * kBlock + threadIdx.x;
    double lx = 0, ly = 0, lz = 0;
    const bool vis = e < a.E && scan_visible(P, a.env + e * a.ld, a.sp, lx, ly, lz);
    const unsigned long long m = __ballot(vis);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_cnt[wid] = __popcll(m);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      const int c = s_cnt[w];
      before += w < wid ? c : 0;
      total += c;
    }
    if (vis) {
      const int64_t idx = base + before + rank;               // index among the frame's visible points
      if (idx % step == 0 && idx / step < a.sp.cap) {
        const int64_t o = idx / step;
        double nx = 0, ny = 0, nz = 0;
        if (a.noise) { const double* q = a.noise + 3 * (doff + o); nx = q[0]; ny = q[1]; nz = q[2]; }
        const int64_t p = poff + o;
        a.cols[p] = (float)(lx + nx);
        a.cols[a.cap + p] = (float)(ly + ny);
        a.cols[2 * a.cap + p] = (float)(lz + nz);
        a.cols[3 * a.cap + p] = (float)a.env[e * a.ld + 3];
      }
    }
    base += total;
    __syncthreads();   // s_cnt is rewritten by the next round
  }
}

}  // namespace mc
