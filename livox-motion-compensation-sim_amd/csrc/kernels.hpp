// kernels.hpp — gfx950 (CDNA4, wave64) device code of the motion-compensation hot path.
//
// Kernels (DESIGN.md §4 has the roofline of each):
//   k_prep              per step, tiny: pose selection + Euler->R per frame (LMC:804-812, 774);
//                       quaternion segment table (SLERP) / IMU record table (CSIM:1482-1516);
//                       per-frame segment windows and their frame-specialised records.
//   k_deskew_frame      Path A, LMC:772-776: p' = R p + t, one pose per frame (SGPR-resident).
//   k_deskew_points<1>  build-added per-point mode: quaternion SLERP + position
//                       LERP of the pose table at each point's time, fused rotate-then-translate.
//   k_deskew_points<2>  Path B, CSIM:1435-1536: gyro LERP at the point timestamp,
//                       theta = w*dt, p' = Rx(-tx) Ry(-ty) Rz(-tz) p.
//   k_trange / k_synth / k_checksum / layout converters: staging, not the per-step path.
//
// Work decomposition: the batch is a "padded CSR" of frames (every frame starts at a multiple of
// 4 points), cut into frame-aligned tiles of up to kTileGroups float4 groups.  A workgroup owns
// one (sub-)tile, so the frame and its pose window are uniform over the workgroup: the pose
// records are read with scalar loads into SGPRs, every column access is a 16-byte-per-lane
// coalesced global_load/store_dwordx4, and stores are non-temporal.  Frames whose points span
// more than two pose/IMU segments stage their window in LDS (one barrier per sub-tile).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include <type_traits>

#include "layout.hpp"

namespace mc {

// Shipping configuration.  The A/B history of every choice below (and of the arms that lost) is in
// profiles/HISTORY_r1-r4.md and profiles/; the kernels carry only the configuration that ships.
//   * output stores: sc1 write-through (st_pol<2>) in the frame, SLERP and IMU kernels — SLERP +7 %
//     vs nt; IMU 327.8-330.1 vs 337.9-343.9 us with sc1 nt (profiles/round3/s46); frame 298.2-298.9
//     vs 300.3-301.3 us with sc1 nt (s48);
//   * non-temporal input loads: SLERP 318.4-322.5 vs 351.7-358.9 us without (profiles/round3/s54);
//   * 4 waves / SIMD for the per-point kernels (128 VGPRs; 5 waves spills, -8 to -11 %, s41);
//   * frames spanning <= 2 segments take the SGPR path, wider ones per-sub-tile windows (§4);
//   * IMU: both window records loaded before the wave's vote, the second one without waiting for the
//     window's W (s21, s23); sub-tile records = segments klo, klo + 1 of the step's IMU segment table
//     (329.1 vs 349.3 us over 5 replicas, s28); the sub-tile window loaded beside the tile record (s35).
constexpr int kStorePol = 2;       // st_pol policy of the deskew kernels' output stores (sc1)
constexpr int kPointsWaves = 4;    // __launch_bounds__ waves / SIMD of k_deskew_points
constexpr int kFastMaxW = 2;       // frames spanning <= this many segments take the SGPR (no-LDS) path

constexpr int kBlock = 256;                    // 4 waves of 64
constexpr int kIters = 2;                      // float4 groups per thread per tile (k_affine_w)
constexpr int kTileGroups = kBlock * kIters;   // 512 groups = 2048 points per tile
constexpr int kSub = kTileGroups / kBlock;     // per-point modes: sub-tiles of kBlock groups
constexpr int kWinMax = 64;                    // LDS window capacity (segments per frame)

// Blocked column layout ("AoSoA"): a batch is a sequence of 256-point blocks, each holding its C
// columns (x, y, z, intensity [, t_ns]) of 256 values back to back.  A wave's float4 access to
// one column is 1 KB contiguous, and a workgroup's whole working set is one contiguous stretch
// of HBM instead of C streams a batch apart (+4-5 % on a 5-in / 4-out pass, tools/layout_probe.hip).
// kBlkPts and the index bidx(C, c, p) live in layout.hpp (shared with the codecs).

struct Tile {
  int64_t pstart;   // padded point index of the first group (multiple of kBlkPts)
  int32_t frame;    // frame id (uniform over the tile)
  int32_t ngroups;  // float4 groups in this tile (<= kTileGroups)
};

// Frame mode pose, one row of [R | t] (LMC:774-775) in float64: the kernels do p' = R p + t in
// float64 on the float32 points and round once on the store, so every output coordinate is the
// reference's float64 value rounded to float32 (<= 2^-24 relative per coordinate, north_star's
// 1e-5 with no scale floor).  3 rows per frame.
struct FrameRow {
  double x, y, z, w;   // R[i][0..2], t_i
};

// One segment [k, k+1] of the pose table (trajectory), built per step by k_prep, float64.  The
// SLERP at alpha is written q(alpha) = cos(alpha th) q0 + alpha sinc(alpha th) v with
// v = th (q1 - cos(th) q0) / sin(th): no division, no small-angle branch, and cos / sinc are even
// polynomials in (alpha th)^2 on th <= pi/2 (slerp_point).
struct PoseSeg {
  double q0[4];   // unit quaternion (x,y,z,w) of orientation_imu[k]
  double v[4];    // th * q_perp, q1 sign-flipped onto q0's hemisphere first (shortest arc)
  double p0[3];   // position[k]
  double dp[3];   // position[k+1] - position[k]
  double th;      // Theta, the angle between q0 and q1 (<= pi/2)
  double t0;      // time[k]
  double inv_dt;  // 1/(time[k+1]-time[k]), 0 for a degenerate segment
  double tf;      // PoseWin: the frame's time (alpha from t_frame + t_ns*1e-9 as the reference forms t)
};

// PoseSeg specialised to one frame (tf set): alpha = clamp(((tf + t_ns*1e-9) - t0) * inv_dt, 0, 1).
typedef PoseSeg PoseWin;

// One IMU record k (CSIM:1482-1516 semantics): gyro(t) = g + alpha*dg,
// alpha = max(0, (t - ts) * inv_dt); the last record has dg = 0, inv_dt = 0.
struct ImuSeg {
  double g[3];
  double dg[3];
  double inv_dt;
  int64_t ts;    // absolute ns in the global table; frame-relative ns in a frame window
};

// Per-frame segment window, written by k_prep: segments [klo, klo+W) cover every point of
// the frame; bnd1 = frame-relative ns where segment klo+1 starts (W >= 2).
struct FrameWin {
  int32_t klo;
  int16_t W;
  int16_t tier;    // polynomial tier covering every point of the window (per_point_tier)
  int64_t bnd1;
};

struct DeskewArgs {
  const float* in;         // blocked columns x|y|z|i[|t_ns], in_C of them
  int64_t in_C;
  int32_t copy_t;          // per-point modes, out != in and out_C == 5: pass t_ns through (CSIM:1472)
  float* out;              // blocked columns, out_C of them
  int64_t out_C;
  const Tile* tiles;
  int32_t n_tiles;
  int32_t xcd_order;       // sub-tiles in XCD-contiguous order (1) or dealt (0): the mode's default or
                           // what mc_tune_order measured faster on this device (deskew_plan)
  const FrameRow* frame_tbl; // frame mode: 3 rows per frame (R row i, t_i), float64
  const double* frame_time;
  const int64_t* frame_start;
  const FrameWin* fwin;    // per-point modes
  const void* frec;        // 2 frame-specialised records per frame (PoseWin or ImuSeg)
  const FrameWin* swin;    // per sub-tile: the same, for frames whose window exceeds kFastMaxW
  unsigned long long* span; // timed launches only (else null): the launch's workgroup span on the wall
                           // clock, [0] = the first workgroup's start, [1 + k] = the end of the k-th of
                           // its last kSpanTail workgroups (launch_span; the slot also keeps the
                           // kernel-argument layout the deskew kernels' register allocation was
                           // measured with: without it the fused SLERP kernel spills more SGPRs)
  const double* pose_time; // T
  const PoseSeg* pose_seg; // nseg
  const int64_t* imu_ts;   // M
  const ImuSeg* imu_seg;   // M
  int64_t nseg;            // segments (SLERP: max(T-1,1); IMU: M)
  int64_t ntab;            // T or M (length of the time table)
  // deskew -> PCD (mc_deskew_pcd, the *_pcd kernels): ASCII PCD text bytes of each output block's
  // valid lines (pcd_value_len sums; index = global block), so the PCD writer needs no measure pass
  int32_t* pcd_len;
  const int64_t* fpoff;    // the output batch's per-frame padded offsets and point counts
  const int64_t* fcount;
};

// ---------------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------------

// Sub-tile order defaults (deskew_plan's default_order; mc_tune_order measures both orders on the
// device at hand, the runtime field DeskewArgs::xcd_order): XCD-contiguous for the frame kernel
// (-7 %, profiles/r13/ab_xcd*.log; tuned XCD in every round-3 line); dealt for SLERP below ~200 M
// points (the slimmed fused next-step kernel streams it fastest: 317-320 vs 342-354 us,
// profiles/round3/s52-s64) and for IMU since its sc1 stores (327.9 vs 349.9 us, s52, s56)
#ifndef MC_XCD_FRAME
#define MC_XCD_FRAME 1
#endif
#ifndef MC_XCD_IMU
#define MC_XCD_IMU 0         // IMU: dealt since its sc1 stores — mc_tune_order picked dealt in every bench
                             // line of s46-s54 (330.8 vs 352.3 us XCD-contiguous, profiles/round3/s52)
#endif
#ifndef MC_XCD_SLERP
#define MC_XCD_SLERP 0
#endif
#ifndef MC_XCD_STAGE
#define MC_XCD_STAGE 1       // the LDS stager pair's tile order
#endif
// 16-byte non-temporal store (output is written once and never re-read by this kernel)
typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
// Output store cache policy (measured with tools/ab.py, interleaved in one process):
//   0 plain, 1 nt (builtin), 2 sc1 write-through.
// The per-point kernels run 10-12% faster with sc1 write-through stores (the line leaves L2 at
// once instead of being retained dirty); the frame kernel is 2% faster with nt.
// sc1 alone has no C-level store builtin, so policy 2 is an inline-asm global_store_dwordx4.  What
// the compiler cannot see about it, and why that is safe:
//   * the store reads its data VGPRs after issue, and on gfx940+ a VALU write to them needs 2 wait
//     states behind the store; the compiler inserts them only after stores it can see, so the asm
//     ends in `s_nop 1` (without it the stager's sc1 build lost the first 8 bytes of chunks,
//     profiles/round3/s08, s24; tests/test_asm_stores.py checks every asm store of the built
//     library's ISA for it);
//   * the compiler's vmcnt bookkeeping does not count the store; on gfx9 vector loads and stores
//     retire from vmcnt in issue order, so an uncounted younger store only makes a wait the
//     compiler places for an older load stricter, never looser.
// The alternative the compiler sees, __builtin_amdgcn_raw_buffer_store_b128 with the SC1 aux bit,
// measured IMU -1.3 %, frame -0.2 %, but SLERP bimodal at 316 / 380-390 us (median +20 %) in two
// interleaved A/Bs (profiles/round4/s10, s11), so the asm store stays.
template <int POL>
__device__ __forceinline__ void st_pol(float* p, const float4& v) {
  static_assert(POL >= 0 && POL <= 2, "store policy 0 / 1 / 2");
  v4f t = {v.x, v.y, v.z, v.w};
  if constexpr (POL == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(t) : "memory");
  } else if constexpr (POL == 1) {
    __builtin_nontemporal_store(t, reinterpret_cast<v4f*>(p));
  } else {
    *reinterpret_cast<v4f*>(p) = t;
  }
}
__device__ __forceinline__ void st_out(float* p, const float4& v) { st_pol<kStorePol>(p, v); }

// 16-byte streaming loads of the input columns
__device__ __forceinline__ float4 ld4(const float* p) {
  const v4f t = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  return make_float4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ int4 ld4(const int32_t* p) {
  const v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
  return make_int4(t.x, t.y, t.z, t.w);
}

__device__ __forceinline__ int ld1(const int32_t* p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// entries of the non-decreasing a[0..n) that are <= x  == numpy searchsorted(a, x, 'right')
template <typename T>
__device__ __forceinline__ int64_t upper_bound(const T* a, int64_t n, T x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// numpy searchsorted(a, x, 'left'): first index with a[i] >= x  (LMC:804)
__device__ __forceinline__ int64_t lower_bound_f64(const double* a, int64_t n, double x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// R = Rz(yaw) Ry(pitch) Rx(roll) == scipy Rotation.from_euler('xyz', rpy).as_matrix() (LMC:774)
__device__ __forceinline__ void euler_xyz_matrix(double r, double p, double y, double R[9]) {
  double sr, cr, sp, cp, sy, cy;
  sincos(r, &sr, &cr);
  sincos(p, &sp, &cp);
  sincos(y, &sy, &cy);
  R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
  R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
  R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

// f64 sin/cos for the per-step prep (k_prep) and the IMU kernel's general tier, whose latency is one
// wave's serial f64 chain: ocml's sincos carries a Payne-Hanek branch (v_trig_preop) inlined at
// every call site (k_prep was 7.2 k instructions), and an out-of-line call costs the deskew kernels
// a call frame (IMU kernel 351 -> 372 us).  Cody-Waite reduction by pi/2 in three 33-bit parts
// (fdlibm's pio2_1/2/3) with fma: each fma forms n * pio2_k exactly and rounds once, so the reduced
// argument is within ~1e-16 + 7e-27 |n| absolute (the first step's result is ~6e-11 |n|) — ~1e-16
// up to |x| ~ 2^30 pi/2, ~1e-11 at 2^50 (the plain products alone are exact only below
// |n| < 2^20).  Then the fdlibm __kernel_sin / __kernel_cos minimax polynomials on |r| <= pi/4
// (<= 2.4 ulp measured against long double over 2e7 arguments).  |x| >= 2^50 rad or non-finite: NaN
// (an angle that large carries an input rounding of >= 0.1 rad; the quadrant index would overflow).
__device__ __forceinline__ void sincos_prep(double x, double* s, double* c) {
  if (!(fabs(x) < 1125899906842624.0)) { *s = *c = __builtin_nan(""); return; }
  const double n = rint(x * 6.36619772367581382433e-01);
  double r = fma(-n, 1.57079632673412561417e+00, x);      // pio2_1: first 33 bits of pi/2
  r = fma(-n, 6.07710050630396597660e-11, r);              // pio2_2
  r = fma(-n, 2.02226624871116645580e-21, r);              // pio2_3
  const double z = r * r;
  double ps = fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
  ps = fma(z, ps, 2.75573137070700676789e-06);
  ps = fma(z, ps, -1.98412698298579493134e-04);
  ps = fma(z, ps, 8.33333333332248946124e-03);
  ps = fma(z, ps, -1.66666666666666324348e-01);
  const double sr = fma(r * z, ps, r);
  double pc = fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
  pc = fma(z, pc, -2.75573143513906633035e-07);
  pc = fma(z, pc, 2.48015872894767294178e-05);
  pc = fma(z, pc, -1.38888888888741095749e-03);
  pc = fma(z, pc, 4.16666666666666019037e-02);
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cr = w + (((1.0 - w) - hz) + z * z * pc);
  const int q = (int)(int64_t)n;
  const double s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
  *s = (q & 2) ? -s0 : s0;
  *c = ((q + 1) & 2) ? -c0 : c0;
}

// euler_xyz_matrix with sincos_prep (k_prep's frame table; the f64 host-array kernels keep ocml)
__device__ __forceinline__ void euler_xyz_matrix_prep(double r, double p, double y, double R[9]) {
  double sr, cr, sp, cp, sy, cy;
  sincos_prep(r, &sr, &cr);
  sincos_prep(p, &sp, &cp);
  sincos_prep(y, &sy, &cy);
  R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
  R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
  R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

// unit quaternion (x,y,z,w) of the same rotation (q = qz * qy * qx)
__device__ __forceinline__ void euler_xyz_quat(double r, double p, double y, double q[4]) {
  double sr, cr, sp, cp, sy, cy;
  sincos_prep(0.5 * r, &sr, &cr);
  sincos_prep(0.5 * p, &sp, &cp);
  sincos_prep(0.5 * y, &sy, &cy);
  q[0] = sr * cp * cy - cr * sp * sy;
  q[1] = cr * sp * cy + sr * cp * sy;
  q[2] = cr * cp * sy - sr * sp * cy;
  q[3] = cr * cp * cy + sr * sp * sy;
}

// One pose sample (time, Euler angles, position) as the prep's registers hold it.
struct PoseSample {
  double t, r[3], p[3];
};
__device__ __forceinline__ PoseSample load_pose(const double* time, const double* pos, const double* rpy,
                                                int64_t k) {
  PoseSample s;
  s.t = time[k];
#pragma unroll
  for (int c = 0; c < 3; ++c) { s.r[c] = rpy[3 * k + c]; s.p[c] = pos[3 * k + c]; }
  return s;
}

// A pose sample with its orientation as a unit quaternion (k_prep's SLERP records: each probe lane
// converts its own sample once, so a record needs no sincos of its two samples' Euler angles — 194
// -> fewer VGPRs for the SLERP prep, which the fused next-step kernel must fit in 128).
struct QSample {
  double t, q[4], p[3];
};
__device__ __forceinline__ QSample qsample_of(const PoseSample& s) {
  QSample r;
  r.t = s.t;
  euler_xyz_quat(s.r[0], s.r[1], s.r[2], r.q);
#pragma unroll
  for (int c = 0; c < 3; ++c) r.p[c] = s.p[c];
  return r;
}

// segment [a, b] of the pose table: shortest-arc quaternion pair, Theta, position delta.
// Theta = 2 atan2(|q1 - q0|, |q1 + q0|) is accurate at every angle (acos(q0.q1) loses half the
// digits below ~1e-4), and q1 - cos(Theta) q0 then has norm sin(Theta) to rounding.
// Theta of the quaternion pair (q0, q1), q1 flipped onto q0's hemisphere first (in place)
__device__ __forceinline__ double quat_theta(const double q0[4], double q1[4]) {
  const double d = q0[0] * q1[0] + q0[1] * q1[1] + q0[2] * q1[2] + q0[3] * q1[3];
  if (d < 0.0) { q1[0] = -q1[0]; q1[1] = -q1[1]; q1[2] = -q1[2]; q1[3] = -q1[3]; }
  double dm = 0.0, dpl = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dm = fma(q1[i] - q0[i], q1[i] - q0[i], dm);
    dpl = fma(q1[i] + q0[i], q1[i] + q0[i], dpl);
  }
  return 2.0 * atan2(sqrt(dm), sqrt(dpl));
}

__device__ __forceinline__ PoseSeg pose_seg_q(const QSample& a, const QSample& b) {
  double q0[4], q1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { q0[i] = a.q[i]; q1[i] = b.q[i]; }
  const double th = quat_theta(q0, q1);
  double sn, cs;
  sincos_prep(th, &sn, &cs);
  const double ratio = th > 0.0 ? th / sn : 1.0;   // th / sin(th), 1 at th = 0
  PoseSeg s;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s.q0[i] = q0[i];
    s.v[i] = ratio * fma(-cs, q0[i], q1[i]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    s.p0[i] = a.p[i];
    s.dp[i] = b.p[i] - a.p[i];
  }
  s.th = th;
  s.t0 = a.t;
  const double dt = b.t - a.t;
  s.inv_dt = dt > 0.0 ? 1.0 / dt : 0.0;
  s.tf = 0.0;
  return s;
}
__device__ __forceinline__ PoseSeg pose_seg_of(const PoseSample& a, const PoseSample& b) {
  return pose_seg_q(qsample_of(a), qsample_of(b));
}

// segment k of the pose table (k + 1 clamped to the last sample)
__device__ __forceinline__ PoseSeg make_pose_seg(const double* time, const double* pos, const double* rpy,
                                                 int64_t T, int64_t k) {
  const int64_t k1 = (k + 1 < T) ? k + 1 : k;
  return pose_seg_of(load_pose(time, pos, rpy, k), load_pose(time, pos, rpy, k1));
}

// One IMU sample (ns timestamp, gyro).
struct ImuSample {
  int64_t ts;
  double g[3];
};
__device__ __forceinline__ ImuSample load_imu(const int64_t* ts, const double* gyro, int64_t k) {
  ImuSample s;
  s.ts = ts[k];
#pragma unroll
  for (int c = 0; c < 3; ++c) s.g[c] = gyro[3 * k + c];
  return s;
}

// IMU record (CSIM:1482-1516): the bracketing pair (a, b), or a alone (last = a is the last sample)
__device__ __forceinline__ ImuSeg imu_seg_of(const ImuSample& a, const ImuSample& b, bool last) {
  ImuSeg s;
  s.g[0] = a.g[0]; s.g[1] = a.g[1]; s.g[2] = a.g[2];
  if (!last) {
    s.dg[0] = b.g[0] - a.g[0]; s.dg[1] = b.g[1] - a.g[1]; s.dg[2] = b.g[2] - a.g[2];
    const int64_t dtn = b.ts - a.ts;
    s.inv_dt = dtn > 0 ? 1.0 / (double)dtn : 0.0;
  } else {
    s.dg[0] = s.dg[1] = s.dg[2] = 0.0;
    s.inv_dt = 0.0;
  }
  s.ts = a.ts;
  return s;
}

// IMU record k: the pair (k, k+1), or the last sample alone
__device__ __forceinline__ ImuSeg make_imu_seg(const int64_t* ts, const double* gyro, int64_t M, int64_t k) {
  const bool last = k + 1 >= M;
  return imu_seg_of(load_imu(ts, gyro, k), load_imu(ts, gyro, last ? k : k + 1), last);
}

__device__ __forceinline__ PoseWin make_pose_win(const PoseSeg& s, double tf) {
  PoseWin w = s;
  w.tf = tf;
  return w;
}

// smallest integer n with tf + n*1e-9 >= t_abs (segment boundary in frame-relative ns)
__device__ __forceinline__ int64_t rel_ns_ceil(double t_abs, double tf) {
  double v = ceil((t_abs - tf) * 1e9);
  if (v > 4.0e18) v = 4.0e18;
  if (v < -4.0e18) v = -4.0e18;
  return (int64_t)v;
}

// ---------------------------------------------------------------------------------------------
// k_prep: everything per step that is per frame or per pose/IMU sample (a few thousand threads)
// ---------------------------------------------------------------------------------------------
struct PrepArgs {
  int mode;
  int pose_select;
  int32_t n_frames;
  const double* time; const double* pos; const double* rpy; int64_t T;   // trajectory
  const int64_t* imu_ts; const double* gyro; int64_t M;                  // IMU
  const double* frame_time; const int64_t* frame_start; const int2* trange;  // frames
  FrameRow* frame_tbl; PoseSeg* pose_seg; ImuSeg* imu_seg;               // outputs
  FrameWin* fwin; void* frec;
  int64_t nseg;
  // per sub-tile windows for frames whose window is wider than kFastMaxW
  const int32_t* ftile;    // first tile of frame f (F+1 entries)
  const int2* strange;     // per sub-tile [min, max] t_ns (recorded with trange)
  FrameWin* swin;
};

// Wave-cooperative searches over a sorted table: 64 lanes probe evenly spaced entries per round,
// so a 3000-pose table takes 2 dependent loads and a 24000-sample IMU table 3 (instead of ~12-15
// for a single-lane binary search).  STRICT=false: entries <= x (searchsorted 'right');
// STRICT=true: entries < x (searchsorted 'left').  Every lane returns the same count.
template <bool STRICT, typename T>
__device__ __forceinline__ int64_t wave_count(const T* a, int64_t n, T x) {
  const int lane = threadIdx.x & 63;
  int64_t lo = 0, hi = n;  // answer in [lo, hi]
  while (hi - lo > 64) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t idx = lo + lane * step;
    const bool in = idx < hi && (STRICT ? a[idx] < x : a[idx] <= x);
    const int c = __popcll(__ballot(in));
    if (c == 0) return lo;
    const int64_t nlo = lo + (int64_t)(c - 1) * step + 1;
    const int64_t nhi = lo + (int64_t)c * step;
    lo = nlo;
    hi = nhi < hi ? nhi : hi;
  }
  const int64_t idx = lo + lane;
  const bool in = idx < hi && (STRICT ? a[idx] < x : a[idx] <= x);
  return lo + __popcll(__ballot(in));
}

// Two searches of the same sorted table in the same rounds (the prep's frame window needs the
// segment of the frame's first and of its last point): round one's probes serve both, later rounds
// issue their two loads together, so the wave waits out one memory latency per round, not two.
template <bool STRICT, typename T>
__device__ __forceinline__ void wave_count2(const T* a, int64_t n, T x0, T x1, int64_t* c0, int64_t* c1) {
  const int lane = threadIdx.x & 63;
  int64_t lo0 = 0, hi0 = n, lo1 = 0, hi1 = n;
  bool done0 = false, done1 = false;
  while (!(done0 && done1)) {
    const bool fine0 = !done0 && hi0 - lo0 <= 64, fine1 = !done1 && hi1 - lo1 <= 64;
    const int64_t st0 = fine0 ? 1 : (hi0 - lo0 + 63) / 64, st1 = fine1 ? 1 : (hi1 - lo1 + 63) / 64;
    const int64_t i0 = lo0 + lane * st0, i1 = lo1 + lane * st1;
    // both loads issued before either compare (the same entry when the two ranges still coincide)
    const T v0 = (!done0 && i0 < hi0) ? a[i0] : T(0);
    const T v1 = (!done1 && i1 < hi1) ? ((i1 == i0 && !done0) ? v0 : a[i1]) : T(0);
    const bool in0 = !done0 && i0 < hi0 && (STRICT ? v0 < x0 : v0 <= x0);
    const bool in1 = !done1 && i1 < hi1 && (STRICT ? v1 < x1 : v1 <= x1);
    const int n0 = __popcll(__ballot(in0)), n1 = __popcll(__ballot(in1));
    if (!done0) {
      if (fine0 || n0 == 0) { *c0 = lo0 + n0 * (fine0 ? 1 : 0); done0 = true; }
      else { const int64_t nlo = lo0 + (int64_t)(n0 - 1) * st0 + 1, nhi = lo0 + (int64_t)n0 * st0;
             lo0 = nlo; hi0 = nhi < hi0 ? nhi : hi0; }
    }
    if (!done1) {
      if (fine1 || n1 == 0) { *c1 = lo1 + n1 * (fine1 ? 1 : 0); done1 = true; }
      else { const int64_t nlo = lo1 + (int64_t)(n1 - 1) * st1 + 1, nhi = lo1 + (int64_t)n1 * st1;
             lo1 = nlo; hi1 = nhi < hi1 ? nhi : hi1; }
    }
  }
}

// A timed launch's workgroup span (DeskewArgs::span): the first workgroup stamps its start and every
// wave its end, folded by atomicMax into one of kSpanTail slots (no wave is missed however the
// workgroups are ordered over the XCDs); the span is the kernel's own execution time, without the
// dispatch gap a start event before the launch includes (~5 us, profiles/round4/s12/roofline_trace.json).
constexpr int kSpanTail = 2048;
__device__ __forceinline__ void span_start(unsigned long long* span) {
  if (span && blockIdx.x == 0 && threadIdx.x == 0) span[0] = (unsigned long long)wall_clock64();
}
__device__ __forceinline__ void span_end(unsigned long long* span) {
  if (span && (threadIdx.x & 63) == 0) {
    const unsigned slot = (blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) & (kSpanTail - 1);
    atomicMax(span + 1 + slot, (unsigned long long)wall_clock64());
  }
}

// ---- k_prep's searches: one load round from an interpolation guess ----------------------------
// The per-step prep is a chain of dependent memory round trips per frame wave (frame record ->
// search rounds -> the records' samples -> math), and its latency is step time: the deskew kernel
// waits for it.  Every table here is a uniform or near-uniform grid (pose samples at gps_rate, IMU
// at its rate), so the wave loads the 64 consecutive entries around the interpolation guess for
// the frame, together with each entry's pose / IMU sample, in ONE round: the search is a ballot
// over the lanes (exact whenever the answer lies inside the window, checked; otherwise the full
// wave-cooperative search), and the samples the records need are shuffled from the lanes that
// hold them (a sample outside the window is loaded).  Frame: 2 memory round trips instead of 5-6.

// first index of the 64-entry window [base, base + 64) around the guess for x in a[0..n)
template <typename T>
__device__ __forceinline__ int64_t probe_base(int64_t n, T a0, T a1, double x) {
  if (n <= 64) return 0;
  const double span = (double)a1 - (double)a0;
  double g = span > 0.0 ? (x - (double)a0) / span * (double)(n - 1) : 0.0;
  g = fmin(fmax(g, 0.0), (double)(n - 1));   // fmax(NaN, 0) = 0
  const int64_t b = (int64_t)g - 31;
  return b < 0 ? 0 : (b > n - 64 ? n - 64 : b);
}

// entries of the sorted a[0..n) that are <= x (STRICT: < x) from the window (lane j holds
// v = a[base + j] when base + j < n); -1 when the answer is not decided inside the window
template <bool STRICT, typename T>
__device__ __forceinline__ int64_t probe_count(T v, int64_t base, int64_t n, T x) {
  const int lane = threadIdx.x & 63;
  const bool in = base + lane < n && (STRICT ? v < x : v <= x);
  const uint64_t m = __ballot(in);
  const bool lo_ok = base == 0 || (m & 1ull);            // everything before the window counts
  const bool hi_ok = base + 64 >= n || !(m >> 63);       // nothing after it does
  return (lo_ok && hi_ok) ? base + (int64_t)__popcll(m) : -1;
}

// entry k of a table whose entries [base, base + 64) the lanes hold (v), else p[stride * k].
// Every lane of the wave must call it (a cross-lane read).
template <typename T>
__device__ __forceinline__ T fetch(T v, int64_t base, int64_t k, const T* p, int stride) {
  const int64_t j = k - base;
  const bool in = j >= 0 && j < 64;
  const T s = __shfl(v, in ? (int)j : 0, 64);
  return in ? s : p[stride * k];
}
__device__ __forceinline__ PoseSample fetch_pose(const PoseSample& v, int64_t base, int64_t k, const PrepArgs& a) {
  PoseSample s;
  s.t = fetch(v.t, base, k, a.time, 1);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    s.r[c] = fetch(v.r[c], base, k, a.rpy + c, 3);
    s.p[c] = fetch(v.p[c], base, k, a.pos + c, 3);
  }
  return s;
}
// QSample k of the pose table whose window [base, base + 64) the lanes hold as QSamples (v); a sample
// outside the window is loaded and converted.  Every lane of the wave must call it.
__device__ __forceinline__ QSample fetch_q(const QSample& v, int64_t base, int64_t k, const PrepArgs& a) {
  const int64_t j = k - base;
  const bool in = j >= 0 && j < 64;
  const int src = in ? (int)j : 0;
  QSample s;
  s.t = __shfl(v.t, src, 64);
#pragma unroll
  for (int c = 0; c < 4; ++c) s.q[c] = __shfl(v.q[c], src, 64);
#pragma unroll
  for (int c = 0; c < 3; ++c) s.p[c] = __shfl(v.p[c], src, 64);
  if (!in) s = qsample_of(load_pose(a.time, a.pos, a.rpy, k));
  return s;
}
// the orientation quaternion of pose sample k alone, the same way
__device__ __forceinline__ void fetch_quat(const QSample& v, int64_t base, int64_t k, const PrepArgs& a, double q[4]) {
  const int64_t j = k - base;
  const bool in = j >= 0 && j < 64;
  const int src = in ? (int)j : 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) q[c] = __shfl(v.q[c], src, 64);
  if (!in) euler_xyz_quat(a.rpy[3 * k], a.rpy[3 * k + 1], a.rpy[3 * k + 2], q);
}
__device__ __forceinline__ ImuSample fetch_imu(const ImuSample& v, int64_t base, int64_t k, const PrepArgs& a) {
  ImuSample s;
  s.ts = fetch(v.ts, base, k, a.imu_ts, 1);
#pragma unroll
  for (int c = 0; c < 3; ++c) s.g[c] = fetch(v.g[c], base, k, a.gyro + c, 3);
  return s;
}

// Polynomial tiers of the per-point sin / cos (see the float64 per-point math below), chosen per
// window by k_prep: SLERP from the window's segment angles Theta (alpha * Theta <= Theta), IMU from
// a bound on the window's angles, |theta| <= max_c (|g_c| + |dg_c|) * max |t_ns| * 1e-9 (alpha in
// [0, 1] for every point a window assigns to a record).
constexpr double kTier0 = 0.0625, kTier1 = 0.25, kTier2 = 1.6;
template <int MODE>
__device__ __forceinline__ int16_t window_tier(double ang) {
  if (MODE == 1) return ang <= kTier0 ? 0 : (ang <= kTier1 ? 1 : 2);
  return ang <= kTier0 ? 0 : (ang <= kTier1 ? 1 : 3);
}
// bound on |theta| over an IMU record's span: |g + alpha dg| <= |g| + |dg|
__device__ __forceinline__ double imu_rate_bound(const ImuSeg& w) {
  const double a = fabs(w.g[0]) + fabs(w.dg[0]), b = fabs(w.g[1]) + fabs(w.dg[1]), c = fabs(w.g[2]) + fabs(w.dg[2]);
  return fmax(a, fmax(b, c));
}
__device__ __forceinline__ double imu_angle_bound(double rate, int2 tr) {   // rate * max |t| * 1e-9, rounded up
  const double tm = fmax(fabs((double)tr.x), fabs((double)tr.y));
  return rate * (tm * 1.000001e-9);
}

// One wave per frame (frame work), then one lane per pose segment / IMU sample (table work).
// MODE = the deskew mode (k_prep dispatches on a.mode).
template <int MODE>
__device__ __forceinline__ void prep_body(const PrepArgs& a, int64_t block) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = block * (kBlock / 64) + (threadIdx.x >> 6);   // global wave id
  if (gw >= a.n_frames) {
    const int64_t k = (gw - a.n_frames) * 64 + lane;
    if (MODE == 1 && k < a.nseg) a.pose_seg[k] = make_pose_seg(a.time, a.pos, a.rpy, a.T, k);
    if (MODE == 2 && k < a.M) a.imu_seg[k] = make_imu_seg(a.imu_ts, a.gyro, a.M, k);
    return;
  }
  const int64_t f = gw;
  if (MODE == 0) {
    // Path A pose selection (LMC:804-812) + Euler->R (LMC:774)
    PoseSample ps;
    if (a.pose_select == 1) {
      ps = load_pose(a.time, a.pos, a.rpy, f);   // explicit per-frame transformation (host checks T == n_frames)
    } else {
      const double tf = a.frame_time[f];
      const int64_t base = probe_base<double>(a.T, a.time[0], a.time[a.T - 1], tf);
      const int64_t pi = base + lane;
      PoseSample pv{};
      if (pi < a.T) pv = load_pose(a.time, a.pos, a.rpy, pi);
      int64_t idx = probe_count<true>(pv.t, base, a.T, tf);
      if (idx < 0) idx = wave_count<true>(a.time, a.T, tf);   // searchsorted 'left'
      if (idx > a.T - 1) idx = a.T - 1;
      ps = fetch_pose(pv, base, idx, a);
    }
    if (lane < 3) {   // lane i writes row i of R and t_i
      double R[9];
      euler_xyz_matrix_prep(ps.r[0], ps.r[1], ps.r[2], R);
      const double t = lane == 0 ? ps.p[0] : (lane == 1 ? ps.p[1] : ps.p[2]);   // no dynamic index (no alloca)
      a.frame_tbl[3 * f + lane] = FrameRow{R[3 * lane], R[3 * lane + 1], R[3 * lane + 2], t};
    }
    return;
  }
  // per-frame window from the frame's time span (recorded when t_ns was staged)
  const int2 tr = a.trange[f];
  const bool has = tr.x <= tr.y;
  const int64_t n_tab = MODE == 1 ? a.T : a.M;
  const double tf = MODE == 1 ? a.frame_time[f] : 0.0;
  const int64_t fs = MODE == 2 ? a.frame_start[f] : 0;
  // the probe window and its samples (one round)
  int64_t base;
  QSample pv{};
  ImuSample iv{};
  if (MODE == 1) {
    const double xm = has ? tf + 0.5e-9 * ((double)tr.x + (double)tr.y) : tf;
    base = probe_base<double>(a.T, a.time[0], a.time[a.T - 1], xm);
    if (base + lane < a.T) pv = qsample_of(load_pose(a.time, a.pos, a.rpy, base + lane));
  } else {
    const double xm = (double)fs + (has ? 0.5 * ((double)tr.x + (double)tr.y) : 0.0);
    base = probe_base<int64_t>(a.M, a.imu_ts[0], a.imu_ts[a.M - 1], xm);
    if (base + lane < a.M) iv = load_imu(a.imu_ts, a.gyro, base + lane);
  }
  int64_t klo = 0, khi = 0;
  if (has) {
    int64_t c0 = -1, c1 = -1;
    if (MODE == 1) {
      const double x0 = tf + (double)tr.x * 1e-9, x1 = tf + (double)tr.y * 1e-9;
      c0 = probe_count<false>(pv.t, base, a.T, x0);
      c1 = probe_count<false>(pv.t, base, a.T, x1);
      if (c0 < 0 || c1 < 0) wave_count2<false>(a.time, a.T, x0, x1, &c0, &c1);
      klo = c0 - 1;
      khi = c1 - 1;
      klo = klo < 0 ? 0 : (klo > a.nseg - 1 ? a.nseg - 1 : klo);
      khi = khi < 0 ? 0 : (khi > a.nseg - 1 ? a.nseg - 1 : khi);
    } else {
      const int64_t x0 = fs + (int64_t)tr.x, x1 = fs + (int64_t)tr.y;
      c0 = probe_count<false>(iv.ts, base, a.M, x0);
      c1 = probe_count<false>(iv.ts, base, a.M, x1);
      if (c0 < 0 || c1 < 0) wave_count2<false>(a.imu_ts, a.M, x0, x1, &c0, &c1);
      klo = c0 - 1;
      khi = c1 - 1;
      klo = klo < 0 ? 0 : klo;
      khi = khi < 0 ? 0 : khi;
    }
  }
  const int64_t W = khi - klo + 1;
  auto clampk = [&](int64_t k) { return k < n_tab - 1 ? k : n_tab - 1; };
  // frame-relative ns where the segment of sample s starts (the LDS path's s_bnd, the SGPR path's bnd1)
  auto bound_pose = [&](const QSample& s) -> int64_t { return rel_ns_ceil(s.t, tf); };
  auto bound_imu = [&](const ImuSample& s) -> int64_t { return s.ts - fs; };
  auto bound_at = [&](int64_t k) -> int64_t { return MODE == 1 ? rel_ns_ceil(a.time[k], tf) : a.imu_ts[k] - fs; };
  // record of segment k from samples k, k+1 (clamped) / IMU k, k+1 (or k alone at the end)
  // s0, s1 come from fetch_pose / fetch_imu; write at dst[slot]
  // a record (its segment's angle measure returned: Theta, or the IMU rate bound)
  auto pose_rec = [&](const QSample& s0, const QSample& s1, void* dst, int64_t slot, bool wr) {
    const PoseSeg sg = pose_seg_q(s0, s1);
    if (wr) reinterpret_cast<PoseWin*>(dst)[slot] = make_pose_win(sg, tf);
    return sg.th;
  };
  auto imu_rec = [&](const ImuSample& s0, const ImuSample& s1, bool last, void* dst, int64_t slot, bool wr) {
    ImuSeg sg = imu_seg_of(s0, s1, last);
    sg.ts -= fs;
    if (wr) reinterpret_cast<ImuSeg*>(dst)[slot] = sg;
    return imu_rate_bound(sg);
  };
  // the frame's two records (lane 0: segment klo + the window header, lane 1: klo + 1); every lane
  // takes part in the fetches
  {
    const int64_t k = clampk(klo + (lane == 1 ? 1 : 0));
    const int64_t k1 = clampk(k + 1);
    const bool writes = lane < 2 && !(lane == 1 && W < 2);
    FrameWin w;
    w.klo = (int32_t)klo;
    w.W = (int16_t)(W > kWinMax ? kWinMax + 1 : W);
    double ang;   // lane 0: segment klo, lane 1: klo + 1
    if (MODE == 1) {
      const QSample s0 = fetch_q(pv, base, k, a), s1 = fetch_q(pv, base, k1, a);
      ang = pose_rec(s0, s1, a.frec, 2 * f + lane, writes);
      w.bnd1 = W >= 2 ? bound_pose(s1) : INT64_MAX;   // lane 0: s1 = sample klo + 1
    } else {
      const ImuSample s0 = fetch_imu(iv, base, k, a), s1 = fetch_imu(iv, base, k1, a);
      ang = imu_rec(s0, s1, k + 1 >= a.M, a.frec, 2 * f + lane, writes);
      w.bnd1 = W >= 2 ? bound_imu(s1) : INT64_MAX;
    }
    const double ang1 = __shfl(ang, 1, 64);
    if (W >= 2) ang = fmax(ang, ang1);
    w.tier = window_tier<MODE>(MODE == 1 ? ang : imu_angle_bound(ang, tr));
    if (lane == 0) a.fwin[f] = w;
  }
  // (IMU: every frame, so the deskew kernel reads only its sub-tile's window, one scalar load)
  if ((MODE == 1 && W <= kFastMaxW) || !a.swin) return;
  // A wide frame (IMU: ~20 samples per 0.1 s frame): each 1024-point sub-tile of a time-ordered
  // frame spans ~1 ms, so its own window is 1-2 segments and takes the SGPR path (no LDS staging,
  // no barrier: -10 % kernel time on SLERP, tools/ab.py).  Lane per sub-tile; segment of t =
  // last k in [klo, khi] with bound(k) <= t (klo if none), as the kernel's window search.
  // A window of <= 64 segments (every IMU frame): lane j holds bound(klo + j) (from the probe
  // window), and a sub-tile's segment is a count over the lanes' bounds; wider windows search the
  // table.
  const bool in_regs = W <= 64;
  int64_t my_bnd = INT64_MAX;
  if (in_regs) {
    const int64_t kb = clampk(klo + lane);
    const int64_t b = MODE == 1 ? rel_ns_ceil(fetch(pv.t, base, kb, a.time, 1), tf) : bound_imu(fetch_imu(iv, base, kb, a));
    my_bnd = lane == 0 ? INT64_MIN : (lane < W ? b : INT64_MAX);
  }
  auto seg_of = [&](int64_t t) {
    if (in_regs) {
      int64_t k = klo - 1;
      for (int j = 0; j < W; ++j) k += (__shfl(my_bnd, j, 64) <= t) ? 1 : 0;
      return k < klo ? klo : k;
    }
    int64_t lo = klo, hi = khi;   // invariant: answer in [lo, hi]
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (bound_at(mid) <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  // SLERP: lane j holds Theta of the probe window's segment base + j (samples base + j and the next);
  // a segment outside the window counts as pi/2, the largest Theta (tier 2 covers every segment)
  double th_lane = 0.0;
  if (MODE == 1) {
    double qn[4], q0[4] = {pv.q[0], pv.q[1], pv.q[2], pv.q[3]};
    fetch_quat(pv, base, clampk(base + lane + 1), a, qn);
    th_lane = quat_theta(q0, qn);
  }
  auto theta_of = [&](int64_t k) {   // every lane must call it (a cross-lane read)
    const int64_t j = k - base;
    const bool in = j >= 0 && j < 64;
    const double v = __shfl(th_lane, in ? (int)j : 0, 64);
    return in ? v : 1.5707963267948966;
  };
  const int64_t st0 = (int64_t)a.ftile[f] * kSub, st1 = (int64_t)a.ftile[f + 1] * kSub;
  for (int64_t sb = st0; sb < st1; sb += 64) {   // a uniform trip count: the shuffles see every lane
    const int64_t st = sb + lane;
    const bool valid = st < st1;
    const int2 r = valid ? a.strange[st] : make_int2(1, 0);
    const bool hs = r.x <= r.y;
    const int64_t s0 = seg_of(hs ? (int64_t)r.x : INT64_MIN), s1 = seg_of(hs ? (int64_t)r.y : INT64_MIN);
    const int64_t k0 = hs ? s0 : klo, n = hs ? s1 - s0 + 1 : 1;
    FrameWin w;
    w.klo = (int32_t)k0;
    w.W = (int16_t)(n > kWinMax ? kWinMax + 1 : n);
    // samples k0, k0 + 1, k0 + 2 (clamped): the boundary of k0 + 1 and the angle bound of segments
    // k0, k0 + 1 (the deskew kernel reads the records themselves from the step's segment table)
    const int64_t ka = clampk(k0), kb = clampk(k0 + 1), kc = clampk(k0 + 2);
    double ang;
    if (MODE == 1) {
      // SLERP: no sub-tile records — the deskew kernel reads segments k0, k0 + 1 of the step's
      // segment table (pose_seg) and adds the frame time; here only the window, its boundary and
      // the tier from the two segments' Theta (building the records here held three samples and two
      // segments live: 200 VGPRs, more than the fused next-step kernel's 128)
      const double t_kb = fetch(pv.t, base, kb, a.time, 1);   // every lane (a cross-lane read)
      w.bnd1 = n >= 2 ? rel_ns_ceil(t_kb, tf) : INT64_MAX;
      ang = theta_of(ka);
      const double ang1 = theta_of(kb);
      if (n >= 2) ang = fmax(ang, ang1);
      (void)kc;
    } else {
      const ImuSample sa = fetch_imu(iv, base, ka, a), sb_ = fetch_imu(iv, base, kb, a);
      const ImuSample sc = fetch_imu(iv, base, kc, a);
      w.bnd1 = n >= 2 ? bound_imu(sb_) : INT64_MAX;
      ang = imu_rec(sa, sb_, ka + 1 >= a.M, nullptr, 0, false);
      if (n >= 2) ang = fmax(ang, imu_rec(sb_, sc, kb + 1 >= a.M, nullptr, 0, false));
    }
    w.tier = window_tier<MODE>(MODE == 1 ? ang : imu_angle_bound(ang, hs ? r : make_int2(0, 0)));
    if (valid) a.swin[st] = w;
  }
}

__global__ __launch_bounds__(kBlock) void k_prep(const PrepArgs a) {
  if (a.mode == 0) prep_body<0>(a, blockIdx.x);
  else if (a.mode == 1) prep_body<1>(a, blockIdx.x);
  else prep_body<2>(a, blockIdx.x);
}

// ---------------------------------------------------------------------------------------------
// Path A: frame mode (LMC:772-776).  One pose per tile -> uniform (SGPR) operands.
// ---------------------------------------------------------------------------------------------
// kW: homogeneous input whose 4th column is w (CSIM:226-229 applies T to (N,4) points as they are),
// p' = A p + b w; otherwise p' = A p + b with the 4th column passed through.
// row r of [R | t] applied to (x, y, z) in float64 (3 FMAs), rounded once to float32; with kW the
// translation is scaled by the homogeneous coordinate w (CSIM:226-229)
template <bool kW = false>
__device__ __forceinline__ float xf_row(const FrameRow& r, float x, float y, float z, float w = 1.f) {
  const double t = kW ? r.w * (double)w : r.w;
  return (float)fma(r.x, (double)x, fma(r.y, (double)y, fma(r.z, (double)z, t)));
}

template <bool kW>
__device__ __forceinline__ void deskew_frame_body(const DeskewArgs& a) {
  for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const Tile tl = ldu(a.tiles + tile);
    const FrameRow r0 = ldu(a.frame_tbl + 3 * tl.frame + 0);
    const FrameRow r1 = ldu(a.frame_tbl + 3 * tl.frame + 1);
    const FrameRow r2 = ldu(a.frame_tbl + 3 * tl.frame + 2);
    // group g of the tile: block pstart/256 + g/64, offset 4 (g % 64) inside it
    const float* ix = a.in + bidx((int)a.in_C, 0, tl.pstart);
    float* ox = a.out + bidx((int)a.out_C, 0, tl.pstart);
    float4 vx[kIters], vy[kIters], vz[kIters], vi[kIters];
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int g = it * kBlock + threadIdx.x;
      if (g < tl.ngroups) {
        const float* q = ix + (int64_t)(g >> 6) * a.in_C * kBlkPts + 4 * (g & 63);
        vx[it] = ld4(q);
        vy[it] = ld4(q + kBlkPts);
        vz[it] = ld4(q + 2 * kBlkPts);
        vi[it] = ld4(q + 3 * kBlkPts);
      }
    }
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int g = it * kBlock + threadIdx.x;
      if (g < tl.ngroups) {
        float4 X = vx[it], Y = vy[it], Z = vz[it], W = vi[it];
        float4 ox4, oy4, oz4;
#define MC_XF(c)                                                  \
  ox4.c = xf_row<kW>(r0, X.c, Y.c, Z.c, W.c);                     \
  oy4.c = xf_row<kW>(r1, X.c, Y.c, Z.c, W.c);                     \
  oz4.c = xf_row<kW>(r2, X.c, Y.c, Z.c, W.c);
        MC_XF(x) MC_XF(y) MC_XF(z) MC_XF(w)
#undef MC_XF
        float* o = ox + (int64_t)(g >> 6) * a.out_C * kBlkPts + 4 * (g & 63);
        st_out(o, ox4);
        st_out(o + kBlkPts, oy4);
        st_out(o + 2 * kBlkPts, oz4);
        st_out(o + 3 * kBlkPts, vi[it]);
      }
    }
  }
}

// Frame kernel, quad decomposition: a workgroup covers 64 float4 groups of a sub-tile and each
// lane ONE column of one group (lane & 3 = x, y, z, intensity): one 16-byte load and one 16-byte
// store per lane (four times the lanes of one group per lane: 293 vs 298-319 us, profiles/round2/s08).  The quad's x / y / z float4s reach
// every lane of the quad through DPP quad broadcasts (no LDS), lane c < 3 forms output column c of
// the four points (R row c . p + t_c in float64, xf_row), lane 3 passes the
// intensities through.  A bare 16 B-in / 16 B-out stream runs at 6.61-6.68 TB/s with one load and
// one store per lane vs 6.12 with four of each (tools/stage_probe.hip, profiles/round2/s07).  Output
// stores sc1 (the deskew kernels' policy): 296.7 vs 306.8 us non-temporal, 303.8 plain
// (profiles/round5/s31).
constexpr int kQuadGroups = kBlock / 4;   // float4 groups per workgroup in the quad decomposition

// kQuadU quarters (64 float4 groups each) per workgroup: each lane issues U column loads before any
// arithmetic, so a wave keeps U KB in flight through its longer float64 chain (frame f64: 294.8 us vs
// 304.0 with U = 1, 308.0 with U = 4, profiles/round3/s05; 299.8-301.0 vs 316.0-319.1 with sc1 stores, s74).
constexpr int kQuadU = 2;
static_assert(kQuadU == 1 || kQuadU == 2 || kQuadU == 4, "quarters per workgroup: 1, 2 or 4");
constexpr int kQuadUnitsPerSub = kBlock / kQuadGroups / kQuadU;   // workgroup units per sub-tile

// PCD: each quarter is one 256-point block; its four waves' text bytes meet in LDS (two barriers per
// workgroup pass, this variant only).
template <bool PCD = false>
__device__ __forceinline__ void deskew_frame_quad(const DeskewArgs& a, const uint32_t pre) {
  const int64_t n_units = (int64_t)a.n_tiles * kSub * kQuadUnitsPerSub;
  const uint32_t nb = gridDim.x - pre;
  const int c = threadIdx.x & 3;
  __shared__ int s_part[PCD ? kQuadU : 1][kBlock / 64];
  for (int64_t it = blockIdx.x - pre; it < n_units; it += nb) {
    const int64_t un = nb >= n_units ? (a.xcd_order ? xcd_unit<1>(it, n_units) : it) : it;
    const int64_t st = un / kQuadUnitsPerSub;
    const Tile tl = ldu(a.tiles + st / kSub);
    const int g0 = (int)(st % kSub) * kBlock + (int)(un % kQuadUnitsPerSub) * kQuadGroups * kQuadU;
    if (g0 >= tl.ngroups) continue;   // uniform: empty part of a short sub-tile
    // lane c's row of [R | t] (lane 3: row 2, unused) as a vector load beside the point load: the
    // 96-byte table row set is L2-resident, and a per-lane select of three SGPR rows would cost 32
    // VALU instructions (two SGPR sources cannot meet in one v_cndmask)
    const FrameRow r = *(a.frame_tbl + 3 * tl.frame + (c < 2 ? c : 2));
    float4 v[kQuadU];
    bool act[kQuadU];
    int64_t p[kQuadU];
#pragma unroll
    for (int u = 0; u < kQuadU; ++u) {
      const int g = g0 + u * kQuadGroups + (threadIdx.x >> 2);
      act[u] = g < tl.ngroups;   // uniform over a quad
      p[u] = tl.pstart + 4 * (int64_t)g;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (act[u]) v[u] = ld4(a.in + bidx((int)a.in_C, c, p[u]));
    }
#pragma unroll
    for (int u = 0; u < kQuadU; ++u) {
      // every lane takes part in the broadcasts (inactive quads carry zeros)
      const float4 w = v[u];
      float4 X, Y, Z;
      X.x = quad_bcast<0>(w.x); X.y = quad_bcast<0>(w.y); X.z = quad_bcast<0>(w.z); X.w = quad_bcast<0>(w.w);
      Y.x = quad_bcast<1>(w.x); Y.y = quad_bcast<1>(w.y); Y.z = quad_bcast<1>(w.z); Y.w = quad_bcast<1>(w.w);
      Z.x = quad_bcast<2>(w.x); Z.y = quad_bcast<2>(w.y); Z.z = quad_bcast<2>(w.z); Z.w = quad_bcast<2>(w.w);
      float4 o;
      o.x = xf_row(r, X.x, Y.x, Z.x);
      o.y = xf_row(r, X.y, Y.y, Z.y);
      o.z = xf_row(r, X.z, Y.z, Z.z);
      o.w = xf_row(r, X.w, Y.w, Z.w);
      if (act[u]) st_out(a.out + bidx((int)a.out_C, c, p[u]), c == 3 ? w : o);
      if constexpr (PCD) {
        // lane c's column of its group's four points (a whole line is the quad's four lanes)
        const float4 val = c == 3 ? w : o;
        const int64_t i0 = p[u] - ldu(a.fpoff + tl.frame), n = ldu(a.fcount + tl.frame);
        PcdCount pc;
        pc.add2(act[u] && i0 < n, val.x, act[u] && i0 + 1 < n, val.y);
        pc.add2(act[u] && i0 + 2 < n, val.z, act[u] && i0 + 3 < n, val.w);
        const int bytes = pc.bytes();   // (every lane: the per-lane variant reduces across the wave)
        if ((threadIdx.x & 63) == 0) s_part[PCD ? u : 0][threadIdx.x >> 6] = bytes;
      }
    }
    if constexpr (PCD) {
      __syncthreads();
      if (threadIdx.x < kQuadU) {
        const int g = g0 + (int)threadIdx.x * kQuadGroups;   // the quarter's first group
        if (g < tl.ngroups) {
          const int* q = s_part[PCD ? threadIdx.x : 0];
          a.pcd_len[(tl.pstart + 4 * (int64_t)g) >> 8] = q[0] + q[1] + q[2] + q[3];
        }
      }
      __syncthreads();   // s_part is rewritten by the next pass
    }
  }
}


__global__ __launch_bounds__(kBlock) void k_deskew_frame(const DeskewArgs a) {
  span_start(a.span);
  deskew_frame_quad(a, 0u);
  span_end(a.span);
}

// Path A with the ASCII PCD text bytes of every output block (mc_deskew_pcd)
__global__ __launch_bounds__(kBlock) void k_deskew_frame_pcd(const DeskewArgs a) { deskew_frame_quad<true>(a, 0u); }

// ---- float64 rows: the reference's own arrays, bit for bit ---------------------------------------
// R p + t (LMC:775: (R @ p.T).T + t) the way numpy's matmul accumulates it: per output an ascending
// FMA chain over k, fma(R[i][2], z, fma(R[i][1], y, R[i][0] * x)), then + t[i] rounded on its own
// (numpy's dgemm, measured on the reference's box: tools/fma_order.py).  P = {R row-major | t}; with
// the host's scipy-faithful R (rot.cpp) the result equals the reference's float64 value exactly.
// A one-point frame is a matrix-vector product for numpy (its dgemv), which accumulates
// fma(R[i][2], z, fma(R[i][0], x, R[i][1] * y)) instead (tools/fma_order.py, single-row cases): `single`.
__device__ __forceinline__ void frame_apply(const double* __restrict__ P, double x, double y, double z, double& ox,
                                            double& oy, double& oz, bool single = false) {
#pragma clang fp contract(off)
  if (single) {
    ox = __builtin_fma(P[2], z, __builtin_fma(P[0], x, P[1] * y)) + P[9];
    oy = __builtin_fma(P[5], z, __builtin_fma(P[3], x, P[4] * y)) + P[10];
    oz = __builtin_fma(P[8], z, __builtin_fma(P[6], x, P[7] * y)) + P[11];
  } else {
    ox = __builtin_fma(P[2], z, __builtin_fma(P[1], y, P[0] * x)) + P[9];
    oy = __builtin_fma(P[5], z, __builtin_fma(P[4], y, P[3] * x)) + P[10];
    oz = __builtin_fma(P[8], z, __builtin_fma(P[7], y, P[6] * x)) + P[11];
  }
}

// the frame of row `row`: last f with doff[f] <= row
__device__ __forceinline__ int32_t row_frame(const int64_t* __restrict__ doff, int32_t F, int64_t row) {
  int32_t lo = 0, hi = F;
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if (doff[mid] <= row) lo = mid; else hi = mid;
  }
  return lo;
}

// Many frames of (n, 4) float64 rows (LMC:802-832 on host arrays, the row pipeline's chunks and the
// zero-copy path): frame f's rows [doff[f], doff[f+1]) get pose[12 f ..] (host frame_poses).  Rows
// [r0, r0 + n) of the concatenated frames; in / out hold (n, ld_in) / (n, 4) rows.
__global__ __launch_bounds__(kBlock) void k_align_rows_f64(const double* __restrict__ in, int64_t ld, int64_t n,
                                                           int64_t r0, const int64_t* __restrict__ doff, int32_t F,
                                                           const double* __restrict__ pose, double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int32_t f = row_frame(doff, F, r0 + i);
    const double* P = pose + 12 * (int64_t)f;
    const double* q = in + i * ld;
    double x, y, z, w;
    if (ld == 4) {
      const double2 p01 = *reinterpret_cast<const double2*>(q);
      const double2 p23 = *reinterpret_cast<const double2*>(q + 2);
      x = p01.x; y = p01.y; z = p23.x; w = p23.y;
    } else {
      x = q[0]; y = q[1]; z = q[2]; w = q[3];
    }
    double ox, oy, oz;
    frame_apply(P, x, y, z, ox, oy, oz, doff[f + 1] - doff[f] == 1);
    double* o = out + 4 * i;
    *reinterpret_cast<double2*>(o) = double2{ox, oy};
    *reinterpret_cast<double2*>(o + 2) = double2{oz, w};
  }
}

// CoordinateTransformer.transform_points (CSIM:214-233): (T @ [p, w].T).T[:, :3] per row with the
// 4x4 T's top 3x4 [A | b] of the row's frame (mats + 12 * frame, or one matrix for all); w = the 4th
// column of (n, 4) homogeneous rows, 1 for (n, 3) rows (CSIM:223-225's column of ones).  numpy's
// accumulation over k = 0..3 for a frame of several rows (dgemm): fma(b_i, w, fma(A_i2, z,
// fma(A_i1, y, A_i0 * x))); for a one-row frame, or every row with per_row (the reference's
// per-point loop, CSIM:2117-2141, one 4x1 product per point — numpy's dgemv):
// (A_i0 x + A_i2 z) + (A_i1 y + b_i w), every product rounded (tools/fma_order.py); out (n, 3).
// per_row == 2 (MC_AFFINE_TRANSLATE): p + b, the UTM branch's plain add (CSIM:2132).
__global__ __launch_bounds__(kBlock) void k_affine_rows_f64(const double* __restrict__ in, int64_t ld, int64_t n,
                                                            const int64_t* __restrict__ doff, int32_t F,
                                                            const double* __restrict__ mats, int32_t n_mats,
                                                            int per_row, double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int32_t f = row_frame(doff, F, i);
    const double* M = mats + (n_mats == 1 ? 0 : 12 * (int64_t)f);
    const bool single = per_row || doff[f + 1] - doff[f] == 1;
    const double* q = in + i * ld;
    const double x = q[0], y = q[1], z = q[2], w = ld == 4 ? q[3] : 1.0;
    double* o = out + 3 * i;
    if (per_row == 2) {
      o[0] = __dadd_rn(x, M[3]);
      o[1] = __dadd_rn(y, M[7]);
      o[2] = __dadd_rn(z, M[11]);
      continue;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma clang fp contract(off)
      const double* m = M + 4 * r;
      o[r] = single ? (m[0] * x + m[2] * z) + (m[1] * y + m[3] * w)
                    : __builtin_fma(m[3], w, __builtin_fma(m[2], z, __builtin_fma(m[1], y, m[0] * x)));
    }
  }
}

// CSIM coordinate transforms with matrices per frame on the f32 batch columns (mc_transform_affine)
__global__ __launch_bounds__(kBlock) void k_affine_w(const DeskewArgs a) { deskew_frame_body<true>(a); }

// ---------------------------------------------------------------------------------------------
// float64 per-point math.  Every per-point quantity (alpha, the interpolated quaternion / gyro, the
// angles, their sin / cos, the rotation, the translation) is formed in float64 from the float32
// point and the float64 tables, and each output coordinate is rounded once to float32 on the store:
// the result is the reference's float64 value to <= 2^-24 relative per coordinate (north_star:
// <= 1e-5 relative per coordinate, no scale floor).  FP64 FMA issues at the FP32 rate on CDNA4
// (16 lanes / SIMD / clock), so the cost is the operation count, kept low by polynomial tiers:
// cos(x) and sin(x)/x are even Taylor polynomials in z = x^2 whose length is picked per wave from
// a bound on |x| (truncation < 2e-17 relative in every tier):
//   tier 0  |x| <= 1/16   cos, sinc to z^4          (4 + 4 FMAs)
//   tier 1  |x| <= 1/4    cos, sinc to z^6          (6 + 6)
//   tier 2  |x| <= 1.6    cos, sinc to z^10         (10 + 10; SLERP's alpha*Theta <= Theta <= pi/2)
//   tier 3  any angle     Cody-Waite reduction + fdlibm kernels (sincos_prep; IMU gyro spikes)
// ---------------------------------------------------------------------------------------------

// Taylor coefficients of cos and sin(x)/x after the leading 1: c[k] of z^(k+1).  They live in
// constant memory and each tier's set is brought into SGPRs by one scalar load per wave where the
// tier is used (poly_load): as immediates the compiler would hoist all ~20 double constants out of
// the sub-tile loop into SGPR pairs and spill them (or keep them in VGPRs behind v_mov copies); as
// SGPR operands every Horner step is one v_fma_f64.  (Not `const`: the compiler would fold the
// initialiser back into immediates.)
template <int K>
struct Poly {
  double c[K];   // cos:  1 + sum c[k] z^(k+1)
  double s[K];   // sinc: 1 + sum s[k] z^(k+1)
};
struct NoPoly {};
#define MC_COS_C -1.0 / 2, 1.0 / 24, -1.0 / 720, 1.0 / 40320, -1.0 / 3628800, 1.0 / 479001600, \
    -1.0 / 87178291200.0, 1.0 / 20922789888000.0, -1.0 / 6402373705728000.0, 1.0 / 2432902008176640000.0
#define MC_SINC_C -1.0 / 6, 1.0 / 120, -1.0 / 5040, 1.0 / 362880, -1.0 / 39916800, 1.0 / 6227020800.0, \
    -1.0 / 1307674368000.0, 1.0 / 355687428096000.0, -1.0 / 121645100408832000.0, 1.0 / 51090942171709440000.0
__constant__ Poly<4> kPoly4 = {{-1.0 / 2, 1.0 / 24, -1.0 / 720, 1.0 / 40320},
                                     {-1.0 / 6, 1.0 / 120, -1.0 / 5040, 1.0 / 362880}};
__constant__ Poly<6> kPoly6 = {{-1.0 / 2, 1.0 / 24, -1.0 / 720, 1.0 / 40320, -1.0 / 3628800, 1.0 / 479001600},
                                     {-1.0 / 6, 1.0 / 120, -1.0 / 5040, 1.0 / 362880, -1.0 / 39916800,
                                      1.0 / 6227020800.0}};
__constant__ Poly<10> kPoly10 = {{MC_COS_C}, {MC_SINC_C}};
#undef MC_COS_C
#undef MC_SINC_C

template <int TIER>
using PolyOf = typename std::conditional<TIER == 0, Poly<4>,
               typename std::conditional<TIER == 1, Poly<6>,
               typename std::conditional<TIER == 2, Poly<10>, NoPoly>::type>::type>::type;

// an SGPR zero the compiler cannot see through: the coefficient load below stays where the tier
// is used instead of being hoisted out of the loop
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
template <int TIER>
__device__ __forceinline__ PolyOf<TIER> poly_load() {
  if constexpr (TIER == 0) return ldu(&kPoly4 + opaque_zero());
  else if constexpr (TIER == 1) return ldu(&kPoly6 + opaque_zero());
  else if constexpr (TIER == 2) return ldu(&kPoly10 + opaque_zero());
  else return NoPoly{};
}

template <int K>
__device__ __forceinline__ double horner1(const double (&c)[K], double z) {   // 1 + sum c[k] z^(k+1)
  double p = c[K - 1];
#pragma unroll
  for (int k = K - 2; k >= 0; --k) p = fma(z, p, c[k]);
  return fma(z, p, 1.0);
}
template <int K>
__device__ __forceinline__ void cos_sinc(const Poly<K>& P, double x, double& c, double& sc) {   // cos(x), sin(x)/x
  const double z = x * x;
  c = horner1<K>(P.c, z);
  sc = horner1<K>(P.s, z);
}
template <typename P>
__device__ __forceinline__ void sincos_tier(const P& poly, double x, double& s, double& c) {
  if constexpr (std::is_same<P, NoPoly>::value) {
    sincos_prep(x, &s, &c);
  } else {
    double sc;
    cos_sinc(poly, x, c, sc);
    s = x * sc;
  }
}

// quaternion SLERP + position LERP at the point's time tq, then p' = R(q) p + pos;
// alpha as the oracle's (t - t_k) / dt; the tier bounds alpha * Theta.  V: float (the batch's
// columns, one rounding per output coordinate on the store) or double (host float64 rows).
template <typename P, typename V>
__device__ __forceinline__ void slerp_core(const PoseWin& w, const P& poly, double tq, V& x, V& y, V& z) {
  double al = (tq - w.t0) * w.inv_dt;
  al = fmin(fmax(al, 0.0), 1.0);
  double cs, sc;
  cos_sinc(poly, al * w.th, cs, sc);
  const double s = al * sc;
  const double qx = fma(s, w.v[0], cs * w.q0[0]);
  const double qy = fma(s, w.v[1], cs * w.q0[1]);
  const double qz = fma(s, w.v[2], cs * w.q0[2]);
  const double qw = fma(s, w.v[3], cs * w.q0[3]);
  const double X = x, Y = y, Z = z;
  // v' = v + 2 (qw t + u x t), t = u x v
  const double tx = fma(qy, Z, -qz * Y);
  const double ty = fma(qz, X, -qx * Z);
  const double tz = fma(qx, Y, -qy * X);
  const double cx = fma(qw, tx, fma(qy, tz, -qz * ty));
  const double cy = fma(qw, ty, fma(qz, tx, -qx * tz));
  const double cz = fma(qw, tz, fma(qx, ty, -qy * tx));
  // (p + alpha dp) + p0 + 2c: one SGPR operand per instruction (no copies of the record into VGPRs)
  x = (V)fma(2.0, cx, fma(al, w.dp[0], X) + w.p0[0]);
  y = (V)fma(2.0, cy, fma(al, w.dp[1], Y) + w.p0[1]);
  z = (V)fma(2.0, cz, fma(al, w.dp[2], Z) + w.p0[2]);
}
// the time formed as the reference forms it, t_frame + t_ns * 1e-9 (no contraction)
__device__ __forceinline__ double slerp_time(double tf, double t_ns) { return __dadd_rn(tf, __dmul_rn(t_ns, 1e-9)); }
template <typename P>
__device__ __forceinline__ void slerp_point(const PoseWin& w, const P& poly, int t, float& x, float& y, float& z) {
  slerp_core(w, poly, slerp_time(w.tf, (double)t), x, y, z);
}

// Path B body (CSIM:1447-1465): w = g + alpha*dg (alpha from the bracketing IMU samples, CSIM:1504-
// 1511), theta = w * dt, dt = (t - frame start) * 1e-9 (CSIM:1454), p' = Rx(-theta_x) Ry(-theta_y)
// Rz(-theta_z) p (CSIM:1518-1536).  dts = t - ts of the record (exact), td = t - frame start (ns).
template <typename P, typename V>
__device__ __forceinline__ void imu_core(const ImuSeg& w, const P& poly, double dts, double td, V& x, V& y, V& z) {
  double al = dts * w.inv_dt;
  al = al > 0.0 ? al : 0.0;
  const double dt = td * 1e-9;
  double sa, ca, sb, cb, sc, cc;
  sincos_tier(poly, fma(al, w.dg[0], w.g[0]) * dt, sa, ca);
  sincos_tier(poly, fma(al, w.dg[1], w.g[1]) * dt, sb, cb);
  sincos_tier(poly, fma(al, w.dg[2], w.g[2]) * dt, sc, cc);
  const double X = x, Y = y, Z = z;
  // Rz(-c)
  const double x1 = fma(cc, X, sc * Y);
  const double y1 = fma(-sc, X, cc * Y);
  // Ry(-b)
  const double x2 = fma(cb, x1, -sb * Z);
  const double z2 = fma(sb, x1, cb * Z);
  // Rx(-a)
  const double y3 = fma(ca, y1, sa * z2);
  const double z3 = fma(-sa, y1, ca * z2);
  x = (V)x2; y = (V)y3; z = (V)z3;
}
// batch form: t = frame-relative int32 ns, tsd = (double)w.ts (frame-relative): t - ts is exact in
// float64 (both integers below 2^53)
template <typename P>
__device__ __forceinline__ void imu_point(const ImuSeg& w, const P& poly, double tsd, int t, float& x, float& y,
                                          float& z) {
  const double td = (double)t;
  imu_core(w, poly, td - tsd, td, x, y, z);
}

// window search: index of the window segment of frame-relative time t (bnd sorted, bnd[0] unused)
__device__ __forceinline__ int win_index(const int64_t* bnd, int W, int64_t t) {
  if (W <= 4) {
    int k = 0;
    for (int j = 1; j < W; ++j) k += (bnd[j] <= t) ? 1 : 0;
    return k;
  }
  int lo = 1, hi = W;   // count entries bnd[1..W) <= t
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (bnd[mid] <= t) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

template <int MODE>
using WinOf = typename std::conditional<MODE == 1, PoseWin, ImuSeg>::type;

// a scheduling fence between the points of a lane: the float64 bodies (~35 live VGPRs each) run
// one after the other instead of interleaved, which keeps the kernels at 4 waves / SIMD (128 VGPRs)
#define MC_POINT_FENCE __builtin_amdgcn_sched_barrier(0);

// one point with a wave-uniform record at a tier
template <int MODE, typename P>
__device__ __forceinline__ void point_at(const WinOf<MODE>& w, const P& poly, int t, float& x, float& y, float& z) {
  if constexpr (MODE == 1) slerp_point(w, poly, t, x, y, z);
  else imu_point(w, poly, (double)w.ts, t, x, y, z);
}
// the general tier of a mode (any angle)
template <int MODE>
constexpr int kTierAny = MODE == 1 ? 2 : 3;

// The 4 points of a lane's float4 group with ONE wave-uniform record (SGPRs) at the tier that
// covers every point of the wave.
template <int MODE, typename P>
__device__ __forceinline__ void points4(const WinOf<MODE>& w, const P& poly, const int4& Tq, float4& X, float4& Y,
                                        float4& Z) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    point_at<MODE>(w, poly, i4c(Tq, c), f4c(X, c), f4c(Y, c), f4c(Z, c));
    MC_POINT_FENCE
  }
}

// Points of one wave that fall into several segments (seg[c] = segment of the lane's point c, -1:
// no point): the wave peels the distinct segments off one at a time, smallest first — rec_of(j)
// returns segment j's record wave-uniformly (scalar loads, or LDS through readfirstlane), so no
// record ever sits in VGPRs and every path keeps the fast path's register budget.
__device__ __forceinline__ int wave_min_u(int v) { return __builtin_amdgcn_readfirstlane(wave_min(v)); }

template <typename T>
__device__ __forceinline__ T uniform_of(const T& v) {   // a value all lanes hold, moved to SGPRs
  static_assert(sizeof(T) % 4 == 0, "dword-multiple type");
  struct Raw { int v[sizeof(T) / 4]; };
  Raw r = __builtin_bit_cast(Raw, v);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) r.v[i] = __builtin_amdgcn_readfirstlane(r.v[i]);
  return __builtin_bit_cast(T, r);
}

template <int MODE, typename RecOf, typename P>
__device__ __forceinline__ void points_peeled(const int seg[4], RecOf rec_of, const P& poly, const int4& Tq, float4& X,
                                              float4& Y, float4& Z) {
  int pend = (seg[0] >= 0 ? 1 : 0) | (seg[1] >= 0 ? 2 : 0) | (seg[2] >= 0 ? 4 : 0) | (seg[3] >= 0 ? 8 : 0);
  while (__any(pend != 0)) {
    int cand = INT_MAX;
#pragma unroll
    for (int c = 0; c < 4; ++c) cand = ((pend >> c) & 1) ? min(cand, seg[c]) : cand;
    const int j = wave_min_u(cand);
    const WinOf<MODE> w = rec_of(j);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (((pend >> c) & 1) && seg[c] == j) {
        point_at<MODE>(w, poly, i4c(Tq, c), f4c(X, c), f4c(Y, c), f4c(Z, c));
        pend &= ~(1 << c);
      }
      MC_POINT_FENCE
    }
  }
}

// a or b by a wave-uniform condition, dword by dword (s_cselect; no private array)
template <typename T>
__device__ __forceinline__ T select_rec(bool second, const T& a, const T& b) {
  struct Raw { int v[sizeof(T) / 4]; };
  const Raw ra = __builtin_bit_cast(Raw, a), rb = __builtin_bit_cast(Raw, b);
  Raw r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) r.v[i] = second ? rb.v[i] : ra.v[i];
  return __builtin_bit_cast(T, r);
}

// The SGPR path of a window of <= 2 segments at tier TIER: each wave votes whether its points all
// sit in one segment; a wave across the boundary peels its two segments.
// set_tf (SLERP sub-tile windows): rec points into the segment table; its records get the frame time tf
// IMU (rec = segment klo of the step's IMU segment table): fs = the frame start (the table's
// absolute ns -> frame-relative), j1 = 1 inside the table, 0 at its last sample.
template <int MODE, int TIER>
__device__ __forceinline__ void fast_path(const WinOf<MODE>* rec, const FrameWin& fw, bool set_tf, double tf,
                                          bool act, const int4& Tq, float4& X, float4& Y, float4& Z,
                                          int64_t fs = 0, int j1 = 1) {
  const PolyOf<TIER> poly = poly_load<TIER>();
  auto load_rec = [&](int j) {
    WinOf<MODE> w = ldu(rec + j);
    if constexpr (MODE == 1) {
      if (set_tf) w.tf = tf;
    } else {
      w.ts -= fs;   // the segment table's absolute ns -> frame-relative
    }
    return w;
  };
  // IMU: both 64-byte records in SGPRs before the vote (their scalar-load latency then overlaps the
  // point loads instead of following the vote), the second one without waiting for the window's W
  // (slot j1 exists for every window); a 144-byte SLERP record pair would not fit
  WinOf<MODE> r0, r1;
  if constexpr (MODE == 2) {
    r0 = load_rec(0);
    r1 = load_rec(j1);
  }
  bool use1 = false, mixed = false;
  if (fw.W == 2) {
    const int64_t b1 = fw.bnd1;
    const bool any1 = act && ((int64_t)Tq.w >= b1 || (int64_t)Tq.x >= b1 || (int64_t)Tq.y >= b1 || (int64_t)Tq.z >= b1);
    const bool any0 = act && ((int64_t)Tq.w < b1 || (int64_t)Tq.x < b1 || (int64_t)Tq.y < b1 || (int64_t)Tq.z < b1);
    const bool w1 = __any(any1), w0 = __any(any0);
    use1 = w1 && !w0;
    mixed = w1 && w0;
  }
  if (!mixed) {
    // every lane computes (a partial wave's idle lanes on zeros, their results never stored): under
    // `if (act)` the compiler sank the record load into the divergent block as 9 per-lane vector
    // loads of the 144-byte record instead of scalar loads
    WinOf<MODE> w;
    if constexpr (MODE == 2) w = select_rec(use1, r0, r1);
    else w = load_rec(use1 ? 1 : 0);
    points4<MODE>(w, poly, Tq, X, Y, Z);
  } else {
    int seg[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) seg[c] = act ? ((int64_t)i4c(Tq, c) >= fw.bnd1 ? 1 : 0) : -1;
    if constexpr (MODE == 2)
      points_peeled<MODE>(seg, [&](int j) { return select_rec(j != 0, r0, r1); }, poly, Tq, X, Y, Z);
    else
      points_peeled<MODE>(seg, [&](int j) { return load_rec(j); }, poly, Tq, X, Y, Z);
  }
}

// Per-point modes: MODE 1 = SLERP, MODE 2 = IMU.  A workgroup works on a sub-tile of kBlock
// float4 groups (1024 points of one frame).  The frame's segment window (k_prep) decides the path,
// uniformly for the whole workgroup:
//   W <= 2      both frame-specialised records come in through scalar loads (SGPRs); each wave
//               votes whether its points all sit in one segment (no LDS, no barrier) and picks the
//               polynomial tier that covers its angles; a wave across the boundary peels its two
//               segments;
//   W <= 64     the window's records are staged into LDS once (one barrier), each point picks its
//               segment by searching the boundaries, the wave peels the segments it holds;
//   W > 64      pathological span: per-point search of the global tables, peeled the same way.
// NEXT: the launch also runs the next step's prep in its first `pre` workgroups (see the
// k_deskew_frame_next comment)
// (NEXT: at least 4 waves / SIMD like the plain kernel — the prep body alone would take 172 VGPRs)
// PCD (mc_deskew_pcd): a wave's 64 groups are one 256-point block of the output batch; it also
// writes that block's ASCII PCD text bytes (a wave reduction, no barrier).
template <int MODE, bool NEXT = false, bool PCD = false>
__global__ __launch_bounds__(kBlock, kPointsWaves) void k_deskew_points(const DeskewArgs a, const PrepArgs pn,
                                                                         const uint32_t pre) {
  span_start(a.span);
  if constexpr (NEXT) {
    if (blockIdx.x < pre) {
      prep_body<MODE>(pn, blockIdx.x);
      return;
    }
  }
  using Win = WinOf<MODE>;
  __shared__ Win s_win[kWinMax];
  __shared__ int64_t s_bnd[kWinMax];
  const int tid = threadIdx.x;
  const int64_t n_sub = (int64_t)a.n_tiles * kSub;
  const Win* frec = reinterpret_cast<const Win*>(a.frec);

  const uint32_t b0 = NEXT ? blockIdx.x - pre : blockIdx.x, nb = NEXT ? gridDim.x - pre : gridDim.x;
  // the points of sub-tile st of tile tl, every lane (a short sub-tile's idle lanes re-read its first
  // group, an empty sub-tile's lanes the tile's first group; their results are never stored): no
  // divergent load block, so nothing makes the point loads wait for the window records, and the
  // records stay scalar loads in uniform control flow
  auto load_sub = [&](int64_t st, const Tile& tl, int4& Tq, float4& X, float4& Y, float4& Z, float4& I) {
    const int g0 = (int)(st % kSub) * kBlock;
    const int g = g0 + tid;
    const int gl = g < tl.ngroups ? g : (g0 < tl.ngroups ? g0 : 0);
    const float* q = a.in + bidx((int)a.in_C, 0, tl.pstart + 4 * (int64_t)gl);
    Tq = ld4(reinterpret_cast<const int32_t*>(q + 4 * kBlkPts));
    X = ld4(q);
    Y = ld4(q + kBlkPts);
    Z = ld4(q + 2 * kBlkPts);
    I = ld4(q + 3 * kBlkPts);
  };
  // one non-empty sub-tile whose points are loaded: records, per-point math, stores
  auto sub_tile = [&](const int64_t st, const Tile& tl, const FrameWin& fw_first, const int4& Tq, float4 X, float4 Y,
                      float4 Z, const float4& I) {
    const int g0 = (int)(st % kSub) * kBlock;
    const int f = tl.frame;
    const int g = g0 + tid;
    const bool act = g < tl.ngroups;
    const int64_t p = tl.pstart + 4 * (int64_t)g;
    // frames wider than the SGPR path take their sub-tile's own window (k_prep writes one for every
    // IMU sub-tile, loaded by the caller beside the tile record).  One scalar load of the chosen
    // record (a select of two loaded structs became a vector load of bnd1 whose wait held back the
    // point loads)
    bool sub = true;
    if constexpr (MODE != 2) sub = ldu(a.fwin + f).W > kFastMaxW;
    const FrameWin fw = MODE == 2 ? fw_first : ldu(sub ? a.swin + st : a.fwin + f);
    // sub-tile windows point into the step's segment table (SLERP: whose records carry no frame time)
    const Win* rec = sub ? (MODE == 1 ? reinterpret_cast<const Win*>(a.pose_seg) : reinterpret_cast<const Win*>(a.imu_seg)) + fw.klo
                         : frec + 2 * f;
    const bool set_tf = MODE == 1 && sub;

    if (fw.W <= kFastMaxW) {
      // the tier k_prep chose for the window: its coefficient load is issued here, beside the point
      // loads, not behind the vote that needs them
      const double tf = set_tf ? ldu(a.frame_time + f) : 0.0;
      // IMU segment-table records: the frame start, and slot 1 only inside the table
      const int64_t fs = MODE == 2 ? ldu(a.frame_start + f) : 0;
      const int j1 = MODE == 2 ? (fw.klo + 1 < a.ntab ? 1 : 0) : 1;
      if (fw.tier == 0) fast_path<MODE, 0>(rec, fw, set_tf, tf, act, Tq, X, Y, Z, fs, j1);
      else if (fw.tier == 1) fast_path<MODE, 1>(rec, fw, set_tf, tf, act, Tq, X, Y, Z, fs, j1);
      else fast_path<MODE, kTierAny<MODE>>(rec, fw, set_tf, tf, act, Tq, X, Y, Z, fs, j1);
    } else if (fw.W <= kWinMax) {
      const int W = fw.W;
      if (tid < W) {
        const int64_t k = fw.klo + tid;
        if constexpr (MODE == 1) {
          const double tf = a.frame_time[f];
          s_win[tid] = make_pose_win(a.pose_seg[k], tf);
          s_bnd[tid] = rel_ns_ceil(a.pose_time[k], tf);
        } else {
          ImuSeg sg = a.imu_seg[k];
          sg.ts -= a.frame_start[f];
          s_win[tid] = sg;
          s_bnd[tid] = sg.ts;
        }
      }
      __syncthreads();
      int seg[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) seg[c] = act ? win_index(s_bnd, W, (int64_t)i4c(Tq, c)) : -1;
      points_peeled<MODE>(seg, [&](int j) { return uniform_of(s_win[j]); }, poly_load<kTierAny<MODE>>(), Tq, X, Y, Z);
      __syncthreads();  // the LDS window is rewritten by the next sub-tile
    } else {
      // pathological span (> kWinMax segments in one sub-tile): each point's segment from the
      // global tables (binary search), as the oracle selects it
      int seg[4];
      if constexpr (MODE == 1) {
        const double tf = a.frame_time[f];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int64_t k = upper_bound(a.pose_time, a.ntab, __dadd_rn(tf, __dmul_rn((double)i4c(Tq, c), 1e-9))) - 1;
          k = k > a.nseg - 1 ? a.nseg - 1 : (k < 0 ? 0 : k);
          seg[c] = act ? (int)k : -1;
        }
        points_peeled<MODE>(seg, [&](int j) { return make_pose_win(ldu(a.pose_seg + j), tf); },
                            poly_load<kTierAny<MODE>>(), Tq, X, Y, Z);
      } else {
        const int64_t fs = a.frame_start[f];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int64_t k = upper_bound(a.imu_ts, a.ntab, fs + (int64_t)i4c(Tq, c)) - 1;
          seg[c] = act ? (int)(k < 0 ? 0 : k) : -1;
        }
        points_peeled<MODE>(seg, [&](int j) {
          ImuSeg w = ldu(a.imu_seg + j);
          w.ts -= fs;
          return w;
        }, poly_load<kTierAny<MODE>>(), Tq, X, Y, Z);
      }
    }
    if (act) {
      float* o = a.out + bidx((int)a.out_C, 0, p);
      st_out(o, X);
      st_out(o + kBlkPts, Y);
      st_out(o + 2 * kBlkPts, Z);
      st_out(o + 3 * kBlkPts, I);
      if (a.copy_t) st_out(o + 4 * kBlkPts, __builtin_bit_cast(float4, Tq));
    }
    if constexpr (PCD) {
      const int64_t i0 = p - ldu(a.fpoff + f), n = ldu(a.fcount + f);
      PcdCount pc;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool v = act && i0 + c < n;
        pc.add2(v, f4g(X, c), f4g(Y, c));
        pc.add2(v, f4g(Z, c), f4g(I, c));
      }
      const int bytes = pc.bytes();      // (every lane: the per-lane variant reduces across the wave)
      const int wg = g0 + (tid & ~63);   // the wave's first group
      if ((tid & 63) == 0 && wg < tl.ngroups) a.pcd_len[(tl.pstart + 4 * (int64_t)wg) >> 8] = bytes;
    }
  };
  // the sub-tile window of an IMU sub-tile does not depend on the tile record, so both scalar loads
  // are in flight together instead of one behind the other
  auto win_first = [&](int64_t st) {
    FrameWin w{};
    if constexpr (MODE == 2) w = ldu(a.swin + st);
    return w;
  };
  for (int64_t it = b0; it < n_sub; it += nb) {
    const int64_t st = nb < n_sub ? it : (a.xcd_order ? xcd_unit<1>(it, n_sub) : it);
    const FrameWin w = win_first(st);
    const Tile tl = ldu(a.tiles + st / kSub);
    if ((int)(st % kSub) * kBlock >= tl.ngroups) continue;  // uniform: empty sub-tile of a short tile
    int4 Tq;
    float4 X, Y, Z, I;
    load_sub(st, tl, Tq, X, Y, Z, I);
    sub_tile(st, tl, w, Tq, X, Y, Z, I);
  }
  span_end(a.span);
}

// ---- the next step's prep inside this step's launch (mc_deskew_steps) --------------------------
// Workgroups [0, pre) run k_prep's body for the NEXT step (its table half), the rest this step's
// deskew over the half the previous launch's prep wrote.  The two halves never alias, and the
// kernel boundary orders the prep's stores before the next launch's reads, so no flag or fence
// inside the launch; the prep workgroups are dispatched first and finish beside the first deskew
// workgroups instead of as a dependent kernel on the queue (~5 us per step).  pre is a multiple of
// the XCD count, so deskew workgroup b - pre sits on the XCD xcd_unit assumes.
__global__ __launch_bounds__(kBlock, 4) void k_deskew_frame_next(const DeskewArgs a, const PrepArgs p,
                                                                 const uint32_t pre) {
  span_start(a.span);
  if (blockIdx.x < pre) {
    prep_body<0>(p, blockIdx.x);
    return;
  }
  deskew_frame_quad(a, pre);
  span_end(a.span);
}

// ---- per-point modes on float64 rows (the reference's own data, no float32 staging) --------------
// The drop-in entry points (MotionCompensator.compensate_point_cloud / compensate_arrays /
// apply_motion_compensation, CSIM:1435-1480 / 2086-2105; LiDARMotionSimulator.deskew_frames) hand
// over float64 coordinates that float32 columns would round by up to 6e-8 |p| — enough to miss
// 1e-5 relative on a coordinate that rotates to near zero.  Here every point is read, computed and
// written in float64 (rows of pinned host memory for small calls, of a device staging buffer for
// large ones): one thread per point, its frame by a binary search of the frame offsets, its
// segment by a binary search of the pose / IMU time table as the oracle selects it (LMC:804-style
// searchsorted 'right' - 1, clamped), the record from the segment table k_prep built (PoseSeg /
// ImuSeg), and the batch kernels' own per-point math (slerp_core / imu_core) at the general tier.
// PCIe-bound by construction (40-56 B of host traffic per point); never the bench's `value`.
struct PointsF64Args {
  const double* pts; int64_t ld; int64_t n;   // (n, ld) rows, ld >= 3: x, y, z [, intensity, ...]
  const int64_t* t_ns;                        // per point, ns since its frame's start
  const int64_t* doff; int32_t F;             // frame f = rows [doff[f], doff[f+1])
  const double* ftime;                        // SLERP: frame time (s) per frame
  const int64_t* fstart;                      // IMU: frame start (ns) per frame
  const double* pose_time; const PoseSeg* pose_seg; int64_t nseg;
  const int64_t* imu_ts; const ImuSeg* imu_seg;
  int64_t ntab;                               // T or M
  double* out;                                // (n, 4): x', y', z', column 3 (0 when ld == 3)
};

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_points_f64(const PointsF64Args a) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * kBlock) {
    int32_t lo = 0, hi = a.F;                    // last f with doff[f] <= i
    while (hi - lo > 1) {
      const int32_t mid = (lo + hi) >> 1;
      if (a.doff[mid] <= i) lo = mid; else hi = mid;
    }
    const double* q = a.pts + i * a.ld;
    double x = q[0], y = q[1], z = q[2];
    const double w = a.ld > 3 ? q[3] : 0.0;
    const int64_t t = a.t_ns[i];
    if constexpr (MODE == 1) {
      const double tf = a.ftime[lo];
      const double tq = slerp_time(tf, (double)t);
      int64_t k = upper_bound(a.pose_time, a.ntab, tq) - 1;
      k = k > a.nseg - 1 ? a.nseg - 1 : (k < 0 ? 0 : k);
      slerp_core(a.pose_seg[k], kPoly10, tq, x, y, z);
    } else {
      const int64_t ta = a.fstart[lo] + t;       // the point's absolute timestamp (CSIM:1447)
      int64_t k = upper_bound(a.imu_ts, a.ntab, ta) - 1;
      k = k < 0 ? 0 : k;                         // before the first sample: the first (CSIM:1496)
      const ImuSeg sg = a.imu_seg[k];
      imu_core(sg, NoPoly{}, (double)(ta - sg.ts), (double)t, x, y, z);
    }
    double* o = a.out + 4 * i;
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
  }
}

// ---------------------------------------------------------------------------------------------
// layout / staging kernels (not the per-step path; PCIe-bound when fed from the host)
// ---------------------------------------------------------------------------------------------
struct LayoutArgs {
  const Tile* tiles; int32_t n_tiles;
  const int64_t* poff; const int64_t* doff; const int64_t* counts;
  float* cols; int32_t C;   // blocked columns x|y|z|i[|t_ns]; C == 5 carries the t_ns column
  int64_t dbase;            // AoS row of the first frame covered (a frame range's fetch: doff[f0]; else 0)
  int32_t* pcd_len;         // stager, MC_BATCH_WITH_PCD_LEN: ASCII PCD bytes per 256-point block, or nullptr
  __device__ __forceinline__ float& col(int c, int64_t p) const { return cols[bidx(C, c, p)]; }
  __device__ __forceinline__ int32_t& tns(int64_t p) const {
    return reinterpret_cast<int32_t*>(cols)[bidx(C, 4, p)];
  }
};

// per element of the padded layout: its frame-local index, or -1 for a padding slot
__device__ __forceinline__ int64_t local_index(const LayoutArgs& a, const Tile& tl, int64_t p) {
  const int64_t i = p - a.poff[tl.frame];
  return i < a.counts[tl.frame] ? i : -1;
}

// The stager pair: the reference's (N, ld) float64 AoS [x,y,z,intensity,...]
// (LMC:770) <-> the padded SoA float32 columns, both on the device.  48 algorithmic bytes per
// point either way.
//
// 256-point units: a workgroup moves 256 points (64 float4 groups, one 256-point block of the batch)
// per unit, so every lane issues ONE 16-byte load and two 16-byte stores (SoA -> AoS) or two loads and
// one store (AoS -> SoA), each wave instruction covering 1 KB contiguous on both sides, transposed
// through a 4 KB LDS tile; non-temporal loads and stores (st_pol<1>).  Bare streams of these lane
// shapes: 6.11 TB/s (16 B in / 32 B out, 1 / 2 per lane) vs 5.22-5.34 with a 2048-point tile's 8 / 16
// per lane; 6.42 TB/s (32 B in / 16 B out, 2 / 1) (tools/stage_probe.hip, profiles/round2/s07).
// Rejected (profiles/HISTORY_r1-r4.md §4, §9): 2048-point LDS tiles (71 / 75 % of peak), register-only quad transposes
// (16-byte holes in every row-side store, profiles/round2/s11-s12), 2 / 4 units per workgroup pass
// (profiles/round3/s09), sc1 / sc1 nt stores (s31), the dealt unit order (s57).
typedef double v2d __attribute__((ext_vector_type(2)));
constexpr int kStageSt = 1;                                // st_pol policy of the stager stores (nt)
constexpr int kStageQuarters = kTileGroups / kQuadGroups;  // 256-point units per tile
constexpr int kUnitRow = kQuadGroups * 4 + 4;              // LDS floats per column (+4: banks)

__device__ __forceinline__ void soa_to_aos_unit(const LayoutArgs& a, double* __restrict__ aos) {
  __shared__ float s[4 * kUnitRow];
  const int64_t n_units = (int64_t)a.n_tiles * kStageQuarters;
  const int t = threadIdx.x;
  for (int64_t it = blockIdx.x; it < n_units; it += gridDim.x) {
    const int64_t un = gridDim.x >= n_units ? xcd_unit<MC_XCD_STAGE>(it, n_units) : it;
    const Tile tl = ldu(a.tiles + un / kStageQuarters);
    const int g0 = (int)(un % kStageQuarters) * kQuadGroups;
    if (g0 >= tl.ngroups) continue;   // uniform
    const int64_t poff = ldu(a.poff + tl.frame), doff = ldu(a.doff + tl.frame), cnt = ldu(a.counts + tl.frame);
    const int64_t p0 = tl.pstart + 4 * (int64_t)g0;   // first point of the unit (a block boundary)
    // column c = t >> 6 of group t & 63: one wave = one column's 1 KB run
    const int c = t >> 6, gi = t & 63;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g0 + gi < tl.ngroups) v = ld4(a.cols + bidx(a.C, c, p0 + 4 * gi));
    *reinterpret_cast<float4*>(&s[c * kUnitRow + 4 * gi]) = v;
    __syncthreads();
    // rows: chunk i = row i >> 1, half i & 1 (x, y | z, w); lane t stores chunks t and 256 + t
    const int64_t loc0 = p0 - poff;
    v2d* d = reinterpret_cast<v2d*>(aos + (doff - a.dbase + loc0) * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + u * kBlock, r = i >> 1, h = i & 1;
      if (loc0 + r < cnt) {
        const v2d w = {(double)s[(2 * h) * kUnitRow + r], (double)s[(2 * h + 1) * kUnitRow + r]};
        st_pol<kStageSt>(reinterpret_cast<float*>(d + i), __builtin_bit_cast(float4, w));
      }
    }
    __syncthreads();   // s is rewritten by the next unit
  }
}

// pcd_len: wave c also sums column c's text bytes over the unit's valid points (PcdCount, one
// wave reduction); the four waves' sums meet in LDS and lane 0 of wave 0 writes the block's total.
__device__ __forceinline__ void aos_to_soa_unit(const LayoutArgs& a, const double* __restrict__ aos) {
  __shared__ float s[4 * kUnitRow];
  __shared__ int s_part[4];
  const int64_t n_units = (int64_t)a.n_tiles * kStageQuarters;
  const int t = threadIdx.x;
  for (int64_t it = blockIdx.x; it < n_units; it += gridDim.x) {
    const int64_t un = gridDim.x >= n_units ? xcd_unit<MC_XCD_STAGE>(it, n_units) : it;
    const Tile tl = ldu(a.tiles + un / kStageQuarters);
    const int g0 = (int)(un % kStageQuarters) * kQuadGroups;
    if (g0 >= tl.ngroups) continue;   // uniform
    const int64_t poff = ldu(a.poff + tl.frame), doff = ldu(a.doff + tl.frame), cnt = ldu(a.counts + tl.frame);
    const int64_t p0 = tl.pstart + 4 * (int64_t)g0;
    const int64_t loc0 = p0 - poff;
    const v2d* s2 = reinterpret_cast<const v2d*>(aos + (doff + loc0) * 4);
    v2d w[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {   // both loads in flight before the LDS writes
      const int i = t + u * kBlock;
      w[u] = (loc0 + (i >> 1) < cnt) ? __builtin_nontemporal_load(s2 + i) : v2d{0.0, 0.0};   // padding: zeros
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + u * kBlock, r = i >> 1, h = i & 1;
      s[(2 * h) * kUnitRow + r] = (float)w[u].x;
      s[(2 * h + 1) * kUnitRow + r] = (float)w[u].y;
    }
    __syncthreads();
    const int c = t >> 6, gi = t & 63;
    const float4 v = *reinterpret_cast<const float4*>(&s[c * kUnitRow + 4 * gi]);
    if (g0 + gi < tl.ngroups) st_pol<kStageSt>(a.cols + bidx(a.C, c, p0 + 4 * gi), v);
    if (a.pcd_len) {   // uniform
      PcdCount pc;
      const int64_t r0 = loc0 + 4 * gi;
      pc.add2(r0 < cnt, v.x, r0 + 1 < cnt, v.y);
      pc.add2(r0 + 2 < cnt, v.z, r0 + 3 < cnt, v.w);
      const int bytes = pc.bytes();
      if (gi == 0) s_part[c] = bytes;
    }
    __syncthreads();
    if (a.pcd_len && t == 0) a.pcd_len[p0 >> 8] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
  }
}

// AoS f64 (dense, row stride ld) -> padded SoA f32 (padding slots zeroed)
__global__ __launch_bounds__(kBlock) void k_aos_to_soa(const LayoutArgs a, const double* __restrict__ aos, int64_t ld) {
  if (ld == 4) {
    aos_to_soa_unit(a, aos);
    return;
  }
  // wider rows (ld > 4: extra columns the reference carries along): one point per lane, one
  // 256-point block (kBlock lanes) per pass, so a block's PCD text bytes are one workgroup sum
  __shared__ int s_part[kBlock / 64];
  for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const Tile tl = ldu(a.tiles + tile);
    const int64_t poff = ldu(a.poff + tl.frame), doff = ldu(a.doff + tl.frame), cnt = ldu(a.counts + tl.frame);
    const int64_t loc0 = tl.pstart - poff;
    const int np = 4 * tl.ngroups;                                      // padded points in the tile
    const int64_t rest = min_i64(np, cnt - loc0);
    const int nv = rest > 0 ? (int)rest : 0;                          // valid ones
    const double* src = aos + (doff + loc0) * ld;
    for (int j0 = 0; j0 < np; j0 += kBlock) {
      const int j = j0 + (int)threadIdx.x;
      float r[4] = {0.f, 0.f, 0.f, 0.f};
      if (j < nv)
        for (int c = 0; c < 4; ++c) r[c] = (float)src[(int64_t)j * ld + c];
      if (j < np)
        for (int c = 0; c < 4; ++c) a.col(c, tl.pstart + j) = r[c];
      if (a.pcd_len) {   // uniform; j0 is a block boundary (tiles start on one)
        PcdCount pc;
        pc.add2(j < nv, r[0], r[1]);
        pc.add2(j < nv, r[2], r[3]);
        const int bytes = pc.bytes();
        if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = bytes;
        __syncthreads();
        if (threadIdx.x == 0) a.pcd_len[(tl.pstart + j0) >> 8] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        __syncthreads();
      }
    }
  }
}

// padded SoA f32 -> dense AoS (N,4) f64  (the (N,4) float64 layout LMC:776 returns)
__global__ __launch_bounds__(kBlock) void k_soa_to_aos(const LayoutArgs a, double* __restrict__ aos) {
  soa_to_aos_unit(a, aos);
}

// dense column (N) <-> blocked column c; DIR 0: dense->blocked (padding zeroed), 1: blocked->dense
template <typename T, int DIR>
__global__ __launch_bounds__(kBlock) void k_column(const LayoutArgs a, int c, const T* __restrict__ src,
                                                   T* __restrict__ dst) {
  T* colv = reinterpret_cast<T*>(a.cols);
  for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const Tile tl = a.tiles[tile];
    const int64_t d0 = a.doff[tl.frame];
    for (int e = threadIdx.x; e < 4 * tl.ngroups; e += kBlock) {
      const int64_t p = tl.pstart + e;
      const int64_t i = local_index(a, tl, p);
      if (DIR == 0) colv[bidx(a.C, c, p)] = i >= 0 ? src[d0 + i] : T(0);
      else if (i >= 0) dst[d0 + i] = colv[bidx(a.C, c, p)];
    }
  }
}

// per-frame [min, max] of t_ns over the valid points (feeds k_prep's frame windows)
__global__ __launch_bounds__(kBlock) void k_trange_init(int2* tr, int32_t F) {
  const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (f < F) tr[f] = make_int2(INT_MAX, INT_MIN);
}
// ... and per sub-tile (kBlock float4 groups), feeding k_prep's sub-tile windows
__global__ __launch_bounds__(kBlock) void k_trange(const LayoutArgs a, int2* tr, int2* str) {
  __shared__ int s_lo[kSub][kBlock / 64], s_hi[kSub][kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const Tile tl = a.tiles[tile];
    int flo = INT_MAX, fhi = INT_MIN;
#pragma unroll
    for (int j = 0; j < kSub; ++j) {
      int lo = INT_MAX, hi = INT_MIN;
      const int e_end = min(4 * tl.ngroups, (j + 1) * 4 * kBlock);
      for (int e = j * 4 * kBlock + threadIdx.x; e < e_end; e += kBlock) {
        const int64_t p = tl.pstart + e;
        if (local_index(a, tl, p) >= 0) {
          const int t = a.tns(p);
          lo = min(lo, t);
          hi = max(hi, t);
        }
      }
      lo = wave_min(lo);
      hi = wave_max(hi);
      if (lane == 0) { s_lo[j][wid] = lo; s_hi[j][wid] = hi; }
      flo = min(flo, lo);
      fhi = max(fhi, hi);
    }
    if (lane == 0 && flo <= fhi) {
      atomicMin(&tr[tl.frame].x, flo);
      atomicMax(&tr[tl.frame].y, fhi);
    }
    __syncthreads();
    if (threadIdx.x < kSub) {
      int lo = INT_MAX, hi = INT_MIN;
      for (int w = 0; w < kBlock / 64; ++w) { lo = min(lo, s_lo[threadIdx.x][w]); hi = max(hi, s_hi[threadIdx.x][w]); }
      str[tile * kSub + threadIdx.x] = make_int2(lo, hi);
    }
    __syncthreads();
  }
}

// ---- synthetic Mid-70 frames (bit-identical to oracle/synth.py) ------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ float u24(uint64_t h) { return (float)(uint32_t)(h >> 40) * 0x1.0p-24f; }

__global__ __launch_bounds__(kBlock) void k_synth(const LayoutArgs a, uint64_t seed, int64_t fid_base) {
#pragma clang fp contract(off)
  for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const Tile tl = a.tiles[tile];
    const int64_t n = a.counts[tl.frame];
    const uint64_t key = mix64((seed + (uint64_t)fid_base + (uint64_t)tl.frame) * kGamma);
    for (int e = threadIdx.x; e < 4 * tl.ngroups; e += kBlock) {
      const int64_t p = tl.pstart + e;
      const int64_t i = local_index(a, tl, p);
      float x = 0.f, y = 0.f, z = 0.f, in = 0.f;
      int32_t t = 0;
      if (i >= 0) {
        const uint64_t c = 4ull * (uint64_t)i;
        const float u0 = u24(mix64(key + (c + 1) * kGamma));
        const float u1 = u24(mix64(key + (c + 2) * kGamma));
        const float u2 = u24(mix64(key + (c + 3) * kGamma));
        const float u3 = u24(mix64(key + (c + 4) * kGamma));
        x = u0 * 0x1.67cccc0p+6f + 0x1.99999a0p-5f;           // depth 0.05 .. 90 m
        const float ah = (u1 * 2.0f - 1.0f) * 0x1.692d20p-1f;  // tan(35.2 deg) half FOV (CSIM:66)
        const float av = (u2 * 2.0f - 1.0f) * 0x1.98b968p-1f;  // tan(38.6 deg) half FOV (CSIM:67)
        y = x * ah;
        z = x * av;
        in = u3;
        t = (int32_t)((i * 100000000ll) / n);                  // spread over the 0.1 s frame
      }
      a.col(0, p) = x; a.col(1, p) = y; a.col(2, p) = z; a.col(3, p) = in;
      if (a.C == 5) a.tns(p) = t;
    }
  }
}

// per-tile f64 partial sums of x,y,z,i,t over valid points (deterministic tree; host sums tiles)
__global__ __launch_bounds__(kBlock) void k_checksum(const LayoutArgs a, double* __restrict__ partial) {
  __shared__ double s[5][kBlock];
  for (int64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const Tile tl = a.tiles[tile];
    double acc[5] = {0, 0, 0, 0, 0};
    for (int e = threadIdx.x; e < 4 * tl.ngroups; e += kBlock) {
      const int64_t p = tl.pstart + e;
      if (local_index(a, tl, p) >= 0) {
        for (int c = 0; c < 4; ++c) acc[c] += (double)a.col(c, p);
        if (a.C == 5) acc[4] += (double)a.tns(p);
      }
    }
    for (int c = 0; c < 5; ++c) s[c][threadIdx.x] = acc[c];
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w)
        for (int c = 0; c < 5; ++c) s[c][threadIdx.x] += s[c][threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x < 5) partial[tile * 5 + threadIdx.x] = s[threadIdx.x][0];
    __syncthreads();
  }
}

}  // namespace mc
